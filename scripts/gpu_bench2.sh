#!/bin/bash
# Bench C1 and C2 and a rocprofv3 kernel summary of each (short runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c1 gpurun_out/prof_c2
for cfg in c1 c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-400
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o run -- \
    python -u bench.py --config $cfg --steps 10 --warmup 2 --latency-steps 5 --no-cpu-baseline --no-fill > gpurun_out/prof_bench_$cfg.log 2>&1 \
    || { tail -30 gpurun_out/prof_bench_$cfg.log; exit 1; }
  f=$(find gpurun_out/prof_$cfg -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-4 "$f" | sed 's/(.*)"/"/' | head -24
done
