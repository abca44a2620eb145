#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (no PMC counters here).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python -u bench.py --steps 10 --warmup 2 --latency-steps 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1 \
  || { tail -30 gpurun_out/prof_bench.log; exit 1; }
tail -1 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -20 "$f"
