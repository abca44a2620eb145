#!/bin/bash
# rocprofv3 kernel trace (per-dispatch start/end) + stats of a short bench run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
out=gpurun_out/trace${TAG}
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
  python -u bench.py --steps 10 --warmup 2 --latency-steps 3 --no-cpu-baseline --no-fill ${BENCH_ARGS} \
  > $out/bench.log 2>&1 || { tail -30 $out/bench.log; exit 1; }
tail -1 $out/bench.log
find $out -name "*.csv" | head
