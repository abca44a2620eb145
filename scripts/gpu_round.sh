#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench (each step under its own time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
