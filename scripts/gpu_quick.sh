#!/bin/bash
# Parity tests, C1/C2 bench and a kernel-trace timeline (each step time-limited).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -40 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1 || { tail -40 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log
bash scripts/gpu_trace.sh
