#!/bin/bash
# Routed N = 1 (bench.py --route): kernel trace per library (in-tree, then
# build_abl/lib_*.so): GPU busy fraction and per-kernel time per batch over 40
# timed batches (scripts/trace_busy.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "" build_abl/lib_*.so; do
  tag=$(basename "${lib:-cur}" .so)
  rm -rf gpurun_out/rtrace_$tag && mkdir -p gpurun_out/rtrace_$tag
  RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rtrace_$tag -o run -- \
    python -u bench.py --route --steps 100 --warmup 3 --latency-steps 3 --pcie-steps 0 --no-cpu-baseline ${KARGS} \
    > gpurun_out/rtrace_$tag.log 2>&1 || { tail -5 gpurun_out/rtrace_$tag.log; exit 1; }
  echo "== $tag"
  python scripts/trace_busy.py gpurun_out/rtrace_$tag/run_kernel_trace.csv 40 > gpurun_out/rtrace_${tag}_busy.txt && \
    head -12 gpurun_out/rtrace_${tag}_busy.txt
  rm -f gpurun_out/rtrace_$tag/run_kernel_trace.csv
done
