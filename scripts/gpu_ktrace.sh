#!/bin/bash
# Kernel trace of one bench command; per-kernel medians over the last TAIL launches.
#   KARGS  bench.py arguments (default: C1 serial = isolated kernels)
#   TAG    output name: gpurun_out/ktrace_<TAG>/ (+ _tail.json)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-c1_serial}
rm -rf gpurun_out/ktrace_$TAG && mkdir -p gpurun_out/ktrace_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktrace_$TAG -o run -- \
  python -u bench.py --steps 50 --warmup 3 --latency-steps 3 --pcie-steps 0 --no-cpu-baseline --prof-every 0 \
  ${KARGS:---config c1 --serial} > gpurun_out/ktrace_$TAG.log 2>&1 || { tail -20 gpurun_out/ktrace_$TAG.log; exit 1; }
tail -1 gpurun_out/ktrace_$TAG.log | cut -c1-200
f=$(find gpurun_out/ktrace_$TAG -name "*kernel_trace.csv" | head -1)
python scripts/kstats_tail.py "$f" ${TAIL:-50} gpurun_out/ktrace_${TAG}_tail.json
rm -f "$f"
