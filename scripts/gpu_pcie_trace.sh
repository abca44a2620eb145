#!/bin/bash
# Memory-copy + kernel trace of the host-fed (PCIe) phase of the default bench
# (short device phase), summarised by scripts/copy_timeline.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/pcie_trace && mkdir -p gpurun_out/pcie_trace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/pcie_trace -o run -- \
  python -u bench.py --steps 20 --warmup 3 --latency-steps 3 --no-cpu-baseline --prof-every 0 --pcie-steps 30 ${KARGS:-} \
  > gpurun_out/pcie_trace.log 2>&1 || { tail -20 gpurun_out/pcie_trace.log; exit 1; }
tail -1 gpurun_out/pcie_trace.log | cut -c1-200
python scripts/copy_timeline.py gpurun_out/pcie_trace > gpurun_out/pcie_timeline.txt 2>&1; cat gpurun_out/pcie_timeline.txt
