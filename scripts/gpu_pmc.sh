#!/bin/bash
# HBM traffic per kernel from rocprofv3 PMC counters: one pass per counter
# (FETCH_SIZE and WRITE_SIZE do not fit one pass), first over the calibration
# probe (tools/pmcprobe.hip: known byte counts for random 64-B sector reads and
# 64-B-per-lane streaming reads), then over a short bench run; then a per-kernel
# summary (scripts/pmc_summary.py -> profiles/traffic_<cfg>.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
cfg=${CFG:-c1}
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_probe_$ctr && mkdir -p gpurun_out/pmc_probe_$ctr
  timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_probe_$ctr -o run -- \
    ./build_tools/pmcprobe > gpurun_out/pmc_probe_$ctr.log 2>&1 || { tail -20 gpurun_out/pmc_probe_$ctr.log; exit 1; }
  rm -rf gpurun_out/pmc_${cfg}_$ctr && mkdir -p gpurun_out/pmc_${cfg}_$ctr
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${cfg}_$ctr -o run -- \
    python -u bench.py --config $cfg --steps 10 --warmup 2 --latency-steps 2 --no-cpu-baseline --pcie-steps 0 \
    > gpurun_out/pmc_${cfg}_$ctr.log 2>&1 || { tail -20 gpurun_out/pmc_${cfg}_$ctr.log; exit 1; }
done
python scripts/pmc_summary.py $cfg
