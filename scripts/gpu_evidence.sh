#!/bin/bash
# Round evidence on one GPU box, every step under its own time limit, chained
# so that the first failure ends the call:
#   1. the -m gpu suite and smoke() (scripts/gpu_round.sh, no bench);
#   2. the default bench (C1) under rocprofv3 --kernel-trace --stats: the bench
#      line (k_table's live HIP-event time) and the trace of the same command,
#      compared over the timed launches (scripts/trace_timed.py);
#   3. C2, C2U and C3 bench lines, the routed path at N = 1;
#   4. (PMC=1) PMC FETCH_SIZE / WRITE_SIZE passes for C1 (scripts/gpu_pmc.sh).
# Outputs under gpurun_out/ev_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SUITE:-1}" = "1" ]; then BENCHES=none bash scripts/gpu_round.sh || exit 1; fi
rm -rf gpurun_out/ev_prof_c1 && mkdir -p gpurun_out/ev_prof_c1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev_prof_c1 -o run -- \
  python -u bench.py > gpurun_out/ev_bench_c1.log 2>&1 || { tail -20 gpurun_out/ev_bench_c1.log; exit 1; }
grep '^{"metric' gpurun_out/ev_bench_c1.log | cut -c1-400
python scripts/trace_timed.py gpurun_out/ev_prof_c1/*/run_kernel_trace.csv gpurun_out/ev_bench_c1.log \
  gpurun_out/ev_trace_timed_c1.json 2>/dev/null || \
  python scripts/trace_timed.py gpurun_out/ev_prof_c1/run_kernel_trace.csv gpurun_out/ev_bench_c1.log \
  gpurun_out/ev_trace_timed_c1.json || exit 1
for cfg in ${CFGS:-c2 c2u c3}; do
  timeout -k 10 500 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ev_bench_$cfg.log 2>&1 \
    || { tail -20 gpurun_out/ev_bench_$cfg.log; exit 1; }
  grep '^{"metric' gpurun_out/ev_bench_$cfg.log | cut -c1-300
done
if [ "${ROUTE:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --route --no-cpu-baseline --pcie-steps 0 > gpurun_out/ev_bench_route.log 2>&1 \
    || { tail -20 gpurun_out/ev_bench_route.log; exit 1; }
  grep '^{"metric' gpurun_out/ev_bench_route.log | cut -c1-300
fi
if [ "${PMC:-0}" = "1" ]; then
  CFG=c1 bash scripts/gpu_pmc.sh > gpurun_out/ev_pmc.log 2>&1 || { tail -20 gpurun_out/ev_pmc.log; exit 1; }
  tail -14 gpurun_out/ev_pmc.log
fi
