# Round 6 final evidence, part B: C2, C2U, C3 and routed benches, then the C1
# and C2 HBM traffic (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for cfg in c2 c2u c3; do
  timeout -k 10 500 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ev_bench_$cfg.log 2>&1 \
    || { tail -20 gpurun_out/ev_bench_$cfg.log; exit 1; }
  grep '^{"metric' gpurun_out/ev_bench_$cfg.log | cut -c1-300
done
timeout -k 10 300 python -u bench.py --route --no-cpu-baseline --pcie-steps 0 > gpurun_out/ev_bench_route.log 2>&1 \
  || { tail -20 gpurun_out/ev_bench_route.log; exit 1; }
grep '^{"metric' gpurun_out/ev_bench_route.log | cut -c1-300
CFG=c1 bash scripts/gpu.sh pmc > gpurun_out/ev_pmc_c1.log 2>&1 || { tail -20 gpurun_out/ev_pmc_c1.log; exit 1; }
tail -14 gpurun_out/ev_pmc_c1.log
CFG=c2 bash scripts/gpu.sh pmc > gpurun_out/ev_pmc_c2.log 2>&1 || { tail -20 gpurun_out/ev_pmc_c2.log; exit 1; }
tail -14 gpurun_out/ev_pmc_c2.log
