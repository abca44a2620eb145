# Round 6: the driver's exact bench command at the final HEAD, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_cmd_$rep.log 2>&1 \
    || { tail -20 gpurun_out/driver_cmd_$rep.log; exit 1; }
  grep '^{"metric' gpurun_out/driver_cmd_$rep.log | cut -c1-260
done
