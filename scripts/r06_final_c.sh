# Round 6 closing check at HEAD: the whole -m gpu suite, smoke(), the driver's
# own bench command, and the default bench under rocprofv3 (timed k_table).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
SUITE=1 PYTEST_TIMEOUT=700 CFGS=" " ROUTE=0 PMC=0 bash scripts/gpu.sh evidence || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_cmd.log 2>&1 \
  || { tail -20 gpurun_out/driver_cmd.log; exit 1; }
grep '^{"metric' gpurun_out/driver_cmd.log | cut -c1-400
