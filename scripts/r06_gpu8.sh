# Round 6: the routed sweep floor test, then isolated per-kernel times (serial
# batches) at C1 and C2, and the C1 HBM traffic per kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_loopback.py -k "sweep" > gpurun_out/r06_sweep_floor.txt 2>&1 || { tail -30 gpurun_out/r06_sweep_floor.txt; exit 1; }
tail -3 gpurun_out/r06_sweep_floor.txt
TAG=c1_serial KARGS="--config c1 --serial" bash scripts/gpu.sh kstats || exit 1
TAG=c2_serial KARGS="--config c2 --serial" bash scripts/gpu.sh kstats || exit 1
TAG=c1_piped KARGS="--config c1" bash scripts/gpu.sh kstats || exit 1
CFG=c1 bash scripts/gpu.sh pmc || exit 1
