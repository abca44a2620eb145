# Round 6: the 32-B wire record and the routed sweep floor (every routed /
# sharded GPU test), then isolated per-kernel times (serial batches) at C1 and
# C2 and the pipelined C1 breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_loopback.py \
  tests/test_gpu_sharded.py tests/test_gpu_multishard.py tests/test_gpu_compact.py tests/test_gpu_prefixed.py \
  > gpurun_out/r06_routed_tests.txt 2>&1 || { tail -40 gpurun_out/r06_routed_tests.txt; exit 1; }
tail -3 gpurun_out/r06_routed_tests.txt
TAG=c1_serial KARGS="--config c1 --serial" bash scripts/gpu.sh kstats || exit 1
TAG=c2_serial KARGS="--config c2 --serial" bash scripts/gpu.sh kstats || exit 1
TAG=c1_piped KARGS="--config c1" bash scripts/gpu.sh kstats || exit 1
