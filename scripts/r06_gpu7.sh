# Round 6: isolated per-kernel times (serial batches) at C1 and C2, and the
# C1 HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=c1_serial KARGS="--config c1 --serial" bash scripts/gpu.sh kstats || exit 1
TAG=c2_serial KARGS="--config c2 --serial" bash scripts/gpu.sh kstats || exit 1
TAG=c1_piped KARGS="--config c1" bash scripts/gpu.sh kstats || exit 1
CFG=c1 bash scripts/gpu.sh pmc || exit 1
