# Round 6: the whole -m gpu suite and smoke() after the snapshot image bump.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
SMOKE=1 BENCHES=none PYTEST_TIMEOUT=700 bash scripts/gpu.sh round
