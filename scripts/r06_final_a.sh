# Round 6 final evidence, part A: the whole -m gpu suite, smoke(), and the
# default bench (C1) under rocprofv3 with k_table's timed-launch average.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
SUITE=1 PYTEST_TIMEOUT=700 CFGS=" " ROUTE=0 PMC=0 bash scripts/gpu.sh evidence
