# Round 6: C2U per-kernel medians, serial batches and pipelined.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=c2u_serial KARGS="--config c2u --serial" bash scripts/gpu.sh kstats || exit 1
TAG=c2u_piped KARGS="--config c2u" bash scripts/gpu.sh kstats || exit 1
