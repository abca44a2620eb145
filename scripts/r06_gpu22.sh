# Round 6: 12 hash keys at C2U and 8 at C2 (40 steps each, self-checked), for
# pathological keys after this round's changes (KEY_DUP, k_late's cue).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
CFG=c2u bash scripts/gpu.sh seed-sweep || exit 1
CFG=c2 SEEDS="21 22 23 24 25 26 27 28" bash scripts/gpu.sh seed-sweep || exit 1
