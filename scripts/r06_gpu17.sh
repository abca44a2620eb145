# Round 6, review item 3: HEAD against the round-4 final tree (5b0485f), C1 x 3
# alternating on one box, with k_table's timed-launch average from a kernel
# trace of each (scripts/ab_head_r04.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_head_r04.sh 3 c1
