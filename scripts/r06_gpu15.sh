# Round 6: C1 A/B of the dup byte array against the previous HEAD, 4 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs.sh "c1" 4 build_abl/lib_head_predup.so
