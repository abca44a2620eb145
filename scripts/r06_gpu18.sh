# Round 6: pipeline depth 3 and 5 against 4 (RL_NBUF), C1 and C2, 2 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs.sh "c1 c2" 2 build_abl/lib_nbuf3.so build_abl/lib_nbuf5.so
