# Round 6: table load factor (--slots-per-key 4 / 2 / 1) at C1 and C2, and
# the history log's 256-partition build, alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/sweep_bench_arg.sh "c1 c2" 2 --slots-per-key "4 2 1" || exit 1
BARGS="" bash scripts/ab_libs.sh "c1 c2" 2 build_abl/lib_lp8.so || exit 1
