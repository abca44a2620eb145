# Round 6: the wire-record validation (routed tests), then the C1 kernel-skip
# probes (how much of the step the empty k_split / large-bucket / k_late
# launches cost) A/B against HEAD on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/ab_libs.sh "c1" 3 build_abl/lib_probe_all.so build_abl/lib_probe_late.so build_abl/lib_probe_split.so build_abl/lib_late64.so
