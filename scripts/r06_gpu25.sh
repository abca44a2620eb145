# Round 6: the whole -m gpu suite with k_late's long-run part on the
# bitmap-walking workgroups for every batch (RL_LATE_CUE=2) and with full
# large-bucket grids for every batch (RL_BIG_CUE=0): both launch shapes of
# each cue under every parity test.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
RL_LATE_CUE=2 RL_BIG_CUE=0 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r06_cues_suite.txt 2>&1 || { tail -40 gpurun_out/r06_cues_suite.txt; exit 1; }
tail -2 gpurun_out/r06_cues_suite.txt
