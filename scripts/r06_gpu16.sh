# Round 6: duplicate marks as KEY_DUP in the arrival-order keys (no partial
# store into each duplicate's record, no extra read at C1): parity suites
# (with the KEY_DUP collision test), then C1 / C2 / C2U A/B against the
# library before the dup change, alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_alias.py \
  tests/test_gpu_parity.py tests/test_gpu_history.py tests/test_gpu_edges.py tests/test_gpu_robustness.py \
  tests/test_gpu_loopback.py > gpurun_out/r06_keydup_tests.txt 2>&1 || { tail -40 gpurun_out/r06_keydup_tests.txt; exit 1; }
tail -2 gpurun_out/r06_keydup_tests.txt
bash scripts/ab_libs.sh "c1 c2 c2u" 3 build_abl/lib_head_predup.so
