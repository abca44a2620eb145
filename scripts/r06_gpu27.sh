# Round 6: k_table's clock reads and their fold only on the sampled batches
# (every 7th, the first sampled one the 7th of the timed region): the
# observability test, then --prof-every 7 against 0 at K = 20 and 200.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_observability.py \
  > gpurun_out/r06_prof_tests.txt 2>&1 || { tail -30 gpurun_out/r06_prof_tests.txt; exit 1; }
tail -1 gpurun_out/r06_prof_tests.txt
bash scripts/r06_gpu26.sh
