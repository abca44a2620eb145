# Round 6: k_part reads the batch's hits array instead of k_prepare's copy
# (4 MB less written per 1M): parity suites, then C1 / C2 A/B, 3 reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_alias.py tests/test_gpu_edges.py tests/test_gpu_compact.py tests/test_gpu_prefixed.py \
  tests/test_gpu_loopback.py > gpurun_out/r06_hita_tests.txt 2>&1 || { tail -40 gpurun_out/r06_hita_tests.txt; exit 1; }
tail -2 gpurun_out/r06_hita_tests.txt
bash scripts/ab_libs.sh "c1 c2" 3 build_abl/lib_head_pre_hita.so
