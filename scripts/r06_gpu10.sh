# Round 6: the wire-record validation (routed tests), then the C1 kernel-skip
# probes (how much of the step the empty k_split / large-bucket / k_late
# launches cost) A/B against HEAD on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_loopback.py \
  tests/test_gpu_sharded.py tests/test_gpu_multishard.py \
  > gpurun_out/r06_routed_tests2.txt 2>&1 || { tail -40 gpurun_out/r06_routed_tests2.txt; exit 1; }
tail -2 gpurun_out/r06_routed_tests2.txt
bash scripts/ab_libs.sh "c1" 3 build_abl/lib_probe_all.so build_abl/lib_probe_late.so build_abl/lib_probe_split.so
