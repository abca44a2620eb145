# Round 6, first GPU pass: the history log's tear tests and the tiny-log
# alias test, the whole -m gpu suite, one default bench line (self-check),
# then the A/B of this tree against the round-4 final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="--timeout 120 --timeout-method thread"
if [ "${NEW:-1}" = "1" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_log_tear.py tests/test_gpu_alias.py tests/test_gpu_history.py -x -v $T \
  > gpurun_out/pytest_new.log 2>&1 || { tail -40 gpurun_out/pytest_new.log; exit 1; }
tail -3 gpurun_out/pytest_new.log
fi
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q $T > gpurun_out/pytest_gpu.log 2>&1 \
  || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c1.log 2>&1 || { tail -20 gpurun_out/bench_c1.log; exit 1; }
grep '^{"metric' gpurun_out/bench_c1.log | cut -c1-600
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_c1.log") if l.startswith('{"metric')][-1])
print("verified", d["verified"], d["self_check"])
print("cpu", {k: d["cpu_baseline"][k] for k in ("value", "cores", "value_1_core", "cores_basis")})
PY
bash scripts/ab_head_r04.sh 3 c1
