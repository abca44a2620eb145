# Round 6: the log-read diagnostic over library builds (product, round-5,
# re-read variants), one default bench line (self-check), the A/B against the
# round-4 tree, then the -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/diag_log_reads.py ${DIAG_REPS:-12} "" $PWD/build_abl/lib_r5.so $PWD/build_abl/lib_rr0.so \
  $PWD/build_abl/lib_rr2.so > gpurun_out/diag_log_reads.txt 2>&1 || { tail -30 gpurun_out/diag_log_reads.txt; exit 1; }
cat gpurun_out/diag_log_reads.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c1.log 2>&1 || { tail -20 gpurun_out/bench_c1.log; exit 1; }
grep '^{"metric' gpurun_out/bench_c1.log | cut -c1-400
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_c1.log") if l.startswith('{"metric')][-1])
print("verified", d["verified"], d["self_check"])
print("cpu", {k: d["cpu_baseline"][k] for k in ("value", "cores", "value_1_core", "cores_basis")})
print("roofline", {k: d["roofline"][k] for k in ("kernel_us", "frac", "stage_ms")})
PY
bash scripts/ab_head_r04.sh 3 c1 || exit 1
T="--timeout 120 --timeout-method thread"
timeout -k 10 480 python -u -m pytest tests -m gpu -q $T > gpurun_out/pytest_gpu.log 2>&1; tail -15 gpurun_out/pytest_gpu.log
