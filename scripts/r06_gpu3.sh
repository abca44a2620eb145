set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_log_reads.py 1 $PWD/build_abl/lib_dbg.so > gpurun_out/diag_dbg.txt 2>&1 || { tail -30 gpurun_out/diag_dbg.txt; exit 1; }
head -60 gpurun_out/diag_dbg.txt
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c1.log 2>&1 || { tail -20 gpurun_out/bench_c1.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_c1.log") if l.startswith('{"metric')][-1])
print("value %.3f G" % (d["value"] / 1e9), "verified", d["verified"], d["self_check"])
print("cpu", {k: d["cpu_baseline"][k] for k in ("value", "cores", "value_1_core", "cores_basis")})
print("roofline", {k: d["roofline"][k] for k in ("kernel_us", "frac", "stage_ms")})
PY
bash scripts/ab_head_r04.sh 3 c1 || exit 1
