# Round 6: the epoch moved into k_b_begin: C1 A/B (in-tree, no guard, the
# round-5 tree, k_table's keys-seen-once blocks first), then the diag, the
# -m gpu suite and smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab5
A="--config c1 --no-cpu-baseline --steps 200 --latency-steps 5 --loaded-steps 0 --pcie-steps 0"
summ() {
python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
r = d["roofline"]
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms" % d["ms_per_step"], "k_table %s us" % r.get("kernel_us"),
      "stages %s" % r["stage_ms"], "verified %s" % d.get("verified"))
PY
}
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py $A > gpurun_out/ab5/cur_$rep.log 2>&1 || { tail -5 gpurun_out/ab5/cur_$rep.log; exit 1; }
  summ gpurun_out/ab5/cur_$rep.log "cur $rep"
  (cd build_abl/r5_tree && timeout -k 10 240 python -u bench.py $A > ../../gpurun_out/ab5/r5_$rep.log 2>&1) || { tail -5 gpurun_out/ab5/r5_$rep.log; exit 1; }
  summ gpurun_out/ab5/r5_$rep.log "r5tree $rep"
  for v in noguard uqf; do
    RL_LIB_PATH=$PWD/build_abl/lib_$v.so timeout -k 10 240 python -u bench.py $A > gpurun_out/ab5/${v}_$rep.log 2>&1 \
      || { tail -5 gpurun_out/ab5/${v}_$rep.log; exit 1; }
    summ gpurun_out/ab5/${v}_$rep.log "$v $rep"
  done
done
timeout -k 10 300 python -u tools/diag_log_reads.py 4 > gpurun_out/diag_fix2.txt 2>&1 || { tail -30 gpurun_out/diag_fix2.txt; exit 1; }
tail -2 gpurun_out/diag_fix2.txt
T="--timeout 120 --timeout-method thread"
timeout -k 10 480 python -u -m pytest tests -m gpu -q $T > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log
[ $rc = 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
