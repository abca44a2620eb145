# Round 6: the refusal fix (diag), then C1 A/B: the in-tree library, the
# round-5 tree, log-protocol variants, the large-bucket cue off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u tools/diag_log_reads.py 6 > gpurun_out/diag_fix.txt 2>&1 || { tail -30 gpurun_out/diag_fix.txt; exit 1; }
tail -3 gpurun_out/diag_fix.txt
A="--config c1 --no-cpu-baseline --steps 200 --latency-steps 5 --loaded-steps 0 --pcie-steps 0"
summ() {
python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
r = d["roofline"]
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms" % d["ms_per_step"], "k_table %s us" % r.get("kernel_us"),
      "stages %s" % r["stage_ms"])
PY
}
for rep in 1 2; do
  timeout -k 10 240 python -u bench.py $A > gpurun_out/ab/cur_$rep.log 2>&1 || { tail -5 gpurun_out/ab/cur_$rep.log; exit 1; }
  summ gpurun_out/ab/cur_$rep.log "cur $rep"
  (cd build_abl/r5_tree && timeout -k 10 240 python -u bench.py $A > ../../gpurun_out/ab/r5_$rep.log 2>&1) || { tail -5 gpurun_out/ab/r5_$rep.log; exit 1; }
  summ gpurun_out/ab/r5_$rep.log "r5tree $rep"
  for v in noorder noguard 2store r5w; do
    RL_LIB_PATH=$PWD/build_abl/lib_$v.so timeout -k 10 240 python -u bench.py $A > gpurun_out/ab/${v}_$rep.log 2>&1 \
      || { tail -5 gpurun_out/ab/${v}_$rep.log; exit 1; }
    summ gpurun_out/ab/${v}_$rep.log "$v $rep"
  done
  RL_BIG_CUE=0 timeout -k 10 240 python -u bench.py $A > gpurun_out/ab/cue0_$rep.log 2>&1 || { tail -5 gpurun_out/ab/cue0_$rep.log; exit 1; }
  summ gpurun_out/ab/cue0_$rep.log "cue0 $rep"
done
