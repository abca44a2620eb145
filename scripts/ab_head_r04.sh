# A/B of the in-tree library + bench against the round-4 final tree
# (build_abl/old_tree, `git archive 5b0485f`, built there), C1, alternating on
# one box: the rate of a plain run, then k_table's timed-launch average from a
# rocprofv3 kernel trace of a second run (scripts/trace_timed.py).
#   bash scripts/ab_head_r04.sh [reps] [cfg]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
REPS=${1:-3}; CFG=${2:-c1}
OUT=$PWD/gpurun_out/ab_r04
mkdir -p $OUT
A="--config $CFG --no-cpu-baseline --steps 200 --warmup 5 --latency-steps 5 --loaded-steps 0 --pcie-steps 0"
for rep in $(seq $REPS); do
  for v in new old; do
    dir=.; [ $v = old ] && dir=build_abl/old_tree
    log=$OUT/${v}_${CFG}_$rep.log
    (cd $dir && timeout -k 10 240 python -u bench.py $A > $log 2>&1) || { tail -5 $log; exit 1; }
    rm -rf $OUT/tr_${v}_$rep
    (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_${v}_$rep -o run -- \
       python -u bench.py $A --prof-every 0 > $OUT/tr_${v}_${CFG}_$rep.log 2>&1) || { tail -5 $OUT/tr_${v}_${CFG}_$rep.log; exit 1; }
    tr=$(find $OUT/tr_${v}_$rep -name "*kernel_trace.csv" | head -1)
    python scripts/trace_timed.py "$tr" $OUT/tr_${v}_${CFG}_$rep.log $OUT/timed_${v}_${CFG}_$rep.json 5 > /dev/null || exit 1
    python scripts/kstats_tail.py "$tr" 200 $OUT/kstats_${v}_${CFG}_$rep.json > $OUT/kstats_${v}_${CFG}_$rep.txt || exit 1
    python - $log $OUT/timed_${v}_${CFG}_$rep.json "$v $CFG $rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
t = json.load(open(sys.argv[2]))
print(sys.argv[3], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms/step" % d["ms_per_step"],
      "k_table timed %.1f us (all %.1f)" % (t["trace_timed_avg_us"], t["trace_all_avg_us"]))
PY
    rm -f "$tr"
  done
done
