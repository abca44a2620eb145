# One bench flag swept, alternating on one box:
#   bash scripts/sweep_bench_arg.sh "<cfgs>" <reps> --flag "v1 v2 ..."
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
CFGS=$1; REPS=$2; FLAG=$3; VALS=$4
mkdir -p gpurun_out/sweep
for rep in $(seq $REPS); do
  for v in $VALS; do
    for cfg in $CFGS; do
      tag=${FLAG#--}_${v}_${cfg}_$rep
      timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 --latency-steps 5 --loaded-steps 0 \
        --pcie-steps 0 $FLAG $v > gpurun_out/sweep/$tag.log 2>&1 || { tail -5 gpurun_out/sweep/$tag.log; exit 1; }
      python - gpurun_out/sweep/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
r = d["roofline"]
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "k_table %s us" % r.get("kernel_us"), "stages %s" % r["stage_ms"],
      "table_gb %s" % d["config"].get("table_hbm_gb"), "verified %s" % d.get("verified"))
PY
    done
  done
done
