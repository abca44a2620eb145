# A/B of an environment knob: bash scripts/_env_ab.sh VAR "v1 v2 ..." "cfgs" reps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
VAR=$1; VALS=$2; CFGS=${3:-c1 c2}; REPS=${4:-2}
for rep in $(seq $REPS); do
  for v in $VALS; do
    for cfg in $CFGS; do
      env $VAR=$v timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 --latency-steps 5 \
        --loaded-steps 0 --pcie-steps 0 > gpurun_out/envab_${v}_${cfg}_$rep.log 2>&1 || { tail -5 gpurun_out/envab_${v}_${cfg}_$rep.log; exit 1; }
      python - gpurun_out/envab_${v}_${cfg}_$rep.log "$VAR=$v $cfg $rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "table %s" % d["roofline"]["stage_ms"].get("table"))
PY
    done
  done
done
