# Round 6: the driver's bench command (--steps 20 --warmup 5) against 200
# timed steps on one box, alternating, 3 reps each (the pipeline's ramp from
# an idle GPU is inside the 20-step timed region).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ramp
for rep in 1 2 3; do
  for k in 20 200; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps $k --warmup 5 --no-cpu-baseline --pcie-steps 0 \
      --latency-steps 5 --loaded-steps 0 > gpurun_out/ramp/k${k}_$rep.log 2>&1 || { tail -5 gpurun_out/ramp/k${k}_$rep.log; exit 1; }
    python - gpurun_out/ramp/k${k}_$rep.log "k=$k rep $rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms/step" % d["ms_per_step"], "verified", d.get("verified"))
PY
  done
done
