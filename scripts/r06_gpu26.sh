# Round 6: the cost of the bench's live k_table timing (every 7th batch) at the
# driver's K = 20 and at K = 200: --prof-every 7 against 0, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_cost
for rep in 1 2 3; do
  for pe in 7 0; do
    for k in 20 200; do
      timeout -k 10 300 python -u bench.py --gpus 1 --steps $k --warmup 5 --no-cpu-baseline --pcie-steps 0 \
        --latency-steps 5 --loaded-steps 0 --prof-every $pe > gpurun_out/prof_cost/pe${pe}_k${k}_$rep.log 2>&1 \
        || { tail -5 gpurun_out/prof_cost/pe${pe}_k${k}_$rep.log; exit 1; }
      python - gpurun_out/prof_cost/pe${pe}_k${k}_$rep.log "prof-every $pe K=$k rep $rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms/step" % d["ms_per_step"], "verified", d.get("verified"))
PY
    done
  done
done
