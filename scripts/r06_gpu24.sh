# Round 6: the bench's per-step call with prebuilt structs: the driver's
# command (K = 20) and K = 200, host time per call in each line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/structs
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/structs/driver_cmd.log 2>&1 \
  || { tail -20 gpurun_out/structs/driver_cmd.log; exit 1; }
for rep in 1 2; do
  for k in 20 200; do
    timeout -k 10 300 python -u bench.py --gpus 1 --steps $k --warmup 5 --no-cpu-baseline --pcie-steps 0 \
      --latency-steps 5 --loaded-steps 0 > gpurun_out/structs/k${k}_$rep.log 2>&1 || { tail -5 gpurun_out/structs/k${k}_$rep.log; exit 1; }
  done
done
for f in gpurun_out/structs/*.log; do
  python - $f <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
print(sys.argv[1].split('/')[-1], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms/step" % d["ms_per_step"],
      "host %.4f ms/call" % d["host_submit_ms"], "verified", d.get("verified"))
PY
done
