# Round 6: the table scan (k_table_info) moved before the warmup, against the
# previous bench (scan between warmup and timed region), the driver's command
# (K = 20) x 4 and K = 200 x 2, alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/scan_move
for rep in 1 2 3 4; do
  for b in bench bench_prev_tmp; do
    timeout -k 10 300 python -u $b.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pcie-steps 0 \
      --latency-steps 5 --loaded-steps 0 > gpurun_out/scan_move/${b}_k20_$rep.log 2>&1 || { tail -5 gpurun_out/scan_move/${b}_k20_$rep.log; exit 1; }
  done
done
for rep in 1 2; do
  for b in bench bench_prev_tmp; do
    timeout -k 10 300 python -u $b.py --gpus 1 --steps 200 --warmup 5 --no-cpu-baseline --pcie-steps 0 \
      --latency-steps 5 --loaded-steps 0 > gpurun_out/scan_move/${b}_k200_$rep.log 2>&1 || { tail -5 gpurun_out/scan_move/${b}_k200_$rep.log; exit 1; }
  done
done
for f in gpurun_out/scan_move/*.log; do
  python - $f <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
print(sys.argv[1].split('/')[-1], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms/step" % d["ms_per_step"], "verified", d.get("verified"))
PY
done
