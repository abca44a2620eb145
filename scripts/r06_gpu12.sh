# Round 6: k_late folded into k_table (tail workgroups) while recent batches had no long runs.
# Parity (alias, parity, history, full-size suites), then C1 and C2 A/B: default (cue + fold)
# against RL_LATE_CUE=0 (k_late a launch of its own, full grid: the round-5 launch).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_alias.py \
  tests/test_gpu_parity.py tests/test_gpu_history.py tests/test_gpu_edges.py tests/test_gpu_robustness.py > gpurun_out/r06_late_tests.txt 2>&1 || { tail -40 gpurun_out/r06_late_tests.txt; exit 1; }
tail -2 gpurun_out/r06_late_tests.txt
mkdir -p gpurun_out/ab_late
for rep in 1 2 3; do
  for mode in 1 0; do
    for cfg in c1 c2; do
      tag=late${mode}_${cfg}_$rep
      RL_LATE_CUE=$mode timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 \
        --latency-steps 5 --loaded-steps 0 --pcie-steps 0 > gpurun_out/ab_late/$tag.log 2>&1 \
        || { tail -5 gpurun_out/ab_late/$tag.log; exit 1; }
      python - gpurun_out/ab_late/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
r = d["roofline"]
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms" % d["ms_per_step"], "k_table %s us" % r.get("kernel_us"),
      "verified %s" % d.get("verified"))
PY
    done
  done
done
