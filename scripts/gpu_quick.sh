#!/bin/bash
# Parity tests + C1/C2 bench lines (no CPU baseline): the inner loop of kernel work.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for cfg in c1 c2; do
  timeout -k 10 300 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/bench_$cfg.log; exit 1; }
  python - "$cfg" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/bench_%s.log" % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.3g dec/s" % d["value"], "ms/step %.4f" % d["ms_per_step"], "p99 %.3f" % d["p99_batch_ms"],
      "frac %.3f" % d["roofline"]["frac"], d["roofline"]["stage_ms"])
PY
done
