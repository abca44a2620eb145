#!/bin/bash
# GPU parity tests, then a short C1/C2 bench (each step under its own limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu ${PYTEST_ARGS} \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in ${CFGS:-c1 c2}; do
  timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --steps 20 --latency-steps 5 \
    > gpurun_out/q_$cfg.log 2>&1 || { tail -5 gpurun_out/q_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/q_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms', d['roofline']['stage_ms'])"
done
