#!/bin/bash
# A/B: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4 on the
# box) for the routed N=1 path (8 streams: the engine's 3 buffer streams, side
# stream and serial stream, the router's partition / forward / return streams)
# and the single-GPU C1/C2 pipeline (5 streams).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag, env, bench args
  env $2 timeout -k 10 200 python -u bench.py $3 --no-cpu-baseline --pcie-steps 0 --latency-steps 5 \
    > gpurun_out/hwq_$1.log 2>&1 || { tail -5 gpurun_out/hwq_$1.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/hwq_$1.log') if l.startswith('{\"metric')][-1]); print('$1', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms', d['roofline']['stage_ms'])"
  grep -h route_host_us gpurun_out/hwq_$1.log || true
}
for rep in 1 2; do
  run route_q4_$rep "RL_DEBUG_ROUTE_TIMING=1" "--route"
  run route_q8_$rep "RL_DEBUG_ROUTE_TIMING=1 GPU_MAX_HW_QUEUES=8" "--route"
  run c1_q4_$rep "RL_NONE=1" "--config c1"
  run c1_q8_$rep "GPU_MAX_HW_QUEUES=8" "--config c1"
  run c2_q4_$rep "RL_NONE=1" "--config c2"
  run c2_q8_$rep "GPU_MAX_HW_QUEUES=8" "--config c2"
done
