#!/bin/bash
# Routed (all_to_all) bench paths on a 1-GPU box: N=1 over RCCL, and a 2-rank
# rehearsal sharing cuda:0 over gloo (the real N>1 run is the driver's, on 8 GPUs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --route --no-cpu-baseline --steps 10 --latency-steps 10 > gpurun_out/bench_route1.log 2>&1 || { tail -30 gpurun_out/bench_route1.log; exit 1; }
tail -1 gpurun_out/bench_route1.log | cut -c1-900
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 \
  bench.py --gpus 2 --dist-backend gloo --one-device --no-cpu-baseline --steps 5 --warmup 2 --latency-steps 3 --tenants 2000000 \
  > gpurun_out/bench_route2.log 2>&1 || { tail -30 gpurun_out/bench_route2.log; exit 1; }
grep '^{' gpurun_out/bench_route2.log | cut -c1-900
