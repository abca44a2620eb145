#!/bin/bash
# C1/C2 bench with alternative builds of the library (build_abl/lib_*.so) and
# HIP hardware-queue counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for q in ${HWQ:-4}; do
for lib in "" build_abl/lib_*.so; do
  for cfg in ${CFGS:-c1 c2}; do
    tag=$(basename "${lib:-default}" .so)_q${q}_$cfg
    GPU_MAX_HW_QUEUES=$q RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --steps 20 --latency-steps 5 \
      > gpurun_out/var_$tag.log 2>&1 || { tail -5 gpurun_out/var_$tag.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/var_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms', d['roofline']['stage_ms'])"
  done
done
done
