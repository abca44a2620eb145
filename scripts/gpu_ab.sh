#!/bin/bash
# A/B: the in-tree library vs build_abl/lib_*.so, alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for lib in "" build_abl/lib_*.so; do
  for cfg in ${CFGS:-c1 c2}; do
    tag=$(basename "${lib:-cur}" .so)_${cfg}_$rep
    RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 --latency-steps 5 --pcie-steps 0 \
      > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms table', d['roofline']['stage_ms']['table'])"
  done
done
done
