#!/bin/bash
# A/B of the stage-event sampling stride (bench --prof-every), alternating on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for pe in 1 4 1000000; do
  for cfg in ${CFGS:-c1 c2}; do
    tag=pe${pe}_${cfg}_$rep
    timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 --latency-steps 5 --prof-every $pe \
      > gpurun_out/pe_$tag.log 2>&1 || { tail -5 gpurun_out/pe_$tag.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/pe_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms runs', d['roofline']['stage_ms']['runs'])"
  done
done
done
