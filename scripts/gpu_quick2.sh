#!/bin/bash
# sortbench variants (build_tools/) + short C1/C2 bench of the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in build_tools/sortbench_*; do
  [ -x "$f" ] || continue
  echo "== $f"
  timeout -k 5 60 $f 1000000 || { echo "FAIL $f"; exit 1; }
done
for cfg in ${CFGS:-c1 c2}; do
  timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --steps 20 --latency-steps 5 \
    > gpurun_out/q_$cfg.log 2>&1 || { tail -5 gpurun_out/q_$cfg.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/q_$cfg.log').read().strip().splitlines()[-1]); print('$cfg', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms', d['roofline']['stage_ms'])"
done
