#!/bin/bash
# Time the run stage with parts of k_runs disabled (RL_ABL builds in build_abl/).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for a in 0 1 2 4 7; do
  RL_LIB_PATH=$PWD/build_abl/lib_abl$a.so timeout -k 10 200 python -u bench.py --config c1 --no-cpu-baseline --steps 10 --latency-steps 3 > gpurun_out/abl_$a.log 2>&1 || { tail -5 gpurun_out/abl_$a.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/abl_$a.log').read().strip().splitlines()[-1]); print('abl', $a, d['roofline']['stage_ms'])"
done
