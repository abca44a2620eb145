#!/bin/bash
# Round evidence for profiles/: rocprofv3 kernel-trace summary of the C1 and C2
# bench commands, then PMC FETCH_SIZE / WRITE_SIZE passes (separate runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in c1 c2; do
  rm -rf gpurun_out/prof_$cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o run -- \
    python -u bench.py --config $cfg \
    > gpurun_out/prof_$cfg.log 2>&1 || { tail -20 gpurun_out/prof_$cfg.log; exit 1; }
  tail -1 gpurun_out/prof_$cfg.log
done
CFG=c1 bash scripts/gpu_pmc.sh
