#!/bin/bash
# One GPU-box pass: parity tests + smoke + default bench (gpu_round.sh), then a
# rocprofv3 kernel-trace summary of the C1 bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit 1
rm -rf gpurun_out/prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o run -- \
  python -u bench.py --config c1 > gpurun_out/prof_c1.log 2>&1 || { tail -20 gpurun_out/prof_c1.log; exit 1; }
tail -1 gpurun_out/prof_c1.log
