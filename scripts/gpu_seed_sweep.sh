#!/bin/bash
# C2 (or CFG) rate per stem-hash key (bench.py --hash-seed): looks for the keys under
# which a C2 batch takes milliseconds.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for seed in ${SEEDS:-1 2 3 4 5 6 7 8 9 10 11 12}; do
  timeout -k 10 120 python -u bench.py --config ${CFG:-c2} --hash-seed $seed --steps 40 --warmup 2 --latency-steps 12 \
    --no-cpu-baseline --pcie-steps 0 > gpurun_out/seed_${CFG:-c2}_$seed.log 2>&1 || { tail -5 gpurun_out/seed_${CFG:-c2}_$seed.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/seed_${CFG:-c2}_$seed.log') if l.startswith('{\"metric')][-1]); print('seed $seed', round(d['value']/1e9,3), 'G/s p50', round(d['p50_batch_ms'],3), 'p99', round(d['p99_batch_ms'],3), d['roofline']['stage_ms'])"
done
