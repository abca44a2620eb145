#!/bin/bash
# k_runs time vs table size (TLB / cache-residency experiment) + counter list.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_all.txt 2>&1 || true
grep -i -E "utcl|tlb|TCC_EA0_RDREQ|TCC_EA0_WRREQ|FETCH_SIZE|WRITE_SIZE|TCC_HIT|TCC_MISS|TA_BUSY|TCP_TCC" gpurun_out/counters_all.txt | head -60 > gpurun_out/counters_sel.txt || true
for T in 100000 1000000 10000000; do
  timeout -k 10 300 python -u bench.py --config c1 --tenants $T --no-cpu-baseline --steps 10 --latency-steps 5 > gpurun_out/size_$T.log 2>&1 || { tail -20 gpurun_out/size_$T.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/size_$T.log').read().strip().splitlines()[-1]); print($T, round(d['value']/1e9,3), d['roofline']['stage_ms'], d['config']['table_slots'])"
done
wc -l gpurun_out/counters_sel.txt
