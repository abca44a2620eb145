#!/bin/bash
# PMC counters of a build_tools/ micro-benchmark (one rocprofv3 pass per counter set).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_tool
T=${TOOL:-build_tools/bucketbench}
A=${ARGS:-"1000000 0"}
i=0
IFS=';' read -ra SETS <<< "${PMC_SETS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU}"
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_tool/p$i -o run -- $T $A > gpurun_out/pmc_tool/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_tool/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/pmc_tool/p*/**/*counter_collection.csv', recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r.get('Kernel_Name', '')[:40]
        acc[(k, r['Counter_Name'])].append(float(r['Counter_Value']))
    for (k, c), v in sorted(acc.items()):
        v = v[2:] if len(v) > 4 else v
        print(f"{k:40s} {c:24s} {sum(v)/len(v):14.0f}")
PY
