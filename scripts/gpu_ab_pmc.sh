#!/bin/bash
# A/B of k_runs HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and longer
# C1 timings: in-tree library vs build_abl/lib_*.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/abpmc
for lib in "" build_abl/lib_*.so; do
  tag=$(basename "${lib:-cur}" .so)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    RL_LIB_PATH=${lib:+$PWD/$lib} timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/abpmc/${tag}_$ctr -o run -- \
      python -u bench.py --config c1 --steps 10 --warmup 2 --latency-steps 2 --no-cpu-baseline > gpurun_out/abpmc/${tag}_$ctr.log 2>&1 \
      || { tail -5 gpurun_out/abpmc/${tag}_$ctr.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, statistics
for d in sorted(glob.glob('gpurun_out/abpmc/*_FETCH_SIZE')) + sorted(glob.glob('gpurun_out/abpmc/*_WRITE_SIZE')):
    vals = {}
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0]
            if k.startswith('rl::k_runs') or k.startswith('rl::k_bucket') or k.startswith('rl::k_prepare'):
                vals.setdefault(k, []).append((int(r['Dispatch_Id']), float(r['Counter_Value'])))
    print(d.split('/')[-1], {k: round(statistics.median([x for _, x in sorted(v)[-10:]]) / 1024, 1) for k, v in vals.items()}, 'MB')
PY
for rep in 1 2 3; do
for lib in "" build_abl/lib_*.so; do
  tag=$(basename "${lib:-cur}" .so)
  RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --config c1 --no-cpu-baseline --steps 200 --latency-steps 2 \
    > gpurun_out/abpmc/t_${tag}_$rep.log 2>&1 || { tail -5 gpurun_out/abpmc/t_${tag}_$rep.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/abpmc/t_${tag}_$rep.log').read().strip().splitlines()[-1]); print('$tag', $rep, round(d['value']/1e9,3), 'G/s runs', d['roofline']['stage_ms']['runs'])"
done
done
