#!/bin/bash
# Per-kernel durations (rocprofv3 kernel-trace stats) of one bench command:
#   KARGS  bench.py arguments (default: C1, serial submission = isolated kernels)
#   TAG    output name: gpurun_out/kstats_<TAG>/ and gpurun_out/kstats_<TAG>.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-c1_serial}
rm -rf gpurun_out/kstats_$TAG && mkdir -p gpurun_out/kstats_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats_$TAG -o run -- \
  python -u bench.py --steps 50 --warmup 3 --latency-steps 3 --no-cpu-baseline --prof-every 0 ${KARGS:---config c1 --serial} \
  > gpurun_out/kstats_$TAG.log 2>&1 || { tail -20 gpurun_out/kstats_$TAG.log; exit 1; }
tail -1 gpurun_out/kstats_$TAG.log | cut -c1-300
f=$(find gpurun_out/kstats_$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kstats_$TAG.csv
python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-24s %6s calls  avg %8.1f us" % (r["Name"].split("(")[0][:24], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
