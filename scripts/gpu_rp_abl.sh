#!/bin/bash
# Routing partition (rl_route_pack) timing: the in-tree library and the
# ablation builds build_abl/lib_rp1.so (RL_RP_ABL=1: no stem moves) and
# lib_rp2.so (RL_RP_ABL=2: no record stores), tools/route_pack_bench.py at 1 and
# 8 owners; then a rocprofv3 kernel trace of the in-tree library's run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "" build_abl/lib_rp*.so; do
  [ -n "$lib" ] && [ ! -e "$lib" ] && continue
  tag=$(basename "${lib:-cur}" .so)
  RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 120 python tools/route_pack_bench.py 1 8 > gpurun_out/rp_$tag.log 2>&1 \
    || { tail -5 gpurun_out/rp_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/rp_$tag.log)"
done
rm -rf gpurun_out/rp_prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_prof -o run -- \
  python tools/route_pack_bench.py 1 > gpurun_out/rp_prof.log 2>&1 || { tail -5 gpurun_out/rp_prof.log; exit 1; }
f=$(find gpurun_out/rp_prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-40s %6s calls  avg %8.1f us" % (r["Name"].split("(")[0][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
