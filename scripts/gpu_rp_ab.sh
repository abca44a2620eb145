#!/bin/bash
# Partition kernel A/B: tools/route_pack_bench.py against side builds in build_abl/ (RL_LIB_PATH).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/route_pack_bench.py 1 8 > gpurun_out/rp_cur.log 2>&1 || { cat gpurun_out/rp_cur.log; exit 1; }
echo "cur $(tail -1 gpurun_out/rp_cur.log)"
for f in build_abl/lib_rp*.so; do
  [ -e "$f" ] || continue
  t=$(basename $f .so)
  RL_LIB_PATH=$PWD/$f timeout -k 10 120 python tools/route_pack_bench.py 1 8 > gpurun_out/rp_$t.log 2>&1 || { cat gpurun_out/rp_$t.log; exit 1; }
  echo "$t $(tail -1 gpurun_out/rp_$t.log)"
done
