#!/bin/bash
# Phase times of k_split's long body on C2U's hot multi-unit runs (device
# printf from measurement builds built with RL_SPLIT_PROF).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${LIBS:-build_abl/lib_sprof.so}; do
  tag=$(basename $lib .so)
  RL_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --config c2u --steps 10 --warmup 2 --latency-steps 2 \
    --pcie-steps 0 --no-cpu-baseline > gpurun_out/split_prof_$tag.log 2>&1 || { tail -5 gpurun_out/split_prof_$tag.log; exit 1; }
  echo "== $tag"; grep split_long gpurun_out/split_prof_$tag.log | tail -4
done
