#!/bin/bash
# A/B of the host-fed phase (bench.py's pcie_fed: compact batch, one PCIe copy
# in, results back) and the routed path at N = 1: the in-tree library vs
# build_abl/lib_*.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for lib in "" build_abl/lib_*.so; do
  tag=$(basename "${lib:-cur}" .so)_pcie_$rep
  RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 --latency-steps 5 \
    > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]); p=d['pcie_fed']; print('$tag', round(d['value']/1e9,3), 'G/s; pcie_fed', round(p['value']/1e9,3), 'G/s, soa', round(p['soa']['value']/1e9,3))"
  if [ "${ROUTE:-1}" = "1" ]; then
    tag=$(basename "${lib:-cur}" .so)_route_$rep
    RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --route --no-cpu-baseline --pcie-steps 0 --latency-steps 5 \
      > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,3), 'G/s')"
  fi
done
done
