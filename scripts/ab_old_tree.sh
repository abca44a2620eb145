set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab_log
A="--no-cpu-baseline --steps 200 --latency-steps 5 --loaded-steps 0 --pcie-steps 0"
for rep in 1 2; do
  for cfg in c1 c2; do
    timeout -k 10 200 python -u bench.py --config $cfg $A > gpurun_out/ab_log/new_${cfg}_$rep.log 2>&1 || exit 1
    (cd build_abl/old_tree && timeout -k 10 200 python -u bench.py --config $cfg $A > ../../gpurun_out/ab_log/old_${cfg}_$rep.log 2>&1) || exit 1
    for v in new old; do
      python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_log/${v}_${cfg}_$rep.log') if l.startswith('{\"metric')][-1])
print('$v $cfg $rep', round(d['value']/1e9,3), d['roofline'].get('kernel_us'), d['roofline']['stage_ms'])"
    done
  done
done
