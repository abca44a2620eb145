# Round 6: one table-stage stream (RL_SB=1; 2 = high priority) against the
# per-batch streams, C1 and C2, alternating on one box; parity under RL_SB=2 first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
RL_SB=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_alias.py \
  tests/test_gpu_parity.py > gpurun_out/r06_sb_tests.txt 2>&1 || { tail -40 gpurun_out/r06_sb_tests.txt; exit 1; }
tail -2 gpurun_out/r06_sb_tests.txt
mkdir -p gpurun_out/ab_sb
for rep in 1 2; do
  for mode in base sb1 sb2 sb2q8; do
    for cfg in c1 c2; do
      tag=${mode}_${cfg}_$rep
      case $mode in
        base) envs="" ;;
        sb1) envs="RL_SB=1" ;;
        sb2) envs="RL_SB=2" ;;
        sb2q8) envs="RL_SB=2 GPU_MAX_HW_QUEUES=8" ;;
      esac
      env $envs timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 \
        --latency-steps 5 --loaded-steps 0 --pcie-steps 0 > gpurun_out/ab_sb/$tag.log 2>&1 \
        || { tail -5 gpurun_out/ab_sb/$tag.log; exit 1; }
      python - gpurun_out/ab_sb/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
r = d["roofline"]
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms" % d["ms_per_step"], "k_table %s us" % r.get("kernel_us"),
      "verified %s" % d.get("verified"))
PY
    done
  done
done
