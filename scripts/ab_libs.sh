# A/B of library builds against the in-tree one, alternating on one box:
#   bash scripts/ab_libs.sh "<cfgs>" <reps> lib1.so [lib2.so ...]   (extra bench args: $BARGS)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
CFGS=$1; REPS=$2; shift 2
mkdir -p gpurun_out/ab
for rep in $(seq $REPS); do
  for lib in "" "$@"; do
    for cfg in $CFGS; do
      tag=$(basename "${lib:-cur}" .so)_${cfg}_$rep
      RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 240 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 \
        --latency-steps 5 --loaded-steps 0 --pcie-steps 0 $BARGS > gpurun_out/ab/$tag.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then  # (a probe build that skips work fails the self-check: report its unverified rate)
        grep -q "SELF-CHECK FAILED" gpurun_out/ab/$tag.log || { tail -5 gpurun_out/ab/$tag.log; exit 1; }
        echo "$tag $(grep -o 'unverified rate [^)]*' gpurun_out/ab/$tag.log) (self-check failed: a probe, not a result)"
        continue
      fi
      python - gpurun_out/ab/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
r = d["roofline"]
print(sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms" % d["ms_per_step"], "k_table %s us" % r.get("kernel_us"),
      "stages %s" % r["stage_ms"], "verified %s" % d.get("verified"))
PY
    done
  done
done
