#!/bin/bash
# One GPU-box pass, every step under its own time limit, chained so that the
# first failure ends the call:
#   PYTEST  pytest arguments (default: the whole -m gpu suite; "none" skips)
#   SMOKE   1 (default) runs __graft_entry__.smoke()
#   BENCHES bench.py argument sets separated by ';' (default: one default run)
# Logs: gpurun_out/pytest_gpu.log, smoke.log, bench_<k>.log.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST=${PYTEST:-"tests -m gpu"}
if [ "$PYTEST" != "none" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-480} python -u -m pytest $PYTEST -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
if [ "${SMOKE:-1}" = "1" ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
k=0
IFS=';' read -ra SETS <<< "${BENCHES-" "}"
for args in "${SETS[@]}"; do
  [ "$args" = "none" ] && continue
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $args > gpurun_out/bench_$k.log 2>&1 \
    || { tail -30 gpurun_out/bench_$k.log; exit 1; }
  echo "bench[$k] $args"; tail -1 gpurun_out/bench_$k.log
  k=$((k + 1))
done
