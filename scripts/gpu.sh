#!/bin/bash
# GPU-box tasks, run through gpurun from the repository root:
#
#   bash scripts/gpu.sh <task> [<task> ...]        e.g.  bash scripts/gpu.sh round ab
#
# Every GPU step runs under its own time limit; the first failure ends the
# call. Outputs go to gpurun_out/. Tasks (environment knobs in brackets):
#
#   round        the -m gpu suite, smoke(), bench lines [PYTEST SMOKE BENCHES]
#   evidence     round's suite, then the default bench (C1) under rocprofv3
#                --kernel-trace --stats with its trace compared to the bench's
#                HIP events (trace_timed.py), C2 / C2U / C3 lines, the routed
#                N = 1 line, PMC traffic [SUITE CFGS ROUTE PMC]
#   ab           A/B: the in-tree library vs build_abl/lib_*.so, alternating,
#                device-resident [CFGS REPS]; MODE=route: bench.py --route;
#                MODE=pcie: the host-fed phase (and the routed line)
#   kstats       per-kernel durations of one bench command (rocprofv3 stats,
#                medians of the last launches: kstats_tail.py) [TAG KARGS]
#   pmc          HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE passes over
#                the calibration probe and a short bench (pmc_summary.py) [CFG]
#   pcie-trace   memory-copy + kernel trace of the host-fed phase
#                (copy_timeline.py) [KARGS]
#   route-trace  routed N = 1 kernel trace per library: GPU busy fraction and
#                kernel time per batch (trace_busy.py) [KARGS]
#   seed-sweep   the rate per stem-hash key [CFG SEEDS]
#   serial-trace kernel + copy trace of serial C1 batches per library (the in-tree
#                one and build_abl/lib_*.so): k_table per batch, fill included [KARGS]
#   split-prof   phase stamps of k_split's long body (build_abl/lib_sprof.so,
#                built with RL_SPLIT_PROF) on C2U [LIBS]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out

# the last bench JSON line of a log: rate, step, table stage (or more fields)
summary() {  # log tag [extra python expression]
  python - "$1" "$2" "${3:-}" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric')][-1])
out = [sys.argv[2], "%.3f G/s" % (d["value"] / 1e9), "%.4f ms" % d["ms_per_step"]]
if d.get("roofline", {}).get("stage_ms"):
    out.append("table %s kern %s" % (d["roofline"]["stage_ms"].get("table"), d["roofline"].get("kernel_us")))
if sys.argv[3]:
    out.append(str(eval(sys.argv[3], {"d": d})))
print(" ".join(out))
PY
}

task_round() {
  local PYTEST=${PYTEST:-"tests -m gpu"}
  if [ "$PYTEST" != "none" ]; then
    timeout -k 10 ${PYTEST_TIMEOUT:-480} python -u -m pytest $PYTEST -x -v --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; return 1; }
    tail -2 gpurun_out/pytest_gpu.log
  fi
  if [ "${SMOKE:-1}" = "1" ]; then
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { cat gpurun_out/smoke.log; return 1; }
    cat gpurun_out/smoke.log
  fi
  local k=0 args
  IFS=';' read -ra SETS <<< "${BENCHES-" "}"
  for args in "${SETS[@]}"; do
    [ "$args" = "none" ] && continue
    timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $args > gpurun_out/bench_$k.log 2>&1 \
      || { tail -30 gpurun_out/bench_$k.log; return 1; }
    echo "bench[$k] $args"; tail -1 gpurun_out/bench_$k.log
    k=$((k + 1))
  done
}

task_pmc() {
  local cfg=${CFG:-c1} ctr
  for ctr in FETCH_SIZE WRITE_SIZE; do  # (one counter per pass: they do not fit one)
    rm -rf gpurun_out/pmc_probe_$ctr && mkdir -p gpurun_out/pmc_probe_$ctr
    timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_probe_$ctr -o run -- \
      ./build_tools/pmcprobe > gpurun_out/pmc_probe_$ctr.log 2>&1 || { tail -20 gpurun_out/pmc_probe_$ctr.log; return 1; }
    rm -rf gpurun_out/pmc_${cfg}_$ctr && mkdir -p gpurun_out/pmc_${cfg}_$ctr
    timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${cfg}_$ctr -o run -- \
      python -u bench.py --config $cfg --steps 10 --warmup 2 --latency-steps 2 --loaded-steps 0 --no-cpu-baseline --pcie-steps 0 \
      > gpurun_out/pmc_${cfg}_$ctr.log 2>&1 || { tail -20 gpurun_out/pmc_${cfg}_$ctr.log; return 1; }
  done
  python scripts/pmc_summary.py $cfg
}

task_evidence() {
  if [ "${SUITE:-1}" = "1" ]; then BENCHES=none task_round || return 1; fi
  rm -rf gpurun_out/ev_prof_c1 && mkdir -p gpurun_out/ev_prof_c1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev_prof_c1 -o run -- \
    python -u bench.py > gpurun_out/ev_bench_c1.log 2>&1 || { tail -20 gpurun_out/ev_bench_c1.log; return 1; }
  grep '^{"metric' gpurun_out/ev_bench_c1.log | cut -c1-400
  local tr
  tr=$(find gpurun_out/ev_prof_c1 -name "*kernel_trace.csv" | head -1)
  python scripts/trace_timed.py "$tr" gpurun_out/ev_bench_c1.log gpurun_out/ev_trace_timed_c1.json || return 1
  local cfg
  for cfg in ${CFGS:-c2 c2u c3}; do
    timeout -k 10 500 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/ev_bench_$cfg.log 2>&1 \
      || { tail -20 gpurun_out/ev_bench_$cfg.log; return 1; }
    grep '^{"metric' gpurun_out/ev_bench_$cfg.log | cut -c1-300
  done
  if [ "${ROUTE:-1}" = "1" ]; then
    timeout -k 10 300 python -u bench.py --route --no-cpu-baseline --pcie-steps 0 > gpurun_out/ev_bench_route.log 2>&1 \
      || { tail -20 gpurun_out/ev_bench_route.log; return 1; }
    grep '^{"metric' gpurun_out/ev_bench_route.log | cut -c1-300
  fi
  if [ "${PMC:-0}" = "1" ]; then CFG=c1 task_pmc > gpurun_out/ev_pmc.log 2>&1 || { tail -20 gpurun_out/ev_pmc.log; return 1; }; tail -14 gpurun_out/ev_pmc.log; fi
}

task_ab() {
  local mode=${MODE:-device} rep lib cfg tag
  for rep in $(seq ${REPS:-2}); do
    for lib in "" build_abl/lib_*.so; do
      [ -n "$lib" ] && [ ! -e "$lib" ] && continue
      if [ "$mode" = "device" ]; then
        for cfg in ${CFGS:-c1 c2}; do
          tag=$(basename "${lib:-cur}" .so)_${cfg}_$rep
          RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --config $cfg --no-cpu-baseline --steps 200 \
            --latency-steps 5 --loaded-steps 0 --pcie-steps 0 > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; return 1; }
          summary gpurun_out/ab_$tag.log $tag
        done
      fi
      if [ "$mode" = "pcie" ]; then
        tag=$(basename "${lib:-cur}" .so)_pcie_$rep
        RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 --latency-steps 5 --loaded-steps 0 \
          > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; return 1; }
        summary gpurun_out/ab_$tag.log $tag \
          '"pcie_fed %.3f G/s, soa %.3f" % (d["pcie_fed"]["value"] / 1e9, d["pcie_fed"]["soa"]["value"] / 1e9)'
      fi
      if [ "$mode" = "route" ] || [ "$mode" = "pcie" ]; then
        tag=$(basename "${lib:-cur}" .so)_route_$rep
        RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 200 python -u bench.py --route --no-cpu-baseline --pcie-steps 0 \
          --latency-steps 5 --loaded-steps 0 > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; return 1; }
        summary gpurun_out/ab_$tag.log $tag
      fi
    done
  done
}

task_kstats() {
  local tag=${TAG:-c1_serial} f
  rm -rf gpurun_out/kstats_$tag && mkdir -p gpurun_out/kstats_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats_$tag -o run -- \
    python -u bench.py --steps 50 --warmup 3 --latency-steps 3 --loaded-steps 0 --no-cpu-baseline --prof-every 0 \
    ${KARGS:---config c1 --serial} > gpurun_out/kstats_$tag.log 2>&1 || { tail -20 gpurun_out/kstats_$tag.log; return 1; }
  tail -1 gpurun_out/kstats_$tag.log | cut -c1-300
  f=$(find gpurun_out/kstats_$tag -name "*kernel_trace.csv" | head -1)
  python scripts/kstats_tail.py "$f" ${TAIL:-50} gpurun_out/kstats_${tag}_tail.json
  rm -f "$f"
}

task_pcie_trace() {
  rm -rf gpurun_out/pcie_trace && mkdir -p gpurun_out/pcie_trace
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/pcie_trace -o run -- \
    python -u bench.py --steps 20 --warmup 3 --latency-steps 3 --loaded-steps 0 --no-cpu-baseline --prof-every 0 --pcie-steps 30 ${KARGS:-} \
    > gpurun_out/pcie_trace.log 2>&1 || { tail -20 gpurun_out/pcie_trace.log; return 1; }
  tail -1 gpurun_out/pcie_trace.log | cut -c1-200
  python scripts/copy_timeline.py gpurun_out/pcie_trace > gpurun_out/pcie_timeline.txt 2>&1
  cat gpurun_out/pcie_timeline.txt
}

task_route_trace() {
  local lib tag f
  for lib in "" build_abl/lib_*.so; do
    [ -n "$lib" ] && [ ! -e "$lib" ] && continue
    tag=$(basename "${lib:-cur}" .so)
    rm -rf gpurun_out/rtrace_$tag && mkdir -p gpurun_out/rtrace_$tag
    RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rtrace_$tag \
      -o run -- python -u bench.py --route --steps 100 --warmup 3 --latency-steps 3 --loaded-steps 0 --pcie-steps 0 --no-cpu-baseline ${KARGS:-} \
      > gpurun_out/rtrace_$tag.log 2>&1 || { tail -5 gpurun_out/rtrace_$tag.log; return 1; }
    echo "== $tag"
    f=$(find gpurun_out/rtrace_$tag -name "*kernel_trace.csv" | head -1)
    python scripts/trace_busy.py "$f" 40 > gpurun_out/rtrace_${tag}_busy.txt && head -12 gpurun_out/rtrace_${tag}_busy.txt
    rm -f "$f"
  done
}

task_serial_trace() {
  local lib tag
  for lib in "" build_abl/lib_*.so; do
    [ -n "$lib" ] && [ ! -e "$lib" ] && continue
    tag=$(basename "${lib:-cur}" .so)
    rm -rf gpurun_out/tr_$tag && mkdir -p gpurun_out/tr_$tag
    RL_LIB_PATH=${lib:+$PWD/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
      -d gpurun_out/tr_$tag -o run -- python -u bench.py --steps 30 --warmup 3 --latency-steps 3 --loaded-steps 0 \
      --no-cpu-baseline --prof-every 0 --pcie-steps 0 --serial ${KARGS:---config c1} > gpurun_out/tr_$tag.log 2>&1 \
      || { tail -20 gpurun_out/tr_$tag.log; return 1; }
    summary gpurun_out/tr_$tag.log $tag
  done
}

task_seed_sweep() {
  local cfg=${CFG:-c2} seed
  for seed in ${SEEDS:-1 2 3 4 5 6 7 8 9 10 11 12}; do
    timeout -k 10 120 python -u bench.py --config $cfg --hash-seed $seed --steps 40 --warmup 2 --latency-steps 12 --loaded-steps 0 \
      --no-cpu-baseline --pcie-steps 0 > gpurun_out/seed_${cfg}_$seed.log 2>&1 || { tail -5 gpurun_out/seed_${cfg}_$seed.log; return 1; }
    summary gpurun_out/seed_${cfg}_$seed.log "seed $seed" '"p50 %.3f p99 %.3f" % (d["p50_batch_ms"], d["p99_batch_ms"])'
  done
}

task_split_prof() {
  local lib tag
  for lib in ${LIBS:-build_abl/lib_sprof.so}; do
    tag=$(basename $lib .so)
    RL_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --config c2u --steps 10 --warmup 2 --latency-steps 2 --loaded-steps 0 \
      --pcie-steps 0 --no-cpu-baseline > gpurun_out/split_prof_$tag.log 2>&1 || { tail -5 gpurun_out/split_prof_$tag.log; return 1; }
    echo "== $tag"; grep split_long gpurun_out/split_prof_$tag.log | tail -4
  done
}

[ $# -gt 0 ] || { sed -n 2,30p "$0"; exit 2; }
for t in "$@"; do
  case "$t" in
    round) task_round ;;
    evidence) task_evidence ;;
    ab) task_ab ;;
    kstats) task_kstats ;;
    pmc) task_pmc ;;
    pcie-trace) task_pcie_trace ;;
    route-trace) task_route_trace ;;
    serial-trace) task_serial_trace ;;
    seed-sweep) task_seed_sweep ;;
    split-prof) task_split_prof ;;
    *) echo "unknown task: $t"; exit 2 ;;
  esac || exit 1
done
