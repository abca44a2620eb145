# Round 6: the routed protocol at C3 shard scale, W = 8 loopback ranks on one
# GPU (62.5M tenants x {sec,min} = 125M keys per rank, 1B over the world;
# 2^28 slots + 2^28 history entries per rank = 206 GB of tables), then the
# same run under a kernel trace for the partition / scan / exchange kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/loopback_c3
timeout -k 10 600 python -u bench.py --loopback 8 --config c3 --steps 40 --warmup 3 \
  > gpurun_out/loopback_c3/bench_w8_c3.log 2>&1 || { tail -20 gpurun_out/loopback_c3/bench_w8_c3.log; exit 1; }
grep '^{"metric' gpurun_out/loopback_c3/bench_w8_c3.log | cut -c1-300
RL_DEBUG_ROUTE_TIMING=1 timeout -k 10 600 python -u bench.py --loopback 8 --config c3 --steps 40 --warmup 3 \
  > gpurun_out/loopback_c3/timing_w8_c3.log 2>&1 || { tail -20 gpurun_out/loopback_c3/timing_w8_c3.log; exit 1; }
grep route_host_us gpurun_out/loopback_c3/timing_w8_c3.log | head -3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/loopback_c3/trace -o run -- \
  python -u bench.py --loopback 8 --config c3 --steps 20 --warmup 3 > gpurun_out/loopback_c3/trace_w8_c3.log 2>&1 \
  || { grep -v "^    @" gpurun_out/loopback_c3/trace_w8_c3.log | tail -20; exit 1; }
f=$(find gpurun_out/loopback_c3/trace -name "*kernel_stats.csv" | head -1)
head -30 "$f"
find gpurun_out/loopback_c3/trace -name "*kernel_trace.csv" -delete
