set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for lib in cur main; do
  rm -rf gpurun_out/tr_$lib && mkdir -p gpurun_out/tr_$lib
  if [ $lib = main ]; then export RL_LIB_PATH=$PWD/build_abl/lib_main.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tr_$lib -o run -- \
    python -u bench.py --steps 30 --warmup 3 --latency-steps 3 --loaded-steps 0 --no-cpu-baseline --prof-every 0 --pcie-steps 0 --config c1 --serial \
    > gpurun_out/tr_$lib.log 2>&1 || { tail -20 gpurun_out/tr_$lib.log; exit 1; }
  tail -1 gpurun_out/tr_$lib.log | cut -c1-200
done
