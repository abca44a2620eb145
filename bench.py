"""Benchmark: rate-limit decisions/sec of the MI355X fixed-window backend.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2]

A step is one DoLimit batch over device-resident packed input (BASELINE.json
configs[1] = C1 by default: 10M tenant stems x {sec, min} per GPU, 500k
requests = 1M descriptors per batch, uniform tenants, `now` +1 s per step).
Before timing, every key is inserted ("warm-up inserts all 20M keys").
N>1 (torch.distributed.run, one process per GPU): the table is hash-sharded
over the GPUs (10M tenants x 2 keys per GPU; --config c3: 62.5M, i.e. 1B keys
on 8), each rank draws its 1M-descriptor slice from the whole node's tenant
space, and every batch is routed to the owning GPUs and back over RCCL by the
library itself (rl_comm_init / rl_do_limit_routed_async, send/recv over xGMI;
--route-impl python: the collectives from ratelimit_amd/sharded.py); weak
scaling, value = all ranks' decisions / max-over-ranks time. --route runs the
routed path at N=1.

Besides the contract line, rank 0 reports:
  roofline      dominant kernel (k_table) achieved GB/s on the canonical
                B_alg = key_len + 16 + 12 + 64 B per decision,
                from HIP events on the library's stream;
  cpu_baseline  the C restatement oracle, key-sharded over the host's cores
                (and on 1 core), on a bounded sample of the same stream.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "rate-limit decisions/sec (whole node) at 10M/1B keys; p99 batch latency"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
LONG_RUN = 32  # rl_kernels.h: runs at least this long take the parallel path (k_late)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c1", choices=["c1", "c2", "c2u", "c3"],
                    help="c1 uniform / c2 Zipf(1.1), hits 1..8 / c2u = c2 with half the hot tenants' sec descriptors overridden to MINUTE (one stem under two units) / c3 = c1 at 62.5M tenants per GPU (1B keys on 8)")
    ap.add_argument("--requests", type=int, default=500_000, help="requests per batch per GPU (2 descriptors each)")
    ap.add_argument("--tenants", type=int, default=0, help="tenants per GPU (default 10M; c3 62.5M)")
    ap.add_argument("--distinct-batches", type=int, default=4)
    ap.add_argument("--latency-steps", type=int, default=1000,
                    help="batches timed one at a time (submit -> outputs ready): p50/p99_batch_ms")
    ap.add_argument("--loaded-steps", type=int, default=1000,
                    help="batches submitted at the measured headline rate with the pipeline full: "
                         "p50/p99_loaded_batch_ms (submit -> outputs ready, rl_batch_progress)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0: the process's CPU share, cpu_share())")
    ap.add_argument("--prof-every", type=int, default=13,
                    help="time every k-th batch's stages with HIP events and k_table's run time on the device "
                         "clock (the roofline's live time; the k-th timed batch first: 1 sample in 20 steps, 15 in "
                         "200; each sample costs its batch a few us, profiles/r06/prof_cost/)")
    ap.add_argument("--no-fill", action="store_true")
    ap.add_argument("--pcie-steps", type=int, default=60, help="host-fed (PCIe) batches timed after the device phase")
    ap.add_argument("--pcie-formats", default="prefixed,compact,soa",
                    help="host-fed formats timed (the first is the reported pcie_fed rate)")
    ap.add_argument("--slots-per-key", type=float, default=0.0,
                    help="table slots per live key, rounded to the power of 2 above (0: 4, c3 2)")
    ap.add_argument("--history-entries", type=int, default=0,
                    help="history log entries (rl_config.history_entries; 0: table slots)")
    ap.add_argument("--jitter", type=int, default=0,
                    help="EXPIRATION_JITTER_MAX_SECONDS (the history horizon: older windows kept div + J s)")
    ap.add_argument("--hash-seed", type=int, default=0, help="stem hash key (0: drawn at random per run; reported)")
    ap.add_argument("--route", action="store_true", help="use the routed (all_to_all) path even at N=1")
    ap.add_argument("--route-impl", default="lib", choices=["lib", "python"],
                    help="routed step: inside the library over RCCL (lib) or collectives from Python")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo + --one-device: rehearse N ranks on one GPU (host-staged exchange)")
    ap.add_argument("--one-device", action="store_true", help="every rank uses cuda:0 (rehearsal only)")
    ap.add_argument("--serial", action="store_true",
                    help="submit every batch on one stream, unpipelined (isolated per-kernel times for profiling)")
    ap.add_argument("--shards", type=int, default=1,
                    help="S > 1 (N = 1): one ctx hash-sharding its table over S shards (rl_config.n_shards) on this "
                         "GPU: host batches are cut into one slice per shard, each routed to its owners and back")
    ap.add_argument("--loopback", type=int, default=0,
                    help="W > 0: W ranks of the library router as threads of this process, all on cuda:0, "
                         "exchanging through the in-process loopback transport (the W-rank protocol on one GPU)")
    args = ap.parse_args()
    if not args.tenants:
        args.tenants = 62_500_000 if args.config == "c3" else 10_000_000
    if not args.slots_per_key:  # c3: 2^28 x 64-B slots (17 GB) + 2^26 ring lines (8.6 GB) per GPU
        args.slots_per_key = 2.0 if args.config == "c3" else 4.0
    return args


def to_dev(a, torch):
    return {k: torch.from_numpy(np.ascontiguousarray(v).view(np.int32) if v.dtype == np.uint32
                                else np.ascontiguousarray(v)).cuda() for k, v in a.items()}


def progress(msg):
    """A phase boundary on stderr (rank 0): long runs (C3's fill) show they are alive."""
    if os.environ.get("RANK", "0") == "0":
        print("[bench] %s" % msg, file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.loopback:
        return loopback_main(args)
    import torch
    import torch.distributed as dist

    from ratelimit_amd import abi, workloads as W
    from ratelimit_amd.limiter import Backend

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.one_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    torch.cuda.set_device(local)
    # every torch op and library call of the benchmark on one non-default
    # stream: the library orders each batch after the work that produced its
    # inputs on it (the default stream's handle is NULL: unordered)
    main_stream = torch.cuda.Stream()
    torch.cuda.set_stream(main_stream)
    routed = world > 1 or args.route
    if routed:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29561")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    def barrier():
        if routed:
            dist.barrier()

    nq = args.requests
    n = 2 * nq
    T = args.tenants
    keys_per_gpu = 2 * T
    # Table at <= 25% load: HBM is plentiful (288 GB) and every extra linear
    # probe is one more random 64-B sector read (tools/slotprobe.hip).
    slots = 1 << max(16, int(np.ceil(np.log2(args.slots_per_key * keys_per_gpu))))
    # a routed owner receives ~n descriptors (binomial spread across sources)
    cap = n if not routed else int(n * 1.05) + 4096
    seed = args.hash_seed
    if not seed and not routed:  # a random key per run, as the library would draw; reported in the line
        import secrets
        seed = secrets.randbits(62) + 1
    if routed and not seed:  # every shard of one table hashes stems under one key: rank 0 draws it
        import secrets
        t = torch.tensor([secrets.randbits(62) + 1 if rank == 0 else 0], dtype=torch.int64,
                         device="cpu" if args.dist_backend == "gloo" else "cuda")
        dist.broadcast(t, 0)
        seed = int(t.item())
    if args.serial:  # isolated kernel timings: each batch's stages serially on the bench stream
        os.environ["RL_DEBUG_SERIAL"] = "1"
    # a routed owner attributes stats per source rank: world x n_rules rule slots
    if args.shards > 1 and routed:
        raise SystemExit("--shards is a single-process option (N = 1, no --route)")
    if args.shards > 1 and not seed:
        import secrets
        seed = secrets.randbits(62) + 1
    sh = dict(n_shards=args.shards, shard_devices=[local] * args.shards) if args.shards > 1 else {}
    NR = args.n_rules = 3 if args.config == "c2u" else 2  # rules per batch (c2u: the override's own stats key)
    be = Backend(0.8, False, table_slots=slots, max_batch=cap, max_rules=max(8, NR * world * args.shards),
                 device=local, hash_seed=seed, max_stem_bytes=64 * cap, history_entries=args.history_entries,
                 jitter=args.jitter, **sh)
    now0 = W.NOW0
    py_route = routed and (args.route_impl == "python" or args.dist_backend == "gloo")
    if routed and not py_route:
        # the routed step inside the library: RCCL send/recv over xGMI (rl_comm.hip)
        from ratelimit_amd.sharded import RcclRouter
        sc = RcclRouter(be)
    elif routed:
        from ratelimit_amd.sharded import DeviceRouteOps, Exchange, ShardedRateLimitCache
        # forward and return collectives on two groups: batch t+1's forward
        # exchange overlaps batch t's owner pipeline and return exchange
        ret_group = dist.new_group(backend=args.dist_backend)
        sc = ShardedRateLimitCache(DeviceRouteOps(be), Exchange(), max_batch=n, max_stem_bytes=64 * n,
                                   device=torch.device("cuda", local), max_recv=cap, max_recv_stem=64 * cap,
                                   ret_exchange=Exchange(ret_group))
    out = {"code": torch.empty(n, dtype=torch.uint8, device="cuda"),
           "limit_remaining": torch.empty(n, dtype=torch.int32, device="cuda"),
           "reset_s": torch.empty(n, dtype=torch.int32, device="cuda"),
           "stats": torch.zeros(NR * 6, dtype=torch.int64, device="cuda")}

    serial_stream = main_stream.cuda_stream

    # the last timed batch writes its own outputs (the self-check reads them;
    # batches in flight share `out`, whose stats several batches add into)
    out_chk = {k: torch.zeros_like(v) for k, v in out.items()}
    check_step = args.warmup + args.steps - 1

    # The library call a C or Go caller makes per batch: its rl_batch /
    # rl_result structs are built once per (distinct batch, output set) and
    # only the clock array's pointer changes per step, so the host time per
    # step is the library's, not Python's struct building (~15 us). Inputs are
    # complete before the timed region (synchronized), so no caller stream.
    structs = {}

    def do_step(inp, bn, bq, o=None, key=None):
        o = out if o is None else o
        if routed:
            sc.submit(inp, bn, bq, NR, o)
        elif args.serial or key is None:
            be.do_limit_device(inp, o, bn, bq, NR, stream=serial_stream)  # (pipelined; --serial: RL_DEBUG_SERIAL)
        else:
            k = (key, o is out)
            if k not in structs:
                structs[k] = (abi.make_batch_struct(inp, bn, bq, NR), abi.make_result_struct(o))
            bs, rs = structs[k]
            bs.now = abi.ptr(inp["now"])
            be.do_limit_structs(bs, rs)

    def sync():
        if routed:
            sc.finish()
        else:
            be.synchronize()

    # ---- fill: every key of the node's tenant space (rank r inserts tenants
    # [r*T, (r+1)*T); routed batches land on their owners). Not timed.
    t_fill = time.perf_counter()
    if not args.no_fill:
        for s0 in range(0, T, nq):
            ids = torch.arange(s0, min(s0 + nq, T), dtype=torch.int64, device="cuda") + rank * T
            a, bn, bq, br = W.c1_batch_dev(ids, now0 - 1)
            do_step(a, bn, bq)
        sync()
    t_fill = time.perf_counter() - t_fill
    progress("fill done (%.1f s)" % t_fill)

    # ---- device-resident input batches + per-step clocks. Requests draw from
    # the whole node's tenant space (world * T): with routing every rank talks
    # to every owner.
    sampler = W.ZipfSampler(world * T, 1.1) if args.config in ("c2", "c2u") else None
    dev_batches = []
    uniq = []  # descriptors k_table answers: keys seen once + runs shorter than LONG_RUN (the rest: k_late)
    host_batches = []
    for a, bn, bq, ten in make_batches(args, W, rank, world * T, sampler):
        _, cnt = np.unique(ten, return_counts=True)
        uniq.append(2 * int(cnt[cnt < LONG_RUN].sum()))  # (a tenant's two stems: one per unit)
        host_batches.append((a, bn, bq))
        dev_batches.append(to_dev(a, torch))
    stem_len = 34
    total_steps = args.warmup + args.steps + args.steps + args.latency_steps + args.loaded_steps
    nows = [torch.full((nq,), now0 + s, dtype=torch.int64, device="cuda") for s in range(total_steps)]
    torch.cuda.synchronize()

    step = [0]
    host_delay = float(os.environ.get("RL_BENCH_HOST_DELAY_US", "0")) * 1e-6
    host_in_call = [0.0]  # host seconds inside the library's submit calls (timed steps only)

    def run_step():
        s = step[0]
        inp = dict(dev_batches[s % len(dev_batches)])
        inp["now"] = nows[s]
        t = time.perf_counter()
        do_step(inp, n, nq, out_chk if s == check_step else None, key=s % len(dev_batches))
        host_in_call[0] += time.perf_counter() - t
        if host_delay:  # (RL_BENCH_HOST_DELAY_US: a slower submitter, to see whether the host paces the GPU)
            while time.perf_counter() - t < host_delay:
                pass
        step[0] += 1

    # (the table counters before the warmup: k_table_info scans the whole
    # table, and run between the warmup and the timed region it would leave
    # the timed batches a cold Infinity Cache; routed runs use the delta per
    # owner batch, warmup batches included)
    info0 = be.table_info()
    # ---- warmup
    for _ in range(args.warmup):
        run_step()
    sync()
    torch.cuda.synchronize()

    # ---- timed region: exactly K steps. The library records HIP events at the
    # stage boundaries on each batch's own stream (pipelined batches are timed
    # as they run, k_table included: the roofline's kernel time).
    be.profile(args.prof_every > 0, args.prof_every)
    be.profile_read()
    recv = []
    if py_route:
        for k in sc.host_s:
            sc.host_s[k] = 0.0
    barrier()
    torch.cuda.synchronize()
    host_in_call[0] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_step()
        if py_route:
            recv.append(sc.last_recv)
    host_submit_ms = host_in_call[0] / args.steps * 1e3
    sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    # (after the timed region) the last timed batch's answers, checked below against the oracle
    last_out = {k: v.cpu().numpy().view(np.uint32) if v.dtype == torch.int32 else v.cpu().numpy()
                for k, v in out_chk.items()}
    last_step = check_step
    assert step[0] - 1 == check_step
    route_host = {k: round(v / args.steps * 1e3, 4) for k, v in sc.host_s.items()} if py_route else None
    info1 = be.table_info()
    if routed and not recv:  # decisions this rank's table answered per owner batch
        recv = [(info1["decisions"] - info0["decisions"]) / max(info1["batches"] - info0["batches"], 1)]
    stage_ms, nb = be.profile_read()
    be.profile(False)
    stage_avg = {k: v / max(nb, 1) for k, v in stage_ms.items() if k != "table_kernel"}
    n_unique = float(np.mean(uniq)) if world == 1 and args.shards == 1 else None  # (routed: owners not tracked)
    n_owner = float(np.mean(recv)) if recv else float(n)
    if routed:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * n * args.steps / elapsed

    progress("timed steps done")
    # ---- batch latency: submit -> outputs ready, one batch at a time
    lat = []
    for i in range(args.latency_steps):
        t1 = time.perf_counter()
        run_step()
        sync()
        lat.append((time.perf_counter() - t1) * 1e3)
        if i % 250 == 249 or lat[-1] > 50:
            progress("latency batch %d: %.2f ms" % (i + 1, lat[-1]))
    lat = np.array(lat) if lat else np.array([float("nan")])
    loaded = None
    if not routed and args.shards == 1 and args.loaded_steps > 0:
        progress("latency done")
        loaded = loaded_latency(be, run_step, args.loaded_steps, elapsed / args.steps)
        progress("loaded latency done")
    pcie = None if (routed or args.pcie_steps <= 0) else pcie_fed(args, be, host_batches, now0 + total_steps)
    info = be.table_info()
    if routed:
        lt = torch.tensor([float(np.percentile(lat, 99))], dtype=torch.float64,
                          device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        p99 = float(lt.item())
    else:
        p99 = float(np.percentile(lat, 99))

    # ---- self-check (outside every timed region): the last timed batch's
    # answers for a tenant subset against the C oracle replaying that subset's
    # whole history (fill, warmup, timed steps, every rank's slices in global
    # order); keys are independent, so the subset's answers must be equal.
    # A wrong-answer fast path cannot post a line.
    check = verify(args, W, last_out, last_step, host_batches[0][1], world, rank, T, now0, sampler)
    if routed:
        ok = torch.tensor([1 if check["verified"] else 0], dtype=torch.int32,
                          device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        check["verified"] = check["verified"] and bool(ok.item())
    if not check["verified"]:
        print("[bench] SELF-CHECK FAILED (rank %d): %s; no result line (unverified rate %.4g decisions/s, %.4f ms "
              "per step)" % (rank, json.dumps(check), value, elapsed / args.steps * 1e3), file=sys.stderr, flush=True)
        be.close()
        raise SystemExit(1)
    progress("self-check: %d descriptors equal to the oracle" % check["checked"])

    if rank != 0:
        be.close()
        if routed:
            dist.destroy_process_group()
        return

    # k_table answers the keys seen once in the batch and the runs shorter than
    # LONG_RUN (replayed in registers): all of C1/C3 but the ~100 hash-prefix
    # collisions, most of C2 but its hot keys' long runs. SURVEY §8(d): 136 B per
    # decision (key = stem + 10-digit window, slot 64 B read, 16 B window
    # write-back, 12 B out).
    b_alg = stem_len + 10 + 16 + 12 + 64
    # k_table's time per launch: its own run time on the device clock (first
    # workgroup start to last workgroup end, as rocprofv3's kernel trace
    # measures it), and the HIP events around the launch on its stream (which
    # also hold the launch's wait behind the other streams' kernels)
    kern_ms = stage_ms.get("table_kernel", 0.0)  # (already a per-batch average, over the sampled timed batches)
    ev_ms = stage_avg["table"]
    achieved = b_alg * n_unique / (kern_ms * 1e-3) / 1e9 if (kern_ms > 0 and n_unique) else None
    achieved_ev = b_alg * n_unique / (ev_ms * 1e-3) / 1e9 if (ev_ms > 0 and n_unique) else None
    pipe_ms = elapsed / args.steps * 1e3
    traffic, traffic_cal = None, None
    tp = os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
    if os.path.exists(tp) and not routed:
        try:
            tj = json.load(open(tp))
            traffic = tj.get("k_table_bytes_per_launch")  # 2 x FETCH_SIZE + WRITE_SIZE (guide)
            rb = tj.get("k_table_read_bytes_bounds")       # probe-calibrated reads (tools/pmcprobe.hip)
            wr = tj["kernels"]["rl::k_table"]["write_size_bytes"]
            traffic_cal = [rb[0] + wr, rb[1] + wr] if rb else None
        except Exception:
            traffic, traffic_cal = None, None
    roofline = {"bound": "hbm", "kernel": "k_table", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                "kernel_us": round(kern_ms * 1e3, 2) if kern_ms > 0 else None,
                "time_basis": "k_table's own run time per launch on the device clock (first workgroup start to "
                              "last workgroup end = rocprofv3 kernel duration), averaged over the sampled timed batches (every --prof-every-th)",
                "event_bracket": {"us": round(ev_ms * 1e3, 2) if ev_ms > 0 else None, "achieved": achieved_ev,
                                  "frac": (achieved_ev / HBM_PEAK_GBS) if achieved_ev else None,
                                  "basis": "HIP events around the k_table launch on its stream (includes its "
                                           "wait behind other streams' kernels)"},
                "traffic_calibrated_bounds": traffic_cal,
                "bytes_alg_per_decision": b_alg, "decisions_per_launch": n_unique,
                # (scripts/trace_timed.py: the timed launches in a kernel trace of this run
                # are the K before the last k_table_launches_after_timed)
                "k_table_launches_after_timed": int(info["batches"] - info1["batches"]),
                "descriptors_per_batch": n_owner,
                "stage_ms": {k: round(v, 4) for k, v in stage_avg.items()},
                "pipeline_achieved": b_alg * n_owner / (pipe_ms * 1e-3) / 1e9 if pipe_ms > 0 else None}
    # the kernels that answer every decision: k_table (keys seen once, short
    # runs) and the long runs' parallel path (k_fast_over, k_late), timed by the
    # table and finish stages (finish also holds k_finish: a conservative figure)
    ans_ms = stage_avg.get("table", 0.0) + stage_avg.get("finish", 0.0)
    if ans_ms > 0 and not routed:
        ach = b_alg * n_owner / (ans_ms * 1e-3) / 1e9
        roofline["answering_kernels"] = {"kernels": "k_table + k_fast_over + k_late + k_finish", "achieved": ach,
                                         "frac": ach / HBM_PEAK_GBS, "decisions_per_batch": n_owner,
                                         "ms_per_batch": ans_ms}

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, W)

    dist_desc = {"c1": "uniform", "c2": "Zipf(1.1), hits 1..8", "c3": "uniform",
                 "c2u": "Zipf(1.1), hits 1..8, half the 16 hottest tenants' sec descriptors overridden to MINUTE"}[args.config]
    line = {
        "metric": METRIC, "value": value, "unit": "decisions/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "%s: %.1fM tenant stems x {sec,min} per GPU (%d live keys node-wide), "
                               "%d-descriptor batches per GPU, %s tenants, now +1 s per batch, all keys pre-inserted"
                               % (args.config.upper(), T / 1e6, 2 * T * world, n, dist_desc),
                   "global_batch": world * n, "batch_per_gpu": n, "live_stem_slots_per_gpu": info["live_slots"],
                   "table_slots": slots, "history_entries": info["history_entries"],
                   "history_appended": info["history_appended"], "history_lost": info["history_lost"], "jitter": args.jitter,
                   "table_hbm_gb": round((slots * 64 + info["history_entries"] * 32) / 1e9, 2), "hash_seed": seed,
                   "parallelism": ("hash-sharded table x%d, %s" % (
                                      world, "RCCL send/recv routing inside the library" if not py_route else
                                      "all_to_all routing from Python (%s)" % args.dist_backend)) if routed else
                                  ("one ctx, table hash-sharded over %d shards on this GPU (loopback routing)"
                                   % args.shards) if args.shards > 1 else "single GPU"},
        "p50_batch_ms": float(np.percentile(lat, 50)), "p99_batch_ms": p99, "latency_batches": int(lat.size),
        "host_submit_ms": round(host_submit_ms, 4),
        **({"p50_loaded_batch_ms": loaded["p50_ms"], "p99_loaded_batch_ms": loaded["p99_ms"],
            "loaded": loaded} if loaded else {}),
        "pcie_fed": pcie,
        "roofline": roofline, "cpu_baseline": cpu, "fill_s": round(t_fill, 2),
        "verified": check["verified"], "self_check": check,
        **({"route_host_ms_per_step": route_host} if py_route else {}),
    }
    print(json.dumps(line), flush=True)
    be.close()
    if routed:
        dist.destroy_process_group()


def make_batches(args, W, rank, tenants, sampler):
    """Rank `rank`'s distinct input batches (deterministic per rank, so any
    rank can regenerate any other's for the self-check): (arrays without
    now, n, n_requests, tenant of each request)."""
    rng = np.random.default_rng((0xC2 if sampler is not None else 0xC1) + 7919 * rank)
    nq = args.requests
    out = []
    for _ in range(args.distinct_batches):
        ten = rng.integers(0, tenants, nq) if sampler is None else sampler.sample(rng, nq)
        if sampler is None:
            a, bn, bq, br = W.c1_batch(ten, W.NOW0)
        elif args.config == "c2u":
            a, bn, bq, br = W.c2u_batch(ten, W.NOW0, rng.integers(1, 9, nq).astype(np.uint32), rng)
        else:
            a, bn, bq, br = W.c1_batch(ten, W.NOW0, rng.integers(1, 9, nq).astype(np.uint32))
        a.pop("now")
        out.append((a, bn, bq, ten))
    return out


def select(a, n, nq, keep, now):
    """Batch a (without now) restricted to the descriptors where keep is True,
    every request at clock `now`."""
    idx = np.nonzero(keep[:n])[0]
    off = a["stem_off"].astype(np.int64)
    L = off[idx + 1] - off[idx]
    o = np.zeros(idx.size + 1, np.uint32)
    o[1:] = np.cumsum(L)
    # (gather the kept stems' bytes with one index array)
    pos = np.repeat(off[idx] - o[:-1], L) + np.arange(int(o[-1]))
    out = {"stem_bytes": a["stem_bytes"][pos], "stem_off": o, "now": np.full(nq, now, np.int64)}
    for k in ("req_idx", "unit", "flags", "limit", "hits", "rule_id"):
        out[k] = a[k][idx]
    return out, idx.size, nq


def verify(args, W, got, last_step, n, world, rank, T, now0, sampler, modulus=128):
    """The bench's answers for the last timed step, checked against the C
    oracle (oracle/rl_oracle.c) on the tenants t % (modulus * world) == 77:
    the oracle replays exactly their history (the fill at now0 - 1, then every
    step s <= last_step: batch s % distinct of every rank, rank-major, at
    now0 + s). Also: the per-rule TotalHits deltas sum to the batch's hits."""
    from oracle.c_oracle import COracle
    t0 = time.perf_counter()
    M = modulus * world
    r0 = 77 % M
    co = COracle(0.8, False, False)
    own = make_batches(args, W, rank, world * T, sampler)
    ranks = [own if q == rank else make_batches(args, W, q, world * T, sampler) for q in range(world)]
    checked, bad = 0, {}
    try:
        if not args.no_fill:
            co.do_limit(*W.c1_batch(np.arange(r0, world * T, M), now0 - 1))
        for s in range(last_step + 1):
            for q in range(world):
                a, bn, bq, ten = ranks[q][s % len(ranks[q])]
                keep = (ten % M == r0)[a["req_idx"]]
                if not keep.any():
                    continue
                o = co.do_limit(*select(a, bn, bq, keep, now0 + s), args.n_rules)
                if q == rank and s == last_step:
                    for f in ("code", "limit_remaining", "reset_s"):
                        g = got[f][:n][keep]
                        if not np.array_equal(g, o[f]):
                            i = np.nonzero(g != o[f])[0]
                            bad[f] = {"mismatches": int(i.size), "first": int(i[0]), "gpu": int(g[i[0]]),
                                      "oracle": int(o[f][i[0]])}
                    checked = int(keep.sum())
    finally:
        co.close()
    a = own[last_step % len(own)][0]
    hits = int(np.maximum(a["hits"], 1).astype(np.int64).sum())
    total_hits = int(got["stats"].reshape(-1, 6)[:, 0].astype(np.int64).sum())
    if total_hits != hits:
        bad["total_hits"] = {"gpu": total_hits, "batch": hits}
    return {"verified": not bad and checked > 0, "checked": checked, "step": last_step,
            "subset": "tenants t %% %d == %d" % (M, r0), "mismatches": bad or None,
            "oracle": "oracle/rl_oracle.c (C restatement), the subset's whole history replayed",
            "seconds": round(time.perf_counter() - t0, 2)}


def loaded_latency(be, run_step, k_steps, interval_s):
    """Batch latency under load: k_steps batches submitted open-loop at the
    measured headline rate (one every interval_s, the pipeline full), each
    timed from its submit call to the moment rl_batch_progress first reports
    its outputs complete (polled between submissions, ~5 us resolution)."""
    sub, done = [], []
    s0, d0 = be.batch_progress()

    def poll():
        _, d = be.batch_progress()
        t = time.perf_counter()
        while len(done) < d - d0:
            done.append(t)

    t0 = time.perf_counter()
    for i in range(k_steps):
        target = t0 + i * interval_s
        while time.perf_counter() < target:
            poll()
        sub.append(time.perf_counter())
        run_step()
        poll()
    while len(done) < k_steps:
        poll()
    el = done[-1] - t0
    lat = (np.array(done[:k_steps]) - np.array(sub)) * 1e3
    return {"p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
            "max_ms": float(lat.max()), "batches": k_steps, "offered_interval_ms": interval_s * 1e3,
            "achieved_interval_ms": el / k_steps * 1e3,
            "method": "open-loop submissions at the timed rate; completion = rl_batch_progress (outputs written)"}


def loopback_main(args):
    """--loopback W: the routed step of an W-GPU node (rl_comm.hip: partition,
    counts, records and stems, owner pipelines, results and stats, scatter)
    with every rank a thread of this process on cuda:0 and the exchanges
    through the loopback transport. Each rank owns `tenants` tenants x {sec,
    min} (all pre-inserted) and submits --requests requests per step drawn
    from the whole world's tenant space. value = W x descriptors per step /
    max-over-ranks time: one GPU does every rank's work, so this measures the
    protocol's cost on the GPU, not scaling."""
    import secrets
    import threading

    import torch

    from ratelimit_amd import workloads as W
    from ratelimit_amd.limiter import Backend
    from ratelimit_amd.sharded import WIRE_BYTES, LibRouter, loopback_id
    R = args.loopback
    nq, n, T = args.requests, 2 * args.requests, args.tenants
    slots = 1 << max(16, int(np.ceil(np.log2(args.slots_per_key * 2 * T))))
    cap = int(n * 1.05) + 4096
    seed = args.hash_seed or secrets.randbits(62) + 1
    torch.cuda.set_device(0)
    uid = loopback_id()
    bes = [Backend(0.8, False, table_slots=slots, max_batch=cap, max_rules=max(8, 2 * R), device=0, hash_seed=seed,
                   max_stem_bytes=64 * cap) for _ in range(R)]
    routers = [LibRouter(be, R, r, uid) for r, be in enumerate(bes)]
    gate = threading.Barrier(R)
    times, fills, errs, stem_mean = [0.0] * R, [0.0] * R, [None] * R, [0.0] * R

    def body(r):
        try:
            torch.cuda.set_device(0)
            torch.cuda.set_stream(torch.cuda.Stream())
            out = {"code": torch.empty(n, dtype=torch.uint8, device="cuda"),
                   "limit_remaining": torch.empty(n, dtype=torch.int32, device="cuda"),
                   "reset_s": torch.empty(n, dtype=torch.int32, device="cuda"),
                   "stats": torch.zeros(2 * 6, dtype=torch.int64, device="cuda")}
            rt = routers[r]
            t = time.perf_counter()
            if not args.no_fill:
                for s0 in range(0, T, nq):
                    ids = torch.arange(s0, min(s0 + nq, T), dtype=torch.int64, device="cuda") + r * T
                    a, bn, bq, _ = W.c1_batch_dev(ids, W.NOW0 - 1)
                    rt.submit(a, bn, bq, 2, out)
                rt.finish()
            fills[r] = time.perf_counter() - t
            rng = np.random.default_rng(0xC1 + 7919 * r)
            batches = []
            for _ in range(args.distinct_batches):
                a, _, _, _ = W.c1_batch(rng.integers(0, R * T, nq), W.NOW0)
                a.pop("now")
                stem_mean[r] = float(a["stem_off"][n]) / n
                batches.append(to_dev(a, torch))
            total = args.warmup + args.steps
            nows = [torch.full((nq,), W.NOW0 + s, dtype=torch.int64, device="cuda") for s in range(total)]
            for s in range(args.warmup):
                rt.submit(dict(batches[s % len(batches)], now=nows[s]), n, nq, 2, out)
            rt.finish()
            torch.cuda.synchronize()
            gate.wait()
            t = time.perf_counter()
            for s in range(args.warmup, total):
                rt.submit(dict(batches[s % len(batches)], now=nows[s]), n, nq, 2, out)
            rt.finish()
            torch.cuda.synchronize()
            times[r] = time.perf_counter() - t
        except Exception as e:  # (a failed rank's peers time out in the loopback transport)
            errs[r] = repr(e)

    ts = [threading.Thread(target=body, args=(r,)) for r in range(R)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    if any(errs):
        raise SystemExit("loopback bench failed: %s" % errs)
    info = [be.table_info() for be in bes]
    for be in bes:
        be.close()
    elapsed = max(times)
    line = {
        "metric": METRIC, "value": R * n * args.steps / elapsed, "unit": "decisions/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "C1 routed: %d loopback ranks on one GPU, %.1fM tenants x {sec,min} per rank, "
                               "%d-descriptor slices per rank per step, uniform over all ranks' tenants"
                               % (R, T / 1e6, n),
                   "global_batch": R * n, "batch_per_rank": n, "table_slots_per_rank": slots, "hash_seed": seed,
                   "live_stem_slots": sum(i["live_slots"] for i in info),
                   "parallelism": "hash-sharded table x%d, library router over the loopback transport" % R},
        "fill_s": round(max(fills), 2),
        # what one remote descriptor moves over the links: its wire record and
        # stem bytes out, its 8-B packed result back ((R-1)/R of a uniform
        # slice is remote; the own chunk moves nothing)
        "wire": {"record_bytes": WIRE_BYTES, "mean_stem_bytes": round(float(np.mean(stem_mean)), 2),
                 "result_bytes": 8,
                 "bytes_per_remote_descriptor": round(WIRE_BYTES + float(np.mean(stem_mean)) + 8, 2),
                 "remote_fraction": (R - 1) / R},
    }
    print(json.dumps(line), flush=True)


def pcie_fed(args, be, host_batches, now):
    """The same batches fed from page-locked host memory: inputs cross PCIe
    while earlier batches compute, outputs come back (code, remaining, reset).
    SURVEY §8(d): with requests arriving in host memory, PCIe is the honest
    bound. Two input formats: the compact one (rl_do_limit_compact_async, one
    46-B-per-descriptor buffer per batch: the reported rate) and the rl_batch
    arrays (rl_do_limit_host_async, 60 B, under "soa"). Rate over
    args.pcie_steps queued batches, then per-batch latency (submit -> outputs
    on the host)."""
    from ratelimit_amd.limiter import PinnedArena
    from ratelimit_amd.packing import PackedBatch, compact_batch, prefixed_batch
    arena = PinnedArena()
    soa, comp, pref = [], [], []
    for a, bn, bq in host_batches:
        arr = {k: arena.like(v) for k, v in a.items()}
        arr["now"] = arena.like(np.full(bq, now, np.int64))  # (time holds: one second for the whole phase)
        soa.append(PackedBatch(arr, bn, bq, args.n_rules))
        comp.append(compact_batch(arr, bn, bq, args.n_rules, alloc=lambda nb: arena.array(nb, np.uint8)))
        pref.append(prefixed_batch(arr, bn, bq, args.n_rules, alloc=lambda nb: arena.array(nb, np.uint8)))
    # outputs as the Go adapter takes them: code and LimitRemaining (5 B per
    # decision); DurationUntilReset is computed host-side (utils.CalculateReset)
    outs = [{k: arena.like(v) for k, v in soa[0].alloc_result(reset=False).items()} for _ in range(4)]
    n = soa[0].n
    bytes_out = n * 5

    def phase(fed, call, bytes_in):
        keep = []
        host_s = [0.0]

        def submit(s):
            t = time.perf_counter()
            keep.append(call(fed[s % len(fed)], outs[s % len(outs)]))
            host_s[0] += time.perf_counter() - t

        for s in range(3):
            submit(s)
        be.synchronize()
        keep.clear()
        host_s[0] = 0.0
        t0 = time.perf_counter()
        for s in range(args.pcie_steps):
            submit(s)
        be.synchronize()
        el = time.perf_counter() - t0
        host_ms = host_s[0] / args.pcie_steps * 1e3
        keep.clear()
        lat = []
        for s in range(20):
            t1 = time.perf_counter()
            submit(s)
            be.synchronize()
            lat.append((time.perf_counter() - t1) * 1e3)
            keep.clear()
        return {"value": n * args.pcie_steps / el, "unit": "decisions/s", "ms_per_step": el / args.pcie_steps * 1e3,
                "p50_batch_ms": float(np.percentile(lat, 50)), "p99_batch_ms": float(np.percentile(lat, 99)),
                "h2d_bytes_per_decision": bytes_in / n, "d2h_bytes_per_decision": bytes_out / n,
                "h2d_GBps": bytes_in * args.pcie_steps / el / 1e9, "steps": args.pcie_steps,
                "host_submit_ms": host_ms}

    soa_in = sum(int(v.nbytes) for k, v in soa[0].arrays.items() if k != "stem_bytes") + \
        int(soa[0].arrays["stem_off"][n])
    fmts = args.pcie_formats.split(",")
    r_soa = phase(soa, be.do_limit_host_async, soa_in) if "soa" in fmts else None
    progress("host-fed soa done")
    r_comp = phase(comp, be.do_limit_compact_async, int(comp[0].buf.size)) if "compact" in fmts else None
    progress("host-fed compact done")
    r_pref = phase(pref, be.do_limit_prefixed_async, int(pref[0].buf.size)) if "prefixed" in fmts else None
    progress("host-fed prefixed done")
    # the link's own rate for one large page-locked copy, the bound to read h2d_GBps against
    import torch
    big = arena.array(256 << 20, np.uint8)
    dst = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(big)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(5):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    peak = 5 * (256 << 20) / (time.perf_counter() - t1) / 1e9
    del dst, src
    arena.close()
    for r in (r_soa, r_comp, r_pref):
        if r:
            r["h2d_peak_GBps"] = peak
            r["frac_of_h2d_peak"] = r["h2d_GBps"] / peak
    named = {"soa": r_soa, "compact": r_comp, "prefixed": r_pref}
    if r_soa:
        r_soa["format"] = "rl_batch arrays (rl_do_limit_host_async: 9 copies per batch)"
    if r_comp:
        r_comp["format"] = "rl_batch_compact (rl_do_limit_compact_async: one buffer, one copy per batch)"
    if r_pref:
        r_pref["format"] = ("rl_batch_prefixed (rl_do_limit_prefixed_async: one buffer, one copy per batch; each "
                            "request's shared stem prefix once)")
    head = named[fmts[0]]
    head["buffers"] = "page-locked (rl_alloc_host); now constant over the phase"
    head["host_numa"] = host_numa()
    keys = ("value", "h2d_bytes_per_decision", "h2d_GBps", "frac_of_h2d_peak", "p99_batch_ms", "host_submit_ms", "format")
    for f in fmts[1:]:
        head[f] = {k: named[f][k] for k in keys}
    return head


def host_numa():
    """Where the fed phase ran: the GPU's NUMA node (sysfs) and the nodes of the
    CPUs this process may run on (pinned buffers are first-touched by it)."""
    out = {}
    try:
        import glob
        nodes = sorted({open(p).read().strip() for p in glob.glob("/sys/class/drm/card*/device/numa_node")})
        out["gpu_numa_nodes"] = nodes
        cpus = sorted(os.sched_getaffinity(0))
        cnodes = set()
        for c in cpus[:256]:
            for p in glob.glob("/sys/devices/system/cpu/cpu%d/node*" % c):
                cnodes.add(os.path.basename(p)[4:])
        out["cpu_numa_nodes"] = sorted(cnodes)
        out["cpus"] = len(cpus)
    except Exception as e:  # (informational only)
        out["error"] = repr(e)
    return out


def cpu_baseline(args, W):
    """The C restatement oracle on a bounded sample of the same stream, sharded by
    stem hash over the host's cores (SURVEY.md §8d CPU baseline (i): independent
    in-process stores, one thread each; bit-equal to the sequential replay,
    tests/test_c_oracle.py), plus the single-thread rate on a shorter sample."""
    from oracle.c_oracle import COracle, COracleMT
    share = cpu_share()
    threads = args.cpu_threads or share["cores"]

    def run(co, seconds, seed):
        rng = np.random.default_rng(seed)
        sampler = W.ZipfSampler(args.tenants, 1.1) if args.config in ("c2", "c2u") else None
        done, spent, k = 0, 0.0, 0
        while spent < seconds and k < 40:
            if sampler is None:
                a, n, nq, nr = W.c1_batch(rng.integers(0, args.tenants, args.requests), W.NOW0 + k)
            elif args.config == "c2u":
                a, n, nq, nr = W.c2u_batch(sampler.sample(rng, args.requests), W.NOW0 + k,
                                           rng.integers(1, 9, args.requests).astype(np.uint32), rng)
            else:
                a, n, nq, nr = W.c1_batch(sampler.sample(rng, args.requests), W.NOW0 + k,
                                          rng.integers(1, 9, args.requests).astype(np.uint32))
            t = time.perf_counter()
            co.do_limit(a, n, nq, nr)
            spent += time.perf_counter() - t
            done += n
            k += 1
        co.close()
        return done / spent, k, spent

    v1, k1, s1 = run(COracle(0.8, False, False), args.cpu_seconds / 3, 0xC1 + 1)
    vt, kt, st = run(COracleMT(0.8, False, False, threads), args.cpu_seconds, 0xC1 + 2)
    return {"value": vt, "unit": "decisions/s", "cores": threads, "kind": "port",
            "value_1_core": v1, "speedup_vs_1_core": vt / v1 if v1 else None,
            "cores_basis": share["basis"], "host_cpus": share,
            "sample": "%d consecutive %s batches x %d descriptors (%.1f s wall), C restatement oracle sharded by "
                      "stem hash over %d threads (one store each, a persistent pool: hash, scatter and replay "
                      "phases O(n / threads) each); 1 thread: %d batches (%.1f s)"
                      % (kt, args.config.upper(), 2 * args.requests, st, threads, k1, s1)}


def cpu_share():
    """The host CPUs this process may use: the affinity mask, capped by the
    cgroup's CPU quota and by OMP_NUM_THREADS (the GPU box sets it to the
    box's CPU share: one GPU's lease is 16 of a node's cores, though its
    affinity mask lists them all)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = max(1, q // per) if q > 0 else None
        except (OSError, ValueError):
            quota = None
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    cores = min([aff] + [x for x in (quota, omp) if x])
    basis = ("all %d CPUs of the affinity mask" % aff if cores == aff else
             "the cgroup CPU quota (%d of %d CPUs in the affinity mask)" % (quota, aff) if cores == quota else
             "OMP_NUM_THREADS=%d, this host's CPU share for the process (%d CPUs in the affinity mask)" % (omp, aff))
    return {"cores": cores, "affinity_cpus": aff, "cgroup_quota_cpus": quota, "omp_num_threads": omp,
            "basis": basis}


if __name__ == "__main__":
    main()
