"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel.

Reads gpurun_out/pmc_<cfg>_{FETCH_SIZE,WRITE_SIZE}/**/*counter_collection.csv
and writes profiles/traffic_<cfg>.json. Per the MI355X guide (HBM section),
FETCH_SIZE on gfx950 counts half of the bytes of wide reads, so the corrected
read bytes are 2 x FETCH_SIZE; WRITE_SIZE is taken as is. Both are in KB.
Only the last `tail` dispatches of each kernel are used (the timed steps,
after table fill and warm-up). The guide leaves other access widths
uncalibrated, so gpurun_out/pmc_probe_* (tools/pmcprobe.hip, known byte
counts) give the measured bytes-per-counted-byte of random 64-B sector reads
and of 64-B-per-lane streaming reads; both are recorded beside the per-kernel
figures, and the k_table line is bracketed by them (its reads are part
streamed records, part random slot sectors).
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(cfg, ctr, tail):
    files = glob.glob(os.path.join(ROOT, "gpurun_out", "pmc_%s_%s" % (cfg, ctr), "**", "*counter_collection.csv"),
                      recursive=True)
    return _collect(files, ctr, tail)


def _collect(files, ctr, tail):
    if not files:
        raise SystemExit("no counter_collection.csv for %s" % ctr)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != ctr:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")
            vals.setdefault(name, []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, v in vals.items():
        v.sort()
        xs = [x for _, x in v[-tail:]]
        out[k] = statistics.median(xs)
    return out


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c1"
    tail = 10
    fetch = per_kernel(cfg, "FETCH_SIZE", tail)
    write = per_kernel(cfg, "WRITE_SIZE", tail)
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("rl::"):
            continue
        f = fetch.get(k, 0.0) * 1024.0
        w = write.get(k, 0.0) * 1024.0
        kernels[k] = {"fetch_size_bytes": f, "write_size_bytes": w, "read_bytes_corrected": 2 * f,
                      "traffic_bytes": 2 * f + w}
    calib = None
    pf = glob.glob(os.path.join(ROOT, "gpurun_out", "pmc_probe_FETCH_SIZE", "**", "*counter_collection.csv"),
                   recursive=True)
    pw = glob.glob(os.path.join(ROOT, "gpurun_out", "pmc_probe_WRITE_SIZE", "**", "*counter_collection.csv"),
                   recursive=True)
    plog = os.path.join(ROOT, "gpurun_out", "pmc_probe_FETCH_SIZE.log")
    if pf and pw and os.path.exists(plog):
        probe = json.loads([l for l in open(plog) if l.startswith('{"tool"')][-1])
        pfk, pwk = _collect(pf, "FETCH_SIZE", 100), _collect(pw, "WRITE_SIZE", 100)
        rd, wr = probe["read_bytes_per_launch"], probe["write_bytes_per_launch"]
        calib = {"probe": probe,
                 "random64_read_bytes_per_fetch_byte": rd / (pfk["k_rand64"] * 1024.0),
                 "seq64_read_bytes_per_fetch_byte": rd / (pfk["k_seq"] * 1024.0),
                 "random64_write_bytes_per_write_byte": wr / max(pwk["k_rand64"] * 1024.0, 1.0)}
    ku = kernels.get("rl::k_table", {})
    res = {"config": cfg, "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate runs; median of the "
                                    "last %d dispatches per kernel; read = 2 x FETCH_SIZE (gfx950 correction)" % tail,
           "calibration": calib,
           "kernels": kernels,
           "k_table_bytes_per_launch": ku.get("traffic_bytes")}
    if calib and ku:
        f = ku["fetch_size_bytes"]
        res["k_table_read_bytes_bounds"] = sorted([f * calib["random64_read_bytes_per_fetch_byte"],
                                                    f * calib["seq64_read_bytes_per_fetch_byte"]])
    # the whole step: every per-batch kernel (not the fill / info / sweep ones)
    per_batch = {k: v for k, v in kernels.items()
                 if not any(x in k for x in ("k_table_info", "k_lc_count", "k_sweep", "k_arena", "k_debug"))}
    res["step_total_bytes"] = sum(v["traffic_bytes"] for v in per_batch.values())
    res["step_kernels"] = sorted(per_batch)
    res["decisions_per_batch"] = 1000000
    # the kernels that answer decisions (C2: the long runs' elements are decided in k_late, not k_table)
    ans = [k for k in ("rl::k_table", "rl::k_late", "rl::k_fast_over") if k in kernels]
    res["answering_kernels_bytes"] = {k: kernels[k]["traffic_bytes"] for k in ans}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    p = os.path.join(ROOT, "profiles", "traffic_%s.json" % cfg)
    json.dump(res, open(p, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["traffic_bytes"]):
        print("%-28s read %8.1f MB  write %8.1f MB" % (k, v["read_bytes_corrected"] / 1e6, v["write_size_bytes"] / 1e6))
    print("whole step: %.1f MB per batch of 1M" % (res["step_total_bytes"] / 1e6))


if __name__ == "__main__":
    main()
