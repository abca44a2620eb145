"""k_table duration from a rocprofv3 kernel trace of one bench.py run, split by
phase: fill + warmup launches, the K timed launches, the latency launches.
The timed-region average is what bench.py's roofline.kernel_us (k_table's
own run time on the device clock, roofline.achieved) must agree with; the whole-run kernel_stats average also holds the fill
batches (20M inserts), which run about twice as long.

usage: python scripts/trace_timed.py <run_kernel_trace.csv> <bench json line file> [out.json]
"""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    d = json.loads([l for l in open(bench) if l.startswith('{"metric')][-1])
    k = d["steps"]
    lat = d["roofline"].get("k_table_launches_after_timed")
    if lat is None:  # (older bench lines)
        lat = 50 if len(sys.argv) < 5 else int(sys.argv[4])
        lat += (d.get("pcie_fed") or {}).get("steps", 0)  # the host-fed phase runs after the latency steps
    rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].startswith("rl::k_table(")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    timed = us[len(us) - lat - k:len(us) - lat]
    out = {
        "kernel": "k_table", "launches": len(us), "timed_launches": len(timed),
        "trace_timed_avg_us": round(sum(timed) / len(timed), 1),
        "events_table_avg_us": round(d["roofline"]["stage_ms"]["table"] * 1e3, 1),
        "bench_kernel_us": d["roofline"].get("kernel_us"),  # device clock, every prof_every-th timed batch
        "trace_other_avg_us": round((sum(us) - sum(timed)) / max(1, len(us) - len(timed)), 1),
        "trace_all_avg_us": round(sum(us) / len(us), 1),
    }
    print(json.dumps(out))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"))


if __name__ == "__main__":
    main()
