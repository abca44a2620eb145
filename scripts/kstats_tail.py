"""Per-kernel durations over the LAST n launches of each kernel in a rocprofv3
kernel trace (the timed / latency steps of a bench run, after its fill
batches): count, median and mean in microseconds, and each kernel's share of
the summed medians.

usage: python scripts/kstats_tail.py <run_kernel_trace.csv> [n=50] [out.json]
"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    runs = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        runs[name].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out = {}
    for k, v in runs.items():
        v.sort()
        us = [d for _, d in v[-n:]]
        out[k] = {"launches": len(v), "tail": len(us), "median_us": round(statistics.median(us), 2),
                  "mean_us": round(sum(us) / len(us), 2)}
    tot = sum(x["median_us"] for k, x in out.items() if k.startswith("rl::"))
    for k in sorted(out, key=lambda k: -out[k]["median_us"]):
        x = out[k]
        if k.startswith("rl::"):
            x["share"] = round(x["median_us"] / tot, 3)
        print("%-28s %5d  med %8.2f us  mean %8.2f us" % (k[:28], x["launches"], x["median_us"], x["mean_us"]))
    if len(sys.argv) > 3:
        json.dump({"source": path, "tail_launches": n, "kernels": out, "rl_sum_of_medians_us": round(tot, 2)},
                  open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
