"""GPU busy fraction over the last K batches of a rocprofv3 kernel trace: the
union of all kernels' [start, end) against the span from the K-th last
k_prepare to the last kernel end, and the summed time per kernel over that
span (per batch).

    python scripts/trace_busy.py <run_kernel_trace.csv> [K=40] [first batch index]

Without a first index the window ends before the last 5 % of batches (bench.py
runs its latency and host-fed phases last).
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+|__amd_\w+|\w*elementwise\w*|ncclDevKernel\w*)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    preps = [t0 for n, t0, _ in ks if n == "k_prepare"]
    if len(preps) < k + 1:
        sys.exit("fewer than %d batches" % (k + 1))
    # the window: K batches ending before the latency steps (skip the last 5 % of batches)
    if len(sys.argv) > 3:
        f = int(sys.argv[3])
        a, b = preps[f], preps[f + k]
    else:
        tail = max(1, len(preps) // 20)
        a, b = preps[-(k + tail)], preps[-tail]
    iv = sorted((max(t0, a), min(t1, b)) for _, t0, t1 in ks if t1 > a and t0 < b)
    busy, cur0, cur1 = 0, None, None
    for s, e in iv:
        if cur1 is None or s > cur1:
            if cur1 is not None:
                busy += cur1 - cur0
            cur0, cur1 = s, e
        else:
            cur1 = max(cur1, e)
    if cur1 is not None:
        busy += cur1 - cur0
    span = b - a
    print("window: %d batches, %.1f us per batch, GPU busy %.1f %%" % (k, span / k / 1e3, 100.0 * busy / span))
    per = defaultdict(float)
    cnt = defaultdict(int)
    for n, t0, t1 in ks:
        if t1 > a and t0 < b:
            per[n] += (min(t1, b) - max(t0, a)) / 1e3
            cnt[n] += 1
    for n in sorted(per, key=lambda n: -per[n]):
        print("  %-28s %6.1f us per batch  (%d launches)" % (n, per[n] / k, cnt[n]))


if __name__ == "__main__":
    main()
