"""Per-batch timeline of a rocprofv3 kernel trace: the n-th launch of every
kernel that runs once per batch belongs to batch n. For a window of K batches
it prints, per kernel, the median start and end relative to the batch's first
kernel, its median run time, and the median gap on the table-order chain
(k_b_begin of batch n after k_late of batch n-1).

    python scripts/batch_timeline.py <run_kernel_trace.csv> [K=40] [first_kernel=k_prepare]
"""
import csv
import re
import statistics as st
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+|__amd_\w+|\w*elementwise\w*|ncclDevKernel\w*)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    first = sys.argv[3] if len(sys.argv) > 3 else "k_prepare"
    by = defaultdict(list)
    for r in rows:
        by[short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    nb = len(by[first])
    # kernels launched once per batch (same count as the first kernel, +-1 for the fill)
    per_batch = [n for n, v in by.items() if abs(len(v) - nb) <= 1 and n.startswith("k_")]
    tail = max(1, nb // 20)
    lo, hi = nb - k - tail, nb - tail
    if lo < 1:
        sys.exit("fewer than %d batches" % (k + 1))
    rel = defaultdict(lambda: ([], [], []))
    for b in range(lo, hi):
        t0 = by[first][b][0]
        for n in per_batch:
            v = by[n]
            j = b + (len(v) - nb)
            if 0 <= j < len(v):
                s, e = v[j]
                rel[n][0].append((s - t0) / 1e3)
                rel[n][1].append((e - t0) / 1e3)
                rel[n][2].append((e - s) / 1e3)
    step = st.median([(by[first][b + 1][0] - by[first][b][0]) / 1e3 for b in range(lo, hi)])
    print("window: batches %d..%d, median interval between batches %.1f us" % (lo, hi, step))
    for n in sorted(per_batch, key=lambda n: st.median(rel[n][0])):
        print("  %-20s start %+8.1f  end %+8.1f  run %7.1f us" % (
            n, st.median(rel[n][0]), st.median(rel[n][1]), st.median(rel[n][2])))
    if "k_b_begin" in by and "k_late" in by:
        bb, kl = by["k_b_begin"], by["k_late"]
        db, dl = len(bb) - nb, len(kl) - nb
        gaps = [(bb[b + db][0] - kl[b - 1 + dl][1]) / 1e3 for b in range(lo, hi)
                if 0 <= b + db < len(bb) and 0 <= b - 1 + dl < len(kl)]
        print("table-order gap (k_b_begin n - k_late n-1 end): median %.1f us, mean %.1f us" % (
            st.median(gaps), st.mean(gaps)))


if __name__ == "__main__":
    main()
