"""Host-fed (PCIe) phase of a rocprofv3 run: memory copies and kernels on one
clock. Per direction: copy count, bytes, busy time, achieved GB/s while busy
and over the span; how much of the span H2D and D2H overlap; the gaps between
consecutive H2D copies.

    python scripts/copy_timeline.py <dir with *memory_copy_trace.csv> [min_bytes]
"""
import csv
import glob
import os
import sys


def col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(names)


def main():
    d = sys.argv[1]
    min_bytes = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    f = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    if not f:
        sys.exit("no memory_copy_trace.csv under %s" % d)
    rows = list(csv.DictReader(open(f[0])))
    print("columns:", list(rows[0].keys()) if rows else [])
    cps = []
    for r in rows:
        kind = col(r, "Direction", "Operation", "Kind")
        try:
            nb = int(col(r, "Bytes", "Size", "Copy_Bytes"))
        except KeyError:  # (rocprofv3 of ROCm 7.2 records no size: durations only)
            nb = -1
        t0, t1 = int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp"))
        cps.append((t0, t1, nb, kind))
    cps.sort()
    by = {}
    for c in cps:
        by.setdefault(c[3], []).append(c)
    for kind, cs in by.items():
        big = [c for c in cs if c[2] >= min_bytes or c[2] < 0]
        if not big:
            continue
        busy = sum(c[1] - c[0] for c in big)
        span = big[-1][1] - big[0][0]
        nb = sum(c[2] for c in big)
        gaps = [b[0] - a[1] for a, b in zip(big, big[1:])]
        gaps.sort()
        print("%-28s %5d copies >= %d B: %8.1f MB, busy %8.1f us (%.1f GB/s), span %8.1f us (%.1f GB/s); "
              "gap p50 %.1f us p90 %.1f us max %.1f us" % (
                  kind, len(big), min_bytes, nb / 1e6, busy / 1e3, nb / max(busy, 1), span / 1e3, nb / max(span, 1),
                  (gaps[len(gaps) // 2] / 1e3) if gaps else 0, (gaps[int(len(gaps) * 0.9)] / 1e3) if gaps else 0,
                  (gaps[-1] / 1e3) if gaps else 0))
        sizes = sorted(set(c[2] for c in big))
        print("   sizes:", sizes[:12], "..." if len(sizes) > 12 else "")
        for c in big[:3] + big[len(big) // 2:len(big) // 2 + 3]:
            print("   %12.1f us  %8.1f us  %10d B  %.1f GB/s" % ((c[0] - big[0][0]) / 1e3, (c[1] - c[0]) / 1e3, c[2],
                                                           c[2] / max(c[1] - c[0], 1)))
    kinds = list(by)
    if len(kinds) >= 2:
        iv = {k: [(c[0], c[1]) for c in by[k] if c[2] >= min_bytes or c[2] < 0] for k in kinds}
        a, b = kinds[0], kinds[1]
        ov = 0
        j = 0
        for s0, e0 in iv[a]:
            for s1, e1 in iv[b]:
                if s1 < e0 and s0 < e1:
                    ov += min(e0, e1) - max(s0, s1)
        print("overlap %s / %s: %.1f us" % (a, b, ov / 1e3))


if __name__ == "__main__":
    main()
