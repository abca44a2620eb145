"""Timeline of a rocprofv3 kernel trace: per-batch kernel starts/ends (us,
relative to the batch's k_prepare start), queue ids, and per-kernel averages.

    python scripts/trace_timeline.py gpurun_out/trace/run_kernel_trace.csv [first_batch] [n_batches]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+|__amd_\w+|\w*elementwise\w*|ncclDevKernel\w*)", name)
    return m.group(1) if m else name[:40]


def main():
    path = sys.argv[1]
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(short(r["Kernel_Name"]), int(r["Queue_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
           int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1), int(r["VGPR_Count"]),
           int(r["Scratch_Size"])) for r in rows]
    preps = [i for i, k in enumerate(ks) if k[0] == "k_prepare"]
    print("batches (k_prepare dispatches):", len(preps))
    for b in range(first, min(first + nb, len(preps))):
        i0 = preps[b]
        t0 = ks[i0][2]
        i1 = preps[b + 1] if b + 1 < len(preps) else len(ks)
        # everything that STARTS between this prepare and the one after next
        i2 = preps[b + 2] if b + 2 < len(preps) else len(ks)
        print("--- batch %d" % b)
        for k in ks[i0:i2]:
            tag = "" if ks.index(k) < i1 else "   (next)"
            print("  q%-2d %-24s %8.1f -> %8.1f  (%6.1f us) grid %6d vgpr %3d scr %d%s" % (
                k[1], k[0], (k[2] - t0) / 1e3, (k[3] - t0) / 1e3, (k[3] - k[2]) / 1e3, k[4], k[5], k[6], tag))
    if len(preps) > 2:
        span = (ks[preps[-1]][2] - ks[preps[first]][2]) / 1e3 / (len(preps) - 1 - first)
        print("mean prepare-to-prepare: %.1f us" % span)
    agg = defaultdict(list)
    for k in ks:
        agg[k[0]].append((k[3] - k[2]) / 1e3)
    print("--- per-kernel mean us (count)")
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print("  %-28s %8.1f (%d)" % (n, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
