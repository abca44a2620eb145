"""Debug aid (GPU): replay a history stream, and for the first descriptor
whose answer differs from the C oracle print every occurrence of its stem
(batch, position, clock, hits, GPU and oracle answers)."""
import sys

import numpy as np

sys.path[:0] = [".", "tests"]
from oracle import c_oracle  # noqa: E402
from ratelimit_amd.limiter import Backend  # noqa: E402
import test_gpu_history as H  # noqa: E402


def main():
    jitter = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    lc = len(sys.argv) > 2 and sys.argv[2] == "lc"
    bs = H._stream(7, 3_000, 6_000, 8, 40, 299, unit=1, hot=200)
    be = Backend(0.8, lc, table_slots=1 << 18, max_batch=1 << 16, max_rules=8, jitter=jitter)
    co = c_oracle.COracle(0.8, lc, horizon=jitter)
    log = []
    bad = None
    for bi, (a, n, nq, nr) in enumerate(bs):
        g = be.do_limit_arrays(a, n, nq, nr, isolate=True)
        o = co.do_limit(a, n, nq, nr)
        L = int(a["stem_off"][1])
        stems = a["stem_bytes"].reshape(n, L)
        log.append((a, stems, g, o))
        if bad is None:
            d = np.nonzero((g["limit_remaining"] != o["limit_remaining"]) | (g["status"] != 0))[0]
            if d.size:
                bad = (bi, int(d[0]), bytes(stems[d[0]]))
                print("first bad: batch", bi, "pos", int(d[0]), "of", d.size, bad[2])
    if bad is None:
        print("no mismatch")
        return
    for bi, (a, stems, g, o) in enumerate(log):
        m = np.nonzero((stems == np.frombuffer(bad[2], np.uint8)).all(1))[0]
        for i in m:
            q = a["req_idx"][i]
            print("batch %d pos %6d now %d hits %d gpu rem %d st %d oracle rem %d" % (
                bi, i, a["now"][q], a["hits"][i], g["limit_remaining"][i], g["status"][i], o["limit_remaining"][i]))
    print(be.table_info())


if __name__ == "__main__":
    main()
