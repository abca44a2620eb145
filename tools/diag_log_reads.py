"""Diagnostic (GPU): the alias stream of test_gpu_override_on_and_off_vs_c_oracle
run REPS times per library build with per-descriptor statuses, reporting the
RL_E_TIME descriptors, rl_table_info's history_lost / history_refused, and
whether every other answer equals the C oracle's.

    python tools/diag_log_reads.py [reps] [lib ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import c_oracle  # noqa: E402
from ratelimit_amd import abi  # noqa: E402
from ratelimit_amd.limiter import Backend  # noqa: E402
import streams  # noqa: E402
import test_gpu_alias as TA  # noqa: E402


def run(lib, lc, seed):
    be = Backend(0.8, lc, False, table_slots=1 << 17, max_batch=1 << 16, max_rules=8, library=lib, hash_seed=seed)
    co = c_oracle.COracle(0.8, lc, False)
    tfail, bad = 0, 0
    try:
        for a, n, nq, nr in TA._stream([38, 40, 40, 41, 59, 60, 61, 60, 100, 100, 101, 120, 121],
                                       p_override=[0.5, 0.0, 0.0, 0.3]):
            g = be.do_limit_arrays(a, n, nq, nr, isolate=True)
            failed = g["status"] != 0
            tfail += int(failed.sum())
            o = co.do_limit(*streams.drop_descriptors(a, n, nq, ~failed), nr)
            for k in ("code", "limit_remaining", "reset_s"):
                bad += int((g[k][~failed] != o[k]).sum())
        info = be.table_info()
    finally:
        be.close()
        co.close()
    return tfail, bad, info["history_lost"], info.get("history_refused")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    libs = [x or None for x in sys.argv[2:]] or [None]
    import ctypes
    for lib in libs:
        if lib:  # (an older build: its own ABI version; rl_table_info's new field stays 0)
            abi.ABI_VERSION = ctypes.CDLL(lib).rl_abi_version()
        tot = [0, 0, 0, 0]
        for r in range(reps):
            for lc in (False, True):
                x = run(lib, lc, 1000 + r)
                if x[0] or x[1] or x[2] or x[3]:
                    print("  %s lc=%d seed=%d: RL_E_TIME %d, mismatches %d, history_lost %d, refused %s"
                          % (os.path.basename(lib or "product"), lc, 1000 + r, *x), flush=True)
                for i in range(4):
                    tot[i] += x[i] or 0
        print("%s: %d runs, RL_E_TIME %d, mismatches %d, history_lost %d, refused %d"
              % (os.path.basename(lib or "product"), 2 * reps, *tot), flush=True)


if __name__ == "__main__":
    main()
