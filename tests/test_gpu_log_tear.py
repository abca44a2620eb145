"""A history-log entry overwritten while a lookup reads it.

The log is 64 append-only rings; when one wraps, an append can overwrite an
entry that another lane's lookup is reading (its key's chain was appended in
an earlier batch). Redis answers such a request from the key as its last
INCRBY left it (src/redis/fixed_cache_impl.go:71-74); the table must answer
from one whole entry or fail the descriptor with RL_E_TIME, never pair one
write's header with another write's record.

These tests run the RL_LOG_TEAR build of the library
(ratelimit_amd/libratelimit_hip_tear.so; same sources, plus a hook in the
lookup): rl_debug_log_tear arms a writer whose stores the reading lane itself
applies between its own loads, following a schedule — how many of the
writer's steps land before the reader's header load, its record load and its
header re-read. Every schedule is run, so every interleaving of the two is
covered deterministically, for an overwrite by another slot's entry and by a
newer entry of the same slot, in the library's writer order (header BUSY,
record, header) and in round 5's (header, record).
"""
import itertools

import numpy as np
import pytest

from oracle import c_oracle
from ratelimit_amd import abi, workloads as W
from ratelimit_amd._lib import TEAR_LIB_PATH
from ratelimit_amd.limiter import Backend

pytestmark = pytest.mark.gpu

T0 = W.NOW0 - W.NOW0 % 60 + 10  # (the three setup clocks stay in one minute)
OWN = 0xFFFFFFFF  # rl_log_tear.entry: the entry's own slot / tag / prev / t_app
STEPS = {0: 3, 1: 2}  # writer steps per protocol: the library's, round 5's


def _schedules(n):
    return [s for s in itertools.product(range(n + 1), repeat=3) if s[0] <= s[1] <= s[2]]


def _run(protocol, sched, entry):
    """One key's SECOND slot holds windows T0, T0+1 (logged) and T0+2 (cur);
    the tear is armed, then one request asks for T0+1: its lookup reads the
    log's newest entry (window T0+1) while the armed writer overwrites it."""
    import ctypes as C
    be = Backend(0.8, False, table_slots=1 << 10, max_batch=1 << 10, max_rules=8, library=TEAR_LIB_PATH)
    co = c_oracle.COracle(0.8, False)
    try:
        for now in (T0, T0 + 1, T0 + 2):
            b = W.c1_batch(np.arange(1), now)
            be.do_limit_arrays(*b, isolate=True)
            co.do_limit(*b)
        arm = abi.RlLogTear(protocol=protocol)
        arm.sched[:] = sched
        arm.entry[:] = entry
        be._check(be.L.rl_debug_log_tear(be.ctx, C.byref(arm), None))
        b = W.c1_batch(np.arange(1), T0 + 1)
        g = be.do_limit_arrays(*b, isolate=True)
        out = abi.RlLogTear()
        be._check(be.L.rl_debug_log_tear(be.ctx, None, C.byref(out)))
        o = co.do_limit(*b)
    finally:
        be.close()
        co.close()
    assert out.armed == 2, "the lookup of window T0+1 did not reach the log"
    seen = list(out.seen)
    before = list(out.before)
    new = [before[k] if k < 4 and entry[k] == OWN else entry[k] for k in range(8)]
    return out.verdict, seen[0:4], seen[4:8], seen[8:12], before, new, g, o


def _cross_owner():
    # another slot's entry (another tag), its record claiming window T0+1
    return [0xFFFFFFFE, 0x1234567, 0xFFFFFFF0, OWN, T0 + 1, 999, T0 + 2, 0]


def _same_slot():
    # a newer entry of the same key (the same slot and tag, another chain
    # link) holding window T0+1 with another count. (With a header equal to
    # the old one bit for bit, a reader that sees it unchanged around the
    # record load gets a whole entry either way.)
    return [OWN, OWN, 0xFFFFFFF0, OWN, T0 + 1, 777, T0 + 2, 0]


@pytest.mark.parametrize("kind", ["cross_owner", "same_slot"])
def test_gpu_log_tear_library_writer_never_pairs_halves(kind):
    """The library's writer and reader: over every schedule, a record the
    lookup uses comes with its own header (both the old entry's, or both the
    new one's); anything else is rejected. Against another slot's entry the
    descriptor is then oracle-exact or RL_E_TIME."""
    entry = _cross_owner() if kind == "cross_owner" else _same_slot()
    verdicts = {}
    for sched in _schedules(STEPS[0]):
        v, h1, r, h2, before, new, g, o = _run(0, sched, entry)
        verdicts[sched] = v
        if v >= 0:
            pair = h1 + r
            assert pair in (before, new), "schedule %s used a mixed entry: %s (before %s, new %s)" % (
                sched, pair, before, new)
        if kind == "cross_owner":
            st = int(g["status"][0])
            assert st in (0, abi.RL_E_TIME), st
            assert (st == 0) == (v == 1), (sched, v, st)
            if st == 0:
                assert int(g["limit_remaining"][0]) == int(o["limit_remaining"][0])
                assert int(g["code"][0]) == int(o["code"][0])
            # the MINUTE descriptor never looks at the log
            assert int(g["status"][1]) == 0 and int(g["limit_remaining"][1]) == int(o["limit_remaining"][1])
    # the untouched schedule answers from the old entry; a half-written one never
    assert verdicts[(0, 0, 0)] == 1
    assert all(verdicts[s] == -1 for s in verdicts if s not in ((0, 0, 0), (3, 3, 3)))
    assert verdicts[(3, 3, 3)] == (-1 if kind == "cross_owner" else 1)


def test_gpu_log_tear_round5_writer_order_pairs_new_header_with_old_record():
    """Round 5's writer (header, then record, no invalidation) under the same
    reader: a lookup that loads the header after the writer's first store and
    the record before its second uses the old entry's record under the new
    entry's header — the hole DESIGN.md §3 closes with the BUSY header."""
    entry = _same_slot()
    mixed = []
    for sched in _schedules(STEPS[1]):
        v, h1, r, h2, before, new, g, o = _run(1, sched, entry)
        if v >= 0 and h1 + r not in (before, new):
            mixed.append(sched)
            assert h1 == new[:4] and r == before[4:]  # new header, old record
    assert mixed == [(1, 1, 1), (1, 1, 2)], mixed
