"""Helpers for diffing the gfx950 engine against the CPU oracle through the shared C ABI."""
import os
import threading
import time

import numpy as np

from swimhip import _abi
from swimhip.cluster import SimulatedCluster

WORDS = ["row", "fd_list", "gossip_list", "events", "gossips_held", "misc"]


def pair(oracle_lib, engine_lib, cfg):
    return SimulatedCluster(oracle_lib, cfg), SimulatedCluster(engine_lib, cfg)


def first_diff(ho, he):
    bad = np.argwhere(ho != he)
    if len(bad) == 0:
        return None
    m, w = bad[0]
    return int(m), WORDS[int(w)], len(bad)


def explain(o, e, member):
    """Readable detail for a mismatching member: differing row entries and list heads."""
    try:
        return _explain(o, e, member)
    except Exception as x:  # noqa: BLE001 - e.g. a replayed oracle tape holds no such readback
        return f"(no member detail: {x})"


def _explain(o, e, member):
    ro, re_ = o.row(member), e.row(member)
    diffs = [(int(s), hex(int(ro[s])), hex(int(re_[s]))) for s in np.nonzero(ro != re_)[0][:8]]
    fo, go, co = o.lists(member)
    fe, ge, ce = e.lists(member)
    go_, ge_ = o.gossips(member), e.gossips(member)
    so, se = set(go_), set(ge_)
    gd = f"gossips oracle-only {sorted(so - se)[:6]} engine-only {sorted(se - so)[:6]} ({len(so)}/{len(se)}); "
    sc = ""
    try:
        import ctypes as C
        names = ["cidCnt", "syncSeq", "gCounter", "nextSync", "fdPeriod", "gPeriod"]
        vals = []
        for c in (o, e):
            fn = c.lib.swimdbg_scalars
            fn.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
            out = (C.c_uint64 * 6)()
            fn(c._h, member, out)
            vals.append(list(out))
        sc = "scalars oracle/engine " + ", ".join(f"{n} {a}/{b}" for n, a, b in zip(names, *vals)) + "; "
    except Exception:  # noqa: BLE001 - debugging detail only
        pass
    return (sc + gd + f"row diffs (subject, oracle, engine): {diffs}; fd len {len(fo)}/{len(fe)} eq={np.array_equal(fo, fe)} "
            f"cursor {co}/{ce}; gossip len {len(go)}/{len(ge)} eq={np.array_equal(go, ge)}")


def assert_same(o, e, where=""):
    ho, he = o.state_hash(), e.state_hash()
    d = first_diff(ho, he)
    if d is not None:
        m, w, n = d
        raise AssertionError(f"{where}: state hash differs at member {m} word {w} ({n} words differ); "
                             + explain(o, e, m))
    co, ce = o.counters(), e.counters()
    keys = ["record_compares", "row_writes", "messages", "gossip_messages", "events", "messages_lost",
            "gossips_created", "sync_merges"]
    for k in keys:
        assert co[k] == ce[k], f"{where}: counter {k} oracle={co[k]} engine={ce[k]} ({co} vs {ce})"


TIMES = {"oracle": 0.0, "engine": 0.0, "wall": 0.0}  # per test, printed by conftest when SWIM_TEST_TIMING is set


def _timed(key, fn, *a):
    t0 = time.perf_counter()
    try:
        return fn(*a)
    finally:
        TIMES[key] += time.perf_counter() - t0


def step_both(o, e, n):
    """Advance the oracle and the engine by n ticks at the same time: the oracle's chunk runs on a helper thread while
    this thread drives the engine (both are ctypes calls, which release the GIL), so a lockstep chunk costs the slower
    of the two instead of their sum. The comparison after the chunk is unchanged."""
    t0 = time.perf_counter()
    err = []

    def run_oracle():
        try:
            _timed("oracle", o.step, n)
        except BaseException as x:  # noqa: BLE001 - re-raised on the caller's thread
            err.append(x)

    th = threading.Thread(target=run_oracle)
    th.start()
    try:
        _timed("engine", e.step, n)
    finally:
        th.join()
        TIMES["wall"] += time.perf_counter() - t0
    if err:
        raise err[0]


def run_lockstep(o, e, ticks, chunk, where="", events=True):
    done = 0
    while done < ticks:
        n = min(chunk, ticks - done)
        step_both(o, e, n)
        done += n
        assert_same(o, e, f"{where} tick {o.tick}")
    if events:
        eo, ee = o.events(), e.events()
        assert eo == ee, f"{where}: event streams differ (oracle {len(eo)} vs engine {len(ee)})"
        return eo
    return None
