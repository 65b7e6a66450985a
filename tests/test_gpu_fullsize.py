"""Parity at the size the headline is timed at: C3 (BASELINE.json configs[2]) at 100 000 members on one GPU against the
CPU oracle, period by period, then the same cluster with membership evolution (the bench's c3dyn line: one
updateIncarnation per period, MembershipProtocolImpl.java:178-190, so gossip, SYNC re-spread, UPDATED events and
metadata fetches run at full size).

The engine runs first in the bench's own configuration (SWIM_FLAG_PROFILE, speculative batches, SYNC_ACK resolution)
and keeps only the per-member state hashes, counters and events; the oracle (~20 B of host RAM per member pair, about
200 GB at 10^5 members, 16 worker threads) runs the same periods beside it on a helper thread. Skipped, with the reason printed, when
the host does not have that much memory available."""
import os
import threading

import numpy as np
import pytest

from swimhip import SimConfig, SimulatedCluster

from parity_util import first_diff

pytestmark = pytest.mark.gpu

N = 100_000
STEADY, DYN = 3, 2
UPDATED = [17, 50_021]  # members whose incarnation is bumped, one per dynamic period
KEYS = ["record_compares", "row_writes", "messages", "gossip_messages", "events", "messages_lost", "gossips_created",
        "sync_merges"]


def mem_available():
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def run(c):
    """Per period: (state hashes, counters); then the events of the whole run."""
    out = []
    for p in range(STEADY + DYN):
        if p >= STEADY:
            c.update_incarnation(UPDATED[p - STEADY])
        c.run_periods(1)
        out.append((c.state_hash().copy(), c.counters()))
    return out, c.events()


def test_c3_headline_size_parity(oracle, engine, monkeypatch):
    need = 21 * N * N  # the oracle's tables and lists (oracle/swimref.cpp Member) plus slack
    avail = mem_available()
    if avail < need:
        msg = f"needs {need / 1e9:.0f} GB of host RAM for the oracle at {N} members, {avail / 1e9:.0f} GB available"
        print("SKIP:", msg, flush=True)
        pytest.skip(msg)
    cfg = SimConfig(n_members=N, profile=True, record_events=True)
    # the oracle (16 worker threads) runs beside the engine on a helper thread: ctypes calls release the GIL
    monkeypatch.setenv("SWIMREF_THREADS", "16")
    got = {}

    def run_oracle():
        try:
            o = SimulatedCluster(oracle, cfg)
            got["o"] = run(o)
            o.close()
        except BaseException as x:  # noqa: BLE001 - re-raised below
            got["err"] = x

    th = threading.Thread(target=run_oracle)
    th.start()
    try:
        e = SimulatedCluster(engine, cfg)
        er, ee = run(e)
        ce = e.counters()
        e.close()
    finally:
        th.join()
    if "err" in got:
        raise got["err"]
    orr, oe = got["o"]
    # every merged payload was either streamed by k_sync_diff or resolved from write logs (k_ack_resolve)
    assert ce["ack_resolved_total"] > 0
    assert ce["ack_resolved_total"] + ce["diff_msgs_total"] == ce["sync_merges"], ce
    steady = er[STEADY - 1][1]
    assert steady["row_writes"] == 0 and steady["events"] == 0  # the headline's steady state

    for p, ((he, ce_), (ho, co)) in enumerate(zip(er, orr)):
        d = first_diff(ho, he)
        assert d is None, f"period {p + 1}: state hash differs at member {d[0]} word {d[1]} ({d[2]} words)"
        for k in KEYS:
            assert ce_[k] == co[k], f"period {p + 1}: counter {k} oracle={co[k]} engine={ce_[k]}"
    assert len(oe) > 0 and oe == ee, f"event streams differ (oracle {len(oe)} vs engine {len(ee)})"
    print(f"C3 at {N} members: {STEADY} steady + {DYN} dynamic periods identical, {len(ee)} events, "
          f"{ce['sync_merges']} payloads merged ({ce['ack_resolved_total']} resolved)", flush=True)
