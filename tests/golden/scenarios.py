"""Golden scenarios: the configs the fixtures in this directory were recorded on.

Each scenario is a list of actions on a SimulatedCluster-like object. The recorder (make_golden.py) runs them on the
CPU oracle and stores, after every period: a digest of the per-member state hashes, the deterministic op counters,
and a digest of that period's MembershipEvents; for C1 the full event list too. tests/test_golden.py replays them on
the oracle (CPU) and on libswimhip (GPU) and requires identical records.
"""
import hashlib

import numpy as np

from swimhip import ClusterConfig, SimConfig, _abi

COUNTERS = ["record_compares", "row_writes", "messages", "gossip_messages", "events", "messages_lost",
            "gossips_created", "sync_merges"]


def _c1():
    cfg = SimConfig(n_members=64, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True)
    return cfg, [("periods", 10), ("kill", 63), ("periods", 60)]


def _c2_small():  # C2-shaped: preconverged, 5 % loss on every link, reduced N
    return SimConfig(n_members=300, record_events=True), [("loss", 5), ("periods", 12)]


def _c4_small():  # C4-shaped: two groups blocked both ways, healed later; seed 0 is in group A
    n = 48
    g = [0] * (n // 2) + [1] * (n // 2)
    return SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), record_events=True), [
        ("partition", g), ("periods", 34), ("unblock", None), ("periods", 40)]


def _c4_mid():  # C4-shaped at 200 members: suspicion timeouts (40 periods) start the DEAD-gossip storm, heal at 45,
    # then SYNC recovery re-adds the other side (ADDED + metadata, re-spread storm). Recorded once (~4 min of oracle
    # time on 8 threads, SWIMREF_THREADS=8 python tests/golden/make_golden.py c4_mid); the CPU suite does not replay it
    n = 200
    g = [0] * (n // 2) + [1] * (n // 2)
    return SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), gossip_slot_cap=1 << 18, pending_fetch_cap=4096,
                     list_slack=4096), [
        ("partition", g), ("periods", 45), ("unblock", None), ("periods", 30)]


def _c2_mid():  # C2-shaped at 2 000 members: 5 % loss on every link; refutations re-spread by SYNC build the gossip
    # storm the bench line measures at 10k. Recorded once (SWIMREF_THREADS=8 python tests/golden/make_golden.py c2_mid)
    return SimConfig(n_members=2000, record_events=True), [("loss", 5), ("periods", 14)]


def _c4_long():  # C4's full schedule at 300 members: partition from period 0, healed at period 200 (as configs[3]),
    # run 40 periods past the heal: suspicion timeouts, the DEAD-gossip storm, then SYNC recovery. Recorded once
    n = 300
    g = [0] * (n // 2) + [1] * (n // 2)
    return SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), gossip_slot_cap=1 << 19, pending_fetch_cap=4096,
                     list_slack=4096), [
        ("partition", g), ("periods", 200), ("unblock", None), ("periods", 40)]


def _c4_large():  # C4's full schedule (BASELINE configs[3]) at 1 000 members: partition from period 0, unblockAll at
    # period 200, run to period 320 (4 SYNC rounds past the heal). Recorded once (SWIMREF_THREADS=8 python
    # tests/golden/make_golden.py c4_large); replayed on 1 and 2 shards by the GPU suite
    n = 1000
    g = [0] * (n // 2) + [1] * (n // 2)
    return SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), gossip_slot_cap=1 << 19, pending_fetch_cap=4096,
                     list_slack=4096), [
        ("partition", g), ("periods", 200), ("unblock", None), ("periods", 120)]


def _c2_full():  # C2 at its configured size (BASELINE configs[1]: 10 000 members, 5 % loss, preconverged) for as many
    # periods as the oracle can hold in this container's 64 GB: it keeps GossipState.infectedFrom as explicit per-holder
    # sets, so its memory grows with the re-spread storm (measured: period 2 4.4 s / 3.4 GB, period 3 152 s / 32 GB with
    # 2.2e4 gossips created and 3.7e8 gossip messages; period 4 creates ~3.5x the gossips and does not fit). Periods 1-3
    # already run the SYNC re-spreads (SYNCs are staggered over the first 300 ticks) and the suspicion refutations.
    # Recorded once (SWIMREF_THREADS=8 python tests/golden/make_golden.py c2_full, ~3 min); replayed on 1 and 2 shards
    return SimConfig(n_members=10_000, record_events=True, event_cap=1 << 22), [("loss", 5), ("periods", 3)]


def _c3_small():  # C3-shaped: steady state SYNC / SYNC_ACK anti-entropy, no loss
    return SimConfig(n_members=1000), [("periods", 35)]


def _c5_small():  # C5-shaped: rumor-only dissemination with 1 % churn per period (SEMANTICS.md §9), reduced N
    return SimConfig(n_members=400, mode=_abi.MODE_RUMOR, churn_per_period=4, record_events=True), [("periods", 30)]


def _c3_full():  # C3 at the headline size (BASELINE configs[2], 100 000 members, the bench's own config with
    # profile=True): the 25 steady periods the default bench line runs (warm-up 5 + 20 timed), then two periods each
    # after one updateIncarnation (the c3dyn line's evolution: gossip, SYNC re-spread, UPDATED events, metadata
    # fetches). Recorded on the GPU box (~210 GB of host RAM: tools/record_golden_box.py c3_full)
    return SimConfig(n_members=100_000, profile=True, record_events=True), [
        ("periods", 25), ("inc", 17), ("periods", 1), ("inc", 50_021), ("periods", 1)]


def _c2_long():  # C2 at its configured 10 000 members past c2_full's 3 periods: as many periods as the GPU box's RAM
    # holds the oracle's explicit infectedFrom sets (tools/record_golden_box.py c2_long stops before its memory cap)
    return SimConfig(n_members=10_000, record_events=True, event_cap=1 << 22), [("loss", 5), ("periods", 12)]


def _c4_50k():  # C4 at its configured 50 000 members (BASELINE configs[3]): groups A = [0, 25 000) and B blocked both
    # ways from period 0, seeds = {0}. The oracle runs on the GPU box through the first SUSPECT wave (pings across the
    # partition time out from period 1, ping-req timeouts suspect, the SUSPECT gossips fill each side) for as many
    # periods as its RAM holds (tools/record_golden_box.py c4_50k)
    n = 50_000
    g = [0] * (n // 2) + [1] * (n // 2)
    return SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), record_events=True, pending_fetch_cap=4096,
                     list_slack=4096), [("partition", g), ("periods", 80)]


SCENARIOS = {"c1": _c1, "c2_small": _c2_small, "c4_small": _c4_small, "c3_small": _c3_small, "c5_small": _c5_small,
             "c4_mid": _c4_mid, "c2_mid": _c2_mid, "c4_long": _c4_long, "c4_large": _c4_large, "c2_full": _c2_full}
# recorded on the GPU box (its host RAM and 16 cores): replayed by their own -m gpu tests, not by test_golden.py
BOX_SCENARIOS = {"c3_full": _c3_full, "c2_long": _c2_long, "c4_50k": _c4_50k}
SLOW_ON_ORACLE = {"c4_mid", "c2_mid", "c4_long", "c4_large", "c2_full"}  # recorded once; replaying it on the oracle takes minutes
FULL_EVENTS = {"c1"}


def digest(a):
    return hashlib.blake2b(np.ascontiguousarray(a).tobytes(), digest_size=16).hexdigest()


def event_rows(evs):
    return [[e.tick, e.observer, e.seq, {"ADDED": 0, "REMOVED": 1, "UPDATED": 2, "GOSSIP": 3}[e.type], e.member,
             -1 if e.oldMetadata is None else e.oldMetadata, -1 if e.newMetadata is None else e.newMetadata] for e in evs]


def record(c, name, limit=None, on_period=None):
    """Run scenario `name` on cluster c (already created from the scenario's SimConfig); return the record.
    limit: stop after that many periods; on_period(out): called after every recorded period."""
    cfg, actions = {**SCENARIOS, **BOX_SCENARIOS}[name]()
    out = {"periods": [], "events": [] if name in FULL_EVENTS else None}
    period = 0
    for what, arg in actions:
        if what == "periods":
            for _ in range(arg):
                if limit is not None and period >= limit:
                    return out
                c.run_periods(1)
                period += 1
                ctr = c.counters()
                rows = event_rows(c.events()) if cfg.record_events else []
                if out["events"] is not None:
                    out["events"].extend(rows)
                out["periods"].append({"period": period, "state": digest(c.state_hash()),
                                       "counters": [int(ctr[k]) for k in COUNTERS],
                                       "events": digest(np.array(rows, dtype=np.int64).reshape(-1, 7))})
                if on_period is not None:
                    on_period(out)
        elif what == "kill":
            c.kill(arg)
        elif what == "loss":
            c.set_default_loss(arg)
        elif what == "partition":
            c.partition(np.array(arg, dtype=np.uint32))
        elif what == "unblock":
            c.unblock_all()
        elif what == "inc":
            c.update_incarnation(arg)
    return out
