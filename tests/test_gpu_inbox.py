"""P4 on a wave per member (member.hip k_inbox_apply) against the golden fixtures.

In a tick after a gossip plane, k_member_tick parks every member with at least Dev::hv routed gossip receipts before
P4; k_inbox_apply then runs each parked member's receipts on a whole wave, 64 at a time (onMembershipGossip ->
updateMembership, MembershipProtocolImpl.java:401-408,475-541: a segmented prefix maximum over the packed keys decides
which receipts override, prefix sums place the metadata fetches and write-log entries in gossip-id order), and a second
k_member_tick launch runs the parked members' P5 and P6. SWIM_CAPS hv=N lowers the threshold, so that every member with
a receipt takes this path; the gossip-heavy scenarios must still reproduce the oracle's records bit for bit: the same
tables, fetch lists, correlation ids, write logs, events and counters as the lane-serial P4."""
import json
from pathlib import Path

import pytest

from swimhip import ClusterConfig, SimConfig
from swimhip.cluster import SimulatedCluster

from parity_util import pair, run_lockstep

GOLDEN = Path(__file__).resolve().parent / "golden"

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,hv", [("c2_small", 1), ("c2_mid", 1), ("c2_mid", 4), ("c4_long", 1), ("c4_large", 1),
                                     ("c1", 1), ("c2_full", 2)])
def test_golden_with_inbox_waves(engine, monkeypatch, name, hv):
    import sys
    sys.path.insert(0, str(GOLDEN))
    from scenarios import SCENARIOS, record
    monkeypatch.setenv("SWIM_CAPS", f"hv={hv}")
    cfg, _ = SCENARIOS[name]()
    c = SimulatedCluster(engine, cfg)
    monkeypatch.delenv("SWIM_CAPS")
    rec = record(c, name)
    c.close()
    want = json.loads((GOLDEN / f"{name}.json").read_text())
    assert len(rec["periods"]) == len(want["periods"])
    for got, exp in zip(rec["periods"], want["periods"]):
        assert got == exp, f"{name} hv={hv} period {exp['period']}: {got} != {exp}"
    if want["events"] is not None:
        assert rec["events"] == want["events"]


@pytest.mark.tape
@pytest.mark.parametrize("seed", [0, 1])
def test_inbox_waves_refutations_and_leaves(oracle, engine, monkeypatch, seed):
    """The receipts k_inbox_apply hands to lane 0 (the member's own record, DEAD records, absent rows, user gossips)
    between its batches: suspicion under loss makes members receive gossips about themselves (refutation), kills and a
    leave spread DEAD records, restarts bring ALIVE records for absent rows, and user gossips mix in."""
    cfg = SimConfig(n_members=120, cluster=ClusterConfig(seedMembers=[0], syncInterval=3000), record_events=True,
                    seed=0x5EED + seed, list_slack=4096, pending_fetch_cap=4096)
    monkeypatch.setenv("SWIM_CAPS", "hv=1")
    o, e = pair(oracle, engine, cfg)
    monkeypatch.delenv("SWIM_CAPS")
    for c in (o, e):
        c.set_default_loss(15)
        for m in range(0, 120, 11):
            c.update_incarnation(m)
    run_lockstep(o, e, 120, 20, "loss 15 + incarnation bumps")
    for c in (o, e):
        c.kill(17)
        c.leave(33)
        c.spread_gossip(5, 77)
        c.spread_gossip(5, 78)
    run_lockstep(o, e, 400, 50, "kill + leave + user gossips")
    o.close()
    e.close()
