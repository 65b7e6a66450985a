"""Capacity growth between ticks (api.hip grow_caps): the gossip slot table, the receipt rings and the per-tick receipt
and replay lists start far too small and are grown, contents moved, before they can overflow. The golden scenarios
(recorded from the oracle, which has no capacities) replay bit for bit, and the handle ends with more device memory
than it started with."""
import dataclasses
import json
from pathlib import Path

import pytest

from swimhip import SimConfig, _abi
from swimhip.cluster import SimulatedCluster

GOLDEN = Path(__file__).resolve().parent / "golden"

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["c2_small", "c4_mid", "c2_mid", "c4_long"])
def test_golden_with_growing_caps(engine, monkeypatch, name):
    import sys
    sys.path.insert(0, str(GOLDEN))
    from scenarios import SCENARIOS, record
    monkeypatch.setenv("SWIM_DELIV_CAP", "16384")  # routed receipts per tick
    monkeypatch.setenv("SWIM_CAPS", "rp=1024")     # replay / slow-path sends per tick
    cfg, _ = SCENARIOS[name]()
    cfg = dataclasses.replace(cfg, gossip_slot_cap=256, gossip_ring_cap=256)
    c = SimulatedCluster(engine, cfg)
    b0 = c.counters()["device_bytes"]
    rec = record(c, name)
    b1 = c.counters()["device_bytes"]
    caps = _abi.debug_caps(c.lib, c._h)
    c.close()
    want = json.loads((GOLDEN / f"{name}.json").read_text())
    assert len(rec["periods"]) == len(want["periods"])
    for got, exp in zip(rec["periods"], want["periods"]):
        assert got == exp, f"{name} period {exp['period']}: {got} != {exp}"
    assert b1 > b0 and caps["growths"] > 0, "no capacity grew"
    print(f"{name}: device bytes {b0} -> {b1}, caps {caps}", flush=True)


def test_growth_off_overflows(engine, monkeypatch):
    """The same tiny caps with growth switched off end in a clean capacity error (the sizes are what grew above)."""
    monkeypatch.setenv("SWIM_NO_GROW", "1")
    cfg = SimConfig(n_members=300, gossip_slot_cap=64, gossip_ring_cap=64)
    c = SimulatedCluster(engine, cfg)
    c.set_default_loss(5)
    with pytest.raises(Exception, match=f"rc={_abi.SWIM_ECAPACITY}"):
        c.run_periods(12)
    c.close()


def test_rumor_defaults_from_churn(engine):
    """RUMOR mode with churn: the slot table and receipt rings are sized from the churn rate when no caps are given
    (about churn x (2 maxSpread + 4 + 2 bitlen(N)) gossip intervals of rumors alive, 2 maxSpread + 3 intervals held
    per member), so a run through the steady state needs at most one growth step."""
    cfg = SimConfig(n_members=4000, mode=_abi.MODE_RUMOR, churn_per_period=40)
    c = SimulatedCluster(engine, cfg)
    caps = _abi.debug_caps(c.lib, c._h)
    assert caps["slots"] >= 850 and caps["ring"] >= 630, caps
    c.run_periods(40)
    assert _abi.debug_caps(c.lib, c._h)["growths"] <= 1
    c.close()


@pytest.mark.parametrize("name", ["c2_mid", "c4_long"])
def test_sharded_golden_with_growing_rings(engine, name):
    """Row-sharded handles (2 shards) grow their receipt rings and incarnation history between gossip ticks
    (api.hip grow_caps_shard): the rings start at 256 entries, the peers' first receipts count towards the fill
    (k_unpack_b), and the golden replays bit for bit with more device memory at the end."""
    import sys
    sys.path.insert(0, str(GOLDEN))
    from scenarios import SCENARIOS, record
    from swimhip.shard import ThreadShardGroup
    cfg, _ = SCENARIOS[name]()
    c = ThreadShardGroup(engine, dataclasses.replace(cfg, gossip_ring_cap=256), 2)
    b0 = c.counters()["device_bytes"]
    rec = record(c, name)
    b1 = c.counters()["device_bytes"]
    c.close()
    want = json.loads((GOLDEN / f"{name}.json").read_text())
    assert len(rec["periods"]) == len(want["periods"])
    for got, exp in zip(rec["periods"], want["periods"]):
        assert got == exp, f"{name} (2 shards) period {exp['period']}: {got} != {exp}"
    assert b1 > b0, "no ring grew"
