"""Golden fixtures (tests/golden/*.json, recorded by tests/golden/make_golden.py from the oracle).

Per period: a digest of every member's state hashes, the eight deterministic op counters and a digest of that period's
MembershipEvents; for C1 the full event list. The CPU tests pin the oracle to the fixtures; the GPU tests replay the
same scenarios on libswimhip, single-GPU and row-sharded, and must reproduce every record bit for bit.
Parity is pinned to the oracle, not to the Java reference, which cannot run here."""
import json
import sys
from pathlib import Path

import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLDEN))

from scenarios import SCENARIOS, SLOW_ON_ORACLE, record  # noqa: E402

from swimhip.cluster import SimulatedCluster  # noqa: E402


def load(name):
    return json.loads((GOLDEN / f"{name}.json").read_text())


def check(rec, want, who):
    assert len(rec["periods"]) == len(want["periods"])
    for got, exp in zip(rec["periods"], want["periods"]):
        assert got == exp, f"{who}: {want['scenario']} period {exp['period']}: {got} != {exp}"
    if want["events"] is not None:
        assert rec["events"] == want["events"], f"{who}: {want['scenario']} event list differs"


@pytest.mark.parametrize("name", [n for n in SCENARIOS if n not in SLOW_ON_ORACLE])
def test_oracle_matches_golden(oracle, name):
    cfg, _ = SCENARIOS[name]()
    c = SimulatedCluster(oracle, cfg)
    check(record(c, name), load(name), "oracle")
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_engine_matches_golden(engine, name):
    cfg, _ = SCENARIOS[name]()
    c = SimulatedCluster(engine, cfg)
    check(record(c, name), load(name), "gfx950")
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("c1", 2), ("c2_small", 3), ("c4_small", 2), ("c3_small", 4), ("c5_small", 3),
                                        ("c4_mid", 2), ("c2_mid", 2), ("c4_long", 2),
                                        ("c4_large", 2), ("c2_full", 2)])
def test_sharded_engine_matches_golden(engine, name, world):
    from swimhip.shard import ThreadShardGroup
    cfg, _ = SCENARIOS[name]()
    g = ThreadShardGroup(engine, cfg, world)
    check(record(g, name), load(name), f"gfx950 x{world} shards")
    g.close()


@pytest.mark.parametrize("name", ["c2_small", "c4_small", "c5_small"])
def test_threaded_oracle_matches_golden(oracle, name, monkeypatch):
    """The oracle with SWIMREF_THREADS=3 (member ranges per worker, lanes merged in member order) reproduces the
    fixtures exactly; bench.py times the CPU baseline this way on all host cores."""
    monkeypatch.setenv("SWIMREF_THREADS", "3")
    cfg, _ = SCENARIOS[name]()
    c = SimulatedCluster(oracle, cfg)
    rec = record(c, name)
    c.close()
    gold = json.loads((GOLDEN / f"{name}.json").read_text())
    assert rec["periods"] == gold["periods"]
