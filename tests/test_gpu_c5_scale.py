"""C5 at its configured size (BASELINE.json configs[4]: 10^6 members, RUMOR mode, 1 % churn per period, 8 GPUs).

The oracle cannot hold 10^6 members, so these tests check size-independent properties:

* rank 0 of 8 slot shards alone on one MI355X with the engine's default capacities (the shard bench.py's
  --rehearse-shard 8 times; its peers' gossip-count deltas are zero), for 5 FD periods:
  - no engine error (no capacity, ring or slot-lifetime overflow);
  - `gossips_created` equals the churn schedule restated here (SEMANTICS.md §9: Philox-chosen churned member and
    origin, gossip id = origin and its counter, GossipProtocolImpl.generateGossipId :207-209), counting the rumors whose
    id hashes to this shard;
  - every member's receipt-ring contents equal its held-bit row (the ring is the member's `gossips` map in receipt
    order, GossipProtocolImpl.java:47-53,171-183), and its gossip count equals those plus the rumors it originated that
    other shards store (no rumor is swept before ~24 periods at this size, ClusterMath.gossipPeriodsToSweep);
  - every first receipt emitted exactly one GOSSIP event (onGossipReq :171-183), folded or pending for the next P4;
* 10^5 members, one handle against two slot shards: identical per-member state hashes and op counters.
"""
import numpy as np
import pytest

from swimhip import SimConfig, _abi
from swimhip.cluster import SimulatedCluster

pytestmark = pytest.mark.gpu

M32 = np.uint64(0xFFFFFFFF)
SALT_CHURN = 0x43485552


def philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 over numpy arrays (swim_common.h philox)."""
    c = [np.asarray(x, dtype=np.uint64) & M32 for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & M32, p1 & M32, ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & M32, p0 & M32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & M32
    return c


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def test_philox_restatement_known_answers():
    for inp, want in [((0, 0, 0, 0, 0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
                      ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822, 0x299F31D0),
                       (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]:
        assert tuple(int(x) for x in philox(*inp)) == want


def churn_schedule(n, churn, periods, seed, world, rank):
    """Per period: how many of its rumors this slot shard stores, and (cumulative) per origin how many rumors it
    originated so far that other shards store."""
    gc = {}  # origin -> gossip counter (RUMOR mode: only churn rumors are created)
    mine_per_period, notmine, acc = [], [], np.zeros(n, dtype=np.int64)
    lo, hi = seed & 0xFFFFFFFF, seed >> 32
    for p in range(periods):
        r = philox(np.full(churn, p), np.arange(churn), 0, 0, lo ^ SALT_CHURN, hi)
        v = (r[0] * np.uint64(n)) >> np.uint64(32)
        o = (r[1] * np.uint64(n - 1)) >> np.uint64(32)
        o = o + (o >= v).astype(np.uint64)
        mine = 0
        for origin in o.tolist():  # event order = each origin's call order (k_user_gossips)
            c = gc.get(origin, 0)
            gc[origin] = c + 1
            if mix64(((origin << 32) | c) ^ 0x510750A4D5) % world == rank:
                mine += 1
            else:
                acc[origin] += 1
        mine_per_period.append(mine)
        notmine.append(acc.copy())
    return mine_per_period, notmine


@pytest.mark.timeout(900)
def test_c5_lone_shard_full_size(engine, monkeypatch):
    from swimhip.shard import LoneExchange, ShardedCluster
    n, world, periods = 1_000_000, 8, 5
    cfg = SimConfig(n_members=n, mode=_abi.MODE_RUMOR, churn_per_period=n // 100)
    want_mine, notmine = churn_schedule(n, n // 100, periods, cfg.seed, world, 0)
    assert 0 < sum(want_mine) < periods * n // 100
    monkeypatch.setenv("SWIM_LONE_SHARD", "1")
    c = ShardedCluster(engine, cfg, 0, world, _abi.TRANSPORT_HOST, exchange=LoneExchange(world))
    try:
        assert c.counters()["device_bytes"] < 280e9
        created = 0
        for p in range(periods):
            c.run_periods(1)  # raises on any engine error (capacities, rings, slot lifetimes)
            created += want_mine[p]
            ctr = c.counters()
            assert ctr["gossips_created"] == created, (p, ctr["gossips_created"], created)
            held, head, tail, pop, pend = _abi.debug_holders(engine, c._h, 0, n).astype(np.int64).T
            ring = (tail - head) % (1 << 32)
            bad = np.nonzero(ring != pop)[0]
            assert len(bad) == 0, f"period {p + 1}: member {bad[0]} ring {ring[bad[0]]} held bits {pop[bad[0]]}"
            # rumors other shards store still count as held by their origin (none is swept this early)
            bad = np.nonzero(held != ring + notmine[p])[0]
            assert len(bad) == 0, (f"period {p + 1}: member {bad[0]} count {held[bad[0]]} ring {ring[bad[0]]} + "
                                   f"{notmine[p][bad[0]]}")
            receipts = int(tail.sum()) - created  # every creation and first receipt appended one ring entry
            assert receipts == ctr["events"] + int(pend.sum()), (p, receipts, ctr["events"], int(pend.sum()))
            assert ctr["gossip_messages"] > 0 and receipts > 0
    finally:
        c.close()


@pytest.mark.timeout(600)
def test_c5_100k_one_vs_two_slot_shards(engine):
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=100_000, mode=_abi.MODE_RUMOR, churn_per_period=1000)
    keys = ["record_compares", "messages", "gossip_messages", "events", "messages_lost", "gossips_created"]

    def trace(make):
        c = make()
        c.set_default_loss(5)
        out = []
        try:
            for p in range(1, 31):
                c.run_periods(1)
                if p % 10 == 0:
                    ctr = c.counters()
                    out.append((p, c.state_hash().copy(), [ctr[k] for k in keys]))
        finally:
            c.close()
        return out

    one = trace(lambda: SimulatedCluster(engine, cfg))
    two = trace(lambda: ThreadShardGroup(engine, cfg, 2))
    for (p, h1, c1), (_, h2, c2) in zip(one, two):
        bad = np.argwhere(h1 != h2)
        assert len(bad) == 0, f"period {p}: state hash differs at member {bad[0][0]} word {bad[0][1]} ({len(bad)})"
        assert c1 == c2, f"period {p}: {dict(zip(keys, c1))} vs {dict(zip(keys, c2))}"
    last = dict(zip(keys, one[-1][2]))
    assert last["gossips_created"] == 30 * 1000 and last["events"] > 10**6, last
