"""The 30-bit incarnation field of the key plane (SEMANTICS.md §8).

MembershipRecord.incarnation is a Java `int` (MembershipRecord.java:12-84): it starts at 0 and grows by one per
refutation or updateIncarnation call (MembershipProtocolImpl.java:178-190,488-509), so 2^31 - 1 is its largest value.
The engine stores a record as the 4-B key `inc << 2 | status` (what k_sync_diff streams), so it holds incarnations up
to 2^30 - 1 and raises SWIM_ECAPACITY (E_INC) instead of truncating above that. These tests put one member's own record
just below the limit (swim_debug_set_incarnation) and check both sides of it: 2^30 - 1 is stored, gossiped and merged
everywhere like any other incarnation; the bump past it fails loudly."""
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster, SwimError

from parity_util import pair, run_lockstep

pytestmark = pytest.mark.gpu

LIMIT = 1 << 30


def test_incarnation_at_the_limit(engine):
    n, m = 40, 11
    c = SimulatedCluster(engine, SimConfig(n_members=n, record_events=True))
    try:
        c.step(3)
        assert _abi.debug_set_incarnation(engine, c._h, m, LIMIT) == -4  # SWIM_ECAPACITY: not representable
        assert _abi.debug_set_incarnation(engine, c._h, m, LIMIT - 2) == 0
        c.update_incarnation(m)  # -> 2^30 - 1, spread as a gossip to every member (UPDATED events after metadata)
        c.step(200)
        for obs in range(n):
            key = int(c.row(obs)[m])
            assert key & 0xFFFFFFFF == LIMIT - 1 and (key >> 32) & 3 == 1, (obs, hex(key))
        upd = {e.observer for e in c.events() if e.isUpdated() and e.member == m}
        assert upd == set(range(n)) - {m}
        c.update_incarnation(m)  # -> 2^30: past the key plane's field
        with pytest.raises(SwimError, match="error bits 0x100000"):
            c.step(2)
    finally:
        c.close()


def test_key16_escape_boundary(oracle, engine):
    """Incarnations around 16 382 (the 16-bit shadow's escape in round 5): far past the 8-bit shadow's, so every
    payload lane holding a mover compares its subjects on the full keys, under loss and SYNCs."""
    n = 64
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(syncInterval=1000), record_events=True, seed=0x16B)
    o, e = pair(oracle, engine, cfg)
    lib = {id(o): oracle, id(e): engine}
    movers = (3, 17, 29, 40)
    for c in (o, e):
        c.set_default_loss(10)
        for j, m in enumerate(movers):  # keys 16 379 << 2 | ALIVE .. : every bump below crosses or nears 0xFFFF
            assert _abi.debug_set_incarnation(lib[id(c)], c._h, m, 16379 + j) == 0
    run_lockstep(o, e, 40, 10, "incarnations below the 16-bit escape")
    for step in range(4):
        for c in (o, e):
            for m in movers:
                c.update_incarnation(m)
        run_lockstep(o, e, 40, 10, f"bump {step + 1} across the escape")
    o.close()
    e.close()


def test_key8_escape_boundary(oracle, engine):
    """The 8-bit shadow the SYNC diff streams on one GPU (key8: the key itself below 0xFF, else the escape 0xFF): movers
    start at incarnations 60-63 and are bumped across 62 / 63 (keys 249-255, DEAD at 63 is the first escaped key) and
    past 64, in different 32-subject lanes of the diff and at a lane boundary (31 / 32), under loss and SYNCs every
    tick; every merged record against the oracle."""
    n = 96
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(syncInterval=1000), record_events=True, seed=0x8B)
    o, e = pair(oracle, engine, cfg)
    lib = {id(o): oracle, id(e): engine}
    movers = (3, 31, 32, 63, 64, 95)
    for c in (o, e):
        c.set_default_loss(10)
        for j, m in enumerate(movers):
            assert _abi.debug_set_incarnation(lib[id(c)], c._h, m, 60 + j % 4) == 0
    run_lockstep(o, e, 30, 10, "incarnations below the 8-bit escape")
    for step in range(4):
        for c in (o, e):
            for m in movers[step % 2::2]:
                c.update_incarnation(m)
        run_lockstep(o, e, 30, 10, f"bump {step + 1} across the 8-bit escape")
    o.close()
    e.close()


@pytest.mark.parametrize("world", [2, 3])
def test_key8_escape_sharded(oracle, engine, world):
    """Row shards stream SYNC payloads from the 8-bit plane too: a local sender's row, and a peer's payload through the
    baseline row's shadow, its shipped chunks (rows that differ from the baseline) as escaped lanes compared on the
    shipped u32 keys. Movers are bumped to incarnation 61 in one tick (one gossip per call) and then across the 8-bit
    escape, under 10 % loss and SYNCs every tick, against the oracle."""
    from swimhip.shard import ThreadShardGroup
    n = 96
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(syncInterval=1000), record_events=True, seed=0x8C,
                    gossip_slot_cap=1 << 12)
    o, e = SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, world)
    movers = (3, 32, 64, 95)
    for c in (o, e):
        c.set_default_loss(10)
        for m in movers:
            for _ in range(61):
                c.update_incarnation(m)
    run_lockstep(o, e, 40, 10, f"W={world}: incarnations 61")
    for step in range(3):
        for c in (o, e):
            for m in movers:
                c.update_incarnation(m)
        run_lockstep(o, e, 30, 10, f"W={world}: bump {step + 1} across the 8-bit escape")
    e.close()
    o.close()
