"""The oracle side of the same-tick SYNC case (no GPU): the directed scenario of
test_gpu_parity.test_sync_same_tick_resurrection and the fast-SYNC fuzz schedules really produce payload records that
equal the receiver's start-of-tick row, differ from its live row and override it (MembershipProtocolImpl.java:456-467,
MembershipRecord.java:67-69). The oracle counts them with SWIMREF_DEBUG (swimdbg_counter 0: equal to the start row
but not to the live one; 1: of those, the ones that override the live row)."""
import ctypes as C

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster


def counters(lib, c):
    fn = lib.swimdbg_counter
    fn.restype, fn.argtypes = C.c_uint64, [C.c_void_p, C.c_uint32]
    return fn(c._h, 0), fn(c._h, 1)


def test_leave_with_fast_sync_resurrects(oracle, monkeypatch):
    monkeypatch.setenv("SWIMREF_DEBUG", "1")
    cc = ClusterConfig(seedMembers=[0], syncInterval=200, syncTimeout=100)
    o = SimulatedCluster(oracle, SimConfig(n_members=8, cluster=cc, record_events=True))
    o.step(7)
    o.leave(0)
    o.step(60)
    equal_start, overriding = counters(oracle, o)
    assert overriding > 0 and equal_start >= overriding
    # a removed leaver re-added by a stale ALIVE record: REMOVED then ADDED of member 0 at one observer
    ev = [x for x in o.events() if x.member == 0]
    readded = {x.observer for x in ev if x.isAdded()} & {x.observer for x in ev if x.isRemoved()}
    assert readded


def test_fast_sync_fuzz_schedules_hit_it(oracle, monkeypatch):
    import test_gpu_fuzz as F
    monkeypatch.setenv("SWIMREF_DEBUG", "1")
    monkeypatch.setattr(F, "run_lockstep", lambda o, e, n, chunk, where: o.step(n))

    class Shadow:
        def __getattr__(self, k):
            return lambda *a, **kw: None

    hits = 0
    for seed in range(200, 210):
        cfg, acts = F.schedule(seed, fast_sync=True)
        o = SimulatedCluster(oracle, cfg)
        F.play(o, Shadow(), acts, "oracle only", cfg.n_dormant)
        hits += counters(oracle, o)[1] > 0
    assert hits >= 2
