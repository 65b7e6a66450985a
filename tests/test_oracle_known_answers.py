"""Pin both libraries to the reference's own known answers, through swim_selftest_eval (include/swimhip_selftest.h).

The oracle evaluates its CPU restatement; libswimhip evaluates, in a gfx950 kernel, the very device functions the
simulation kernels call (the `-m gpu` cases).
* MembershipRecordTest.java:34-108 (cluster/src/test/java/io/scalecube/cluster/membership/) — the full isOverrides
  truth table, the only known-answer test on the hot path, plus the equal-record cases.
* ClusterMath.java:99-135 — ceilLog2 = bit length and the spread / sweep / suspicion closed forms, read from each
  library's own implementation; the table in SURVEY.md §8's header is the fixture.
* Philox4x32-10 known-answer vectors (Random123 kat_vectors), the injected selector of SEMANTICS.md §2.
"""
import ctypes as C

import pytest

from swimhip import _abi

A, S, D, NULL = _abi.ST_ALIVE, _abi.ST_SUSPECT, _abi.ST_DEAD, _abi.ST_ABSENT

R0 = {"null": (NULL, 0), "A0": (A, 0), "A1": (A, 1), "A2": (A, 2), "S0": (S, 0), "S1": (S, 1), "S2": (S, 2),
      "D0": (D, 0), "D1": (D, 1), "D2": (D, 2)}

# MembershipRecordTest.testDeadOverride (:47-63), testAliveOverride (:66-82), testSuspectOverride (:85-101)
TRUTH = {
    (D, 1): {"null": 0, "A0": 1, "A1": 1, "A2": 1, "S0": 1, "S1": 1, "S2": 1, "D0": 0, "D1": 0, "D2": 0},
    (A, 1): {"null": 1, "A0": 1, "A1": 0, "A2": 0, "S0": 1, "S1": 0, "S2": 0, "D0": 0, "D1": 0, "D2": 0},
    (S, 1): {"null": 0, "A0": 1, "A1": 1, "A2": 0, "S0": 1, "S1": 0, "S2": 0, "D0": 0, "D1": 0, "D2": 0},
}
# testEqualRecordNotOverriding (:103-108)
EQUAL = [((st, 1), (st, 1)) for st in (A, S, D)]
CASES = [(r1, R0[name], TRUTH[r1][name]) for r1 in TRUTH for name in R0] + [(a, b, 0) for a, b in EQUAL]

# Random123 kat_vectors, philox4x32 with 10 rounds: ctr[4], key[2] -> out[4]
PHILOX_KAT = [
    ((0, 0, 0, 0, 0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 6, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]

# ClusterMath.ceilLog2 / gossipPeriodsToSpread / gossipPeriodsToSweep / suspicionTimeout at repeatMult 3, mult 5,
# pingInterval 1000 ms = 10 ticks of 100 ms
CLUSTER_MATH = [  # N, bitlen, spread, sweep, suspicion ms  
    (64, 7, 21, 44, 35000), (10_000, 14, 42, 86, 70000), (50_000, 16, 48, 98, 80000),
    (100_000, 17, 51, 104, 85000), (1_000_000, 20, 60, 122, 100000)]


def check_truth_table(lib):
    got = _abi.selftest_eval(lib, _abi.SELFTEST_OVERRIDES, [(r1[0], r1[1], r0[0], r0[1]) for r1, r0, _ in CASES])
    for (r1, r0, want), (g,) in zip(CASES, got):
        assert g == want, (r1, r0, want, g)
    assert len(CASES) == 33


def check_philox(lib):
    got = _abi.selftest_eval(lib, _abi.SELFTEST_PHILOX, [i for i, _ in PHILOX_KAT])
    for (inp, want), g in zip(PHILOX_KAT, got):
        assert g == want, (inp, [hex(x) for x in g])


def check_cluster_math(lib):
    got = _abi.selftest_eval(lib, _abi.SELFTEST_CLUSTER_MATH, [(n, 3, 5, 10) for n, *_ in CLUSTER_MATH])
    for (n, bl, spread, sweep, susp), g in zip(CLUSTER_MATH, got):
        assert g == (bl, spread, sweep, susp // 100), (n, g)
    # the WAN preset (ClusterConfig.java:39-44): suspicionMult 6, pingInterval 5000 ms; edge sizes 0, 1, 2
    got = _abi.selftest_eval(lib, _abi.SELFTEST_CLUSTER_MATH, [(0, 3, 6, 50), (1, 3, 6, 50), (2, 2, 6, 50)])
    assert got == [(0, 0, 2, 0), (1, 3, 8, 300), (2, 4, 10, 600)]


def check_network_settings(lib):
    """TransportTest.testNetworkSettings (transport/src/test/.../TransportTest.java:130-153): 1000 messages from
    client to server with a 50 % loss link setting; the server receives fewer than total / 100 * (50 + 5). The rolls
    are the library's own loss draw (K_PING = 3, one correlation id per message), for three seeds."""
    total, lost_pct = 1000, 50
    for seed in (0x5EED5EED, 1, 0xDEADBEEF12345678):
        rows = [(3, 0, 1, 7, 0, i, seed & 0xFFFFFFFF, seed >> 32) for i in range(total)]
        received = sum(1 for (r,) in _abi.selftest_eval(lib, _abi.SELFTEST_LOSS_ROLL, rows) if not r < lost_pct)
        assert received < total // 100 * lost_pct + total // 100 * 5, received
        assert received > total // 100 * lost_pct - total // 100 * 5, received  # and not a degenerate draw
    rolls = _abi.selftest_eval(lib, _abi.SELFTEST_LOSS_ROLL, [(3, 0, 1, t, 0, 0, 7, 0) for t in range(4000)])
    assert sorted(set(r for (r,) in rolls)) == list(range(100))  # every roll in [0, 100) occurs


def test_network_settings_loss_statistics(oracle):
    check_network_settings(oracle)


def test_is_overrides_truth_table(oracle):
    check_truth_table(oracle)
    for r1, r0, want in CASES:  # the exported scalar helper too
        assert oracle.swim_is_overrides(r1[0], r1[1], r0[0], r0[1]) == want


def test_philox_known_answers(oracle):
    check_philox(oracle)


@pytest.mark.parametrize("n,bl,spread,sweep,susp", CLUSTER_MATH)
def test_cluster_math(oracle, n, bl, spread, sweep, susp):
    assert oracle.swim_ceil_log2(n) == bl
    check_cluster_math(oracle)
    assert oracle.swim_ceil_log2(0) == 0 and oracle.swim_ceil_log2(1) == 1 and oracle.swim_ceil_log2(2) == 2


@pytest.mark.gpu
def test_engine_device_known_answers(engine):
    """The same known answers through libswimhip's device functions (a gfx950 kernel)."""
    check_truth_table(engine)
    check_philox(engine)
    check_cluster_math(engine)
    check_network_settings(engine)
    # the same rolls on both libraries (the device draw is the oracle's)


def test_default_config_matches_cluster_config(oracle):
    c = _abi.SwimConfig()
    oracle.swim_default_config(C.byref(c))
    # ClusterConfig.java:27-36,57
    assert (c.sync_interval_ms, c.sync_timeout_ms, c.suspicion_mult) == (30000, 3000, 5)
    assert (c.ping_interval_ms, c.ping_timeout_ms, c.ping_req_members) == (1000, 500, 3)
    assert (c.gossip_interval_ms, c.gossip_fanout, c.gossip_repeat_mult, c.metadata_timeout_ms) == (200, 3, 3, 3000)


def test_invalid_config_rejected(oracle):
    c = _abi.SwimConfig()
    oracle.swim_default_config(C.byref(c))
    c.n_members = 8
    c.ping_timeout_ms = 1000  # ClusterConfig.java:413-415
    h = C.c_void_p()
    assert oracle.swim_create(C.byref(c), C.byref(h)) == _abi.SWIM_EINVAL
