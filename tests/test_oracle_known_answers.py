"""Pin the oracle to the reference's own known answers.

* MembershipRecordTest.java:34-108 (cluster/src/test/java/io/scalecube/cluster/membership/) — the full isOverrides
  truth table, the only known-answer test on the hot path.
* ClusterMath.java:99-135 — ceilLog2 = bit length and the spread / sweep / suspicion closed forms; the table in
  SURVEY.md §8 header is the fixture.
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


@pytest.mark.parametrize("r1", list(TRUTH))
def test_is_overrides_truth_table(oracle, r1):
    for name, (s0, i0) in R0.items():
        assert oracle.swim_is_overrides(r1[0], r1[1], s0, i0) == TRUTH[r1][name], (r1, name)


def test_equal_records_do_not_override(oracle):  # testEqualRecordNotOverriding (:103-108)
    for st in (A, S, D):
        assert oracle.swim_is_overrides(st, 1, st, 1) == 0


# ClusterMath.ceilLog2 / gossipPeriodsToSpread / gossipPeriodsToSweep / suspicionTimeout at repeatMult 3, mult 5
CLUSTER_MATH = [  # N, bitlen, spread, sweep, suspicion ms  
    (64, 7, 21, 44, 35000), (10_000, 14, 42, 86, 70000), (50_000, 16, 48, 98, 80000),
    (100_000, 17, 51, 104, 85000), (1_000_000, 20, 60, 122, 100000)]


@pytest.mark.parametrize("n,bl,spread,sweep,susp", CLUSTER_MATH)
def test_cluster_math(oracle, n, bl, spread, sweep, susp):
    assert oracle.swim_ceil_log2(n) == bl
    assert 3 * bl == spread and 2 * (spread + 1) == sweep and 5 * bl * 1000 == susp
    assert oracle.swim_ceil_log2(0) == 0 and oracle.swim_ceil_log2(1) == 1 and oracle.swim_ceil_log2(2) == 2


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
