"""The oracle's swim_debug_set_incarnation (include/swimhip_debug.h), which the 16-bit escape-boundary parity test
(test_gpu_incarnation_limit.py) drives in lockstep with the engine: it sets one member's own record and refuses an
incarnation the engine's 30-bit key field cannot hold, like the engine does (SEMANTICS.md §8). CPU only."""
from swimhip import SimConfig, _abi
from swimhip.cluster import SimulatedCluster


def test_oracle_sets_own_incarnation(oracle):
    c = SimulatedCluster(oracle, SimConfig(n_members=16))
    try:
        assert _abi.debug_set_incarnation(oracle, c._h, 5, 1 << 30) == -4  # SWIM_ECAPACITY
        assert _abi.debug_set_incarnation(oracle, c._h, 99, 3) != 0        # no such member
        assert _abi.debug_set_incarnation(oracle, c._h, 5, 16383) == 0
        key = int(c.row(5)[5])
        assert key & 0xFFFFFFFF == 16383 and (key >> 32) & 3 == 1, hex(key)
        c.update_incarnation(5)  # applied in P0 of the next tick: one above the value set
        c.step(1)
        assert int(c.row(5)[5]) & 0xFFFFFFFF == 16384
    finally:
        c.close()
