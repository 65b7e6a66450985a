"""Every device allocation of the engine is filled with 0xA5 before initialisation (SWIM_POISON), so state the
engine reads without having written it would change the result. Parity with the oracle must still be bit-exact.
(This caught copy-on-write SYNC snapshots that left the row padding unwritten.)"""
import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, _abi

from parity_util import pair, run_lockstep

pytestmark = pytest.mark.gpu


@pytest.fixture
def poisoned(monkeypatch):
    monkeypatch.setenv("SWIM_POISON", "1")


def test_poisoned_loss_and_kill(oracle, engine, poisoned):
    cfg = SimConfig(n_members=300, record_events=True)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(5)
    run_lockstep(o, e, 60, 20, "poisoned loss5")
    for c in (o, e):
        c.kill(17)
        c.update_incarnation(200)
    run_lockstep(o, e, 120, 40, "poisoned kill")
    e.close()


def test_poisoned_cold_join_partition(oracle, engine, poisoned):
    n = 40
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, n - 1]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 60, 20, "poisoned join")
    g = np.array([0] * (n // 2) + [1] * (n // 2), dtype=np.uint32)
    for c in (o, e):
        c.partition(g)
    run_lockstep(o, e, 200, 50, "poisoned partition")
    for c in (o, e):
        c.unblock_all()
    run_lockstep(o, e, 200, 50, "poisoned heal")
    e.close()
