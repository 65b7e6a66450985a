"""Oracle tapes (tests/tape.py) on the CPU: the record / replay round trip, and every committed tape against the live
oracle (a prefix of its calls, the ones whose arguments the tape holds in full), so an oracle change that makes a tape
stale fails here rather than on the GPU box."""
import json
import time

import numpy as np
import pytest

import tape
from swimhip import ClusterConfig, SimConfig, _abi  # noqa: F401  (names for the recorded SimConfig reprs)
from swimhip.cluster import SimulatedCluster


def _same(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b))
    if isinstance(a, tuple) and isinstance(b, tuple):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    return a == b


def test_tape_record_replay_round_trip(oracle, tmp_path, monkeypatch):
    cfg = SimConfig(n_members=40, cluster=ClusterConfig(syncInterval=1000), record_events=True)
    monkeypatch.setenv("SWIM_ORACLE_TAPE", "record")
    monkeypatch.setenv("SWIM_TAPE_OUT", str(tmp_path))
    nodeid = "tests/test_tapes.py::roundtrip[x]"

    def script(c):
        out = []
        c.set_default_loss(10)
        c.step(30)
        out.append(c.state_hash())
        c.kill(3)
        c.update_incarnation(5)
        c.step(40)
        out += [c.counters(), c.events(), c.lists(7), c.row(7), c.gossips(7), c.tick, c.records(1)]
        return out

    tape.begin(nodeid, True)
    live = script(SimulatedCluster(oracle, cfg))
    tape.end(True)
    f = tmp_path / f"{tape.tape_name(nodeid)}.npz"
    assert f.exists()
    monkeypatch.delenv("SWIM_ORACLE_TAPE")
    monkeypatch.setattr(tape, "TAPES", tmp_path)
    tape.begin(nodeid, True)
    c = SimulatedCluster(oracle, cfg)
    assert isinstance(c, tape.TapeCluster) and tape.mode() == "replay"
    again = script(c)
    tape.end(True)
    assert len(again) == len(live) and all(_same(a, b) for a, b in zip(again, live))
    # a different call sequence is refused
    tape.begin(nodeid, True)
    c = SimulatedCluster(oracle, cfg)
    c.set_default_loss(10)
    with pytest.raises(tape.TapeError, match="stale tape"):
        c.step(31)
    tape.end(False)


def _reissue(c, name, args, kwargs):
    if name == "tick":
        return c.tick
    return getattr(c, name)(*args, **kwargs)


@pytest.mark.parametrize("path", sorted(tape.TAPES.glob("*.npz")), ids=lambda p: p.stem)
def test_committed_tape_matches_live_oracle(oracle, path):
    """Re-issue a tape's calls on the live oracle, in order, while their arguments are plain values and the oracle has
    run at most ~60 ticks (CPU time), and require the recorded results."""
    t = tape.load(path)
    live, checked, ticks = {}, 0, 0
    t0 = time.time()
    for rec in t["calls"]:
        name, args, kwargs = json.loads(rec["args"])
        if name == "__create__":
            cfg = eval(args[0], {"SimConfig": SimConfig, "ClusterConfig": ClusterConfig})  # noqa: S307 (our own file)
            live[rec["c"]] = SimulatedCluster(oracle, cfg)
            continue
        if any(isinstance(a, dict) for a in args):  # an array argument: the tape keeps only its digest
            break
        c = live[rec["c"]]
        if name in ("step", "run_periods"):
            n = args[0] * (c.cfg.cluster.pingInterval // c.cfg.tick_ms if name == "run_periods" else 1)
            if ticks + n > 60 or time.time() - t0 > 20:
                break
            ticks += n
        got = _reissue(c, name, args, kwargs)
        want = tape._dec(rec["res"], t["arrays"])
        assert _same(got, want), f"{path.name} call {name}{args}: the live oracle differs from the tape (re-record)"
        checked += 1
    for c in live.values():
        c.close()
    assert checked > 0
