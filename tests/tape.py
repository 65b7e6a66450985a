"""Oracle tapes: the CPU oracle's side of a lockstep parity test, recorded once and replayed on the GPU box.

TEST INFRASTRUCTURE. The slowest -m gpu tests spend their time in the CPU oracle (a 160-member SYNC storm under loss runs
~0.15 s per tick on the oracle and ~1 ms on the engine), which put the GPU suite near the driver's 900-s limit. A test
marked `@pytest.mark.tape` gets, for every `SimulatedCluster(oracle, cfg)` it builds, a TapeCluster:

* record (SWIM_ORACLE_TAPE=record): the real oracle cluster runs, and every call the test makes on it (name, arguments,
  result: state hashes, counters, events, rows, lists, gossips, ticks) is appended to the test's tape, written to
  $SWIM_TAPE_OUT (default gpurun_out/tapes) when the test passes;
* replay (the default when the test's tape exists under tests/golden/tapes): no oracle runs; each call must match the
  recorded call (same method and arguments, same SimConfig at creation) and returns the recorded result, so every
  assertion of the test compares the engine against exactly what the oracle returned when the tape was recorded;
* live (no tape, or SWIM_ORACLE_TAPE=off): the real oracle, as before.

The comparison is the same bit-exact one as with the live oracle; only the oracle's cost moves out of the GPU run.
tests/test_tapes.py replays a prefix of every tape against the live oracle on the CPU, so a change to the oracle that
would make a tape stale fails the CPU suite.
"""
import dataclasses
import hashlib
import io
import json
import os
import re
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
TAPES = HERE / "golden" / "tapes"

_state = {"test": None, "mode": "live", "tape": None, "clusters": 0, "recorded": None}


class TapeError(AssertionError):
    pass


def tape_name(nodeid):
    """tests/test_x.py::test_y[a-b] -> test_x__test_y_a-b_"""
    path, _, test = nodeid.partition("::")
    return Path(path).stem + "__" + re.sub(r"[^A-Za-z0-9_.\-]+", "_", test)


def tape_path(nodeid):
    return TAPES / f"{tape_name(nodeid)}.npz"


# -- encoding of arguments and results -------------------------------------------------------------------------------
def _enc(v, arrays):
    from swimhip.cluster import MembershipEvent, MembershipRecord
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    if isinstance(v, np.integer):
        return int(v)
    if isinstance(v, np.ndarray):
        key = f"a{len(arrays)}"
        arrays[key] = v
        return {"__nd__": key}
    if isinstance(v, dict):
        return {"__dict__": [[_enc(k, arrays), _enc(x, arrays)] for k, x in v.items()]}
    if isinstance(v, tuple):
        return {"__tuple__": [_enc(x, arrays) for x in v]}
    if isinstance(v, list):
        if v and all(isinstance(x, MembershipEvent) for x in v):
            rows = np.array([[e.tick, e.observer, e.seq, ["ADDED", "REMOVED", "UPDATED", "GOSSIP"].index(e.type),
                              e.member, -1 if e.oldMetadata is None else e.oldMetadata,
                              -1 if e.newMetadata is None else e.newMetadata, e.gossipCounter] for e in v],
                            dtype=np.int64)
            key = f"a{len(arrays)}"
            arrays[key] = rows
            return {"__events__": key}
        if v and all(isinstance(x, MembershipRecord) for x in v):
            return {"__records__": [dataclasses.astuple(x) for x in v]}
        return [_enc(x, arrays) for x in v]
    if dataclasses.is_dataclass(v):
        return {"__repr__": repr(v)}
    raise TypeError(f"tape cannot encode {type(v)}")


def _dec(v, arrays):
    from swimhip.cluster import MembershipEvent, MembershipRecord
    if isinstance(v, list):
        return [_dec(x, arrays) for x in v]
    if not isinstance(v, dict):
        return v
    if "__nd__" in v:
        return arrays[v["__nd__"]].copy()
    if "__dict__" in v:
        return {_dec(k, arrays): _dec(x, arrays) for k, x in v["__dict__"]}
    if "__tuple__" in v:
        return tuple(_dec(x, arrays) for x in v["__tuple__"])
    if "__events__" in v:
        types = ["ADDED", "REMOVED", "UPDATED", "GOSSIP"]
        out = []
        for r in arrays[v["__events__"]].tolist():
            old = None if r[5] == -1 else r[5]
            new = None if r[6] == -1 else r[6]
            out.append(MembershipEvent(r[0], r[1], r[2], types[r[3]], r[4], old, new, r[7]))
        return out
    if "__records__" in v:
        return [MembershipRecord(*x) for x in v["__records__"]]
    raise TypeError(f"tape cannot decode {v}")


def _args_key(name, args, kwargs):
    norm = json.dumps([name, _plain(args), _plain(kwargs)], sort_keys=True)
    return hashlib.blake2b(norm.encode(), digest_size=12).hexdigest(), norm


def _plain(v):
    if isinstance(v, np.ndarray):
        return {"nd": hashlib.blake2b(np.ascontiguousarray(v).tobytes(), digest_size=12).hexdigest(), "shape": v.shape}
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _plain(x) for k, x in v.items()}
    if isinstance(v, np.integer):
        return int(v)
    if dataclasses.is_dataclass(v):
        return repr(v)
    return v


# -- the cluster stand-in --------------------------------------------------------------------------------------------
class TapeCluster:
    """A SimulatedCluster(oracle, cfg) of a taped test: records the real one's calls, or replays them."""

    def __init__(self, real_lib, cfg):
        idx = _state["clusters"]
        _state["clusters"] += 1
        self._idx = idx
        self.cfg = cfg
        self.n = cfg.n_members
        self._mode = _state["mode"]
        self._real = None
        if self._mode == "record":
            from swimhip.cluster import SimulatedCluster
            self._real = object.__new__(SimulatedCluster)
            self._real.__init__(real_lib, cfg)
            self.lib, self._h = self._real.lib, self._real._h
        else:
            self.lib, self._h = None, None
        self._call("__create__", (repr(cfg),), {}, lambda: None)

    def _call(self, name, args, kwargs, fn):
        key, norm = _args_key(name, args, kwargs)
        if self._mode == "record":
            res = fn()
            _state["recorded"]["calls"].append({"c": self._idx, "name": name, "key": key, "args": norm,
                                                "res": _enc(res, _state["recorded"]["arrays"])})
            return res
        tape = _state["tape"]
        pos = tape["pos"]
        if pos >= len(tape["calls"]):
            raise TapeError(f"oracle tape {tape['path'].name} ends before call {name}{args} (re-record: "
                            f"SWIM_ORACLE_TAPE=record)")
        rec = tape["calls"][pos]
        if rec["c"] != self._idx or rec["key"] != key:
            raise TapeError(f"oracle tape {tape['path'].name} call {pos}: the test made {norm} on cluster {self._idx}, "
                            f"the tape holds {rec['args']} on cluster {rec['c']} (stale tape: re-record with "
                            f"SWIM_ORACLE_TAPE=record)")
        tape["pos"] = pos + 1
        return _dec(rec["res"], tape["arrays"])

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        if name == "tick":
            return self._call("tick", (), {}, lambda: self._real.tick)
        from swimhip.cluster import SimulatedCluster
        if not callable(getattr(SimulatedCluster, name, None)):
            raise AttributeError(f"TapeCluster has no {name}")

        def method(*args, **kwargs):
            if name in ("close", "__del__"):
                if self._real is not None:
                    self._real.close()
                return None
            return self._call(name, args, kwargs, lambda: getattr(self._real, name)(*args, **kwargs))

        return method

    def close(self):
        if self._real is not None:
            self._real.close()


# -- per-test set-up (conftest) ----------------------------------------------------------------------------------
def begin(nodeid, taped):
    """Called before each test: picks the mode for the oracle clusters the test builds."""
    _state.update(test=nodeid, clusters=0, tape=None, recorded=None, mode="live")
    if not taped:
        return
    want = os.environ.get("SWIM_ORACLE_TAPE", "")
    p = tape_path(nodeid)
    if want == "record":
        _state["mode"] = "record"
        _state["recorded"] = {"calls": [], "arrays": {}}
    elif want != "off" and p.exists():
        _state["mode"] = "replay"
        _state["tape"] = load(p)


def load(p):
    z = np.load(p, allow_pickle=False)
    meta = json.loads(bytes(z["__tape__"]).decode())
    arrays = {k: z[k] for k in z.files if k != "__tape__"}
    return {"path": p, "calls": meta["calls"], "arrays": arrays, "pos": 0}


def end(passed):
    """After each test: write a recorded tape (record mode, test passed); check a replay consumed its whole tape."""
    mode, rec, tape = _state["mode"], _state["recorded"], _state["tape"]
    nodeid = _state["test"]
    _state.update(mode="live", recorded=None, tape=None)
    if mode == "record" and passed and rec is not None:
        out = Path(os.environ.get("SWIM_TAPE_OUT", str(HERE.parent / "gpurun_out" / "tapes")))
        out.mkdir(parents=True, exist_ok=True)
        meta = json.dumps({"test": nodeid, "calls": rec["calls"]}, separators=(",", ":")).encode()
        buf = io.BytesIO()
        np.savez_compressed(buf, __tape__=np.frombuffer(meta, dtype=np.uint8), **rec["arrays"])
        (out / f"{tape_name(nodeid)}.npz").write_bytes(buf.getvalue())
    if mode == "replay" and passed and tape["pos"] != len(tape["calls"]):
        raise TapeError(f"oracle tape {tape['path'].name}: the test made {tape['pos']} of its {len(tape['calls'])} "
                        f"recorded calls (stale tape: re-record with SWIM_ORACLE_TAPE=record)")


def mode():
    return _state["mode"]
