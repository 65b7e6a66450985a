"""Wire-format export (include/swimhip_wire.h): the TCP frames the reference's transport would write.

A frame is a 4-byte big-endian length (LengthFieldPrepender, transport/.../TransportImpl.java:370-384) and the Jackson
JSON of a Message (JacksonMessageCodec.java:41-52). The expected bytes are restated here independently, field by field,
from the reference classes (Message.java, SyncData.java:11-41, MembershipRecord.java:12-56, Member.java:12-13,
Address.java:14-15, GossipRequest.java, Gossip.java). The reference's own test is a Jackson round trip
(GossipRequestTest.java:41-69: data type, correlation id, gossip list, inner message data survive), restated as a
parse of our frame; no serialized bytes ship with the reference, so byte order within the accessor-derived
properties is parity unpinned (see the header)."""
import json
import struct

import pytest

from swimhip import LIB_PATH, _abi

A, S, D = _abi.ST_ALIVE, _abi.ST_SUSPECT, _abi.ST_DEAD


@pytest.fixture(scope="module")
def lib():
    if not LIB_PATH.exists():
        pytest.skip("libswimhip.so not built")
    return _abi.load(LIB_PATH)  # the encoders are host code: no device is touched


def member(i):
    return {"id": str(i), "address": {"host": f"10.{(i >> 16) & 255}.{(i >> 8) & 255}.{i & 255}", "port": 4801}}


def record(i, st, inc):
    name = {A: "ALIVE", S: "SUSPECT", D: "DEAD"}[st]
    return {"member": member(i), "status": name, "incarnation": inc, "alive": st == A, "suspect": st == S,
            "dead": st == D}


def expected_sync(kind, sender, recs, cid=None, group="default"):
    headers = {"q": "sc/membership/sync" if kind == _abi.WIRE_SYNC else "sc/membership/syncAck"}
    if cid is not None:
        headers["cid"] = cid
    msg = {"headers": headers,
           "data": {"@class": "io.scalecube.cluster.membership.SyncData",
                    "membership": [record(*r) for r in recs], "syncGroup": group},
           "sender": member(sender)["address"]}
    return json.dumps(msg, separators=(",", ":")).encode()


def unframe(b):
    (n,) = struct.unpack(">I", b[:4])
    assert n == len(b) - 4
    return b[4:]


def test_sync_frame_bytes(lib):
    recs = [(0, A, 0), (1, S, 3), (7, A, 12), (70000, A, 2), (5, D, 1)]
    for kind, cid in ((_abi.WIRE_SYNC, None), (_abi.WIRE_SYNC_ACK, "17-4"), (_abi.WIRE_SYNC, 'q"\\x')):
        got = _abi.wire_sync_frame(lib, kind, 70000, recs, cid=cid)
        assert unframe(got) == expected_sync(kind, 70000, recs, cid), got


def test_gossip_request_round_trip(lib):
    """GossipRequestTest.testSerializationAndDeserialization (:41-69) restated on our bytes."""
    got = json.loads(unframe(_abi.wire_gossip_frame(lib, 3, 9, 41, (9, S, 5))))
    assert got["headers"] == {"q": "sc/gossip/req"}
    assert got["data"]["@class"] == "io.scalecube.cluster.gossip.GossipRequest"
    assert got["data"]["from"] == "3"
    (g,) = got["data"]["gossips"]
    assert g["gossipId"] == "9-41"  # generateGossipId: <origin id>-<counter> (GossipProtocolImpl.java:207-209)
    inner = g["message"]
    assert inner["headers"] == {"q": "sc/membership/gossip"} and "sender" not in inner  # NON_NULL
    assert inner["data"] == {"@class": "io.scalecube.cluster.membership.MembershipRecord", **record(9, S, 5)}
    assert got["sender"] == member(3)["address"]
    assert list(inner["data"]) == ["@class", "member", "status", "incarnation", "alive", "suspect", "dead"]


def test_capacity_and_max_frame(lib):
    import ctypes as C
    _abi.bind_wire(lib)
    arr = (_abi.SwimWireRecord * 1)(_abi.SwimWireRecord(1, A, 0))
    n = C.c_size_t()
    buf = (C.c_uint8 * 8)()
    assert lib.swim_wire_sync_frame(1, 0, None, b"default", arr, 1, buf, 8, C.byref(n)) == _abi.SWIM_ECAPACITY
    assert n.value == len(_abi.wire_sync_frame(lib, 1, 0, [(1, A, 0)]))
    # TransportConfig.DEFAULT_MAX_FRAME_LENGTH = 2 MB (TransportConfig.java:9): a 20k-record SYNC is beyond it
    big = _abi.wire_sync_frame(lib, 1, 0, [(i, A, 0) for i in range(20_000)])
    assert len(big) - 4 > 2 * 1024 * 1024


@pytest.mark.gpu
def test_export_live_table_matches_oracle(oracle, engine):
    """A SYNC frame exported from the engine's live table equals the one encoded from the oracle's table."""
    from swimhip import ClusterConfig, SimConfig
    from swimhip.cluster import SimulatedCluster
    cfg = SimConfig(n_members=64, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN)
    o, e = SimulatedCluster(oracle, cfg), SimulatedCluster(engine, cfg)
    for c in (o, e):
        c.step(60)
        c.kill(63)
        c.step(30)
    for obs in (0, 17, 62):
        row = o.row(obs)
        recs = [(s, (int(v) >> 32) & 3, int(v) & 0xFFFFFFFF) for s, v in enumerate(row) if v]
        want = _abi.wire_sync_frame(engine, _abi.WIRE_SYNC, obs, recs)
        assert _abi.export_sync_frame(engine, e._h, obs) == want
        assert json.loads(unframe(want))["data"]["membership"][0]["member"]["id"] == str(recs[0][0])
    e.close()
