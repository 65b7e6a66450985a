"""SimulatedCluster: N scalecube members behind one libswimhip handle.

It mirrors the outward surface of the reference's per-member stack:
  * MembershipEvent (membership/MembershipEvent.java:11-123): type ADDED/REMOVED/UPDATED, member, old/new metadata.
  * Cluster.listenMembership / MembershipProtocol.listen (Cluster.java:247, ClusterImpl.java:287-294): here events()
    drains them in (tick, observer, seq) order.
  * MembershipProtocol.members / member(id) (MembershipProtocol.java:14-65): members(observer).
  * MembershipProtocolImpl.getMembershipRecords (:678-680): records(observer).
  * NetworkEmulator.block / unblockAll / setDefaultLinkSettings (transport/.../NetworkEmulator.java:113-192).
The failure behaviour follows the C ABI: any negative return raises SwimError carrying swim_last_error().
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _abi
from .config import SimConfig


class SwimError(RuntimeError):
    pass


@dataclass(frozen=True)
class MembershipEvent:
    tick: int
    observer: int
    seq: int
    type: str  # "ADDED" | "REMOVED" | "UPDATED" | "GOSSIP" (listenGossips: member = origin, metadata = payload lo / hi)
    member: int
    oldMetadata: Optional[int]
    newMetadata: Optional[int]
    # GOSSIP events: the gossip's counter (its id is (member, gossipCounter)); not part of equality
    gossipCounter: int = field(default=0, compare=False, repr=False)

    def isAdded(self):
        return self.type == "ADDED"

    def isRemoved(self):
        return self.type == "REMOVED"

    def isUpdated(self):
        return self.type == "UPDATED"

    def isGossip(self):
        return self.type == "GOSSIP"

    def payload(self):
        """64-bit payload of a GOSSIP event (Cluster.spreadGossip message)."""
        return (self.newMetadata << 32) | self.oldMetadata


@dataclass(frozen=True)
class MembershipRecord:
    member: int
    status: str  # "ALIVE" | "SUSPECT"
    incarnation: int
    has_metadata: bool
    suspicion_deadline: Optional[int]


_TYPES = {_abi.EV_ADDED: "ADDED", _abi.EV_REMOVED: "REMOVED", _abi.EV_UPDATED: "UPDATED", _abi.EV_GOSSIP: "GOSSIP"}
_STATUS = {_abi.ST_ALIVE: "ALIVE", _abi.ST_SUSPECT: "SUSPECT", _abi.ST_DEAD: "DEAD"}  # DEAD: a leaving member's own


def _meta(v):
    return None if v == _abi.META_NONE else int(v)


class SimulatedCluster:
    def __init__(self, lib, cfg: SimConfig):
        self.lib = lib
        self.cfg = cfg
        self.n = cfg.n_members
        self._h = C.c_void_p()
        a = cfg.to_abi()
        rc = lib.swim_create(C.byref(a), C.byref(self._h))
        if rc != 0:
            raise SwimError(f"swim_create failed rc={rc}")
        self._groups = {cfg.cluster.syncGroup: 0}  # MembershipConfig.syncGroup names -> ABI ids

    # -- lifecycle ------------------------------------------------------------------------------------------
    def close(self):
        if self._h:
            self.lib.swim_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc, what):
        if rc != 0:
            msg = self.lib.swim_last_error(self._h)
            raise SwimError(f"{what} failed rc={rc}: {msg.decode() if msg else ''}")

    # -- driving --------------------------------------------------------------------------------------------
    def step(self, ticks=1):
        self._ck(self.lib.swim_step(self._h, ticks), "swim_step")

    def run_periods(self, n):
        self._ck(self.lib.swim_run_periods(self._h, n), "swim_run_periods")

    def sync(self):
        self._ck(self.lib.swim_sync(self._h), "swim_sync")

    @property
    def tick(self):
        t = C.c_uint64()
        self._ck(self.lib.swim_current_tick(self._h, C.byref(t)), "swim_current_tick")
        return t.value

    # -- fault injection (NetworkEmulator) ------------------------------------------------------------------
    def kill(self, member):
        self._ck(self.lib.swim_kill(self._h, member), "swim_kill")

    def set_default_loss(self, pct):
        self._ck(self.lib.swim_set_default_loss(self._h, pct), "swim_set_default_loss")

    def partition(self, group_of_member):
        g = np.ascontiguousarray(np.asarray(group_of_member, dtype=np.uint32))
        assert g.shape == (self.n,)
        self._ck(self.lib.swim_set_partition(self._h, g.ctypes.data_as(C.POINTER(C.c_uint32))), "swim_set_partition")

    def update_incarnation(self, member):
        self._ck(self.lib.swim_update_incarnation(self._h, member), "swim_update_incarnation")

    def update_metadata(self, member):
        """Cluster.updateMetadata: a new metadata version for member, then updateIncarnation (ClusterImpl.java:254)."""
        self._ck(self.lib.swim_update_metadata(self._h, member), "swim_update_metadata")

    def unblock_all(self):
        self._ck(self.lib.swim_unblock_all(self._h), "swim_unblock_all")

    def join(self, member, seeds=()):
        """Cluster.join of a new process for a dormant member (SimConfig.n_dormant) with its own seedMembers."""
        arr = (C.c_uint32 * max(1, len(seeds)))(*[int(x) for x in seeds])
        self._ck(self.lib.swim_join(self._h, member, arr, len(seeds)), "swim_join")

    def set_member_config(self, member, cc):
        """Member `member` runs with its own ClusterConfig `cc` (ClusterImpl.join0 builds every member from its own
        config): its FailureDetectorConfig (ping interval / timeout / ping-req members) and its syncGroup. Before the
        first step, or for a dormant member before join()."""
        cc.validate()
        mc = _abi.SwimMemberConfig()
        mc.ping_interval_ms = cc.pingInterval
        mc.ping_timeout_ms = cc.pingTimeout
        mc.ping_req_members = cc.pingReqMembers
        mc.sync_group = self._groups.setdefault(cc.syncGroup, len(self._groups))
        self._ck(self.lib.swim_set_member_config(self._h, member, C.byref(mc)), "swim_set_member_config")

    def spread_gossip(self, member, payload):
        """Cluster.spreadGossip(message): a user gossip from member carrying a 64-bit payload (ClusterImpl.java:208)."""
        self._ck(self.lib.swim_spread_gossip(self._h, member, int(payload) & (2**64 - 1)), "swim_spread_gossip")

    def leave(self, member):
        """Cluster.shutdown(): graceful leave (MembershipProtocolImpl.leaveCluster, ClusterImpl.doShutdown)."""
        self._ck(self.lib.swim_leave(self._h, member), "swim_leave")

    def set_link_loss(self, src, dst, pct):
        """NetworkEmulator.setLinkSettings on src's emulator for destination dst; 100 = block(dst)."""
        self._ck(self.lib.swim_set_link_loss(self._h, src, dst, pct), "swim_set_link_loss")

    def set_default_link_settings(self, loss, mean_delay_ms):
        """NetworkEmulator.setDefaultLinkSettings(lossPercent, meanDelay) (NetworkEmulator.java:113-125)."""
        self._ck(self.lib.swim_set_default_link_settings(self._h, loss, mean_delay_ms), "swim_set_default_link_settings")

    def set_link_settings(self, src, dst, loss, mean_delay_ms):
        """NetworkEmulator.setLinkSettings(dst, lossPercent, meanDelay) on src's emulator (NetworkEmulator.java:97-111)."""
        self._ck(self.lib.swim_set_link_settings(self._h, src, dst, loss, mean_delay_ms), "swim_set_link_settings")

    def emulator_counters(self):
        """Every member's (totalMessageSentCount, totalMessageLostCount) (NetworkEmulator.java:200-222), shape (n, 2)."""
        out = np.zeros(2 * self.n, dtype=np.uint64)
        self._ck(self.lib.swim_emulator_counters(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), out.size),
                 "swim_emulator_counters")
        return out.reshape(self.n, 2)

    def block(self, src, *dsts):
        """NetworkEmulator.block(destinations) on src's emulator (NetworkEmulator.java:141-150)."""
        for dst in dsts:
            self.set_link_loss(src, dst, 100)

    def unblock(self, src, *dsts):
        """NetworkEmulator.unblock(destinations) on src's emulator (NetworkEmulator.java:158-175)."""
        for dst in dsts:
            self._ck(self.lib.swim_unblock_link(self._h, src, dst), "swim_unblock_link")

    # -- readback -------------------------------------------------------------------------------------------
    def row(self, observer) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.uint64)
        self._ck(self.lib.swim_read_row(self._h, observer, out.ctypes.data_as(C.POINTER(C.c_uint64)), self.n),
                 "swim_read_row")
        return out

    def records(self, observer) -> List[MembershipRecord]:
        row = self.row(observer)
        recs = []
        for s in np.nonzero(row)[0]:
            v = int(row[s])
            st = (v >> 32) & 3
            dl = v >> 35
            recs.append(MembershipRecord(int(s), _STATUS[st], v & 0xFFFFFFFF, bool((v >> 34) & 1), dl or None))
        return recs

    def members(self, observer):
        return [r.member for r in self.records(observer)]

    def trusted(self, observer):
        return [r.member for r in self.records(observer) if r.status == "ALIVE"]

    def suspected(self, observer):
        return [r.member for r in self.records(observer) if r.status == "SUSPECT"]

    def lists(self, observer):
        cap = max(self.n * 2, 16)
        fd = np.zeros(cap, dtype=np.uint32)
        gl = np.zeros(cap, dtype=np.uint32)
        fl, glen = C.c_uint32(), C.c_uint32()
        cur = (C.c_int32 * 2)()
        P = C.POINTER(C.c_uint32)
        self._ck(self.lib.swim_read_lists(self._h, observer, fd.ctypes.data_as(P), C.byref(fl), gl.ctypes.data_as(P),
                                          C.byref(glen), cap, cur), "swim_read_lists")
        return fd[: fl.value].copy(), gl[: glen.value].copy(), (cur[0], cur[1])

    def gossips(self, observer, cap=1 << 20):
        ids = np.zeros(cap, dtype=np.uint64)
        inf = np.zeros(cap, dtype=np.uint32)
        n = C.c_size_t()
        self._ck(self.lib.swim_read_gossips(self._h, observer, ids.ctypes.data_as(C.POINTER(C.c_uint64)),
                                            inf.ctypes.data_as(C.POINTER(C.c_uint32)), cap, C.byref(n)),
                 "swim_read_gossips")
        return [(int(ids[i] >> 32), int(ids[i] & 0xFFFFFFFF), int(inf[i])) for i in range(n.value)]

    def state_hash(self) -> np.ndarray:
        out = np.zeros(self.n * _abi.HASH_WORDS, dtype=np.uint64)
        self._ck(self.lib.swim_state_hash(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), out.size),
                 "swim_state_hash")
        return out.reshape(self.n, _abi.HASH_WORDS)

    def counters(self):
        c = _abi.SwimCounters()
        self._ck(self.lib.swim_counters_get(self._h, C.byref(c)), "swim_counters_get")
        return c.as_dict()

    def events(self, cap=1 << 16) -> List[MembershipEvent]:
        out = []
        buf = (_abi.SwimEvent * cap)()
        n = C.c_size_t()
        while True:
            self._ck(self.lib.swim_drain_events(self._h, buf, cap, C.byref(n)), "swim_drain_events")
            for i in range(n.value):
                e = buf[i]
                if e.type == _abi.EV_GOSSIP:  # payload words, not metadata versions
                    out.append(MembershipEvent(e.tick, e.observer, e.seq, "GOSSIP", e.subject, int(e.old_meta),
                                               int(e.new_meta), int(e.pad)))
                else:
                    out.append(MembershipEvent(e.tick, e.observer, e.seq, _TYPES[e.type], e.subject,
                                               _meta(e.old_meta), _meta(e.new_meta)))
            if n.value < cap:
                return out
