"""Host-side mirror of the reference's configuration surface.

ClusterConfig (cluster/src/main/java/io/scalecube/cluster/ClusterConfig.java:24-419) implements FailureDetectorConfig,
GossipConfig and MembershipConfig. The field names, defaults (:27-36,57), presets (:39-55) and the one validation rule
(pingTimeout < pingInterval, :412-416) are kept. to_abi() lowers the config into the POD swim_config of include/swimhip.h.
"""
from dataclasses import dataclass, field, replace
from typing import List

from . import _abi

DEFAULT_SYNC_GROUP = "default"


@dataclass(frozen=True)
class ClusterConfig:
    # MembershipConfig (membership/MembershipConfig.java:7-26)
    seedMembers: List[int] = field(default_factory=list)
    syncInterval: int = 30_000
    syncTimeout: int = 3_000
    suspicionMult: int = 5
    syncGroup: str = DEFAULT_SYNC_GROUP
    metadataTimeout: int = 3_000
    # FailureDetectorConfig (fdetector/FailureDetectorConfig.java:3-10)
    pingInterval: int = 1_000
    pingTimeout: int = 500
    pingReqMembers: int = 3
    # GossipConfig (gossip/GossipConfig.java:3-10)
    gossipInterval: int = 200
    gossipFanout: int = 3
    gossipRepeatMult: int = 3

    @staticmethod
    def defaultLanConfig():
        return ClusterConfig()

    @staticmethod
    def defaultWanConfig():  # ClusterConfig.java:39-44
        return ClusterConfig(suspicionMult=6, syncInterval=60_000, pingTimeout=3_000, pingInterval=5_000, gossipFanout=4)

    @staticmethod
    def defaultLocalConfig():  # ClusterConfig.java:48-55
        return ClusterConfig(suspicionMult=3, syncInterval=15_000, pingTimeout=200, pingInterval=1_000,
                             gossipRepeatMult=2, pingReqMembers=1, gossipInterval=100)

    def with_(self, **kw):
        return replace(self, **kw)

    def validate(self):
        if self.pingTimeout >= self.pingInterval:  # ClusterConfig.java:413-415
            raise ValueError("Ping timeout can't be bigger than ping interval")
        return self


@dataclass(frozen=True)
class SimConfig:
    """What the deterministic harness adds on top of ClusterConfig (SEMANTICS.md §1-3)."""
    n_members: int
    cluster: ClusterConfig = field(default_factory=ClusterConfig)
    init_mode: int = _abi.INIT_PRECONVERGED
    seed: int = 0x5EED5EED
    tick_ms: int = 100
    latency_ticks: int = 1
    record_events: bool = False
    profile: bool = False
    profile_all: bool = False  # SWIM_FLAG_PROFILE_ALL: every k_sync_diff launch timed (+ member / gossip kernels)
    implicit_views: bool = False  # SWIM_FLAG_IMPLICIT_VIEWS (RUMOR mode): tables / lists computed, not stored
    emulator_counters: bool = False  # SWIM_FLAG_EMULATOR_COUNTERS: per-member NetworkEmulator sent / lost counts
    gossip_slot_cap: int = 0
    gossip_ring_cap: int = 0  # gossips one member can hold at once (0: the engine's default)
    delay_cap_ms: int = 0  # the largest mean link delay this handle will be given (sizes the engine's delay queues)
    pending_fetch_cap: int = 0
    event_cap: int = 0
    list_slack: int = 0
    mode: int = _abi.MODE_FULL  # MODE_RUMOR: gossip layer only, churn_per_period rumors per period (SEMANTICS.md §9)
    churn_per_period: int = 0
    n_dormant: int = 0  # COLD_JOIN: the last n_dormant members start only on join()
    device: int = 0
    n_gpus: int = 1  # > 1: one handle row-sharded over n_gpus devices in this process (swim_create)

    def to_abi(self):
        c = self.cluster.validate()
        a = _abi.SwimConfig()
        a.n_members = self.n_members
        a.tick_ms = self.tick_ms
        a.latency_ticks = self.latency_ticks
        a.init_mode = self.init_mode
        a.seed = self.seed
        a.sync_interval_ms = c.syncInterval
        a.sync_timeout_ms = c.syncTimeout
        a.suspicion_mult = c.suspicionMult
        a.ping_interval_ms = c.pingInterval
        a.ping_timeout_ms = c.pingTimeout
        a.ping_req_members = c.pingReqMembers
        a.gossip_interval_ms = c.gossipInterval
        a.gossip_fanout = c.gossipFanout
        a.gossip_repeat_mult = c.gossipRepeatMult
        a.metadata_timeout_ms = c.metadataTimeout
        a.mode = self.mode
        a.churn_per_period = self.churn_per_period
        a.n_dormant = self.n_dormant
        a.flags = (_abi.FLAG_RECORD_EVENTS if self.record_events else 0) | (_abi.FLAG_PROFILE if self.profile or self.profile_all else 0) \
            | (_abi.FLAG_PROFILE_ALL if self.profile_all else 0) \
            | (_abi.FLAG_IMPLICIT_VIEWS if self.implicit_views else 0) \
            | (_abi.FLAG_EMULATOR_COUNTERS if self.emulator_counters else 0)
        seeds = list(dict.fromkeys(c.seedMembers))
        if len(seeds) > 16:
            raise ValueError("at most 16 seed members")
        a.n_seeds = len(seeds)
        for i, s in enumerate(seeds):
            a.seeds[i] = s
        a.gossip_slot_cap = self.gossip_slot_cap
        a.gossip_ring_cap = self.gossip_ring_cap
        a.delay_cap_ms = self.delay_cap_ms
        a.pending_fetch_cap = self.pending_fetch_cap
        a.event_cap = self.event_cap
        a.n_gpus = self.n_gpus
        a.device = self.device
        a.list_slack = self.list_slack
        return a
