/*
 * swimhip.h — C ABI of libswimhip, the MI355X SWIM membership engine.
 *
 * This header is the drop-in boundary. The reference has no SPI. Its hot path sits behind constructor-injected
 * interfaces wired in ClusterImpl.join0 (cluster/src/main/java/io/scalecube/cluster/ClusterImpl.java:85-152):
 *   FailureDetector    (cluster/.../fdetector/FailureDetector.java:12-25)     start/stop/listen
 *   GossipProtocol     (cluster/.../gossip/GossipProtocol.java:12-29)        start/stop/spread/listen
 *   MembershipProtocol (cluster/.../membership/MembershipProtocol.java:14-65)  start/stop/listen/members/member
 *   MetadataStore      (cluster/.../metadata/MetadataStore.java:11-67)
 *   Transport          (transport/.../Transport.java:74-135)                 send/requestResponse/listen
 * One swim_handle simulates N members, each one a full FD + gossip + membership + metadata stack. The handle replaces
 * those five objects for all N members at once. The MembershipEvent flux (ClusterImpl.java:287-294) becomes
 * swim_drain_events. Configuration is the ClusterConfig field set (ClusterConfig.java:27-36,57).
 *
 * Conventions: every call returns 0 on success or a negative SWIM_E* code; swim_last_error() gives details.
 * The caller owns all buffers. A handle is NOT thread-safe (one host thread per handle, mirroring the single
 * scheduler per member, ClusterImpl.java:93). Semantics: SEMANTICS.md.
 */
#ifndef SWIMHIP_H
#define SWIMHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWIM_ABI_VERSION 1u

/* error codes */
#define SWIM_OK 0
#define SWIM_EINVAL -1    /* bad argument / config (e.g. pingTimeout >= pingInterval, ClusterConfig.java:413-415) */
#define SWIM_ENOMEM -2    /* device or host allocation failed */
#define SWIM_EDEVICE -3   /* HIP / RCCL failure, or no GPU present */
#define SWIM_ECAPACITY -4 /* a fixed-capacity structure overflowed (gossip slots, pending fetches, arenas), or an
                           stored incarnation reached 2^30 (the device key plane holds inc << 2 | status) */
#define SWIM_EUNSUPPORTED -5

/* init_mode */
#define SWIM_INIT_COLD_JOIN 0u    /* every member joins at tick 0 through the seeds (ClusterImpl.join0) */
#define SWIM_INIT_PRECONVERGED 1u /* full views, ALIVE inc 0, shuffled lists (SEMANTICS.md §3) */

/* mode */
#define SWIM_MODE_FULL 0u
#define SWIM_MODE_RUMOR 1u /* gossip layer only (SEMANTICS.md §9): no FD, SYNC or metadata; churn_per_period rumors per period */

/* event types: MembershipEvent.Type (membership/MembershipEvent.java:13-17) */
#define SWIM_EV_ADDED 0u
#define SWIM_EV_REMOVED 1u
#define SWIM_EV_UPDATED 2u
#define SWIM_EV_GOSSIP 3u /* Cluster.listenGossips(): first receipt of a user gossip; subject = origin, old/new_meta = payload lo/hi */
#define SWIM_META_NONE 0xFFFFFFFFu

/* status codes used by swim_read_row: MemberStatus (membership/MemberStatus.java:6-15); 0 = no row */
#define SWIM_ST_ABSENT 0u
#define SWIM_ST_ALIVE 1u
#define SWIM_ST_SUSPECT 2u

/* flags */
#define SWIM_FLAG_RECORD_EVENTS 1u /* keep full event records for swim_drain_events (hashes are always kept) */
#define SWIM_FLAG_PROFILE 2u       /* time a SAMPLE of the k_sync_diff launches with HIP events on the engine stream:
                                      one GPU: the launches of ticks k % 10 == 0; sharded or with PROFILE_ALL: every
                                      launch (swim_counters diff_ns / diff_launches / diff_msgs cover the same set) */
#define SWIM_FLAG_IMPLICIT_VIEWS 8u /* RUMOR mode: the (unchanging) tables and lists are computed, not stored; always
                                      on above 65536 members (C5: 10^6 members would need 8 TB of tables) */
#define SWIM_FLAG_PROFILE_ALL 4u   /* also time k_member_tick and k_gossip_send (member_ns, gossip_ns); ~10 % slower */
#define SWIM_FLAG_EMULATOR_COUNTERS 16u /* keep every member's NetworkEmulator sent / lost counters
                                           (swim_emulator_counters; the oracle always keeps them) */

typedef struct swim_config {
  uint32_t n_members;
  uint32_t tick_ms;       /* virtual time per tick; every interval must be a multiple */
  uint32_t latency_ticks; /* one-way message latency */
  uint32_t init_mode;
  uint64_t seed;
  /* ClusterConfig (ClusterConfig.java:27-36,57) */
  uint32_t sync_interval_ms;    /* 30000 */
  uint32_t sync_timeout_ms;     /* 3000 */
  uint32_t suspicion_mult;      /* 5 */
  uint32_t ping_interval_ms;    /* 1000 */
  uint32_t ping_timeout_ms;     /* 500 */
  uint32_t ping_req_members;    /* 3 */
  uint32_t gossip_interval_ms;  /* 200 */
  uint32_t gossip_fanout;       /* 3 */
  uint32_t gossip_repeat_mult;  /* 3 */
  uint32_t metadata_timeout_ms; /* 3000 */
  uint32_t mode;
  uint32_t flags;
  uint32_t n_seeds;
  uint32_t seeds[16]; /* seed member ids (ClusterConfig.seedMembers) */
  /* engine capacities (0 = default) */
  uint32_t gossip_slot_cap;   /* concurrent gossip ids */
  uint32_t pending_fetch_cap; /* concurrent metadata fetches per member */
  uint32_t event_cap;         /* buffered event records */
  uint32_t n_gpus;            /* > 1: one handle row-sharded over n_gpus devices of this process (RCCL between them;
                                 host exchange when the process sees fewer devices), DESIGN.md §6 */
  uint32_t device;            /* first HIP device */
  uint32_t list_slack;        /* FD / gossip list entries beyond N (duplicates after reordered ADDED / REMOVED) */
  uint32_t churn_per_period;  /* SWIM_MODE_RUMOR: churn events (one rumor each) drawn at the start of every FD period */
  uint32_t n_dormant;         /* COLD_JOIN: the last n_dormant members are not started; each starts on swim_join */
  uint32_t gossip_ring_cap;   /* gossips one member can hold at once (its receipt ring; rounded up to a power of two) */
  uint32_t delay_cap_ms;      /* the largest mean link delay the handle will be given (swim_set_*link_settings); it sizes
                                 the engine's delay queues and replay window. 0: delays that reach a tick are refused
                                 by the engine (the oracle ignores it) */
  uint32_t reserved[2];
} swim_config;

/* One member's own configuration where it differs from the handle's config. The reference builds every member from its own
 * ClusterConfig (ClusterImpl.java:85-152); FailureDetectorTest.testTrustedDespiteDifferentPingTimings runs members with
 * different ping timings (FailureDetectorTest.java:150-178). The FailureDetectorConfig fields drive the member's
 * doPing schedule, ping / ping-req timeouts and helper count, and its suspicion timeout
 * (ClusterMath.suspicionTimeout(mult, size, pingInterval), MembershipProtocolImpl.java:597-606). sync_group is
 * MembershipConfig.syncGroup as an id: a member ignores SYNC / SYNC_ACK data of another group (checkSyncGroup,
 * MembershipProtocolImpl.java:320-331,431-437); members configured by swim_config alone are in group 0. */
typedef struct swim_member_config {
  uint32_t ping_interval_ms;
  uint32_t ping_timeout_ms; /* < ping_interval_ms (ClusterConfig.java:413-415) */
  uint32_t ping_req_members;
  uint32_t sync_group;
  uint32_t reserved[4];
} swim_member_config;

typedef struct swim_event {
  uint32_t tick;
  uint32_t observer;
  uint32_t seq; /* per-observer emission sequence */
  uint32_t type;
  uint32_t subject;
  uint32_t old_meta;
  uint32_t new_meta;
  uint32_t pad;
} swim_event;

/* deterministic op counters; identical on both backends */
typedef struct swim_counters {
  uint64_t tick;
  uint64_t record_compares;   /* R */
  uint64_t row_writes;        /* W */
  uint64_t messages;          /* M: non-gossip messages sent */
  uint64_t gossip_messages;   /* G: GOSSIP_REQ sent */
  uint64_t events;            /* E */
  uint64_t messages_lost;     /* sends failed by loss / block / dead destination */
  uint64_t gossips_created;
  uint64_t sync_merges;       /* SYNC + SYNC_ACK payloads merged */
  /* engine-side measurements (0 on the oracle); *_ns need SWIM_FLAG_PROFILE */
  uint64_t device_bytes;  /* HBM allocated for the simulation state */
  uint64_t diff_ns;       /* k_sync_diff time of the TIMED launches only (see SWIM_FLAG_PROFILE): average per launch =
                             diff_ns / diff_launches; a total needs x (all launches / timed launches) */
  uint64_t member_ns;     /* k_member_tick: per-member protocol control */
  uint64_t gossip_ns;     /* k_gossip_send: gossip data plane */
  uint64_t diff_launches;
  uint64_t exchange_ns; /* sharded handles: host time spent in the per-tick shard exchanges */
  uint64_t diff_msgs;   /* SYNC / SYNC_ACK payloads streamed by the timed k_sync_diff launches (diff_launches) */
  uint64_t ack_resolved; /* SYNC_ACK payloads of those ticks resolved from write logs instead (one GPU; k_ack_resolve) */
  uint64_t ack_resolved_total; /* the same over every tick (payloads streamed = those merged minus these) */
  uint64_t diff_msgs_total;    /* SYNC / SYNC_ACK payloads streamed by every k_sync_diff launch (timed or not) */
  uint64_t diff_key_bytes;     /* key bytes the timed k_sync_diff launches compared: 2 x 2 B per subject for a payload
                                  read from the 16-bit key shadow plane (one GPU, live-row payloads), 2 x 4 B otherwise */
  uint64_t diff_key_bytes_total; /* the same over every k_sync_diff launch */
} swim_counters;

typedef struct swim_handle swim_handle;

/* fills *cfg with the reference defaults (ClusterConfig.java:27-36,57), tick 100 ms, latency 1 tick */
void swim_default_config(swim_config* cfg);
uint32_t swim_abi_version(void);

int swim_create(const swim_config* cfg, swim_handle** out);
int swim_destroy(swim_handle* h);

/* advance the simulation */
int swim_step(swim_handle* h, uint32_t n_ticks);
int swim_run_periods(swim_handle* h, uint32_t n_periods); /* n * pingInterval */
int swim_sync(swim_handle* h);                            /* wait for queued device work */

/* fault injection, effective from the next tick (NetworkEmulator.java:113-192) */
int swim_kill(swim_handle* h, uint32_t member);
int swim_set_default_loss(swim_handle* h, uint32_t loss_percent);
int swim_set_partition(swim_handle* h, const uint32_t* group_of_member); /* n_members entries */
int swim_unblock_all(swim_handle* h); /* also clears every per-link setting (NetworkEmulator.unblockAll :186-192) */
/* NetworkEmulator.setLinkSettings(destination, loss, 0) / block(destination) on member src's emulator (:97-150):
 * a custom loss for messages src -> dst (100 = blocked) that replaces the default and partition settings for that link;
 * swim_set_partition overwrites it on cross-group links, as block() does */
int swim_set_link_loss(swim_handle* h, uint32_t src, uint32_t dst, uint32_t loss_percent);
/* NetworkEmulator.unblock(destination) on member src's emulator (:158-175): back to the default settings */
int swim_unblock_link(swim_handle* h, uint32_t src, uint32_t dst);
/* NetworkEmulator.setDefaultLinkSettings(loss, meanDelay) (:113-125) and setLinkSettings(destination, loss, meanDelay)
 * on member src's emulator (:97-111): loss as above plus a mean delay in ms. A message that is not lost is delayed
 * exponentially (NetworkLinkSettings.evaluateDelay :64-74) and delivered floor(delay / tick_ms) ticks after its
 * normal tick (SEMANTICS.md §2). mean_delay_ms <= 11 * tick_ms (larger means reach delays of 256 ticks: SWIM_EINVAL).
 * swim_set_default_loss keeps the default mean delay; swim_set_link_loss sets a link's mean delay to 0. */
int swim_set_default_link_settings(swim_handle* h, uint32_t loss_percent, uint32_t mean_delay_ms);
int swim_set_link_settings(swim_handle* h, uint32_t src, uint32_t dst, uint32_t loss_percent, uint32_t mean_delay_ms);
/* every member's NetworkEmulator counters (totalMessageSentCount / totalMessageLostCount, NetworkEmulator.java:200-222):
 * out[2m] = sent, out[2m + 1] = lost, cap >= 2 * n_members. tryFail and tryDelay each count a send, so a delivered
 * message counts 2 and a lost one 1 (+1 lost); sends to a dead member fail before the emulator and are not counted.
 * The engine needs SWIM_FLAG_EMULATOR_COUNTERS (else SWIM_EUNSUPPORTED). On an n_gpus handle: the sum over its
 * shards; on one shard of swim_create_sharded: the sends that shard evaluated (its observers' FD / SYNC / metadata
 * messages, the gossip sends to its targets), so the shards' arrays add up to the cluster's. */
int swim_emulator_counters(swim_handle* h, uint64_t* out, size_t cap);
/* MembershipProtocolImpl.updateIncarnation (:178-190): the member bumps its own incarnation and spreads it, at the
 * start (P0) of the next tick; what ClusterImpl.updateMetadata does after storing new metadata */
int swim_update_incarnation(swim_handle* h, uint32_t member);
/* ClusterImpl.updateMetadata (:254-258): metadataStore.updateMetadata, then membership.updateIncarnation. The member's
 * metadata version (what GET_METADATA_RESP carries, MetadataStoreImpl.java:202-241) is bumped at once, between ticks;
 * the incarnation bump and its gossip follow at P0 of the next tick, as swim_update_incarnation */
int swim_update_metadata(swim_handle* h, uint32_t member);
/* ClusterImpl.shutdown -> MembershipProtocolImpl.leaveCluster (ClusterImpl.java:297-313, MembershipProtocolImpl.java:197-206):
 * at the start (P0) of the next tick the member's own record becomes DEAD inc+1 and is spread as gossip; when that
 * gossip is swept at the member (the leave Mono completes), the member stops as if killed, from the next tick */
int swim_leave(swim_handle* h, uint32_t member);
/* Cluster.spreadGossip(message) -> GossipProtocolImpl.spread (ClusterImpl.java:208-211, GossipProtocolImpl.java:124-128):
 * at the start (P0) of the next tick the member creates a user gossip carrying the 64-bit payload, before any
 * incarnation bump or leave queued for the same tick, in call order. Every other member that receives it first emits a
 * SWIM_EV_GOSSIP event (listenGossips, ClusterImpl.java:213-216); membership ignores it (MembershipProtocolImpl :401-408) */
int swim_spread_gossip(swim_handle* h, uint32_t member, uint64_t payload);
/* Cluster.join(config) of a new process (ClusterImpl.join0 -> MembershipProtocolImpl.start0, ClusterImpl.java:85-152,
 * MembershipProtocolImpl.java:216-251) for a dormant member (swim_config.n_dormant): at the next tick it starts with
 * its own seed list (seedMembers, deduplicated, self skipped; at most 16), its schedules starting at that tick. A
 * restart of a crashed member is swim_kill of the old id plus swim_join of a dormant id (a restarted member has a new
 * id in the reference, FailureDetectorTest.java:345-401). A member joins at most once. */
int swim_join(swim_handle* h, uint32_t member, const uint32_t* seeds, uint32_t n_seeds);
/* the member's own FailureDetectorConfig / syncGroup (swim_member_config). Allowed before the first swim_step, or for a
 * dormant member before its swim_join (a running member's config is fixed, as a Cluster's is) */
int swim_set_member_config(swim_handle* h, uint32_t member, const swim_member_config* mc);

/* readback */
int swim_current_tick(swim_handle* h, uint64_t* tick);
/* row of one observer: keys[s] = inc | status<<32 | meta_present<<34 | timer_deadline<<35 (SEMANTICS.md §8); the
 * device stores it as two u32 planes (key32 = inc << 2 | status, and the bits from 34 up), joined here */
int swim_read_row(swim_handle* h, uint32_t observer, uint64_t* keys_out, size_t cap);
/* per-observer hashes: out[6*m + {0:row, 1:fd list, 2:gossip list, 3:events, 4:gossips held, 5:counters}] */
int swim_state_hash(swim_handle* h, uint64_t* out, size_t cap);
/* FD pingMembers and gossip remoteMembers lists, plus cursors */
int swim_read_lists(swim_handle* h, uint32_t observer, uint32_t* fd_out, uint32_t* fd_len, uint32_t* gossip_out,
                    uint32_t* gossip_len, size_t cap, int32_t* cursors_out /* [pingIdx, remoteIdx] */);
/* gossips held by one observer (GossipProtocolImpl.gossips, GossipState.java:8-38): id = origin << 32 | counter,
 * infection period; sorted by id */
int swim_read_gossips(swim_handle* h, uint32_t observer, uint64_t* ids_out, uint32_t* inf_period_out, size_t cap,
                      size_t* n_out);
int swim_drain_events(swim_handle* h, swim_event* out, size_t cap, size_t* n_out);
int swim_counters_get(swim_handle* h, swim_counters* out);
const char* swim_last_error(swim_handle* h);

/* the reference's pure helpers, exported for known-answer tests */
int swim_is_overrides(uint32_t r1_status, uint32_t r1_inc, uint32_t r0_status, uint32_t r0_inc); /* status 3 = DEAD */
uint32_t swim_ceil_log2(uint32_t n);

#ifdef __cplusplus
}
#endif
#endif
