// engine.h — device-resident state of libswimhip and the per-tick kernel pipeline.
//
// Layout in HBM, one GPU, N members (all arrays are SoA; "per member" = indexed by observer id):
//   rowk, rowa u32[N][NS] x 2      membership table: key plane (inc << 2 | status) and aux plane (metadata bit,
//                                  suspicion deadline), swim_common.h
//   fdl, gl    u32[N][LCAP]       FailureDetectorImpl.pingMembers / GossipProtocolImpl.remoteMembers
//   S          u32[N][SLOTS]      holder x gossip slot: creation tick + 1 | SWEPT | REBORN (stale past a recycle: s_get)
//   logs       per member ring of the last LOGW gossip rounds: (tick, spread, targets[F])
//   subs/paths/fetches/groups      fixed-capacity per-member request state (virtual remote hops)
//   msgs       SYNC / SYNC_ACK records, double-buffered by tick parity; payload = the sender's live row
//              (copy-on-write into the arena if the sender writes its row later in the same tick)
#pragma once
#include <stdint.h>

#include "swim_common.h"

namespace swim {

constexpr uint32_t NEVER = 0xFFFFFFFFu;
constexpr uint32_t MAX_EPOCHS = 8;
constexpr uint32_t DTAB = 16;  // distinct mean delays per handle (delay index 0: none)
constexpr uint32_t SUBCAP = 8, PATHCAP = 8, FREC = 8, GREC = 8;
// pending virtual hops per member with link delays (swim_config.delay_cap_ms > 0): a delayed ping-req chain stays
// open for up to 4 x (lat + EMAX) ticks, several FD periods, so more of them overlap (Dev::PCAP <= 32)
constexpr uint32_t PATHCAP_DELAY = 32;
constexpr uint32_t CH = 2048;  // subjects per SYNC-diff work item (256 threads x 8) and per shipped payload chunk
constexpr uint32_t MCH = 1024;  // subjects per candidate-list segment (chunk_meta): one wave of 16-bit keys
constexpr uint32_t TRK = 16;   // subjects written in one tick's P1 that are re-checked against later payloads (sorted list)
constexpr uint32_t TRKL = 64;  // of them listed per member for clearing its written-subject bitmap (more: the whole row)
// deferred copy-on-write (member.hip cow): row writes logged per member and tick while a snapshot is open, open
// snapshots per member, deferred snapshots per k_member_tick block
constexpr uint32_t ULOG = 1024, CREQ = 4, CWMAX = 32;  // ULOG: the largest undo log (Dev::ULOGC is the stride in use)
constexpr uint32_t SPQ = 32;  // gossips a member creates in one tick before their slots are taken together
constexpr uint32_t KP = 64;   // FD-list inserts of one member's tick applied together (member.hip fd_flush)
constexpr uint32_t MQ = 16;   // inbound SYNC messages of one tick sorted in registers (more: selected by list walks)
constexpr uint32_t SORT_MAX = 4096;  // receipts of one member and tick sorted in LDS at once (more: runs + merges)

// S entry flags (gossip slot x member), as s_get returns them
constexpr uint32_t S_SWEPT = 1u << 30, S_REBORN = 1u << 31;
constexpr uint32_t S_TICK_MASK = (1u << 29) - 1u;
// stored S entries are 16 bits: REBORN | SWEPT | EVER | the creation tick's low 13 bits. s_get rebuilds the tick as the
// latest one at or before the entry's newest possible tick (now + lat) with those bits, exact while every entry is
// younger than 8192 ticks: a slot may live SLIFE ticks (E_SLIFE past it), and every SCRUB ticks k_s_scrub clears the
// entries of recycled slots, so a stale entry is at most SLIFE + SCRUB < 8192 - lat ticks old
constexpr uint16_t S16_REBORN = 1u << 15, S16_SWEPT = 1u << 14, S16_EVER = 1u << 13, S16_TICK = (1u << 13) - 1u;
constexpr uint32_t SLIFE = 4096, SCRUB = 2048;
// the creation tick of a stored entry: the latest tick at or before ref (the newest an entry can carry: now + lat)
// with the stored low 13 bits
__host__ __device__ __forceinline__ uint32_t s16_tick(uint16_t e, uint32_t ref) {
  return ref - ((ref - (uint32_t)(e & S16_TICK)) & (uint32_t)S16_TICK);
}

// device error bits
constexpr uint32_t E_SLOTS = 1, E_FETCH = 2, E_SUBS = 4, E_PATHS = 8, E_GROUPS = 16, E_MSGS = 32, E_ARENA = 64,
                   E_POOL = 128, E_LIST = 256, E_DELIV = 512, E_RECEIPTS = 1024, E_CONTACTS = 2048,
                   E_REBORN = 4096, E_LOGWIN = 8192, E_EPOCH = 16384, E_EVENTS = 32768, E_SORTCAP = 65536,
                   E_XCAP = 1u << 17, E_LINKHIST = 1u << 18, E_DEATHS = 1u << 19,
                   E_INC = 1u << 20,  // an incarnation >= 2^30 would not fit the key plane (swim_common.h)
                   E_PIN = 1u << 21,  // a later SYNC payload of a receiver's tick had no readable copy (pin)
                   E_RING = 1u << 22,  // a member held more gossips than its receipt ring (gossip_ring_cap)
                   E_DELAYQ = 1u << 23,  // more delayed first receipts due in one tick than the delay queue holds
                   E_SYNCQ = 1u << 24,   // more delayed SYNC / SYNC_ACK messages in flight than the SYNC delay store holds
                   E_SLIFE = 1u << 25;   // a gossip slot stayed in use SLIFE ticks (its 16-bit holder entries could alias)
// per-link NetworkEmulator settings (setLinkSettings / block / unblock): hash of (src, dst) -> change history
constexpr uint32_t LKCAP = 4096, LKH = 8;  // keys, history entries per key
constexpr uint32_t CIN_SLOW = 0xFFFFFFFEu;
constexpr uint32_t RX_ALL = 0xFFFFFFFFu;
constexpr uint32_t MDU = 64;  // members with updated metadata per handle
// cached contact events per (sender, target): n, oldest[2], last inbound, then per event tick, slot | dir | loss % |
// spread, and the sender's rounds before the event's tick
constexpr uint32_t CEV = 6, CEVW = 4 + 3 * CEV;
// gossip incarnation history entry: 3 header words + HKEEP creation ticks of swept incarnations (small clusters
// under loss re-infect a member with the same gossip many times: each late sender restarts the chain)
constexpr uint32_t HREC = 11, HKEEP = 16;
constexpr uint32_t LK_NONE = 0xFFFFFFFFu, LK_TRUNC = 0x80000000u;  // link values: loss % | delay index << 8

// row sharding: SyncMsg.payload values
constexpr uint32_t PAY_RX = 0x40000000u;  // received from another shard: PAY_RX | rx index (dirty chunks + baseline)
constexpr uint32_t RRW = 12;              // words per gossip-round record: m, cnt, spread, period, targets[8]
constexpr uint32_t NSW = 8;               // words per new-gossip-slot record
// exchange byte-count words: low 48 bits = bytes; bit 62 = the sender has gossip slots in use this tick
// bit 61 = the sender has a region larger than the inline block for some peer (a send/recv group follows)
constexpr unsigned long long XCNT_MASK = (1ull << 48) - 1, XFLAG_GOSSIP = 1ull << 62, XFLAG_OVER = 1ull << 61;
// exchange B record (slot << 32 | low word): low = target id (< 2^31), or XD_EXT | tick: a delayed send queued on its
// target's shard keeps the slot until tick + EXPB (delay_push), and every shard must recycle it at the same tick
constexpr uint32_t XD_EXT = 0x80000000u;
constexpr uint32_t XINL = 16384;  // RCCL: bytes per peer moved by the fixed-size all-to-all (count word + region head)

// counters (swim_counters order after .tick)
// 8..12: SWIM_EXP & 4 (and 16..19: the gossip plane's work units per tick, for algorithmic bytes; tools/pmc_gossip.py)
constexpr uint32_t CSH = 64, CSTRIDE = 64;  // Dev::ctr_sh rows, 512 B apart
enum Ctr { C_R = 0, C_W, C_M, C_G, C_E, C_LOST, C_GCREATED, C_SYNCMERGE, C_DIFFMSG = 13, C_XU = 16, C_ACKRES = 24, C_ACKRES_ALL = 25, C_DIFFMSG_ALL = 26, C_DIFFWIDE = 27, C_DIFFWIDE_ALL = 28, C_NCTR = 29 };

// capacity fallbacks that fired (include/swimhip_debug.h; counted only when Dev::fb is allocated: SWIM_CAPS or
// SWIM_FALLBACKS set at create). Each one is an exact slow path taken when a fixed-capacity fast structure is full.
enum Fb {
  FB_TRK_WALK = 0,  // merge_payload merged a later payload with the written-subject bitmap (more than trk_cap tracked)
  FB_ULOG,          // cow_now: a member's undo log was full (ulog_cap), its open snapshots copied by its lane
  FB_CREQ,          // cow_now: a member had creq_cap snapshots open
  FB_CWMAX,         // copy_row_to: the block's deferred snapshot list was full (cwmax_cap), the lane copied the row
  FB_CEV_SLOW,      // k_gossip_send_slow: sends of a pair whose contact list overflowed the cache (cev_cap)
  FB_REPLAY,        // k_gossip_replay: sends of a pair with a cached contact (isInfected replay)
  FB_MQ,            // P1: more than mq_cap inbound SYNC messages, selected in key order by list walks
  FB_SORT_MERGE,    // k_seg_sort: a receipt segment above sort_cap sorted in runs and merged
  FB_RX_ALL,        // a contact pair without an RX row (more than rx_cap this tick): its whole window replayed
  FB_N = 16
};

struct SyncMsg {
  uint32_t src, dst, kind, seq, cid_iss, cid_cnt;
  uint32_t payload;  // NEVER = sender's live row, else arena row index
  uint32_t psize;    // records in the payload = the sender's table size when it sent
  uint32_t ncand;    // filled by k_sync_diff: payload records that differ from the receiver's row
  uint32_t pad;
  // arena row that k_sync_diff fills with a copy of a live-row payload (NEVER: none). Set when the receiver has
  // several SYNC / SYNC_ACK payloads in one tick: the member kernel then reads later payloads' records directly (the
  // sender may write its live row meanwhile), for the subjects an earlier payload of that tick changed
  uint32_t pin;
  uint32_t due;  // delayed message (kind has KF_DEFER): the tick of its P1 delivery
  uint32_t tln;  // SYNC_ACK with KF_RES: the sender's tick write-log length when it sent (k_ack_resolve)
};
constexpr uint32_t KF_DEFER = 0x100u;  // SyncMsg.kind flag: delivered after the next tick (k_sync_defer stores it)
// k_sync_diff: a SYNC payload lacks a record the receiver holds (its SYNC_ACK cannot be resolved from write logs)
constexpr uint32_t KF_ABS = 0x200u;
// a SYNC_ACK sent in the tick its SYNC was merged: k_ack_resolve derives its diff from the two write logs instead of
// k_sync_diff streaming it (cleared there when it cannot)
constexpr uint32_t KF_RES = 0x400u;
// k_sync_diff's list entries (Dev::dlist, dlist_w: 16 B = message, sender, receiver, payload place): the payload place
// is the message's payload (arena row or PAY_RX | rx index), NEVER for the live row, DESC_PIN | arena row for a pinned
// live row, DESC_DEFER for a delayed message (kernels.hip desc_pay)
constexpr uint32_t DESC_PIN = 0x80000000u, DESC_DEFER = 0xFFFFFFFEu;
constexpr uint32_t KF_LATE = 0x800u;  // a delayed message put back by k_sync_redeliver
constexpr uint32_t KF_FLAGS = KF_DEFER | KF_ABS | KF_RES | KF_LATE;
constexpr uint32_t TL = 16;  // per-member tick write log (ack resolution); past it the member's ACKs are streamed
// exchange A's SYNC entry: the message, its first chunk slot + pad, the chunk mask, the sender's write-log prefix
__host__ __device__ __forceinline__ uint64_t sync_entry_size(uint32_t MW) { return sizeof(SyncMsg) + 8 + 8ull * MW + 4ull * TL; }

// a member's body-only state (member_tick_body's ML fields): one 128-B line per member
struct alignas(16) MS {
  uint32_t tsize, fdLen, gLen, fdPeriod;
  uint32_t gPeriod, gCounter, cidCnt, syncSeq;
  uint32_t evSeq, initDeadline, initCidBase, initN;
  uint32_t nsub, npath, nfetch, fnext;  // fnext: earliest tick at which a pending metadata fetch needs the member
  int32_t pingIdx, remoteIdx;
  uint64_t evHash;
  uint32_t pad[12];
};
static_assert(sizeof(MS) == 128, "one cache line per member");

struct Dev {
  // ---- configuration ----
  uint32_t N, NS, F, kreq, ping_t, pingTimeout_t, gossip_t, sync_t, syncTimeout_t, md_t, lat, suspMult, repeatMult;
  uint32_t seed_lo, seed_hi, init_mode, flags, n_seeds;
  uint32_t n_dormant;    // COLD_JOIN: members [N - n_dormant, N) start only on swim_join
  uint32_t* start_tick;  // [N] tick of start0 (0: initial COLD_JOIN members; NEVER: PRECONVERGED or not joined yet)
  uint32_t* jseed_n;     // [N] seeds of a joined member (NONE32: the config's seeds)
  uint32_t* jseeds;      // [N][16]
  // per-member FailureDetectorConfig + syncGroup (swim_set_member_config): [N][4] = ping_t, pingTimeout_t,
  // pingReqMembers, sync group; read only when permember (else the swim_config values above)
  uint32_t permember;
  uint32_t* mcfg;
  uint32_t* md_uidx;  // [N] column of a member whose metadata was updated (swim_update_metadata), NONE32 if never
  uint32_t* md_ver;   // [NL][MDU] metadata version each observer stores for those members (the others: 0 if known)
  uint32_t mode, churn;  // SWIM_MODE_RUMOR: gossip layer only, churn rumors per FD period (SEMANTICS.md §9)
  uint64_t* churn_q;     // [churn][2] (origin, payload) of this period's rumors
  uint32_t* ucnt;        // [N] scratch of the user-gossip queue: its entries per member (zero between launches)
  uint32_t seeds[16];
  uint32_t NMETA;  // candidate-list segments per payload: NS / MCH rounded up
  uint32_t LCAP, FCAP, GRCAP, LOGW, SLOTS, MSGCAP, NCHUNK, POOLCAP, EVCAP, DCAP, RCAP, ARENA_ROWS, LOOKBACK, HCAP;
  uint32_t gt_mul;  // floor(2^32 / gossip_t) (2^32 - 1 for 1): rounds_before divides by multiply-high + one correction

  // ---- network / fault history (NetworkEmulator settings per epoch) ----
  uint32_t* dead_tick;  // [N] tick from which the member is dead, NEVER = alive
  // the epoch table and the link count are held in Dev itself: a kernel reads them with scalar loads at the tick's
  // (uniform) epoch, not as a chain of dependent vector loads in every send (xmit_ep)
  uint32_t ep_from[MAX_EPOCHS];   // first tick of each settings epoch (NEVER = unused)
  uint32_t ep_loss[MAX_EPOCHS];
  uint32_t ep_part[MAX_EPOCHS];   // partition active
  uint32_t ep_delay[MAX_EPOCHS];  // default mean delay (its delay index)
  // NetworkLinkSettings.meanDelay (SEMANTICS.md §2): a link value is loss % | delay index << 8; each index has the
  // thresholds on the 32-bit delay draw whose count the draw reaches is the message's delay in ticks past lat
  uint32_t dly_on;      // a delay that reaches a tick was set (the gossip plane queues delayed first receipts)
  uint32_t EMAX;        // largest delay in ticks past lat under swim_config.delay_cap_ms
  uint32_t* dly_thr;    // [DTAB][256]
  uint32_t* dly_len;    // [DTAB]
  unsigned long long* em;  // [2N] SWIM_FLAG_EMULATOR_COUNTERS: every member's emulator (sent, lost); null otherwise
  uint64_t* dq;         // [EMAX + 2][DQCAP] delayed first-receipt candidates (slot << 32 | target) by delivery tick
  uint32_t* dq_n;       // [EMAX + 2]
  uint32_t DQCAP;
  uint32_t* dmark;      // [N] tick + 1 at which the target joined the tick's target list by a delayed receipt
  // delayed SYNC / SYNC_ACK messages (KF_DEFER) between their send and the tick before their delivery: the record and
  // the payload as it was sent (k_sync_defer), put back into the message buffer then (k_sync_redeliver)
  uint32_t DSCAP;
  SyncMsg* ds_msg;      // [DSCAP]
  uint32_t* ds_row;     // [DSCAP][NS]
  uint32_t* ds_used;    // [DSCAP]
  uint32_t* ds_free;    // [DSCAP] free entries (a stack)
  int32_t* ds_top;      // [1]
  uint32_t* ep_group;   // [MAX_EPOCHS][N]
  uint32_t* md_version; // [N]
  uint32_t link_n;      // keys in the link table (0: no per-link setting was ever made)
  uint64_t* link_key;   // [LKCAP] (src << 32 | dst) + 1, 0 = empty slot
  uint32_t* link_hist;  // [LKCAP][LKH][2] (from tick, loss % or LK_NONE), oldest first; [0][0] | LK_TRUNC if older ones dropped

  // ---- per member scalars ----
  // the triage's words, one array each ([N], coalesced loads over every member of a wave)
  uint32_t *nextPing, *nextGossip, *nextSync, *held, *timerMin, *initFlags, *firstGossip;
  // the rest of a member's state, read and written only by its own lane's body: one 128-B record per member (MS),
  // loaded and stored as five 16-B words, so that the busy members a block compacts into its first waves touch one
  // cache line each instead of a line per field
  MS* ms;  // [N]
  uint32_t* sel;  // [N][8]

  uint32_t* rowk;  // [N][NS] key plane: row stride NS = N rounded up to 8 (32-B aligned rows for 16-B loads)
  uint8_t* rowk8;  // [N][NS8] or null: the key plane's 8-bit shadow (key8) that k_sync_diff streams for live-row
                   // payloads on one GPU (1 B + 1 B per record compare instead of 4 B + 4 B); written with every key
  uint32_t NS8;    // its row stride: N rounded up to 16 (16-B aligned rows for 16-B loads)
  uint32_t* rowa;  // [N][NS] aux plane
  uint32_t *fdl, *gl;  // [N][LCAP]

  uint32_t* subs;    // [N][SUBCAP][4]  cnt, kind, target, deadline
  uint32_t* paths;   // [N][PCAP][5] cnt, stage, tick, a, b
  uint32_t PCAP;     // PATHCAP, or PATHCAP_DELAY when link delays are enabled
  uint32_t* fetch;   // [N][FCAP][FREC]
  uint32_t* groups;  // [N][GRCAP][GREC]  pending Mono.whenDelayError groups (SYNC replies, initial sync)

  // ---- gossip round of the current tick ----
  uint32_t *tround, *tcnt, *tspread, *tperiod, *T, *tcontact;  // T, tcontact: [N][F]
  uint32_t* spchg;  // [N] tick of the member's latest gossip round whose spread differs from the round before
  uint64_t* slow;  // [SLOWCAP] (slot << 32 | m * F + s) sends deferred to k_gossip_send_slow
  uint32_t* slow_n;
  uint32_t SLOWCAP;
  uint32_t* cin;    // [N][F] latest cached contact t -> m of (m, T[m][s]); NEVER: none, CIN_SLOW: list overflowed
  uint64_t* rp;  // [RPCAP] (slot << 32 | m * F + s): sends of pairs with a cached contact, for k_gossip_replay
  uint32_t* rp_n;
  uint32_t RPCAP;
  uint32_t* cev;  // [N][F][CEVW] contact events of (m, T[m][s]) cached by k_gossip_contacts when tcontact is set
  uint32_t *log_tick, *log_spread, *log_cnt, *log_tg, *log_pos;  // [N][LOGW], tg [N][LOGW][F], pos [N]

  // ---- holder state (gossip.hip) ----
  // Bit planes indexed by slot id, member-major: HB = held (GossipProtocolImpl.gossips contains the id), kept up to
  // date by every creation, first receipt and sweep; WB = inside the member's spread window as of its latest round
  // (selectGossipsToSend :239-250), rebuilt incrementally at each of its rounds. QW = SLOTS / 64 words per row.
  unsigned long long *HB, *WB;  // [N][QW]
  uint32_t QW;
  // The member's held gossips in receipt order: a ring of (slot | infection period & 1023 << 22) entries. The
  // infection period (rounds before the receipt) never decreases along the ring, so the sweep (:283-308) removes a
  // prefix and the window is a suffix; a round only walks the entries whose status changes.
  uint32_t* rg;                                 // [N][BCAP]
  uint32_t *rhead, *rwin, *rseen, *rtail;       // [N] positions: first held, first in WB, first not yet in WB, end
  uint32_t BCAP;                                // ring entries per member (power of two)
  uint32_t* rwl;                                // [N] round members whose ring needs work this tick
  uint32_t* nrwl;
  uint32_t *rsend, *rwnew;                      // [N] planned sweep end / window start (k_round_plan)
  // groups of 64 slot ids with a slot in use (GU), and with a DEAD membership record (DM: first receipts of those
  // stamp dead_rx); the active groups of a tick in ascending order
  unsigned long long *GU, *DM;                  // [QW]
  uint32_t *agroup, *nagroup;                   // [QW], [2] = count, span (last active group + 1)
  // this tick's (sender, target) pairs by target: a target's senders are processed together, so first receipts
  // are deduplicated without atomics (target-major send)
  uint32_t *tin_cnt, *tin_off, *tin_fill, *tin;  // [N], [N], [N], [N * F] = m * F + s
  uint32_t *tlist, *ntl;                         // targets with senders this tick
  uint32_t* rt0;                                 // [N] a target's ring end before this tick's receipts
  // pairs with a logged contact: only the sender's window gossips received no later than the latest contact can
  // have the target in infectedFrom (replayed); the rest are sent normally. RX row r marks the former for one pair.
  uint32_t* crow;                                // [N * F] RX row of the pair (m, s), RX_ALL: every window gossip
  unsigned long long* RX;                        // [CRCAP][QW]
  uint32_t* rxl;                                 // [CRCAP][3] (m * F + s, first, end ring position)
  uint32_t *nrx, CRCAP;
  uint32_t *cfl, *ncfl;                          // [N * F] pairs with a logged contact this tick (k_contact_cache)
  uint32_t EXPB;  // ticks after its latest creation or receipt by which every holder has swept a gossip (slot_exp)

  // ---- gossip slots ----
  uint64_t* slot_gid;
  uint32_t* slot_subj;
  uint32_t* slot_ctick;  // creation tick of the gossip (origin's spread)
  uint64_t* slot_key;  // inc | status<<32 (status may be DEAD)
  uint32_t* slot_exp;  // tick from which no member holds the gossip any more: the slot is recycled (k_gossip_free)
  uint32_t* slot_used;
  uint16_t* S;  // [N][SLOTS] creation tick (13 low bits) | EVER | SWEPT | REBORN of each member's latest incarnation
                // (replay, hashes); entries older than the slot's gossip (slot_ctick) are stale (s_get)
  uint32_t* free_list;
  int32_t* free_top;
  uint64_t* xd;  // W > 1: (slot << 32) | target, this shard's first receipts of the tick (exchange B)
  uint32_t* xd_n;
  // receipts produced at tick k, consumed in P4 of tick k+1
  uint64_t* rc_raw;  // (member << 32) | slot
  uint32_t* rc_n;
  uint32_t *rc_cnt, *rc_off, *rc_fill;  // [N]
  uint32_t* scan_part;                  // block partial sums of the exclusive scan
  uint32_t* rc_slot;  // [RCAP] sorted by member then gossip id
  uint32_t* rc_ndrop;  // [N] receipts k_gossip_apply did not route (they cannot change the row): counted in P4
  uint32_t* dead_rx;   // [N] tick whose P4 receives a DEAD membership record (set by the delivering sender)
  uint32_t* leaving;   // [N] 1 once the member's leave was requested (its own DEAD record may travel in SYNC data)
  uint64_t* rc_key;   // [RCAP] gossip id sort key
  uint32_t* rc_slot2;  // [RCAP] merge scratch of k_seg_sort (segments above SORT_MAX)
  uint32_t *ap_list, *nap;  // [N], [1] targets with more than APPLY_LANE first receipts this tick (k_gossip_apply_big)
  uint32_t *sg_list, *nsg;  // [N], [1] members with two routed receipts or more this tick (the segments to sort)
  uint64_t* rc_key2;
  uint32_t* fexp;   // [SLOTS] slots recycled at the end of this tick (k_gossip_free)
  uint32_t* nfexp;
  uint64_t* hist;  // [HCAP][HREC] incarnation history: tag, gid, member | n << 32, HKEEP x u32 creation ticks
  uint32_t* hist_n;  // [1] W == 1: entries in use (grow_caps)

  // ---- SYNC messages (double-buffered by tick parity) ----
  SyncMsg* msgs[2];
  uint32_t* nmsg;  // [2]
  uint32_t* arena[2];  // [ARENA_ROWS][NS] key-plane snapshots (a payload carries keys only)
  uint32_t* arena_used;  // [2]
  uint32_t* m_next; // [2][MSGCAP] next message of msgs[b] to the same destination
  uint32_t* m_head; // [2][N] first message of msgs[b] to each destination, NEVER if none (reset by the consumer)
  uint32_t* pending_inc; // [N] host requests for the next tick's P0: bits 2.. updateIncarnation calls, bit 1 leaveCluster
  uint32_t* next_evt; // [N] earliest tick at which a pending path / subscription / fetch needs the member
  uint32_t* mdone;  // finished k_member_tick blocks this tick (the last one runs the end-of-tick resets)
  // speculative batches (W == 1, gossip plane idle): tick + 1 of the member kernel after which the gossip plane was
  // needed (0: none); every later k_sync_diff / k_member_tick launch of the batch returns at once
  uint32_t* halt;
  uint32_t* trk;    // [NL][TRKL] per receiver: subjects its row changed earlier in this tick's P1 (member.hip)
  unsigned long long* tbm;  // [NL][NW] the same subjects as a bitmap (zero between ticks): merged in subject order
  uint32_t NW;       // u64 words per bitmap row ((N + 63) / 64; no SYNC with implicit views: 0)
  uint32_t* ulog;   // [NL][ULOGC][2] per member: (subject, old key) of its row writes this tick after a SYNC send
  uint32_t ULOGC;   // undo-log entries per member (1024 up to 65 536 members, 256 above; ulog_cap <= ULOGC)
  uint32_t* spq;    // [NL][SPQ][8] per member: gossips created this tick, waiting for their slots (member.hip)
  uint32_t* fpend;  // [NL][KP][2] per member: this tick's pending FD-list inserts (subject, final position)
  uint32_t* chunk_meta;                      // [MSGCAP][NMETA][2] (pool offset, count) per MCH subjects
  uint64_t* pool;                            // candidate (subject << 34 | key)
  uint32_t* pool_used;
  // SYNC_ACK resolution (W == 1): per member and tick parity, the subjects whose key its row changed in
  // that tick plus the candidates of the payloads it merged (first TL of them), their count (> TL: overflowed) and the
  // tick they belong to; the messages k_sync_diff streams this tick (the others are resolved)
  uint32_t ackres;
  uint32_t* tlog;     // [2][NL][TL]
  uint32_t* tl_n;     // [2][NL]
  uint32_t* tl_tick;  // [2][NL]
  uint32_t* dlist;    // [MSGCAP] 16-B entries: payloads k_sync_diff streams from the 8-bit plane (k_ack_resolve)
  uint32_t* dlist_w;  // [MSGCAP] 16-B entries: payloads it streams on 4-B keys
  uint32_t* ndlw;
  uint32_t* ndl;
  // W > 1: the sender's write-log prefix (SyncMsg.tln entries) of each message of the inbound list committed this tick,
  // by its index there: copied by k_pack_all for this shard's senders and shipped in exchange A for the peers'
  uint32_t* mlog;     // [MSGCAP][TL]
  // P4 of the members with many routed gossip receipts (W == 1, ticks after a gossip plane): k_member_tick parks a
  // member with at least hv receipts before P4 (its pending live-row payload chain and write-log tail kept here),
  // k_inbox_apply runs its P4 a wave per member, and a second k_member_tick launch runs its P5 and P6
  uint32_t hv;
  uint32_t rr_atomic;  // a round's holder-row changes up to this many go to the rows by global atomics (k_round_apply)
  uint32_t *hv_list, *nhv, *hv_pend, *hv_tlast;  // [NL], [1], [NL], [NL]

  // ---- outputs ----
  uint32_t* ev;  // [EVCAP][8] swim_event
  uint32_t* ev_n;
  unsigned long long* ctr;  // [C_NCTR]
  // counters 0-7 as the member kernel adds them: one row of CSTRIDE per block residue (blockIdx % CSH), summed by the
  // host with ctr. ~1 400 waves adding to one word per tick serialise at its L2 channel (~13 ns each) and held every
  // later memory access of the waves still running (k_member_tick 44 -> 31 us at C3)
  unsigned long long* ctr_sh;  // [CSH][CSTRIDE]
  unsigned long long* wt;   // SWIM_EXP & 512: per-wave timestamps of the latest k_member_tick [waves][16]
  uint32_t* err;            // [8] bits, info...
  const Dev* self;          // device-resident copy of this struct (kernels index it through a pointer)
  uint32_t* hflag;          // host-mapped: [0] gossip slots in use after this tick's member control (W == 1);
                            // [1] the halt tick read back after a speculative batch; with rfill: the previous gossip
                            // plane's largest receipt-ring fill [2], routed receipts [3], replay and slow-path sends
                            // [4], [5], history entries in use [6]
  uint32_t* hsh;            // [8] device copy of what hflag holds (tick_flag writes host memory only on a change):
                            // hsh[0] mirrors hflag[0], hsh[1..5] mirror hflag[2..6]
  uint32_t* rfill;          // [1] W == 1: largest ring fill (rtail - rhead) after this tick's receipts (grow_caps)
  uint32_t* dbg_send;       // debugging aid (SWIM_SEND_LOG=cap): [cap][5] tick, sender, gid lo, gid hi, target
  uint32_t* dbg_send_n;
  uint32_t dbg_send_cap;
  uint32_t exp;  // timing experiments only (SWIM_EXP): 1 = no infectedFrom replay, 2 = no per-target work
  // runtime capacities of the fast structures (<= the compile-time sizes TRK, ULOG, CREQ, CWMAX, CEV, MQ, SORT_MAX);
  // SWIM_CAPS lowers them so that tests drive every exact fallback path (include/swimhip_debug.h)
  uint32_t trk_cap, ulog_cap, creq_cap, cwmax_cap, cev_cap, mq_cap, sort_cap;
  unsigned long long* fb;  // [FB_N] fallback counters, or null (not counted)

  // ---- row sharding (W > 1) ----
  // This shard owns observers [lo, hi): their rows, lists, subscriptions, paths, fetches and groups are stored
  // at local index m - lo. Everything in the gossip plane (slots, S, round logs, hist) is replicated and kept
  // identical on every shard by applying the union of every shard's gossip records each tick.
  uint32_t W, rank, lo, hi, NL, SPR, MW;  // SPR: gossip slots owned per shard; MW: u64 words per chunk mask
  uint32_t NSCAP, RRCAP, RQCAP, RXCAP, CHCAP;
  uint64_t XA_PEER, XB_PEER;  // bytes per peer region of the two exchange buffers
  uint64_t* rdirty;    // [NL][MW] per own observer: the 2048-record chunks of its key plane ever written with a key
                       // that differs from base_row (conservative: never cleared); a payload ships exactly these
  uint64_t* arena_dirty[2];  // [ARENA_ROWS][MW] the sender's rdirty at copy-on-write time
  uint32_t* base_row;  // [NS] baseline key plane: a remote SYNC payload ships only its chunks that differ
  uint8_t* base_row8;  // [NS8] with rowk8: base_row's 8-bit shadow (narrow items of peers' payloads)
  uint32_t* xn;        // [8] 0 new slots, 1 round records, 2 sweeps, 4 inbound msgs (mtmp), 5 rx payloads
  uint32_t* ns_rec;    // [NSCAP][NSW] gossips created on this shard this tick
  uint32_t* rr_rec;    // [RRCAP][RRW] gossip rounds of this shard's members this tick
  SyncMsg* mtmp;       // [MSGCAP] inbound list of the next tick while it is assembled
  uint64_t* rx_mask;   // [RXCAP][MW]
  uint64_t* rx_off;    // [RXCAP] byte offset (in xa_recv) of the first shipped chunk of a received payload
  uint8_t *xa_send, *xa_recv, *xb_send, *xb_recv;  // [W][X*_PEER]
  unsigned long long *xa_scnt, *xa_rcnt, *xb_scnt, *xb_rcnt;  // [W] bytes per peer region
  uint8_t *xi_send, *xi_recv;    // [W][XINL] inline all-to-all blocks
  uint32_t XI;                   // bytes per peer the inline all-to-all moves (XINL; SWIM_CAPS xinl= lowers it)
  unsigned long long* xi_host;   // host-mapped [2W]: send and receive count words of the last exchange
  uint32_t* xdone;  // [2 W] k_pack_all: [0] peer columns done, [1 + q] blocks of column q done (the last writes q's inline block)
  uint32_t inl;     // RCCL transport: exchange A's inline blocks are written by k_pack_all

  // ---- slot sharding (RUMOR mode with W > 1) ----
  // Every shard runs all N members (their scalar state is replicated and evolves identically) but holds only the
  // gossips it owns (slot_mine): their holder table, sends, first receipts and sweeps stay on that shard. The only
  // cross-shard state is each member's gossip count (doSpreadGossip returns early without gossips): the shards'
  // per-tick receipt / sweep deltas are summed with one all-reduce. Kernels see W = 1; XW / xrank name the slot shard.
  uint32_t XW, xrank;
  int32_t* held_delta;  // [N] this tick's change of the member's gossip count from this shard's slots

  // ---- RUMOR mode at scale ----
  // implicit: no table or list is stored; a row is the PRECONVERGED row and list position p of observer m is
  // list_at (the Feistel permutation k_init_lists would have written). Tables and lists never change in RUMOR mode;
  // a gossip-list wrap would need a reshuffle and raises E_LIST.
  // fastp4 (RUMOR, events not recorded): the GOSSIP events of first receipts are hashed (an order-independent sum)
  // and counted where the receipts are applied, into evp_*, and folded into the member at P4 of the next tick: no
  // receipt routing.
  uint32_t implicit, fastp4;
  unsigned long long* evp_hash;  // [N]
  uint32_t* evp_n;               // [N]
};

// PRECONVERGED list w (0: pingMembers, 1: remoteMembers) of observer m: position p holds the other member of rank
// feistel(p) (SEMANTICS.md §3; k_init_lists, and computed on the fly with implicit views)
__host__ __device__ __forceinline__ FeistelPerm list_perm(const Dev& d, uint32_t m, uint32_t w) {
  uint32_t k[4];
  for (uint32_t r = 0; r < 4; ++r) k[r] = philox(m, 16 + 4 * w + r, 0, 0, d.seed_lo ^ SALT_INIT, d.seed_hi).x;
  return make_perm(d.N - 1, k[0], k[1], k[2], k[3]);
}
__host__ __device__ __forceinline__ uint32_t list_at(const FeistelPerm& P, uint32_t m, uint32_t p) {
  const uint32_t j = feistel(P, p);
  return j < m ? j : j + 1;
}
// the PRECONVERGED record every row holds in RUMOR mode (k_init_rows)
constexpr uint64_t PRE_REC = ((uint64_t)ST_ALIVE << 32) | META_BIT;

// the slot shard that owns gossip gid (slot sharding; always this shard otherwise)
__host__ __device__ __forceinline__ bool slot_mine(const Dev& d, uint64_t gid) {
  return d.XW <= 1 || (uint32_t)(mix64(gid ^ 0x510750A4D5ull) % d.XW) == d.xrank;
}

// local index of an observer owned by this shard
__host__ __device__ __forceinline__ size_t lidx(const Dev& d, uint32_t m) { return (size_t)(m - d.lo); }
// first observer of shard r: contiguous ranges floor(r N / W)
__host__ __device__ __forceinline__ uint32_t shard_lo(uint32_t N, uint32_t W, uint32_t r) {
  return (uint32_t)((uint64_t)r * N / W);
}
__host__ __device__ __forceinline__ uint32_t shard_of(uint32_t N, uint32_t W, uint32_t m) {
  uint32_t r = (uint32_t)((uint64_t)m * W / N);
  while (r > 0 && m < shard_lo(N, W, r)) --r;
  while (r + 1 < W && m >= shard_lo(N, W, r + 1)) ++r;
  return r;
}

// optional per-tick timing of the three main kernels (HIP events on the engine's stream)
struct TickEvents {
  void* ev[6];  // hipEvent_t: diff start/stop, member start/stop, gossip-send start/stop
  int all;      // 0: only the diff pair is recorded (each timed event costs ~5 us of stream time)
};

// host-side kernel launchers (one HIP stream)
void launch_init(const Dev& d, void* stream);
// single GPU, per tick k: launch_diff(k) (k > 0), launch_member(k) (+ host flag), then launch_gossip(k) if the flag
// says a gossip slot is in use; launch_diff(k+1) may be queued before launch_gossip(k)
// spec: a launch of a speculative batch (it returns at once once d.halt is set)
void launch_diff(const Dev& d, uint32_t k, void* stream, const TickEvents* prof = nullptr, bool spec = false);
// split: the previous tick ran the gossip plane (routed receipts for P4: k_member_tick parks the members with many,
// k_inbox_apply runs their P4, a second k_member_tick launch their P5 and P6)
void launch_member(const Dev& d, uint32_t k, void* stream, const TickEvents* prof = nullptr, bool spec = false,
                   bool split = false);
void launch_gossip(const Dev& d, uint32_t k, void* stream, const TickEvents* prof = nullptr);
// sharded tick (W > 1): A = SYNC diff + member control + pack exchange A; B = unpack A, gossip sends, pack
// exchange B; C = unpack B, apply receipts, routing, slot recycling. The host runs the exchanges in between and
// skips the gossip half (and exchange B) when no shard has a gossip slot in use.
// spec: a launch of a speculative sharded batch (RCCL, gossip plane idle): every kernel returns at once once d.halt is
// set; k_unpack_a (after exchange A's inline all-to-all) raises it at the first tick whose exchange needs the host (a
// gossip slot in use on some shard, or a region past the inline block)
void launch_tick_a(const Dev& d, uint32_t k, void* stream, const TickEvents* prof = nullptr, bool spec = false);
void launch_tick_b(const Dev& d, uint32_t k, void* stream, const TickEvents* prof, bool gossip, bool spec = false);
void launch_tick_c(const Dev& d, uint32_t k, void* stream, bool gossip);
void launch_inline_out(const Dev& d, const uint8_t* send, uint64_t cap, const unsigned long long* scnt, void* stream);
void launch_inline_in(const Dev& d, uint8_t* recv, uint64_t cap, const unsigned long long* scnt, unsigned long long* rcnt,
                      void* stream, bool spec = false);
void launch_user_gossips(const Dev& d, uint32_t k, const uint64_t* q, uint32_t n, void* stream);
void launch_churn(const Dev& d, uint32_t k, void* stream);
void launch_md_column(const Dev& d, uint32_t m, uint32_t u, void* stream);
void launch_join(const Dev& d, uint32_t m, uint32_t k, const uint32_t* seeds, uint32_t n, void* stream);  // RUMOR mode, at ticks k % ping_t == 0
void launch_hash(const Dev& d, uint64_t* out, uint32_t now, void* stream);
void launch_held_add(const Dev& d, const int32_t* sum, void* stream);
void launch_s_scrub(const Dev& d, uint32_t now, void* stream);  // every SCRUB ticks: stale S entries cleared
void launch_ring_move(const uint32_t* rg, uint32_t* rg2, const uint32_t* rhead, const uint32_t* rtail, uint32_t N,
                      uint32_t B, uint32_t B2, void* stream);  // capacity growth of the receipt rings
void launch_hist_rehash(const uint64_t* h1, uint32_t cap1, uint64_t* h2, uint32_t cap2, void* stream);
void launch_dbg_holders(const Dev& d, uint32_t first, uint32_t n, uint32_t* out, void* stream);  // swim_debug_holders

}  // namespace swim
