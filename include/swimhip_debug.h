/*
 * swimhip_debug.h — test surface of libswimhip (not part of the simulation API; the CPU oracle has no such paths).
 *
 * The engine keeps its hot per-tick state in fixed-capacity fast structures and falls back to an exact slow path
 * when one is full. Those fallbacks must give the same bits as the fast path, so tests force them:
 * the environment variable SWIM_CAPS, read by swim_create, lowers the capacities, e.g.
 *   SWIM_CAPS="trk=1,ulog=2,creq=1,cwmax=1,cev=1,mq=1,sort=2"
 *   trk    subjects tracked per receiver and tick in a sorted list for later SYNC payloads (more: the written-subject
 *          bitmap is walked in subject order),
 *          MembershipProtocolImpl.syncMembership (:456-467) with several payloads in one tick
 *   ulog   row writes logged after a SYNC send of the same tick (more: the lane copies its open snapshots),
 *          prepareSyncDataMsg (:446-454) snapshot semantics
 *   creq   copy-on-write snapshots open per member and tick (more: the lane copies them)
 *   cwmax  deferred snapshots per k_member_tick block (more: the lane copies the row)
 *   cev    cached contact events per (sender, target) pair (more: k_gossip_send_slow scans both round logs),
 *          GossipProtocolImpl.selectGossipsToSend isInfected (:239-250)
 *   mq     inbound SYNC messages of one tick sorted in registers (more: selection by list walks), onMessage (:320-331)
 *   sort   first receipts of one member and tick sorted in LDS at once (more: sorted runs merged), P4 order
 *   rx     contact pairs per tick whose replay is limited to the gossips received before the contact (more: the
 *          whole window is replayed), GossipProtocolImpl isInfected (:247)
 *   xinl   bytes per peer of the RCCL inline all-to-all of a sharded tick (more: a send/recv group; speculative
 *          sharded batches halt on the overflow flag), every rank the same value
 *   rp     replay / slow-path gossip sends per tick (grow_caps enlarges the lists; SWIM_DELIV_CAP sets the routed
 *          receipts per tick the same way)
 * With SWIM_CAPS (or SWIM_FALLBACKS=1) set, the handle counts how often each fallback fired.
 */
#ifndef SWIMHIP_DEBUG_H
#define SWIMHIP_DEBUG_H

#include <stddef.h>
#include <stdint.h>

#include "swimhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* indices into swim_debug_fallbacks' output */
#define SWIM_FB_TRK_WALK 0u    /* later SYNC payloads merged with the written-subject bitmap (trk) */
#define SWIM_FB_ULOG 1u        /* snapshot copies forced by a full undo log (ulog) */
#define SWIM_FB_CREQ 2u        /* snapshot copies forced by too many open snapshots (creq) */
#define SWIM_FB_CWMAX 3u       /* lane row copies, block list full (cwmax) */
#define SWIM_FB_CEV_SLOW 4u    /* gossip sends replayed from a full log scan (cev) */
#define SWIM_FB_REPLAY 5u      /* gossip sends replayed from the contact cache (pairs with a logged contact) */
#define SWIM_FB_MQ 6u          /* receivers with more than mq inbound SYNC messages in one tick */
#define SWIM_FB_SORT_MERGE 7u  /* receipt segments sorted as runs and merged (sort) */
#define SWIM_FB_RX_ALL 8u      /* contact pairs that replayed their whole window (rx: rows of window gossips received
                                  before the contact, per tick) */
#define SWIM_FB_COUNT 9u

/* counts of the fallbacks fired since create, n <= 16 entries (summed over shards); SWIM_EUNSUPPORTED when the
 * handle was created without SWIM_CAPS / SWIM_FALLBACKS */
int swim_debug_fallbacks(swim_handle* h, uint64_t* out, size_t n);

/* the current sizes of the structures that grow between ticks (api.hip grow_caps), n <= 8 entries:
 * gossip slots per shard, receipt-ring entries per member, routed receipts per tick, replay / slow-path sends per
 * tick, incarnation-history entries, and how many growth steps ran. One GPU (a sharded handle: SWIM_EUNSUPPORTED). */
#define SWIM_CAP_SLOTS 0u
#define SWIM_CAP_RING 1u
#define SWIM_CAP_RECEIPTS 2u
#define SWIM_CAP_REPLAY 3u
#define SWIM_CAP_HISTORY 4u
#define SWIM_CAP_GROWTHS 5u
int swim_debug_caps(swim_handle* h, uint64_t* out, size_t n);

/* the holder bookkeeping of members [first, first + n), out[5 * i + j] for member first + i: j = 0 its gossip count
 * (GossipProtocolImpl.gossips.size(), what doSpreadGossip's early return reads, :141-146), 1 / 2 the receipt-ring
 * positions of its first held entry and of the ring end (absolute: every creation and first receipt appends one entry,
 * every sweep advances the first), 3 the popcount of its held-bit row, 4 first receipts of the last tick whose GOSSIP
 * events the next P4 folds (RUMOR mode without recorded events; 0 otherwise). One GPU or one shard of a slot-sharded
 * RUMOR cluster (a row-sharded or multi-device handle: SWIM_EUNSUPPORTED). */
int swim_debug_holders(swim_handle* h, uint32_t first, uint32_t n, uint32_t* out);

/* sets member m's own record in its own table to incarnation inc, status unchanged, between steps (one GPU): the
 * boundary test of the 30-bit incarnation field of the key plane (SEMANTICS.md §8). inc >= 2^30: SWIM_ECAPACITY.
 * The write bypasses the row's copy-on-write and write-log bookkeeping, so it is refused (SWIM_EINVAL) while a SYNC /
 * SYNC_ACK that m sent in the last tick still carries m's live row as its payload. */
int swim_debug_set_incarnation(swim_handle* h, uint32_t m, uint32_t inc);

#ifdef __cplusplus
}
#endif
#endif
