// member.hip — k_member_tick: one thread per simulated member runs phases P1..P6 of SEMANTICS.md §4.
//
// This kernel is the control plane of the protocol stack of every member: FailureDetectorImpl, MembershipProtocolImpl,
// MetadataStoreImpl and the selection half of GossipProtocolImpl. Its work per member per tick is O(1) in the
// common case. The O(N) work runs elsewhere: the SYNC-payload diff (k_sync_diff) and the gossip data plane
// (gossip.hip). Remote hops of stateless request handlers (onPing, onPingReq, onTransitPingAck,
// onMetadataRequest) are evaluated at the issuer, at the hop's own tick and against that tick's network
// settings. The payload they would carry is only the correlation id, so no message is materialised.
#include "dev_util.h"

namespace swim {

enum Reason : uint32_t { R_FD = 0, R_GOSSIP = 1, R_SYNC = 2, R_INITIAL = 3, R_TIMEOUT = 4 };
enum : uint32_t { INIT_ACTIVE = 1, INIT_RECEIVED = 2 };
enum : uint32_t { GF_USED = 1, GF_ERROR = 2, GF_SEALED = 4 };
// path stages: 1..3 = pending hop at `tick`, 9 = ack arrives at `tick`
enum : uint32_t { P_DIRECT = 0x10, P_REQ = 0x20, P_ARRIVE = 9 };

struct ML {
  const Dev* d;
  uint32_t m, k, N;
  uint32_t tsize, fdLen, gLen, fdPeriod, gPeriod, gCounter, nextPing, nextGossip, nextSync, cidCnt, syncSeq, evSeq,
      held, timerMin, initFlags, initDeadline, initCidBase, initN, nsub, npath, nfetch;
  int ep;          // NetworkEmulator settings epoch of tick k (epoch_at, looked up once)
  uint32_t fnext;  // earliest tick at which a pending fetch needs the member (hop, arrival or timeout); NEVER: none
  int32_t pingIdx, remoteIdx;
  uint64_t evHash;
  uint32_t *rk, *ra;  // this observer's row: key plane and aux plane (swim_common.h)
  uint64_t* rd;       // W > 1: its dirty-chunk mask against base_row (Dev::rdirty), else null
  uint32_t *fdl, *gl, *subs, *paths, *fetch, *groups;
  uint32_t c[8];  // this tick's op counters (one member, one tick: u32; summed per wave in u64)
  uint32_t pend;  // this tick's SYNC messages that carry the live row: a chain through SyncMsg.pad (NEVER = none)
  uint32_t tround;
  // subjects whose key changed in this tick's P1 (several payloads only): the first TRKL listed, all of them in the
  // bitmap tb (one bit per subject); ntrk counts them
  uint32_t* trk;
  uint32_t ntrk;
  bool trk_on;
  // deferred copy-on-write (cow): open snapshots of this member (indices into the block's list cw) and its undo log
  uint4* cw;       // block list (LDS): member, arena row, first log entry, log length at the end of the body
  uint32_t* cw_n;  // LDS counter of cw
  uint32_t* ulog;  // this member's log: (subject, key before the write) per row write while a snapshot is open
  uint32_t ncreq, nlog;  // open snapshots (their cw entries carry this member's id), logged writes
  uint32_t* spq;  // gossips created this tick that wait for their slots (flush_spreads): [SPQ][8] gid, subj, key
  uint32_t nsp;
  // ArrayList.add(index) inserts of this tick not applied to fdl yet (fd_flush), sorted by their final position;
  // fdLen counts them
  uint32_t* fpend;
  uint32_t npend;
  // SYNC_ACK resolution (d.ackres): this tick's write log (Dev::tlog), its length (> TL: overflowed) and last entry;
  // the group of the SYNC merged just now whose SYNC_ACK may be resolved (-1: none)
  uint32_t* tl;
  uint32_t ntl, tlast;
  // the FD list entry the P6 ping takes and its dead_tick, loaded with the member state when the ping is due and the
  // cursor needs no reshuffle (compared only at the ping, so nothing waits for them before); pre = NEVER when not
  // loaded or once the list changes in this tick
  uint32_t pre, pre_dt;
  // the last SYNC / SYNC_ACK this lane linked into its receiver's inbound list (W == 1): the list-link exchange's old
  // head, written to m_next with the pins at the next send or at the end of the body (link_flush), so that the
  // exchange's round trip overlaps the lane's next loads instead of holding them (NEVER: none pending)
  uint32_t lk_i, lk_o;
  // the earliest pending path tick and subscription deadline, kept in registers once P2 and P5 have walked the lists
  // (NEVER: none), so the next-event minimum at the end of the body needs no loads of entries just stored; ev_ok says
  // whether they are known (not in a resumed launch, whose P2 ran in the launch before)
  uint32_t pmin, smin;
  bool ev_ok;
  int rgrp;
  bool spec;  // a launch of a one-GPU speculative batch: a member that takes a gossip slot raises d.halt (k_member_tick)
};

// a subject whose key this member's row changed in this tick, or a candidate of a payload it merged (k_ack_resolve)
__device__ __forceinline__ void tl_add(ML& L, uint32_t s) {
  if (L.ntl && L.tlast == s) return;  // merge_record's candidate, then its row_put
  if (L.ntl < TL) L.tl[L.ntl] = s;
  if (L.ntl <= TL) L.ntl++;
  L.tlast = s;
}

// the selector counters live in memory (Dev::sel), not in the member's registers: draws are rare next to the
// registers every member-kernel wave would hold for them
__device__ __forceinline__ uint32_t draw_at(const ML& L, uint32_t stream, uint32_t c) {
  return philox(L.m, stream, c, 0, L.d->seed_lo ^ SALT_SEL, L.d->seed_hi).x;
}
__device__ __forceinline__ uint32_t draw(ML& L, uint32_t stream) {
  uint32_t* p = L.d->sel + (size_t)L.m * 8 + stream;
  const uint32_t c = *p;
  *p = c + 1u;
  return draw_at(L, stream, c);
}

// Collections.shuffle: for i = size..2: swap(i-1, nextInt(i))
__device__ __forceinline__ void shuffle_list(ML& L, uint32_t* v, uint32_t n, uint32_t stream) {
  uint32_t* p = L.d->sel + (size_t)L.m * 8 + stream;
  uint32_t c = *p;
  if (n > 1) *p = c + (n - 1u);
  for (uint32_t i = n; i > 1; --i) {
    uint32_t j = next_int(draw_at(L, stream, c++), i);
    uint32_t t = v[i - 1];
    v[i - 1] = v[j];
    v[j] = t;
  }
}

// copy-on-write of the live row for SYNC payloads sent earlier in this tick. The payloads take an
// arena row; the copy itself is deferred to the end of k_member_tick, where the member's whole block copies the row
// (coalesced) and then undoes, newest first, the writes the member logged after this point (row_put). One lane
// copying N words would hold the whole kernel (~3 ms per tick at 100k members when a SYNC sender also merges a
// gossip in the same tick). Past CREQ open snapshots, ULOG logged writes or CWMAX snapshots per block, the copy is
// made here, by this lane (cow_now).
__device__ __forceinline__ void copy_row_to(ML& L, uint32_t r) {
  const Dev& d = *L.d;
  const uint32_t b = L.k & 1;
  const uint4* src4 = (const uint4*)L.rk;  // keys only, with the zero padding k_sync_diff reads up to NS
  uint4* dst4 = (uint4*)(d.arena[b] + (size_t)r * d.NS);
#pragma unroll 16
  for (uint32_t s = 0; s < d.NS / 4; ++s) dst4[s] = src4[s];
  if (L.rd)
    for (uint32_t w = 0; w < d.MW; ++w) d.arena_dirty[b][(size_t)r * d.MW + w] = L.rd[w];
}

// the open snapshots, now: live row, then the logged writes since each one opened undone newest first
__device__ __forceinline__ void cow_now(ML& L) {
  const Dev& d = *L.d;
  const uint32_t b = L.k & 1;
  const uint32_t n = min(*L.cw_n, d.cwmax_cap);
  for (uint32_t q = 0; q < n; ++q) {
    uint4& e = L.cw[q];
    if (e.x != L.m) continue;  // another member's (entries are NEVER until written)
    copy_row_to(L, e.y);
    uint32_t* dst = d.arena[b] + (size_t)e.y * d.NS;
    for (uint32_t j = L.nlog; j-- > e.z;) dst[L.ulog[2 * j]] = L.ulog[2 * j + 1];
    e.x = NEVER;  // done: the block epilogue skips it
  }
  L.ncreq = 0;
  L.nlog = 0;
}

__device__ __forceinline__ void cow(ML& L) {
  const Dev& d = *L.d;
  uint32_t b = L.k & 1;
  uint32_t r = atomicAdd(&d.arena_used[b], 1u);
  if (r >= d.ARENA_ROWS) {
    set_err(d, E_ARENA);
    L.pend = NEVER;
    return;
  }
  for (uint32_t i = L.pend; i != NEVER; i = d.msgs[b][i].pad) d.msgs[b][i].payload = r;
  L.pend = NEVER;
  if (L.ncreq == d.creq_cap) {  // rare: many send-then-write rounds in one tick
    fb_add(d, FB_CREQ);
    cow_now(L);
  }
  const uint32_t idx = atomicAdd(L.cw_n, 1u);  // LDS
  if (idx >= d.cwmax_cap) {  // the block's list is full: this snapshot now, by this lane
    fb_add(d, FB_CWMAX);
    copy_row_to(L, r);
    return;
  }
  L.cw[idx] = make_uint4(L.m, r, L.nlog, 0u);
  L.ncreq++;
}

__device__ __forceinline__ uint64_t row_ld(const ML& L, uint32_t s) { return rec_join(L.rk[s], L.ra[s]); }
__device__ __forceinline__ uint32_t row_status(const ML& L, uint32_t s) { return L.rk[s] & 3u; }

// old: the key the row holds for s now (callers that loaded it already pass it: no load after this lane's stores)
__device__ __forceinline__ void row_put(ML& L, uint32_t s, uint64_t v, uint32_t old) {
  const uint32_t k = key32(v);
  if (rec_inc(v) >= INC_LIMIT) set_err(*L.d, E_INC);
  if (L.pend != NEVER && old != k) cow(L);
  if (L.ncreq && old != k) {  // an open snapshot: log the key this write replaces
    if (L.nlog == L.d->ulog_cap) {
      fb_add(*L.d, FB_ULOG);
      cow_now(L);
    } else {
      L.ulog[2 * L.nlog] = s;
      L.ulog[2 * L.nlog + 1] = old;
      L.nlog++;
    }
  }
  if (L.trk_on && old != k) {  // merge_payload re-checks it against the later payloads
    unsigned long long* tw = L.d->tbm + lidx(*L.d, L.m) * L.d->NW + (s >> 6);
    const unsigned long long bit = 1ull << (s & 63u), old = *tw;
    if (!(old & bit)) {
      *tw = old | bit;
      if (L.ntrk < TRKL) L.trk[L.ntrk] = s;
      L.ntrk++;
    }
  }
  if (L.d->ackres && old != k) tl_add(L, s);
  L.rk[s] = k;
  if (L.d->rowk8) L.d->rowk8[lidx(*L.d, L.m) * L.d->NS8 + s] = key8(k);
  if (L.rd && k != L.d->base_row[s]) L.rd[(s / CH) >> 6] |= 1ull << ((s / CH) & 63);
  L.ra[s] = aux32(v);
}
__device__ __forceinline__ void row_put(ML& L, uint32_t s, uint64_t v) { row_put(L, s, v, L.rk[s]); }

__device__ __forceinline__ void link_flush(ML& L) {
  if (L.lk_i == NEVER) return;
  const Dev& d = *L.d;
  const uint32_t b = L.k & 1, i = L.lk_i, old = L.lk_o;
  d.m_next[(size_t)b * d.MSGCAP + i] = old;
  if (old != NEVER) {  // a receiver with several payloads this tick: both pinned (pin_msg)
    pin_msg(d, b, i);
    pin_msg(d, b, old);
  }
  L.lk_i = NEVER;
}

// prepareSyncDataMsg (MembershipProtocolImpl.java:446-454) + transport.send; false if the send failed
// res: a SYNC_ACK sent in the tick its SYNC was merged (k_ack_resolve may derive its diff from the write logs)
__device__ __forceinline__ bool send_sync(ML& L, uint32_t kind, uint32_t dst, uint32_t ciss, uint32_t ccnt,
                                          bool res = false) {
  const Dev& d = *L.d;
  uint32_t seq = L.syncSeq++;
  L.c[C_M]++;
  const int e = xmit_ep(d, L.ep, kind, L.m, dst, L.k, L.m, seq);
  if (e < 0) {
    L.c[C_LOST]++;
    return false;
  }
  uint32_t b = L.k & 1;
  // one atomic per wave for the lanes sending here together: ~1 300 SYNC / SYNC_ACK sends per tick at C3 on one
  // counter would otherwise serialise at its L2 channel (~90 per µs)
  uint32_t i = wave_append(&d.nmsg[b]);
  if (i >= d.MSGCAP) {
    set_err(d, E_MSGS);
    return true;
  }
  SyncMsg mm;
  mm.src = L.m;
  mm.dst = dst;
  // a delayed one is stored at the end of the tick (k_sync_defer)
  mm.kind = kind | (e > 0 ? KF_DEFER : (res && d.ackres && L.ntl <= TL ? KF_RES : 0u));
  mm.seq = seq;
  mm.cid_iss = ciss;
  mm.cid_cnt = ccnt;
  mm.payload = NEVER;
  mm.psize = L.tsize;
  mm.ncand = 0;
  mm.pad = L.pend;  // chained so that a later row write can redirect the payload to a snapshot (cow)
  // every field but `pin`: pin_msg of another sender may set that one by atomics in this same tick (from another
  // XCD, whose L2 is not this one's), so this sender never stores it. It is NEVER already: the receiver of the
  // slot's previous message reset it after use (P1 below), or the buffer's initialisation did. Without a store to it
  // no release fence is needed (one per send cost an L2 write-back and invalidate: ~14 us per tick at C3).
  SyncMsg* q = &d.msgs[b][i];
  q->src = mm.src, q->dst = mm.dst, q->kind = mm.kind, q->seq = mm.seq, q->cid_iss = mm.cid_iss;
  q->cid_cnt = mm.cid_cnt, q->payload = mm.payload, q->psize = mm.psize, q->ncand = mm.ncand, q->pad = mm.pad;
  q->due = L.k + d.lat + (uint32_t)e;
  q->tln = L.ntl;
  L.pend = i;
  if (e > 0) return true;  // not linked to the receiver's inbound list before its delivery tick
  // the receiver's inbound list for the next tick (sharded handles build it when the exchange commits the list);
  // a receiver with several payloads gets them pinned (pin_msg)
  if (d.W == 1) {
    link_flush(L);
    L.lk_o = atomicExch(&d.m_head[(size_t)b * d.N + dst], i);
    L.lk_i = i;
  }
  return true;
}

// ArrayList.remove(Object) on one lane: find subj, then shift the tail down by one in blocks of 8 (the loads of a
// block are independent of the stores before it, so they are in flight together instead of one load per element)
__device__ __forceinline__ bool list_remove(uint32_t* a, uint32_t len, uint32_t subj) {
  uint32_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint32_t v[8];
#pragma unroll
    for (uint32_t t = 0; t < 8; ++t) v[t] = a[i + t];
    bool hit = false;
#pragma unroll
    for (uint32_t t = 0; t < 8; ++t) hit |= v[t] == subj;
    if (hit) break;
  }
  for (; i < len && a[i] != subj; ++i) {
  }
  if (i >= len) return false;
  uint32_t j = i + 1;
  for (; j + 8 <= len; j += 8) {
    uint32_t v[8];
#pragma unroll
    for (uint32_t t = 0; t < 8; ++t) v[t] = a[j + t];
#pragma unroll
    for (uint32_t t = 0; t < 8; ++t) a[j + t - 1] = v[t];
  }
  for (; j < len; ++j) a[j - 1] = a[j];
  return true;
}

// The FD list with its pending inserts applied: one pass over the part of the list at or above the first insert,
// instead of one tail shift per ArrayList.add(index, e). Entry p (ascending final positions f_0 < ... < f_{k-1}) ends
// at f_p; the originals between f_p and f_{p+1} move up by p + 1, segment by segment from the top (8 loads in flight,
// then 8 stores), so no original is overwritten before it is read.
__device__ __noinline__ void fd_flush(uint32_t* a, const uint32_t* pend, uint32_t k, uint32_t len) {
  for (int p = (int)k - 1; p >= 0; --p) {
    const uint32_t fp = pend[2 * p + 1], fnext = (uint32_t)p + 1 < k ? pend[2 * p + 3] : len;
    const uint32_t s = (uint32_t)p + 1, lo = fp + 1 - s, hi = fnext - s;  // originals [lo, hi) move to [lo + s, hi + s)
    uint32_t j = hi;
    for (; j >= lo + 8; j -= 8) {
      uint32_t v[8];
#pragma unroll
      for (uint32_t t = 0; t < 8; ++t) v[t] = a[j - 8 + t];
#pragma unroll
      for (uint32_t t = 0; t < 8; ++t) a[j - 8 + t + s] = v[t];
    }
    for (; j > lo; --j) a[j - 1 + s] = a[j - 1];
    a[fp] = pend[2 * p];
  }
}
__device__ __forceinline__ void fd_ready(ML& L) {
  if (L.npend) {
    fd_flush(L.fdl, L.fpend, L.npend, L.fdLen);
    L.npend = 0;
  }
}

__device__ __forceinline__ void on_member_event(ML& L, uint32_t type, uint32_t subj) {
  const Dev& d = *L.d;
  L.pre = NEVER;
  if (type == 1) {  // REMOVED: FailureDetectorImpl.onMemberEvent (:321-325), GossipProtocolImpl (:187-189)
    fd_ready(L);
    if (list_remove(L.fdl, L.fdLen, subj)) L.fdLen--;
    if (list_remove(L.gl, L.gLen, subj)) L.gLen--;
  } else if (type == 0) {  // ADDED: insert at nextInt(size) (:326-331); append (:190-192)
    if (L.fdLen >= d.LCAP || L.gLen >= d.LCAP) {
      set_err(d, E_LIST);
      return;
    }
    const uint32_t idx = L.fdLen > 0 ? next_int(draw(L, S_FD_INSERT), L.fdLen) : 0;
    if (L.npend == KP) fd_ready(L);
    // ArrayList.add(index, e), deferred: the pending inserts at or above idx move up by one, the new one takes idx
    uint32_t j = L.npend;
    for (; j > 0 && L.fpend[2 * j - 1] >= idx; --j) {
      L.fpend[2 * j] = L.fpend[2 * j - 2];
      L.fpend[2 * j + 1] = L.fpend[2 * j - 1] + 1u;
    }
    L.fpend[2 * j] = subj;
    L.fpend[2 * j + 1] = idx;
    L.npend++;
    L.fdLen++;
    L.gl[L.gLen++] = subj;
  }
}

// pad: the gossip counter of a GOSSIP event (its id is (subject, pad)), 0 otherwise. RUMOR mode hashes the events
// as a sum (SEMANTICS.md §9), so slot shards that each emit a member's events for their own gossips add up.
__device__ __forceinline__ void emit_event(ML& L, uint32_t type, uint32_t subj, uint32_t oldm, uint32_t newm,
                                           uint32_t pad = 0) {
  const Dev& d = *L.d;
  uint32_t seq = L.evSeq++;
  if (d.mode == 1u) {  // SWIM_MODE_RUMOR
    L.evHash += hpair(hpair(((uint64_t)L.k << 32) | ((uint64_t)type << 30) | subj, ((uint64_t)oldm << 32) | newm), pad);
  } else {
    L.evHash = hpair(L.evHash, ((uint64_t)L.k << 32) | ((uint64_t)type << 30) | subj);
    L.evHash = hpair(L.evHash, ((uint64_t)oldm << 32) | newm);
  }
  L.c[C_E]++;
  if (d.flags & 1u) {
    uint32_t i = atomicAdd(d.ev_n, 1u);
    if (i < d.EVCAP) {
      uint32_t* e = d.ev + (size_t)i * 8;
      e[0] = L.k;
      e[1] = L.m;
      e[2] = seq;
      e[3] = type;
      e[4] = subj;
      e[5] = oldm;
      e[6] = newm;
      e[7] = pad;
    } else {
      set_err(d, E_EVENTS);
    }
  }
  on_member_event(L, type, subj);
}

// createAndPutGossip (GossipProtocolImpl.java:163-169): gossip slot g becomes a new gossip held by member m since tick
// k (slot_create: slot tables and the creator's holder state, ring position pos); with row shards it is replicated on
// the other shards from exchange A
__device__ __forceinline__ void slot_init(const Dev& d, uint32_t g, uint32_t m, uint32_t k, uint64_t gid, uint32_t subj,
                                          uint64_t key, uint32_t pos) {
  slot_create(d, g, m, k, gid, subj, key, pos);
  if (d.W > 1) {
    uint32_t i = atomicAdd(&d.xn[0], 1u);
    if (i >= d.NSCAP) {
      set_err(d, E_XCAP);
      return;
    }
    uint32_t* r = d.ns_rec + (size_t)i * NSW;
    r[0] = g;
    r[1] = (uint32_t)gid;
    r[2] = (uint32_t)(gid >> 32);
    r[3] = subj;
    r[4] = k;
    r[5] = (uint32_t)key;
    r[6] = (uint32_t)(key >> 32);
    r[7] = m;
  }
}

// the member's queued gossips of this tick get their slots with one atomic on the free stack: a member that re-spreads
// hundreds of SYNC records in one tick (C2) would otherwise wait for one round trip on that hot word per gossip
__device__ __forceinline__ void flush_spreads(ML& L) {
  const uint32_t n = L.nsp;
  if (n == 0) return;
  L.nsp = 0;
  const Dev& d = *L.d;
  if (L.spec) *(volatile uint32_t*)d.halt = L.k + 1u;  // a slot in use: the batch stops after this tick
  const int base = atomicSub(d.free_top, (int)n) - (int)n;
  uint32_t rt = d.rtail[L.m];  // only this lane appends to the member's ring in this kernel
  for (uint32_t i = 0; i < n; ++i) {
    const int pos = base + (int)i;
    if (pos < 0) {
      set_err(d, E_SLOTS);
      continue;
    }
    const uint4 e0 = *(const uint4*)(L.spq + 8 * i), e1 = *(const uint4*)(L.spq + 8 * i + 4);
    slot_init(d, d.free_list[pos], L.m, L.k, ((uint64_t)e0.y << 32) | e0.x, e0.z, ((uint64_t)e1.x << 32) | e0.w, rt++);
    L.c[C_GCREATED]++;
  }
  d.rtail[L.m] = rt;
}

// GossipProtocolImpl.spread -> createAndPutGossip (:124-128,163-169): a membership gossip held by this member; its
// slot is taken at the end of the member's tick (flush_spreads: slot ids are not observable)
__device__ __forceinline__ void spread(ML& L, uint32_t subj, uint32_t st, uint32_t inc) {
  uint64_t gid = ((uint64_t)L.m << 32) | L.gCounter++;
  if (slot_mine(*L.d, gid)) {  // slot sharding: only the owning shard stores it; every shard counts it as held
    if (L.nsp == SPQ) flush_spreads(L);
    const uint64_t key = rec_key(st, inc);
    *(uint4*)(L.spq + 8 * L.nsp) = make_uint4((uint32_t)gid, (uint32_t)(gid >> 32), subj, (uint32_t)key);
    *(uint4*)(L.spq + 8 * L.nsp + 4) = make_uint4((uint32_t)(key >> 32), 0u, 0u, 0u);
    L.nsp++;
  }
  L.held++;
}

// Cluster.spreadGossip (ClusterImpl.java:208-211) queued by swim_spread_gossip: user gossips of this shard's live
// members, in call order, at P0 of tick k (before the member kernel loads gCounter / held). Only the order of one
// member's calls is observable (its gossip counters follow them, GossipProtocolImpl.generateGossipId :207-209), so
// the queue runs one thread per entry in three passes: count the entries per member, create each gossip with
// counter gCounter[m] + (its rank among the member's entries), then advance the member's counter and gossip count
// once. Slot ids are not observable; a wave takes its slots with one atomic on the free stack.
__device__ __forceinline__ bool ug_live(const Dev& d, uint32_t m, uint32_t k) {
  return m >= d.lo && m < d.hi && !dead_at(d, m, k);
}
__global__ void k_ug_count(Dev d, uint32_t k, const uint64_t* q, uint32_t n, uint32_t* ucnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t m = (uint32_t)q[2 * i];
  if (ug_live(d, m, k)) atomicAdd(&ucnt[m], 1u);
}
// rank of entry i among the queue entries of member m before it (members with one entry: 0, no scan), and among
// those whose gossip this (slot) shard stores (its ring position); gc0 = the member's gossip counter before the queue
struct UgRank {
  uint32_t all, mine;
};
__device__ __forceinline__ UgRank ug_rank(const Dev& d, const uint64_t* q, uint32_t i, uint32_t m, uint32_t cnt,
                                          uint32_t gc0) {
  UgRank r{0, 0};
  if (cnt <= 1) return r;
  for (uint32_t j = 0; j < i; ++j)
    if ((uint32_t)q[2 * j] == m) r.mine += slot_mine(d, ((uint64_t)m << 32) | (gc0 + r.all++)) ? 1u : 0u;
  return r;
}
__global__ void __launch_bounds__(256) k_ug_create(Dev d, uint32_t k, const uint64_t* q, uint32_t n, const uint32_t* ucnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t m = i < n ? (uint32_t)q[2 * i] : 0u;
  bool mine = false;
  uint64_t gid = 0;
  UgRank rk{0, 0};
  if (i < n && ug_live(d, m, k)) {
    rk = ug_rank(d, q, i, m, ucnt[m], d.ms[m].gCounter);
    gid = ((uint64_t)m << 32) | (d.ms[m].gCounter + rk.all);
    mine = slot_mine(d, gid);  // slot sharding: only the owning shard stores it; every shard counts it as held
  }
  const uint64_t bm = __ballot(mine);
  const uint32_t lane = __lane_id(), nb = (uint32_t)__popcll(bm);
  int top = 0;
  if (lane == 0 && nb) top = atomicSub(d.free_top, (int)nb);
  top = __shfl(top, 0);
  if (mine) {
    const int pos = top - (int)nb + (int)__popcll(bm & ((1ull << lane) - 1ull));
    if (pos < 0)
      set_err(d, E_SLOTS);
    else  // ring position: the member's stored gossips of this queue take consecutive positions in call order
      slot_init(d, d.free_list[pos], m, k, gid, USER_SUBJ, q[2 * i + 1], d.rtail[m] + rk.mine);
  }
  if (lane == 0 && nb) atomicAdd(&d.ctr[C_GCREATED], (unsigned long long)nb);
}
__global__ void k_ug_finish(Dev d, uint32_t k, const uint64_t* q, uint32_t n, uint32_t* ucnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t m = (uint32_t)q[2 * i];
  if (!ug_live(d, m, k)) return;
  const uint32_t c = ucnt[m], gc0 = d.ms[m].gCounter;
  if (c > 1 && ug_rank(d, q, i, m, c, gc0).all != 0) return;  // the member's first entry advances it once
  uint32_t mine = 0;  // ring entries this shard appended for the member
  for (uint32_t r = 0; r < c; ++r) mine += slot_mine(d, ((uint64_t)m << 32) | (gc0 + r)) ? 1u : 0u;
  d.ms[m].gCounter = gc0 + c;
  d.held[m] += c;
  d.rtail[m] += mine;
  ucnt[m] = 0;
}
void launch_ug(const Dev& d, uint32_t k, const uint64_t* q, uint32_t n, hipStream_t st) {
  if (n == 0) return;
  const dim3 g((n + 255) / 256), b(256);
  hipLaunchKernelGGL(k_ug_count, g, b, 0, st, d, k, q, n, d.ucnt);
  hipLaunchKernelGGL(k_ug_create, g, b, 0, st, d, k, q, n, d.ucnt);
  hipLaunchKernelGGL(k_ug_finish, g, b, 0, st, d, k, q, n, d.ucnt);
}

// RUMOR-mode churn of period p = k / ping_t (SEMANTICS.md §9): event i picks the churned member v and an origin
// o != v; the rumor (p << 32 | v) is then spread by o through k_user_gossips, in event order
__global__ void k_churn(Dev d, uint32_t k) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.churn) return;
  const uint32_t p = k / d.ping_t;
  const u32x4 r = philox(p, i, 0, 0, d.seed_lo ^ SALT_CHURN, d.seed_hi);
  const uint32_t v = next_int(r.x, d.N);
  uint32_t o = next_int(r.y, d.N - 1);
  o += o >= v ? 1u : 0u;
  d.churn_q[2 * i] = o;
  d.churn_q[2 * i + 1] = ((uint64_t)p << 32) | v;
}

void launch_churn(const Dev& d, uint32_t k, void* stream) {
  hipLaunchKernelGGL(k_churn, dim3((d.churn + 255) / 256), dim3(256), 0, (hipStream_t)stream, d, k);
  launch_ug(d, k, d.churn_q, d.churn, (hipStream_t)stream);
}

void launch_user_gossips(const Dev& d, uint32_t k, const uint64_t* q, uint32_t n, void* stream) {
  launch_ug(d, k, q, n, (hipStream_t)stream);
}

// the metadata version this observer stores for subj (MetadataStoreImpl.membersMetadata), NONE32 if unknown
__device__ __forceinline__ uint32_t known_meta(const ML& L, uint32_t subj, uint64_t v) {
  if (!(v & META_BIT)) return NONE32;
  const Dev& d = *L.d;
  const uint32_t u = d.md_uidx[subj];
  return u == NONE32 ? 0u : d.md_ver[lidx(d, L.m) * MDU + u];
}

__device__ __forceinline__ uint32_t* grp(ML& L, int g) { return L.groups + (size_t)g * GREC; }
// a fetch whose timeout fired while its request was still in flight (a delay): only its hops remain
constexpr uint32_t FETCH_ORPHAN = 0xFFFFFFFEu;

__device__ __forceinline__ void complete_group(ML& L, int g) {
  uint32_t* G = grp(L, g);
  uint32_t kind = G[0], flags = G[5];
  G[5] = 0;
  if (kind == 0) {
    // onSync doOnSuccess (MembershipProtocolImpl.java:351-365): SYNC_ACK with the post-merge table
    if (!(flags & GF_ERROR)) send_sync(L, K_SYNC_ACK, G[1], G[2], G[3], g == L.rgrp);
  } else {
    // start0 doFinally (:244-248): schedulePeriodicSync
    L.initFlags &= ~INIT_ACTIVE;
    L.nextSync = L.k + L.d->sync_t;
  }
}

// one inner Mono of Mono.whenDelayError terminated
__device__ __forceinline__ void finish(ML& L, int g, bool error) {
  if (g < 0) return;
  uint32_t* G = grp(L, g);
  if (error) G[5] |= GF_ERROR;
  if ((G[5] & GF_SEALED) && G[4] == 0) complete_group(L, g);
}

__device__ __forceinline__ int alloc_group(ML& L, uint32_t kind, uint32_t reply, uint32_t ciss, uint32_t ccnt) {
  for (int g = 0; g < (int)L.d->GRCAP; ++g) {
    uint32_t* G = grp(L, g);
    if (!(G[5] & GF_USED)) {
      G[0] = kind;
      G[1] = reply;
      G[2] = ciss;
      G[3] = ccnt;
      G[4] = 0;
      G[5] = GF_USED;
      return g;
    }
  }
  set_err(*L.d, E_GROUPS);
  return -1;
}

// doFinally of updateMembership (:526-539)
__device__ __forceinline__ void do_finally(ML& L, uint32_t subj, uint32_t st, uint32_t inc, uint32_t reason) {
  if (reason != R_GOSSIP && reason != R_INITIAL) spread(L, subj, st, inc);
}

// MetadataStoreImpl.fetchMetadata (:149-186); the response hop is evaluated in P3 at k + lat
// dd: whether subj is dead at this tick, when the caller loaded it already (-1: look it up)
__device__ __forceinline__ void fetch_md(ML& L, uint32_t subj, uint32_t st, uint32_t inc, uint32_t reason, uint32_t added, int g,
                                         int dd = -1) {
  const Dev& d = *L.d;
  uint32_t cnt = L.cidCnt++;
  L.c[C_M]++;
  const int e = xmit_ep(d, L.ep, K_GMD_REQ, L.m, subj, L.k, L.m, cnt, dd);
  if (e < 0) {
    L.c[C_LOST]++;
    if (g >= 0) grp(L, g)[5] |= GF_ERROR;
    do_finally(L, subj, st, inc, reason);
    return;
  }
  if (L.nfetch >= d.FCAP) {
    set_err(d, E_FETCH);
    return;
  }
  uint32_t* f = L.fetch + (size_t)(L.nfetch++) * FREC;
  f[0] = cnt;
  f[1] = subj;
  f[2] = inc;
  f[3] = st | (reason << 8) | (added << 16) | (1u << 24);  // stage 1: response hop pending
  f[4] = (uint32_t)g;
  f[5] = L.k + d.md_t;
  f[6] = L.k + d.lat + (uint32_t)e;
  f[7] = NONE32;
  L.fnext = min(L.fnext, min(f[5], f[6]));
  if (g >= 0) grp(L, g)[4]++;
}

// MembershipProtocolImpl.updateMembership (:475-541) + emitMembershipEvent (:543-588)
__device__ __forceinline__ void update_membership(ML& L, uint32_t subj, uint32_t s1, uint32_t i1, uint32_t reason, int g) {
  const Dev& d = *L.d;
  uint64_t v0 = row_ld(L, subj);
  uint32_t s0 = rec_status(v0), i0 = rec_inc(v0);
  if (!overrides(s1, i1, s0, i0)) return;
  if (subj == L.m) {  // :488-509 refute with max(inc)+1, keep r0's status, spread, no event
    uint32_t ni = (i0 > i1 ? i0 : i1) + 1u;
    row_put(L, subj, (v0 & ~KEY_MASK) | rec_key(s0, ni));
    L.c[C_W]++;
    spread(L, subj, s0, ni);
    return;
  }
  if (s1 == ST_DEAD) {
    row_put(L, subj, 0);  // row removed; REMOVED below removes the metadata; the timer is cancelled
    L.tsize--;
  } else {
    if (s0 == ST_ABSENT) L.tsize++;
    uint64_t v = (v0 & ~KEY_MASK) | rec_key(s1, i1);
    if (s1 == ST_SUSPECT) {  // scheduleSuspicionTimeoutTask (:597-606): computeIfAbsent
      if (rec_timer(v) == 0) {
        uint32_t dl = L.k + suspicion_ticks(d, L.tsize, mc_ping_t(d, L.m));
        v = rec_with_timer(v, dl);
        if (dl < L.timerMin) L.timerMin = dl;
      }
    } else {
      v = rec_with_timer(v, 0);  // cancelSuspicionTimeoutTask (:590-595)
    }
    row_put(L, subj, v);
  }
  L.c[C_W]++;
  if (s1 == ST_DEAD) {
    uint32_t oldm = known_meta(L, subj, v0);  // metadataStore.removeMetadata
    emit_event(L, 1, subj, oldm, NONE32);
    finish(L, g, false);
    do_finally(L, subj, s1, i1, reason);
    return;
  }
  if (s0 == ST_ABSENT && s1 == ST_ALIVE) {
    fetch_md(L, subj, s1, i1, reason, 1, g);
    return;
  }
  if (s0 != ST_ABSENT && i0 < i1) {
    fetch_md(L, subj, s1, i1, reason, 0, g);
    return;
  }
  finish(L, g, false);
  do_finally(L, subj, s1, i1, reason);
}

// onFailureDetectorEvent (:370-398)
__device__ __forceinline__ void on_fd_event(ML& L, uint32_t target, uint32_t status) {
  uint64_t v0 = row_ld(L, target);
  uint32_t s0 = rec_status(v0);
  if (s0 == ST_ABSENT || s0 == status) return;
  if (status == ST_ALIVE) {
    send_sync(L, K_SYNC, target, NONE32, 0);
  } else {
    L.c[C_R]++;
    update_membership(L, target, ST_SUSPECT, rec_inc(v0), R_FD, -1);
  }
}

__device__ __forceinline__ void add_sub(ML& L, uint32_t cnt, uint32_t kind, uint32_t target, uint32_t deadline) {
  if (L.nsub >= SUBCAP) {
    set_err(*L.d, E_SUBS);
    return;
  }
  uint32_t* s = L.subs + (size_t)(L.nsub++) * 4;
  s[0] = cnt;
  s[1] = kind;
  s[2] = target;
  s[3] = deadline;
  L.smin = min(L.smin, deadline);
}
__device__ __forceinline__ void add_path(ML& L, uint32_t cnt, uint32_t stage, uint32_t tick, uint32_t a, uint32_t b) {
  if (L.npath >= L.d->PCAP) {
    set_err(*L.d, E_PATHS);
    return;
  }
  uint32_t* p = L.paths + (size_t)(L.npath++) * 5;
  p[0] = cnt;
  p[1] = stage;
  p[2] = tick;
  p[3] = a;
  p[4] = b;
  L.pmin = min(L.pmin, tick);
}

// doPing error branch (FailureDetectorImpl.java:159-175), selectPingReqMembers (:349-361), doPingReq (:178-213)
__device__ __forceinline__ void ping_req_step(ML& L, uint32_t target, uint32_t cnt) {
  const Dev& d = *L.d;
  uint32_t helpers[8];
  uint32_t nh = 0;
  const uint32_t kreq = mc_kreq(d, L.m);
  if (kreq > 0) {
    fd_ready(L);
    uint32_t pos = L.fdLen;
    for (uint32_t i = 0; i < L.fdLen; ++i)
      if (L.fdl[i] == target) {
        pos = i;
        break;
      }
    uint32_t n = L.fdLen - (pos < L.fdLen ? 1u : 0u);
    if (n > 0) {
      uint32_t kk = kreq < n ? kreq : n;
      uint32_t ovp[16], ovv[16], nov = 0;  // positions touched by the partial Fisher-Yates
      auto get = [&](uint32_t i) -> uint32_t {
        for (uint32_t q = 0; q < nov; ++q)
          if (ovp[q] == i) return ovv[q];
        return L.fdl[i < pos ? i : i + 1];
      };
      auto set = [&](uint32_t i, uint32_t v) {
        for (uint32_t q = 0; q < nov; ++q)
          if (ovp[q] == i) {
            ovv[q] = v;
            return;
          }
        ovp[nov] = i;
        ovv[nov] = v;
        nov++;
      };
      for (uint32_t i = 0; i < kk; ++i) {
        uint32_t j = i + next_int(draw(L, S_PINGREQ), n - i);
        uint32_t vi = get(i), vj = get(j);
        set(i, vj);
        set(j, vi);
      }
      for (uint32_t i = 0; i < kk; ++i) helpers[i] = get(i);
      nh = kk;
    }
  }
  int timeLeft = (int)mc_ping_t(d, L.m) - (int)mc_timeout_t(d, L.m);
  if (timeLeft <= 0 || nh == 0) {
    on_fd_event(L, target, ST_SUSPECT);
    return;
  }
  for (uint32_t q = 0; q < nh; ++q) {
    uint32_t h = helpers[q];
    L.c[C_M]++;
    const int e = xmit_ep(d, L.ep, K_PING_REQ, L.m, h, L.k, L.m, cnt);
    if (e < 0) {
      L.c[C_LOST]++;
      on_fd_event(L, target, ST_SUSPECT);
      continue;
    }
    add_sub(L, cnt, 1, target, L.k + (uint32_t)timeLeft);
    add_path(L, cnt, P_REQ | 1, L.k + d.lat + (uint32_t)e, h, target);
  }
}

// doPing (:128-176) + selectPingMember (:338-347)
__device__ __forceinline__ void do_ping(ML& L) {
  const Dev& d = *L.d;
  L.fdPeriod++;
  if (L.fdLen == 0) return;
  fd_ready(L);
  if (L.pingIdx >= (int32_t)L.fdLen) {
    L.pingIdx = 0;
    shuffle_list(L, L.fdl, L.fdLen, S_FD_SHUFFLE);
  }
  uint32_t target;
  int dd = -1;  // the target's liveness, when loaded with the member state (L.pre)
  if (L.pre != NEVER) {
    target = L.pre;
    dd = L.k >= L.pre_dt ? 1 : 0;
    L.pingIdx++;
  } else {
    target = L.fdl[L.pingIdx++];
  }
  uint32_t cnt = L.cidCnt++;
  L.c[C_M]++;
  const int e = xmit_ep(d, L.ep, K_PING, L.m, target, L.k, L.m, cnt, dd);
  if (e < 0) {
    L.c[C_LOST]++;
    ping_req_step(L, target, cnt);
    return;
  }
  add_sub(L, cnt, 0, target, L.k + mc_timeout_t(d, L.m));
  add_path(L, cnt, P_DIRECT | 1, L.k + d.lat + (uint32_t)e, target, 0);
}

// doSpreadGossip (GossipProtocolImpl.java:139-157) target selection (:252-273). The sends and the sweep run in
// the gossip data plane (gossip.hip) from T / tspread / tperiod; the round is logged for infectedFrom replay.
__device__ __forceinline__ void do_spread_gossip(ML& L) {
  const Dev& d = *L.d;
  uint32_t period = L.gPeriod++;
  if (L.held == 0) return;
  uint32_t F = d.F;
  uint32_t* T = d.T + (size_t)L.m * F;
  uint32_t cnt;
  if (d.implicit) {  // RUMOR at scale: the PRECONVERGED permutation, read where a stored list would be (engine.h)
    const FeistelPerm P = list_perm(d, L.m, 1);
    if (L.gLen < F) {
      for (uint32_t i = 0; i < L.gLen; ++i) T[i] = list_at(P, L.m, i);
      cnt = L.gLen;
    } else {
      if (L.remoteIdx < 0 || (uint32_t)L.remoteIdx + F > L.gLen) {
        set_err(d, E_LIST);  // the reshuffle of a wrapped cursor needs a stored list (N / F rounds: never at C5)
        L.remoteIdx = 0;
      }
      for (uint32_t i = 0; i < F; ++i) T[i] = list_at(P, L.m, L.remoteIdx + i);
      L.remoteIdx += (int32_t)F;
      cnt = F;
    }
  } else if (L.gLen < F) {
    for (uint32_t i = 0; i < L.gLen; ++i) T[i] = L.gl[i];
    cnt = L.gLen;
  } else {
    if (L.remoteIdx < 0 || (uint32_t)L.remoteIdx + F > L.gLen) {
      shuffle_list(L, L.gl, L.gLen, S_GOSSIP_SHUFFLE);
      L.remoteIdx = 0;
    }
    for (uint32_t i = 0; i < F; ++i) T[i] = L.gl[L.remoteIdx + i];
    L.remoteIdx += (int32_t)F;
    cnt = F;
  }
  uint32_t sp = spread_of(d, L.gLen + 1);
  L.tround = 1;
  d.tcnt[L.m] = cnt;
  d.tspread[L.m] = sp;
  d.tperiod[L.m] = period;
  uint32_t pos = d.log_pos[L.m] % d.LOGW;
  size_t lo = (size_t)L.m * d.LOGW + pos;
  if (d.log_pos[L.m] > 0 && d.log_spread[(size_t)L.m * d.LOGW + (d.log_pos[L.m] - 1) % d.LOGW] != sp) d.spchg[L.m] = L.k;
  d.log_tick[lo] = L.k;
  d.log_spread[lo] = sp;
  d.log_cnt[lo] = cnt;
  for (uint32_t i = 0; i < cnt; ++i) d.log_tg[lo * F + i] = T[i];
  d.log_pos[L.m]++;
  if (d.W > 1) {  // the round is replayed into the other shards' replicated logs from exchange A
    uint32_t i = atomicAdd(&d.xn[1], 1u);
    if (i >= d.RRCAP) {
      set_err(d, E_XCAP);
      return;
    }
    uint32_t* r = d.rr_rec + (size_t)i * RRW;
    r[0] = L.m;
    r[1] = cnt;
    r[2] = sp;
    r[3] = period;
    for (uint32_t j = 0; j < cnt; ++j) r[4 + j] = T[j];
  }
}

// the member's seedMembers: its own list if it joined through swim_join, else the config's (deduplicated; self is
// skipped by the callers, MembershipProtocolImpl.java:160-166)
__device__ __forceinline__ const uint32_t* member_seeds(const Dev& d, uint32_t m, uint32_t* n) {
  const uint32_t jn = d.jseed_n[m];
  if (jn != NONE32) {
    *n = jn;
    return d.jseeds + (size_t)m * 16;
  }
  *n = d.n_seeds;
  return d.seeds;
}

__device__ __forceinline__ bool is_seed(const Dev& d, uint32_t m, uint32_t s) {
  if (s == m) return false;
  uint32_t n;
  const uint32_t* sd = member_seeds(d, m, &n);
  for (uint32_t i = 0; i < n; ++i)
    if (sd[i] == s) return true;
  return false;
}

// doSync (MembershipProtocolImpl.java:298-314) + selectSyncAddress (:410-421)
__device__ __forceinline__ void do_sync(ML& L) {
  const Dev& d = *L.d;
  uint32_t extra = 0, nsd;
  const uint32_t* sd = member_seeds(d, L.m, &nsd);
  for (uint32_t i = 0; i < nsd; ++i) {
    uint32_t s = sd[i];
    if (s != L.m && row_status(L, s) == ST_ABSENT) extra++;
  }
  uint32_t count = (L.tsize - 1u) + extra;
  if (count == 0) return;
  uint32_t i = next_int(draw(L, S_SYNC_PICK), count);
  uint32_t target;
  if (L.tsize == L.N) {
    target = i < L.m ? i : i + 1u;
  } else {
    target = NONE32;
    for (uint32_t s = 0; s < L.N; ++s) {
      bool in = (s != L.m && row_status(L, s) != ST_ABSENT) || is_seed(d, L.m, s);
      if (!in) continue;
      if (i == 0) {
        target = s;
        break;
      }
      --i;
    }
  }
  send_sync(L, K_SYNC, target, NONE32, 0);
}

// payload record r1 (key32 k1) of subject s against the live row: `.filter(r1 -> !r1.equals(table.get(id)))`, then
// updateMembership (:462-464)
__device__ __forceinline__ void merge_record(ML& L, uint32_t s, uint32_t k1, uint32_t reason, int g) {
  if ((k1 & 3u) == ST_ABSENT || k1 == L.rk[s]) return;
  if (L.d->ackres) tl_add(L, s);
  const uint64_t key = key34(k1);
  update_membership(L, s, rec_status(key), rec_inc(key), reason, g);
}

// syncMembership (:456-467) of one payload. The reference filters every payload record against the live table when
// that payload is processed. k_sync_diff extracted the records that differ from the receiver's row as it stood at
// the start of the tick, in subject order; that is exact for the first payload of the tick. A later payload can
// also hold, for a subject an earlier payload changed, a record equal to the start row but not to the live one (a
// leaver's own DEAD record removes it, then another member's ALIVE record of the old incarnation re-adds it,
// MembershipRecord.java:67-69). Those subjects are read from the payload itself and merged into the candidate walk
// in subject order: up to trk_cap of them from the sorted list L.trk, more from the bitmap Dev::tbm, word by word with the
// next word's load in flight (C2's receivers change hundreds of subjects in one P1: comparing every later payload with
// the whole row on one lane held the member kernel).
__device__ __forceinline__ void merge_payload(ML& L, uint32_t mi, uint32_t reason, int g) {
  const Dev& d = *L.d;
  const uint32_t b = (L.k - 1) & 1;
  const SyncMsg& mm = d.msgs[b][mi];
  L.c[C_R] += mm.psize;
  L.c[C_SYNCMERGE]++;
  const uint32_t nt = L.ntrk;
  const bool bmap = nt > d.trk_cap;  // many subjects changed earlier in this tick: walk the bitmap
  if (bmap) fb_add(d, FB_TRK_WALK);
  if (d.exp & 128) {  // timing experiments: full walks, largest candidate count
    if (bmap) atomicAdd(&d.ctr[14], 1ull);
    atomicMax(&d.ctr[15], (unsigned long long)mm.ncand);
  }
  if (mm.ncand == 0 && nt == 0) return;  // steady state: nothing differs, skip the chunk walk
  if (!bmap)
    for (uint32_t i = 1; i < nt; ++i)  // the tracked subjects in ascending order (insertion sort, at most TRK)
      for (uint32_t j = i; j > 0 && L.trk[j - 1] > L.trk[j]; --j) {
        const uint32_t t = L.trk[j];
        L.trk[j] = L.trk[j - 1];
        L.trk[j - 1] = t;
      }
  // One walk with a single merge site: update_membership is large, and each inlined copy of it costs instruction
  // cache in every wave of this kernel. The next record comes from the candidate pool and the tracked subjects merged
  // in subject order (a tracked candidate takes the pool's record).
  uint32_t ti = 0, c = 0, e = 0, n = 0, off = 0;
  bool pool = mm.ncand != 0;
  // the bitmap cursor: word wi - 1 is being consumed (bits left: wcur), word wi is loading (wnxt)
  uint32_t wi = 0;
  unsigned long long wcur = 0, wnxt = 0;
  const unsigned long long* tb = d.tbm + lidx(d, L.m) * d.NW;
  if (bmap && d.NW) {
    wcur = tb[0];
    wnxt = d.NW > 1 ? tb[1] : 0ull;
    wi = 1;
  }
  auto tnext = [&]() -> uint32_t {  // the next tracked subject in ascending order (bitmap mode), NEVER at the end
    while (wcur == 0ull) {
      if (wi >= d.NW) return NEVER;
      wcur = wnxt;
      ++wi;
      wnxt = wi < d.NW ? tb[wi] : 0ull;
    }
    const uint32_t v = (wi - 1u) * 64u + (uint32_t)(__ffsll((long long)wcur) - 1);
    wcur &= wcur - 1ull;
    return v;
  };
  uint32_t tsb = bmap ? tnext() : NEVER;
  for (;;) {
    uint32_t subj, k1;
    {
      while (pool && e == n) {
        if (c == d.NMETA) {
          pool = false;
          break;
        }
        const uint32_t* cm = d.chunk_meta + ((size_t)mi * d.NMETA + c) * 2;
        off = cm[0];
        n = cm[1];
        e = 0;
        ++c;
      }
      uint64_t prec = 0;
      uint32_t ps = NEVER;
      if (pool) {
        prec = d.pool[(size_t)off + e];
        ps = (uint32_t)(prec >> 34);
      }
      const uint32_t ts = bmap ? tsb : ti < nt ? L.trk[ti] : NEVER;
      if (ps == NEVER && ts == NEVER) break;
      if (ts < ps) {
        subj = ts;
        k1 = payload_key_at(d, mm, b, ts);
        if (bmap) tsb = tnext(); else ++ti;
      } else {
        subj = ps;
        k1 = key32(prec & KEY_MASK);
        ++e;
        if (ts == ps) {
          if (bmap) tsb = tnext(); else ++ti;
        }
      }
    }
    merge_record(L, subj, k1, reason, g);
  }
}

// Triage (k_member_triage): the idle fast path. Most members have nothing due in most ticks (a ping every 10 ticks,
// a SYNC every 300); they only advance an empty gossip round here. Returns whether the member needs the full
// control path of k_member_tick this tick, and its work class: 1 = a ping and / or a periodic SYNC is due (P6) and
// nothing else, 2 = only request-state events (ping hops, ack arrivals, timeouts), 3 = both, 0 = anything else (SYNC
// receipt, gossip receipts or round, timers, host requests, start).
__device__ __forceinline__ bool member_triage(const Dev& d, uint32_t m, uint32_t k, uint32_t& cls, uint32_t& drops,
                                              uint32_t& evs) {
  // A dead member does nothing itself, but the remote hops of its in-flight requests still run at the live
  // responders (their sends fail against the dead issuer), so those hops are still evaluated for the counters.
  // every word is loaded up front (no short-circuit chain of dependent loads); the SoA loads coalesce per wave
  const uint32_t mh = d.m_head[(size_t)((k - 1) & 1) * d.N + m], rc = d.rc_cnt[m], pi = d.pending_inc[m],
                 ne = d.next_evt[m], tm = d.timerMin[m], np = d.nextPing[m], ns = d.nextSync[m], inf = d.initFlags[m],
                 ng = d.nextGossip[m], held = d.held[m], dt = d.dead_tick[m], st = d.start_tick[m],
                 nd = d.rc_ndrop[m];
  const bool dead = k >= dt;
  cls = 0;
  drops = 0;
  if (d.fastp4) {  // RUMOR mode: P4's GOSSIP events of this tick, hashed and counted when they were applied
    const uint32_t pn = d.evp_n[m];
    if (pn) {
      if (!dead) {  // a member crashed since holds no P4 (its receipts are dropped, as rc_cnt below)
        d.ms[m].evHash += d.evp_hash[m];
        d.ms[m].evSeq += pn;
        evs = pn;
      }
      d.evp_hash[m] = 0;
      d.evp_n[m] = 0;
    }
  }
  if (nd) {  // receipts that could not change the row: P4's record compares (none for a dead member)
    d.rc_ndrop[m] = 0;
    if (!dead) drops = nd;
  }
  if (dead) {
    d.rc_cnt[m] = 0;
    d.rc_fill[m] = 0;
    if (k > 0 && mh != NEVER) {  // dropped payloads: their pins go back to NEVER (send_sync)
      const uint32_t pb = (k - 1) & 1;
      for (uint32_t q = mh; q != NEVER; q = d.m_next[(size_t)pb * d.MSGCAP + q]) d.msgs[pb][q].pin = NEVER;
      d.m_head[(size_t)pb * d.N + m] = NEVER;
    }
  } else {
    const bool busy = (k > 0 && mh != NEVER) | (rc != 0) | (pi != 0) | (ne <= k) | (tm <= k) | (k == np) | (k == ns) |
                      ((inf & INIT_ACTIVE) != 0) | (k == st);
    // a periodic SYNC send (doSync, P6) is scheduled with the pings (P6 too), not with the SYNC receivers: in one wave
    // their chains would run one after the other
    const bool other = (k > 0 && mh != NEVER) | (rc != 0) | (pi != 0) | (tm <= k) | ((inf & INIT_ACTIVE) != 0) |
                       (k == st) | (k == ng && held != 0);
    cls = other ? 0u : (k == np || k == ns ? 1u : 0u) | (ne <= k ? 2u : 0u);
    if (!busy) {
      if (k != ng) {
        d.tround[m] = 0;
        return false;
      }
      if (held == 0) {  // doSpreadGossip with no gossips: period++ only (GossipProtocolImpl.java:141-146)
        d.ms[m].gPeriod++;
        d.nextGossip[m] = ng + d.gossip_t;
        d.tround[m] = 0;
        return false;
      }
    }
  }
  if (dead && d.ms[m].npath == 0 && (d.ms[m].nfetch == 0 || d.ms[m].fnext > k)) {
    d.tround[m] = 0;
    return false;
  }
  return true;
}

// the member's state as member_tick_body holds it (one lane per member; k_inbox_apply: every lane of the member's wave)
__device__ __forceinline__ void ml_init(ML& L, const Dev& d, uint32_t m, uint32_t k, uint4* cw, uint32_t* cw_n, bool spec) {
  L.d = &d;
  L.m = m;
  L.k = k;
  L.N = d.N;
  {  // the body-only state: one 128-B record, five 16-B loads
    const uint4* mp = (const uint4*)(d.ms + m);
    const uint4 w0 = mp[0], w1 = mp[1], w2 = mp[2], w3 = mp[3], w4 = mp[4];
    L.tsize = w0.x, L.fdLen = w0.y, L.gLen = w0.z, L.fdPeriod = w0.w;
    L.gPeriod = w1.x, L.gCounter = w1.y, L.cidCnt = w1.z, L.syncSeq = w1.w;
    L.evSeq = w2.x, L.initDeadline = w2.y, L.initCidBase = w2.z, L.initN = w2.w;
    L.nsub = w3.x, L.npath = w3.y, L.nfetch = w3.z, L.fnext = w3.w;
    L.pingIdx = (int32_t)w4.x, L.remoteIdx = (int32_t)w4.y, L.evHash = ((uint64_t)w4.w << 32) | w4.z;
  }
  L.nextPing = d.nextPing[m];
  L.nextGossip = d.nextGossip[m];
  L.nextSync = d.nextSync[m];
  L.held = d.held[m];
  L.timerMin = d.timerMin[m];
  L.initFlags = d.initFlags[m];
  L.ep = epoch_at(d, k);
  const size_t li = lidx(d, m);  // per-observer arrays hold only this shard's rows
  L.rk = d.rowk + li * d.NS;
  L.ra = d.rowa + li * d.NS;
  L.rd = d.W > 1 ? d.rdirty + li * d.MW : nullptr;
  L.fdl = d.fdl + li * d.LCAP;
  L.gl = d.gl + li * d.LCAP;
  L.subs = d.subs + li * SUBCAP * 4;
  L.paths = d.paths + li * d.PCAP * 5;
  L.fetch = d.fetch + li * d.FCAP * FREC;
  L.groups = d.groups + li * d.GRCAP * GREC;
  L.fpend = d.fpend + li * KP * 2;
  L.npend = 0;
  for (int i = 0; i < 8; ++i) L.c[i] = 0;
  L.pend = NEVER;
  L.tround = 0;
  L.trk = d.trk + li * TRKL;
  L.ntrk = 0;
  L.trk_on = false;
  L.cw = cw;
  L.cw_n = cw_n;
  L.spec = spec;
  L.ulog = d.ulog + li * d.ULOGC * 2;
  L.ncreq = 0;
  L.nlog = 0;
  L.spq = d.spq + li * SPQ * 8;
  L.nsp = 0;
  L.tl = d.ackres ? d.tlog + ((size_t)(k & 1) * d.NL + li) * TL : nullptr;
  L.ntl = 0;
  L.tlast = NEVER;
  L.rgrp = -1;
  L.pre = NEVER;
  L.lk_i = NEVER;
  L.pmin = L.smin = NEVER;
  L.ev_ok = false;
}

// member_tick_body's state back (everything but next_evt and tround, which only a finished tick stores)
__device__ __forceinline__ void ml_store(ML& L) {
  link_flush(L);
  const Dev& d = *L.d;
  const uint32_t m = L.m, k = L.k;
  const size_t li = lidx(d, m);
  {  // the body-only state: five 16-B stores into the member's record
    uint4* mp = (uint4*)(d.ms + m);
    mp[0] = make_uint4(L.tsize, L.fdLen, L.gLen, L.fdPeriod);
    mp[1] = make_uint4(L.gPeriod, L.gCounter, L.cidCnt, L.syncSeq);
    mp[2] = make_uint4(L.evSeq, L.initDeadline, L.initCidBase, L.initN);
    mp[3] = make_uint4(L.nsub, L.npath, L.nfetch, L.fnext);
    mp[4] = make_uint4((uint32_t)L.pingIdx, (uint32_t)L.remoteIdx, (uint32_t)L.evHash, (uint32_t)(L.evHash >> 32));
  }
  d.nextPing[m] = L.nextPing;
  d.nextGossip[m] = L.nextGossip;
  d.nextSync[m] = L.nextSync;
  d.held[m] = L.held;
  d.timerMin[m] = L.timerMin;
  d.initFlags[m] = L.initFlags;
  if (L.ntl) {  // (no entry this tick: the stale tick stamp reads as an empty log)
    d.tl_n[(size_t)(k & 1) * d.NL + li] = L.ntl;
    d.tl_tick[(size_t)(k & 1) * d.NL + li] = k;
  }
}

// mode: BODY_FULL = the whole tick; BODY_SPLIT = the whole tick, except that a member with at least Dev::hv routed
// gossip receipts stops before P4 and is listed for k_inbox_apply (P4, a wave per member) and the resumed launch;
// BODY_RESUME = P5 and P6 of a listed member (its P0-P4 ran in the two launches before)
enum : uint32_t { BODY_FULL = 0, BODY_SPLIT = 1, BODY_RESUME = 2 };
template <uint32_t mode>
__device__ __forceinline__ void member_tick_body(const Dev& d, uint32_t m, uint32_t k, unsigned long long (&cnt)[8],
                                                 uint4* cw, uint32_t* cw_n, bool spec) {
  const bool dead = dead_at(d, m, k);
  ML L;
  ml_init(L, d, m, k, cw, cw_n, spec);
  const size_t li = lidx(d, m);
  if (mode == BODY_RESUME) {  // what the parked member kept between the launches (k_inbox_apply updated it)
    L.pend = d.hv_pend[li];
    L.tlast = d.hv_tlast[li];
    if (d.ackres && d.tl_tick[(size_t)(k & 1) * d.NL + li] == k) L.ntl = d.tl_n[(size_t)(k & 1) * d.NL + li];
  }
  // P1's inbound list head, loaded with the state above (P0's sends link into the other buffer)
  const uint32_t head0 = (mode != BODY_RESUME && !dead && k > 0) ? d.m_head[(size_t)((k - 1) & 1) * d.N + m] : NEVER;
  // the P6 ping's target and its liveness, loaded now (do_ping's loads would wait for this tick's stores)
  if (!dead && k == L.nextPing && L.fdLen > 0 && L.pingIdx >= 0 && L.pingIdx < (int32_t)L.fdLen) {
    L.pre = L.fdl[L.pingIdx];
    L.pre_dt = d.dead_tick[L.pre];
  }
  // SWIM_EXP & 16 (timing experiment): shader cycles per phase summed over members, ctr[8..12]
  // SWIM_EXP & 128: the largest per-member cycles of each phase instead (which phase makes the longest lane)
  const bool prof = (d.exp & (16 | 128)) != 0;
  unsigned long long tp = prof ? clock64() : 0;
  // SWIM_EXP & 512: the wave's first busy lane stamps the wall clock after each phase group (wt[4 + slot])
  // (the first lane active at the lap stamps it: a lap inside a branch times the lanes that took it)
  auto lap = [&](int slot) {
    if ((d.exp & 512) && (threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)__ballot(1)) - 1))
      d.wt[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + 4 + slot] = wall_clock64();
    if (!prof || slot > 4) return;  // (slots 5-10: finer wall-clock laps only)
    const unsigned long long t = clock64();
    if (d.exp & 16)
      atomicAdd(&d.ctr[8 + slot], t - tp);
    else
      atomicMax(&d.ctr[8 + slot], t - tp);
    tp = t;
  };

  if (mode != BODY_RESUME) {  // P0 - P4
  // ---- P0 host requests: updateIncarnation (MembershipProtocolImpl.java:178-190), then leaveCluster (:197-206) ----
  const uint32_t preq = dead ? 0u : d.pending_inc[m];
  if (preq) {
    d.pending_inc[m] = 0;
    for (uint32_t b = preq >> 2; b > 0; --b) {  // one bump and one gossip per swim_update_incarnation call
      uint64_t v0 = row_ld(L, m);
      uint32_t ni = rec_inc(v0) + 1u;
      row_put(L, m, (v0 & ~KEY_MASK) | rec_key(ST_ALIVE, ni));
      L.c[C_W]++;
      spread(L, m, ST_ALIVE, ni);
    }
    if (preq & 2u) {  // the own record becomes DEAD inc+1 (the only DEAD record a table keeps) and is spread
      uint64_t v0 = row_ld(L, m);
      uint32_t ni = rec_inc(v0) + 1u;
      row_put(L, m, (v0 & ~KEY_MASK) | rec_key(ST_DEAD, ni));
      L.c[C_W]++;
      spread(L, m, ST_DEAD, ni);
    }
  }

  // ---- P0 start: ClusterImpl.join0 -> MembershipProtocolImpl.start0 (:216-251): COLD_JOIN members at tick 0, joined
  // (swim_join) members at their join tick, with their own seeds ----
  if (!dead && k == d.start_tick[m]) {
    uint32_t nsd;
    const uint32_t* sd = member_seeds(d, m, &nsd);
    uint32_t ns = 0;
    for (uint32_t i = 0; i < nsd; ++i)
      if (sd[i] != m) ns++;
    if (ns == 0) {
      L.nextSync = k + d.sync_t;
    } else {
      L.initFlags = INIT_ACTIVE;
      L.initDeadline = k + d.syncTimeout_t;
      L.initCidBase = L.cidCnt;
      L.initN = ns;
      uint32_t failed = 0;
      for (uint32_t i = 0; i < nsd; ++i) {
        if (sd[i] == m) continue;
        uint32_t cnt = L.cidCnt++;
        if (!send_sync(L, K_SYNC, sd[i], m, cnt)) failed++;
      }
      if (failed == ns) {
        L.initFlags = 0;
        L.nextSync = k + d.sync_t;
      }
    }
  }

  // ---- P1 SYNC / SYNC_ACK (onMessage :320-331, onSync :346-367, onSyncAck :337-343) ----
  // the senders linked this member's inbound messages into a list; they are handled in (src, syncSeq) order
  const uint32_t* mnext = d.m_next + (size_t)((k - 1) & 1) * d.MSGCAP;
  if (head0 != NEVER) {
    const uint32_t pb = (k - 1) & 1;
    const uint32_t head = head0;
    uint64_t key[MQ];
    uint32_t idx[MQ], n = 0;
    bool more = false;
    for (uint32_t q = head; q != NEVER; q = mnext[q]) {
      if (n == d.mq_cap) {
        more = true;
        fb_add(d, FB_MQ);
        break;
      }
      const SyncMsg& mq = d.msgs[pb][q];
      uint64_t kq = ((uint64_t)mq.src << 32) | mq.seq;
      uint32_t j = n++;
      while (j > 0 && key[j - 1] > kq) {
        key[j] = key[j - 1];
        idx[j] = idx[j - 1];
        --j;
      }
      key[j] = kq;
      idx[j] = q;
    }
    // (reset after the walk's loads: on gfx950 a load issued after this lane's store waits for the store)
    d.m_head[(size_t)pb * d.N + m] = NEVER;
    lap(5);
    uint64_t last = 0;
    L.trk_on = n > 1 || more;  // several payloads: later ones re-check the subjects earlier ones changed
    for (uint32_t r = 0;; ++r) {
      uint32_t mi;
      if (!more) {
        if (r == n) break;
        mi = idx[r];
      } else {  // rare: more than MQ messages in one tick (a seed during a cold join): select the next key
        uint64_t best = ~0ull;
        mi = NEVER;
        for (uint32_t q = head; q != NEVER; q = mnext[q]) {
          const SyncMsg& mq = d.msgs[pb][q];
          uint64_t kq = ((uint64_t)mq.src << 32) | mq.seq;
          if ((r == 0 || kq > last) && kq < best) {
            best = kq;
            mi = q;
          }
        }
        if (mi == NEVER) break;
        last = best;
      }
      SyncMsg mm = d.msgs[pb][mi];
      const uint32_t mflags = mm.kind & KF_FLAGS;
      mm.kind &= ~KF_FLAGS;
      if (mc_group(d, mm.src) != mc_group(d, m)) continue;  // checkSyncGroup (:320-321,431-437): another group's data
      if (mm.kind == K_SYNC && mm.ncand == 0 && L.ntrk == 0 && L.nfetch == 0) {
        // onSync with nothing to merge (the steady state): merge_payload finds no record, and with no fetch pending
        // every group is free, so the group alloc_group would take completes at once; its SYNC_ACK goes out without
        // the group table's round trips (a free group's fields are never read before alloc_group rewrites them)
        L.c[C_R] += mm.psize;
        L.c[C_SYNCMERGE]++;
        send_sync(L, K_SYNC_ACK, mm.src, mm.cid_iss, mm.cid_cnt, !(mflags & (KF_ABS | KF_LATE)));
        continue;
      }
      // one merge_payload / finish site for the three cases (each inlined copy is large)
      int g = -1;
      uint32_t reason = R_SYNC;
      bool grouped = false;
      if (mm.kind == K_SYNC) {
        g = alloc_group(L, 0, mm.src, mm.cid_iss, mm.cid_cnt);
        grouped = true;
      } else if (mm.cid_iss == NONE32) {
      } else if (mm.cid_iss == m && (L.initFlags & INIT_ACTIVE) && !(L.initFlags & INIT_RECEIVED) &&
                 mm.cid_cnt >= L.initCidBase && mm.cid_cnt < L.initCidBase + L.initN) {
        L.initFlags |= INIT_RECEIVED;  // mergeDelayError(...).take(1) (:239-243)
        g = alloc_group(L, 1, NONE32, NONE32, 0);
        reason = R_INITIAL;
        grouped = true;
      } else {
        continue;  // a SYNC_ACK of another initial sync or of an expired one (:326-328)
      }
      merge_payload(L, mi, reason, g);
      if (grouped && g >= 0) {
        grp(L, g)[5] |= GF_SEALED;
        // its SYNC_ACK, if sent now, may be resolved unless the payload lacked records this row holds or came late
        L.rgrp = (mm.kind == K_SYNC && !(mflags & (KF_ABS | KF_LATE))) ? g : -1;
        finish(L, g, false);
        lap(8);
        L.rgrp = -1;
      }
    }
    L.trk_on = false;
    if (L.ntrk) {  // the written-subject bitmap back to zero: the listed subjects' words, or the whole row
      unsigned long long* tb = d.tbm + li * d.NW;
      if (L.ntrk <= TRKL)
        for (uint32_t q = 0; q < L.ntrk; ++q) tb[L.trk[q] >> 6] = 0ull;
      else
        for (uint32_t q = 0; q < d.NW; ++q) tb[q] = 0ull;
      L.ntrk = 0;
    }
    if (n > 1 || more)  // the pins of this tick's payloads go back to NEVER for the slots' next use (send_sync)
      for (uint32_t q = head; q != NEVER; q = mnext[q]) d.msgs[pb][q].pin = NEVER;
  }

  lap(0);  // P0 + P1
  // ---- P2 FD: remote hops of pending pings, then PING_ACK arrivals in cid order ----
  L.ev_ok = mode != BODY_RESUME;  // this launch walks the path list (P2) and the subscriptions (P5)
  if (L.npath) {
    // arrivals stay in the compacted list this pass, marked by their new index (at most PATHCAP_DELAY = 32 entries)
    uint32_t arrmask = 0;
    uint32_t w = 0, pm = NEVER;
    for (uint32_t p = 0; p < L.npath; ++p) {
      uint32_t* P = L.paths + (size_t)p * 5;
      uint32_t cnt = P[0], stage = P[1], tk = P[2], a = P[3], b = P[4];
      bool keep = true, arr = false;
      if (tk == k) {
        lap(9);
        uint32_t kind = stage & 0xF0, st = stage & 0xF;
        if (st == P_ARRIVE) {
          if (dead) keep = false;
          else arrmask |= 1u << w, arr = true;
        } else if (kind == P_DIRECT) {  // onPing at the target (:230-255): PING_ACK back to the issuer
          if (dead_at(d, a, k)) {
            keep = false;
          } else {
            L.c[C_M]++;
            const int e = xmit_ep(d, L.ep, K_PING_ACK, a, m, k, m, cnt);
            if (e < 0) {
              L.c[C_LOST]++;
              keep = false;
            } else {
              stage = P_DIRECT | P_ARRIVE;
              tk = k + d.lat + (uint32_t)e;
            }
          }
        } else {  // ping-req chain: helper a, target b
          uint32_t who = st == 2 ? b : a;
          if (dead_at(d, who, k)) {
            keep = false;
          } else {
            L.c[C_M]++;
            int e;
            if (st == 1)  // onPingReq (:258-284): transit PING helper -> target
              e = xmit_ep(d, L.ep, K_PING, a, b, k, m, cnt);
            else if (st == 2)  // onPing at the target: PING_ACK target -> helper
              e = xmit_ep(d, L.ep, K_PING_ACK, b, a, k, m, cnt);
            else  // onTransitPingAck (:290-315): PING_ACK helper -> issuer
              e = xmit_ep(d, L.ep, K_PING_ACK, a, m, k, m, cnt);
            if (e < 0) {
              L.c[C_LOST]++;
              keep = false;
            } else {
              stage = P_REQ | (st == 3 ? P_ARRIVE : st + 1);
              tk = k + d.lat + (uint32_t)e;
            }
          }
        }
        lap(10);
      }
      if (keep) {
        uint32_t* Q = L.paths + (size_t)w * 5;
        Q[0] = cnt;
        Q[1] = stage;
        Q[2] = tk;
        Q[3] = a;
        Q[4] = b;
        w++;
        if (!arr) pm = min(pm, tk);  // (an arrival leaves the list below)
      }
    }
    L.npath = w;
    L.pmin = min(L.pmin, pm);
    lap(6);
    // arrivals: every pending subscription on the cid takes the first PING_ACK (TransportImpl.java:205-232), in cid
    // order; then the arrived entries leave the list
    const uint32_t narr = __popc(arrmask);
    for (uint32_t done = 0, last = 0; done < narr;) {
      uint32_t cnt = NEVER;  // the smallest arrived cid above the last one handled
      for (uint32_t q = 0; q < w; ++q) {
        const uint32_t c = L.paths[(size_t)q * 5];
        if (((arrmask >> q) & 1u) && (done == 0 || c > last) && c < cnt) cnt = c;
      }
      for (uint32_t q = 0; q < w; ++q) done += ((arrmask >> q) & 1u) && L.paths[(size_t)q * 5] == cnt;
      last = cnt;
      uint32_t hit[SUBCAP], nh = 0, w2 = 0;
      for (uint32_t s = 0; s < L.nsub; ++s) {
        uint32_t* S4 = L.subs + (size_t)s * 4;
        if (S4[0] == cnt) {
          hit[nh++] = S4[2];
        } else {
          uint32_t* D4 = L.subs + (size_t)w2 * 4;
          D4[0] = S4[0];
          D4[1] = S4[1];
          D4[2] = S4[2];
          D4[3] = S4[3];
          w2++;
        }
      }
      L.nsub = w2;
      lap(11);
      for (uint32_t q = 0; q < nh; ++q) on_fd_event(L, hit[q], ST_ALIVE);  // publishPingResult(ALIVE)
    }
    lap(7);
    if (arrmask) {
      uint32_t w3 = 0;
      for (uint32_t p = 0; p < w; ++p)
        if (!((arrmask >> p) & 1u)) {
          if (w3 != p)
            for (uint32_t q = 0; q < 5; ++q) L.paths[(size_t)w3 * 5 + q] = L.paths[(size_t)p * 5 + q];
          w3++;
        }
      L.npath = w3;
    }
  }

  // ---- P3 metadata: response hops at the subject, then GET_METADATA_RESP arrivals in cid order ----
  // One pass over the pending fetches (kept in cid order), only when one of them is due: the response hops due now
  // (onMetadataRequest at the subject, MetadataStoreImpl.java:202-241) and the responses arriving now, compacted in
  // place. A hop reads nothing an arrival writes (its loss draw is keyed by the message, SEMANTICS.md §2), so one pass
  // runs both. A dead issuer keeps only its pending hops (their responses still count as sent at the live subject).
  if (L.nfetch && L.fnext <= k) {
    uint32_t w = 0, fn = NEVER;
    const uint32_t nf = L.nfetch;  // no fetch is issued in P3
    for (uint32_t q = 0; q < nf; ++q) {
      uint32_t* f = L.fetch + (size_t)q * FREC;
      uint4 lo = *(const uint4*)f, hi = *(const uint4*)(f + 4);  // cnt subj inc w3 | g deadline hop meta
      uint32_t stage = lo.w >> 24;
      bool keep = true, mod = false;
      if (stage == 1 && hi.z == k) {
        mod = true;
        const uint32_t subj = lo.y;
        if (dead_at(d, subj, k)) {
          lo.w &= 0x00FFFFFFu;
        } else {
          L.c[C_M]++;
          const int e = xmit_ep(d, L.ep, K_GMD_RESP, subj, m, k, m, lo.x);
          if (e < 0) {
            L.c[C_LOST]++;
            lo.w &= 0x00FFFFFFu;
          } else {
            lo.w = (lo.w & 0x00FFFFFFu) | (2u << 24);
            hi.z = k + d.lat + (uint32_t)e;
            hi.w = d.md_version[subj];
          }
        }
        keep = (!dead && hi.x != FETCH_ORPHAN) || (lo.w >> 24) == 1;
      } else if (stage == 2 && hi.z == k) {
        keep = false;
        if (!dead && hi.x != FETCH_ORPHAN) {  // doOnSuccess (:563-567, :576-581): updateMetadata then sink.next
          const uint32_t subj = lo.y, inc = lo.z, w3 = lo.w, meta = hi.w;
          const int g = (int)hi.x;
          const uint32_t st = w3 & 0xFF, reason = (w3 >> 8) & 0xFF, added = (w3 >> 16) & 0xFF;
          uint64_t v = row_ld(L, subj);
          uint32_t oldm = known_meta(L, subj, v);
          L.ra[subj] = aux32(v | META_BIT);
          const uint32_t u = d.md_uidx[subj];
          if (u != NONE32) d.md_ver[lidx(d, m) * MDU + u] = meta;
          if (added)
            emit_event(L, 0, subj, NONE32, meta);
          else
            emit_event(L, 2, subj, oldm, meta);
          if (g >= 0) grp(L, g)[4]--;
          finish(L, g, false);
          do_finally(L, subj, st, inc, reason);
        }
      } else if (dead) {
        keep = stage == 1;
      }
      if (keep) {
        if (w != q || mod) {
          uint32_t* o = L.fetch + (size_t)w * FREC;
          *(uint4*)o = lo;
          *(uint4*)(o + 4) = hi;
        }
        w++;
        const uint32_t ns = lo.w >> 24;  // the next due event (P5 recomputes it after its own pass)
        fn = min(fn, dead ? (ns == 1 ? hi.z : NEVER) : (ns != 0 ? min(hi.y, hi.z) : hi.y));
      }
    }
    L.nfetch = w;
    L.fnext = fn;
  }

  lap(1);  // P2 + P3
  if (dead) {
    fd_ready(L);
    link_flush(L);
    d.tround[m] = 0;
    d.ms[m].npath = L.npath;
    d.ms[m].nfetch = L.nfetch;
    d.ms[m].fnext = L.fnext;
    d.next_evt[m] = NEVER;
    if (L.ntl) {
      d.tl_n[(size_t)(k & 1) * d.NL + li] = L.ntl;
      d.tl_tick[(size_t)(k & 1) * d.NL + li] = k;
    }
    for (int i = 0; i < 8; ++i) cnt[i] += L.c[i];
    return;
  }

  // ---- P4 gossip first receipts in gossip-id order -> onMembershipGossip (:401-408) ----
  // only the receipts that can change the row were routed (receipt_matters, kernels.hip); the others were counted
  // as record compares by the triage
  {
    uint32_t off = d.rc_off[m], n = d.rc_cnt[m];
    if (mode == BODY_SPLIT && n >= d.hv) {  // many receipts: P4 in k_inbox_apply, P5 and P6 in the resumed launch
      d.hv_list[wave_append(d.nhv)] = m;
      d.hv_pend[li] = L.pend;
      d.hv_tlast[li] = L.tlast;
      flush_spreads(L);
      fd_ready(L);
      if (L.ncreq)  // this launch's epilogue completes the open snapshots, undoing the writes logged so far
        for (uint32_t q = 0, nq = min(*L.cw_n, d.cwmax_cap); q < nq; ++q)
          if (L.cw[q].x == m) L.cw[q].w = L.nlog;
      ml_store(L);
      for (int i = 0; i < 8; ++i) cnt[i] += L.c[i];
      return;
    }
    if (n) {
      d.rc_cnt[m] = 0;  // the next receipt routing counts from zero
      d.rc_fill[m] = 0;
    }
    // batches of PB receipts: their slot words and the rows they touch are loaded together (independent loads in
    // flight at once), then the updates run in order; update_membership re-reads the row (cache-hot), so a batch
    // that touches one subject twice still sees its own earlier write. (A member with many receipts in a tick after a
    // gossip plane runs them on a wave of its own instead: k_inbox_apply.)
    constexpr uint32_t PB = 8;
    for (uint32_t q0 = 0; q0 < n; q0 += PB) {
      const uint32_t nb = min(PB, n - q0);
      uint32_t gs[PB], subj[PB];
      uint64_t key[PB];
#pragma unroll
      for (uint32_t i = 0; i < PB; ++i) gs[i] = i < nb ? d.rc_slot[off + q0 + i] : 0u;
#pragma unroll
      for (uint32_t i = 0; i < PB; ++i) {
        subj[i] = i < nb ? d.slot_subj[gs[i]] : USER_SUBJ;
        key[i] = i < nb ? d.slot_key[gs[i]] : 0ull;
      }
      uint32_t warm = 0;
#pragma unroll
      for (uint32_t i = 0; i < PB; ++i)
        if (subj[i] != USER_SUBJ) warm += L.rk[subj[i]] + L.ra[subj[i]];
      asm volatile("" ::"v"(warm));  // keep the warming loads
      for (uint32_t i = 0; i < nb; ++i) {
        if (subj[i] == USER_SUBJ) {  // sink.next -> ClusterImpl.listenGossips (:213-216), not membership
          const uint64_t gid = d.slot_gid[gs[i]];
          emit_event(L, 3, (uint32_t)(gid >> 32), (uint32_t)key[i], (uint32_t)(key[i] >> 32), (uint32_t)gid);
          continue;
        }
        L.c[C_R]++;
        update_membership(L, subj[i], rec_status(key[i]), rec_inc(key[i]), R_GOSSIP, -1);
      }
    }
  }

  lap(2);  // P4
  }  // P0 - P4
  // ---- P5 timers ----
  if (L.nsub) {  // FD subscription timeouts in (cid, subscription) order
    uint32_t dcnt[SUBCAP], dkind[SUBCAP], dtgt[SUBCAP], nd = 0, w = 0, sm = NEVER;
    for (uint32_t s = 0; s < L.nsub; ++s) {
      uint32_t* S4 = L.subs + (size_t)s * 4;
      if (S4[3] == k) {
        uint32_t j = nd++;
        while (j > 0 && dcnt[j - 1] > S4[0]) {
          dcnt[j] = dcnt[j - 1];
          dkind[j] = dkind[j - 1];
          dtgt[j] = dtgt[j - 1];
          --j;
        }
        dcnt[j] = S4[0];
        dkind[j] = S4[1];
        dtgt[j] = S4[2];
      } else {
        uint32_t* D4 = L.subs + (size_t)w * 4;
        D4[0] = S4[0];
        D4[1] = S4[1];
        D4[2] = S4[2];
        D4[3] = S4[3];
        w++;
        sm = min(sm, S4[3]);
      }
    }
    L.nsub = w;
    L.smin = sm;  // (no subscription was added in this body before this pass)
    for (uint32_t q = 0; q < nd; ++q) {
      if (dkind[q] == 0)
        ping_req_step(L, dtgt[q], dcnt[q]);  // ping timeout (:159-175)
      else
        on_fd_event(L, dtgt[q], ST_SUSPECT);  // ping-req timeout (:204-212)
    }
  }
  if (L.nfetch && L.fnext <= k) {  // metadata timeouts: onErrorResume(TimeoutException) swallows the event (:568,582)
    uint32_t w = 0, fn = NEVER;
    const uint32_t nf = L.nfetch;  // no fetch is issued in P5
    for (uint32_t q = 0; q < nf; ++q) {
      uint32_t* f = L.fetch + (size_t)q * FREC;
      const uint4 lo = *(const uint4*)f, hi = *(const uint4*)(f + 4);
      uint4 h2 = hi;
      if (hi.y == k) {
        const int g = (int)hi.x;
        if (g >= 0) grp(L, g)[4]--;
        finish(L, g, false);
        do_finally(L, lo.y, lo.w & 0xFF, lo.z, (lo.w >> 8) & 0xFF);
        if ((lo.w >> 24) != 1) continue;
        // the request is still in flight (delayed past the timeout): the subject still answers it, into nothing
        h2.x = FETCH_ORPHAN;
        h2.y = NEVER;
      }
      fn = min(fn, (lo.w >> 24) != 0 ? min(h2.y, h2.z) : h2.y);
      if (w != q || h2.x != hi.x) {
        uint32_t* o = L.fetch + (size_t)w * FREC;
        *(uint4*)o = lo;
        *(uint4*)(o + 4) = h2;
      }
      w++;
    }
    L.nfetch = w;
    L.fnext = fn;
  }
  if ((L.initFlags & INIT_ACTIVE) && !(L.initFlags & INIT_RECEIVED) && k == L.initDeadline) {
    L.initFlags &= ~INIT_ACTIVE;  // .timeout(syncTimeout) (:241) -> doFinally -> schedulePeriodicSync
    L.nextSync = k + d.sync_t;
  }
  if (L.timerMin <= k) {  // suspicion timeouts (:608-618), ascending subject; lazy minimum
    uint32_t nmin = NEVER;
    // one lane scans the whole aux plane: 16-B loads, four subjects each (rows are 32-B aligned); processing
    // subject s writes only entry s, so the loaded words of the later subjects stay current
    for (uint32_t s4 = 0; s4 < L.N; s4 += 4) {
     const uint4 a4 = *(const uint4*)(L.ra + s4);
     const uint32_t av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
     for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t s = s4 + j, a = av[j];  // the aux plane alone holds the deadline
      uint32_t dl = rec_timer((uint64_t)a << 34);
      if (dl == 0 || s >= L.N) continue;
      const uint64_t v = rec_join(L.rk[s], a);
      if (dl == k) {
        L.ra[s] = aux32(rec_with_timer(v, 0));
        if (rec_status(v) != ST_ABSENT) {
          L.c[C_R]++;
          update_membership(L, s, ST_DEAD, rec_inc(v), R_TIMEOUT, -1);
        }
      } else if (dl < nmin) {
        nmin = dl;
      }
     }
    }
    L.timerMin = nmin;
  }

  lap(3);  // P5
  // ---- P6 periodic tasks (schedulePeriodically) ----
  if (k == L.nextPing) {
    L.nextPing += mc_ping_t(d, m);
    do_ping(L);
  }
  if (k == L.nextGossip) {
    L.nextGossip += d.gossip_t;
    do_spread_gossip(L);
  }
  if (k == L.nextSync) {
    L.nextSync += d.sync_t;
    do_sync(L);
  }

  lap(4);  // P6
  flush_spreads(L);
  // the next due event
  uint32_t nev = L.fnext;
  if (L.ev_ok) {  // from registers (P2, P5 and every add since)
    nev = min(nev, min(L.pmin, L.smin));
  } else {  // a resumed launch: the first four paths and subscriptions loaded together (one round trip)
    uint32_t t[8];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      t[q] = q < L.npath ? L.paths[(size_t)q * 5 + 2] : NEVER;
      t[4 + q] = q < L.nsub ? L.subs[(size_t)q * 4 + 3] : NEVER;
    }
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) nev = min(nev, t[q]);
    for (uint32_t q = 4; q < L.npath; ++q) nev = min(nev, L.paths[(size_t)q * 5 + 2]);
    for (uint32_t q = 4; q < L.nsub; ++q) nev = min(nev, L.subs[(size_t)q * 4 + 3]);
  }
  if (L.ncreq)  // the log length the block epilogue undoes from
    for (uint32_t q = 0, n = min(*L.cw_n, d.cwmax_cap); q < n; ++q)
      if (L.cw[q].x == m) L.cw[q].w = L.nlog;
  fd_ready(L);
  d.next_evt[m] = nev;
  d.tround[m] = L.tround;
  ml_store(L);
  for (int i = 0; i < 8; ++i) cnt[i] += L.c[i];
}

// ---- P4 of a parked member on one wave (k_inbox_apply) ----
// A member with many routed gossip receipts (C2: a few hundred in a tick) ran them one after another on its lane,
// each a chain of dependent loads, while 63 lanes of another member's wave waited. Here the member's receipts are taken
// 64 at a time in gossip-id order. A receipt of the common case (another member's present row, a record that is not
// DEAD) touches only its subject's row entry, the metadata-fetch list, the correlation counter and the write log, and
// on a present row isOverrides (MembershipRecord.java:66-84) is the order of the packed keys: a receipt is accepted iff
// its key is above the largest of the row's and every earlier same-subject key of the batch (a segmented prefix
// maximum). Its correlation id, fetch-list place and write-log place are prefix sums in gossip-id order, so every
// per-member sequence is the one the lane-serial P4 produces. Any other receipt (the member's own record, a DEAD
// record, an absent row, a user gossip) runs the full update on lane 0 between batches.

// one batch: lanes [0, cnt) hold common-case receipts (subject s, record s1 / i1, row entry k0 / a0 before the batch)
__device__ __forceinline__ void inbox_batch(ML& L, uint32_t lane, uint32_t cnt, uint32_t s, uint32_t s1, uint32_t i1,
                                            uint32_t k0, uint32_t a0, bool dead) {
  const Dev& d = *L.d;
  const bool act = lane < cnt;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const uint32_t kk = (i1 << 2) | s1;
  uint32_t pm = 0;  // the largest earlier key of this subject in the batch
  for (uint32_t o = 0; o < cnt; ++o) {
    const uint32_t so = __shfl(s, (int)o), ko = __shfl(kk, (int)o);
    if (o < lane && so == s) pm = max(pm, ko);
  }
  const uint32_t run = max(k0, pm);  // the subject's key just before this receipt
  const bool acc = act && kk > run;
  const unsigned long long am = __ballot(acc);
  // the accepted receipts before this one: of any subject (write log) and of this subject (suspicion timer)
  uint32_t pacc = 0, prev = L.tlast;
  bool alive_before = false, acc_before = false, acc_later = false;
  for (uint32_t o = 0; o < cnt; ++o) {
    if (!((am >> o) & 1ull)) continue;
    const uint32_t so = __shfl(s, (int)o), sto = __shfl(s1, (int)o);
    if (o < lane) {
      acc_before = true;
      prev = so;
      if (so == s) {
        pacc = sto;
        alive_before |= sto == ST_ALIVE;
      }
    } else if (o > lane && so == s) {
      acc_later = true;
    }
  }
  // scheduleSuspicionTimeoutTask (:597-606, computeIfAbsent) / cancelSuspicionTimeoutTask (:590-595) along the chain:
  // every deadline set in this tick is the same
  const uint32_t dl = L.k + suspicion_ticks(d, L.tsize, mc_ping_t(d, L.m));
  const uint64_t v0 = rec_join(k0, a0);
  const uint32_t T0 = rec_timer(v0);
  if (__ballot(acc && s1 == ST_SUSPECT && (pacc == ST_ALIVE || (pacc == 0 && T0 == 0)))) L.timerMin = min(L.timerMin, dl);
  if (acc && !acc_later) {  // the subject's last accepted record is what the row holds after the batch
    uint64_t v = (v0 & ~KEY_MASK) | rec_key(s1, i1);
    v = rec_with_timer(v, s1 == ST_SUSPECT ? ((alive_before || T0 == 0) ? dl : T0) : 0u);
    L.rk[s] = key32(v);
    L.ra[s] = aux32(v);
    if (d.rowk8) d.rowk8[lidx(d, L.m) * d.NS8 + s] = key8(key32(v));
  }
  if (act) L.c[C_R]++;
  if (acc) L.c[C_W]++;
  if (d.ackres) {  // tl_add of each accepted write, in order
    const bool flag = acc && !((L.ntl > 0 || acc_before) && prev == s);
    const unsigned long long fm = __ballot(flag);
    const uint32_t p = L.ntl + (uint32_t)__popcll(fm & lt);
    if (flag && p < TL) L.tl[p] = s;
    L.ntl = min(TL + 1u, L.ntl + (uint32_t)__popcll(fm));
    if (am) L.tlast = __shfl(s, 63 - (int)__clzll(am));
  }
  // fetchMetadata for an incarnation increase (:572-584): ids and fetch-list places in gossip-id order
  const bool fet = acc && (run >> 2) < i1;
  const unsigned long long fm = __ballot(fet);
  int e = -1;
  if (fet) {
    L.c[C_M]++;
    e = xmit_ep(d, L.ep, K_GMD_REQ, L.m, s, L.k, L.m, L.cidCnt + (uint32_t)__popcll(fm & lt), dead ? 1 : 0);
    if (e < 0) L.c[C_LOST]++;
  }
  L.cidCnt += (uint32_t)__popcll(fm);
  const bool kept = fet && e >= 0;
  const unsigned long long km = __ballot(kept);
  uint32_t fn = NEVER;
  if (kept) {
    const uint32_t q = L.nfetch + (uint32_t)__popcll(km & lt);
    if (q >= d.FCAP) {
      set_err(d, E_FETCH);
    } else {
      uint32_t* f = L.fetch + (size_t)q * FREC;
      const uint32_t cid = L.cidCnt - (uint32_t)__popcll(fm) + (uint32_t)__popcll(fm & lt);
      *(uint4*)f = make_uint4(cid, s, i1, s1 | (R_GOSSIP << 8) | (1u << 24));
      *(uint4*)(f + 4) = make_uint4(0xFFFFFFFFu, L.k + d.md_t, L.k + d.lat + (uint32_t)e, NONE32);
      fn = min(L.k + d.md_t, L.k + d.lat + (uint32_t)e);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) fn = min(fn, (uint32_t)__shfl_xor(fn, o));
  L.nfetch = min(d.FCAP, L.nfetch + (uint32_t)__popcll(km));
  L.fnext = min(L.fnext, fn);
}

// lane 0's member state to every lane of the wave (after a receipt lane 0 ran alone)
__device__ __forceinline__ void ml_bcast(ML& L) {
  L.tsize = __shfl(L.tsize, 0), L.fdLen = __shfl(L.fdLen, 0), L.gLen = __shfl(L.gLen, 0);
  L.cidCnt = __shfl(L.cidCnt, 0), L.evSeq = __shfl(L.evSeq, 0), L.held = __shfl(L.held, 0);
  L.gCounter = __shfl(L.gCounter, 0), L.timerMin = __shfl(L.timerMin, 0), L.nfetch = __shfl(L.nfetch, 0);
  L.fnext = __shfl(L.fnext, 0), L.ntl = __shfl(L.ntl, 0), L.tlast = __shfl(L.tlast, 0), L.nsp = __shfl(L.nsp, 0);
  L.npend = __shfl(L.npend, 0), L.pend = __shfl(L.pend, 0);
  const uint32_t hl = __shfl((uint32_t)L.evHash, 0), hh = __shfl((uint32_t)(L.evHash >> 32), 0);
  L.evHash = ((uint64_t)hh << 32) | hl;
}

__device__ void inbox_member(const Dev& d, uint32_t m, uint32_t k, uint32_t lane) {
  ML L;
  ml_init(L, d, m, k, nullptr, nullptr, false);  // every lane holds the member's state
  const size_t li = lidx(d, m);
  L.pend = d.hv_pend[li];
  L.tlast = d.hv_tlast[li];
  if (d.ackres && d.tl_tick[(size_t)(k & 1) * d.NL + li] == k) L.ntl = d.tl_n[(size_t)(k & 1) * d.NL + li];
  const uint32_t off = d.rc_off[m], n = d.rc_cnt[m];
  // a SYNC / SYNC_ACK of this tick still carries the live row: its snapshot, copied by the wave before the first batch
  // that may write the row (an accepted receipt's key is above the row's; lane 0's receipts may write), not before
  auto snapshot = [&]() {
    const uint32_t b = k & 1;
    uint32_t r = 0;
    if (lane == 0) r = atomicAdd(&d.arena_used[b], 1u);
    r = __shfl(r, 0);
    if (r >= d.ARENA_ROWS) {
      if (lane == 0) set_err(d, E_ARENA);
    } else {
      const uint4* src4 = (const uint4*)L.rk;
      uint4* dst4 = (uint4*)(d.arena[b] + (size_t)r * d.NS);
      for (uint32_t q = lane; q < d.NS / 4; q += 64) dst4[q] = src4[q];
      if (lane == 0)
        for (uint32_t i = L.pend; i != NEVER; i = d.msgs[b][i].pad) d.msgs[b][i].payload = r;
    }
    L.pend = NEVER;
    __threadfence_block();
  };
  for (uint32_t pos = 0; pos < n;) {
    const uint32_t j = pos + lane;
    const bool act = j < n;
    const uint32_t g = act ? d.rc_slot[off + j] : 0u;
    const uint32_t s = act ? d.slot_subj[g] : USER_SUBJ;
    const uint64_t key = act ? d.slot_key[g] : 0ull;
    const bool mem = act && s != USER_SUBJ;
    const uint32_t k0 = mem ? L.rk[s] : 0u, a0 = mem ? L.ra[s] : 0u, dt = mem ? d.dead_tick[s] : NEVER;
    const uint32_t s1 = rec_status(key), i1 = rec_inc(key);
    const bool fast = mem && s != m && (k0 & 3u) != ST_ABSENT && s1 != ST_DEAD && i1 < INC_LIMIT;
    const unsigned long long slow = __ballot(act && !fast);
    const uint32_t f = slow ? (uint32_t)__ffsll((long long)slow) - 1u : 64u;
    const uint32_t cnt = min(f, n - pos);
    if (L.pend != NEVER && __ballot((lane < cnt && key32(key) > k0) || (f < 64u && lane == f))) snapshot();
    if (cnt) inbox_batch(L, lane, cnt, s, s1, i1, k0, a0, k >= dt);
    __threadfence_block();  // the batch's row writes, before any lane reads the row again
    if (f == 64u) {
      pos += cnt;
      continue;
    }
    const uint32_t gs = __shfl(g, (int)f), ss = __shfl(s, (int)f);
    const uint32_t klo = __shfl((uint32_t)key, (int)f), khi = __shfl((uint32_t)(key >> 32), (int)f);
    const uint64_t kf = ((uint64_t)khi << 32) | klo;
    if (lane == 0) {
      if (ss == USER_SUBJ) {  // sink.next -> ClusterImpl.listenGossips (:213-216)
        const uint64_t gid = d.slot_gid[gs];
        emit_event(L, 3, (uint32_t)(gid >> 32), (uint32_t)kf, (uint32_t)(kf >> 32), (uint32_t)gid);
      } else {
        L.c[C_R]++;
        update_membership(L, ss, rec_status(kf), rec_inc(kf), R_GOSSIP, -1);
      }
    }
    ml_bcast(L);
    __threadfence_block();
    pos += f + 1;
  }
  if (lane == 0) {  // the gossips lane 0 created (refutations) take their slots; the FD list inserts land
    flush_spreads(L);
    fd_ready(L);
  }
  unsigned long long* cs = d.ctr_sh + (size_t)(blockIdx.x % CSH) * CSTRIDE;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    unsigned long long v = L.c[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)v, o), hi = __shfl_xor((uint32_t)(v >> 32), o);
      v += ((unsigned long long)hi << 32) | lo;
    }
    if (lane == 0 && v) atomicAdd(&cs[i], v);
  }
  if (lane != 0) return;
  ml_store(L);
  d.hv_pend[li] = L.pend;
  d.hv_tlast[li] = L.tlast;
  d.rc_cnt[m] = 0;  // the next receipt routing counts from zero
  d.rc_fill[m] = 0;
}

__global__ void __launch_bounds__(256) k_inbox_apply(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  const uint32_t nh = *d.nhv, lane = threadIdx.x & 63u;
  for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < nh; i += gridDim.x * 4) inbox_member(d, d.hv_list[i], k, lane);
}

// One launch per tick for member control. Each block triages its 256 members (the idle fast path, one thread per
// member, unconditional coalesced loads) and places the busy ones in an LDS list grouped by work class, each class
// starting on a wave boundary when they fit (block-local ballot prefixes, no atomics). Its waves then run the full
// control path for them: a wave holds one kind of work, so it does not serialise the latency chains of a ping, a
// ping hop and an ack arrival, and no wave runs mostly idle lanes. Counters are summed across the wave first: 10^4
// pingers per tick adding to one word would serialise on that address. With `flag` (W == 1) the block that finishes
// last runs the end-of-tick resets and raises the host flag. flag: 1 = W == 1 (end-of-tick work), 2 = a launch of a
// speculative batch.
// (MODE: BODY_FULL, or the two launches around k_inbox_apply, BODY_SPLIT and BODY_RESUME: three kernels, each with its
// own register allocation, so the steady-state one keeps the code it had before the split)
template <uint32_t MODE>
__global__ void __launch_bounds__(256, 2) k_member_tick_t(const Dev* __restrict__ dp, uint32_t k, uint32_t flag) {
  const Dev& d = *dp;  // global, not kernarg: taking its address must not copy ~1 KB into per-lane scratch
  if (flag & 2u) {  // a speculative batch halted at an earlier tick (this tick's own halt is raised while it runs)
    const uint32_t hv = *(volatile uint32_t*)d.halt;
    if (hv != 0u && hv - 1u < k) return;
  }
  // a speculative launch resets the next tick's counters at its start (nothing in this kernel uses them), so no block
  // waits for the last one at its end: the halt that tick_flag would raise is raised by the member taking a slot
  if ((flag & 3u) == 3u && blockIdx.x == 0 && threadIdx.x == 0) tick_reset(d, k);
  // SWIM_EXP & 512 (timing experiment): wall clock of each wave at entry, after triage, after its bodies, at exit
  const bool wtime = (d.exp & 512) != 0;
  unsigned long long* wt = wtime ? d.wt + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 : nullptr;
  if (wtime && (threadIdx.x & 63) == 0) wt[0] = wall_clock64();
  __shared__ uint32_t wc[4][4];  // [wave][class] busy members
  __shared__ uint32_t list[256];
  __shared__ uint4 cw[CWMAX];  // deferred copy-on-write snapshots of this block's members (cow)
  __shared__ uint32_t cw_n;
  if (threadIdx.x == 0) cw_n = 0;
  if (threadIdx.x < CWMAX) cw[threadIdx.x].x = NEVER;  // no member until written (cow scans by member)
  constexpr bool resume = MODE == BODY_RESUME;  // the parked members' P5 and P6 (one lane each, from the list)
  const uint32_t m = d.lo + blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t cls = 0, drops = 0, evs = 0;
  const bool busy = !resume && m < d.hi && member_triage(d, m, k, cls, drops, evs);
  {  // the triage's record compares and folded RUMOR events, one atomic each per wave
    uint32_t v = drops, e = evs;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o), e += __shfl_xor(e, o);
    unsigned long long* cs = d.ctr_sh + (size_t)(blockIdx.x % CSH) * CSTRIDE;
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&cs[C_R], (unsigned long long)v);
    if ((threadIdx.x & 63) == 0 && e) atomicAdd(&cs[C_E], (unsigned long long)e);
  }
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t b0 = __ballot(busy && cls == 0), b1 = __ballot(busy && cls == 1), b2 = __ballot(busy && cls == 2),
                 b3 = __ballot(busy && cls == 3);
  if (lane == 0) {
    wc[w][0] = (uint32_t)__popcll(b0);
    wc[w][1] = (uint32_t)__popcll(b1);
    wc[w][2] = (uint32_t)__popcll(b2);
    wc[w][3] = (uint32_t)__popcll(b3);
  }
  list[threadIdx.x] = NEVER;
  __syncthreads();
  uint32_t aligned = 0, dense = 0, all = 0, before = 0;
  for (uint32_t c = 0; c < 4; ++c) {
    const uint32_t t = wc[0][c] + wc[1][c] + wc[2][c] + wc[3][c];
    all += (t + 63u) & ~63u;
    if (c < cls) aligned += (t + 63u) & ~63u, dense += t;
  }
  const uint32_t start = all <= 256 ? aligned : dense;  // classes on wave boundaries when they fit, else packed
  for (uint32_t j = 0; j < w; ++j) before += wc[j][cls];
  const uint64_t bal = cls == 0 ? b0 : cls == 1 ? b1 : cls == 2 ? b2 : b3;
  uint32_t slot = start + before + __popcll(bal & ((1ull << lane) - 1ull));
  if (busy) list[slot] = m | (cls << 30);  // m < 2^30
  __syncthreads();
  uint32_t ent = list[threadIdx.x];
  if (resume) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    ent = i < *d.nhv ? d.hv_list[i] : NEVER;  // class 0
  }
  const uint32_t me = ent == NEVER ? NEVER : (ent & 0x3FFFFFFFu), mcls = ent >> 30;
  if (wtime) {  // [1]: after triage, with the wave's class mix in the top byte
    const uint64_t cm = (__ballot(me != NEVER && mcls == 0) ? 1ull : 0ull) | (__ballot(me != NEVER && mcls == 1) ? 2ull : 0ull) |
                        (__ballot(me != NEVER && mcls == 2) ? 4ull : 0ull) | (__ballot(me != NEVER && mcls == 3) ? 8ull : 0ull);
    const uint32_t nb = (uint32_t)__popcll(__ballot(me != NEVER));
    if ((threadIdx.x & 63) == 0) wt[1] = wall_clock64() | (cm << 56) | ((uint64_t)nb << 48);
  }
  // SWIM_EXP & 32 / 64 (timing experiments, wrong results): skip the bodies of class 0 / of classes 1-3
  if (__ballot(me != NEVER)) {  // waves with no busy member skip to the end
    unsigned long long cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool skip = ((d.exp & 32) && mcls == 0) || ((d.exp & 64) && mcls != 0);
    if (me != NEVER && !skip)
      member_tick_body<MODE>(d, me, k, cnt, cw, &cw_n, (flag & 3u) == 3u);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      unsigned long long v = cnt[i];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, o), hi = __shfl_xor((uint32_t)(v >> 32), o);
        v += ((unsigned long long)hi << 32) | lo;
      }
      if (lane == 0 && v) atomicAdd(&d.ctr_sh[(size_t)(blockIdx.x % CSH) * CSTRIDE + i], v);
    }
  }
  if (wtime && (threadIdx.x & 63) == 0) wt[2] = wall_clock64();
  // deferred copy-on-write: the block copies each snapshot's row (final for this tick: only its member writes it),
  // then one lane undoes the member's logged writes since the snapshot opened, newest first
  __syncthreads();
  const uint32_t ncw = min(cw_n, d.cwmax_cap);
  for (uint32_t q = 0; q < ncw; ++q) {
    const uint4 e = cw[q];
    if (e.x == NEVER) continue;  // made by its lane already (cow_now)
    const uint32_t b = k & 1;
    const size_t li = lidx(d, e.x);
    const uint4* src4 = (const uint4*)(d.rowk + li * d.NS);
    uint4* dst4 = (uint4*)(d.arena[b] + (size_t)e.y * d.NS);
    for (uint32_t s = threadIdx.x; s < d.NS / 4; s += blockDim.x) dst4[s] = src4[s];
    if (d.W > 1)
      for (uint32_t w = threadIdx.x; w < d.MW; w += blockDim.x)
        d.arena_dirty[b][(size_t)e.y * d.MW + w] = d.rdirty[li * d.MW + w];
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t* dst = d.arena[b] + (size_t)e.y * d.NS;
      const uint32_t* lg = d.ulog + li * d.ULOGC * 2;
      for (uint32_t j = e.w; j-- > e.z;) dst[lg[2 * j]] = lg[2 * j + 1];
    }
    __syncthreads();
  }
  if (wtime && (threadIdx.x & 63) == 0) wt[3] = wall_clock64();
  if ((flag & 3u) != 1u) return;
  if (!last_block_ticket(d.mdone, gridDim.x) || threadIdx.x != 0) return;
  *d.mdone = 0;
  if (resume) *d.nhv = 0;  // every block has read the list
  tick_flag(d, k);
}

template __global__ void k_member_tick_t<BODY_FULL>(const Dev* __restrict__, uint32_t, uint32_t);
template __global__ void k_member_tick_t<BODY_SPLIT>(const Dev* __restrict__, uint32_t, uint32_t);
template __global__ void k_member_tick_t<BODY_RESUME>(const Dev* __restrict__, uint32_t, uint32_t);

}  // namespace swim
