// gossip.hip — the gossip data plane: GossipProtocolImpl.doSpreadGossip (:139-157), selectGossipsToSend (:239-250),
// onGossipReq (:171-183) and sweepGossips (:283-308) for every member at once.
//
// Holder state. Per member, the held gossips are a bit row HB over slot ids and a ring of (slot, infection period)
// entries in receipt order. The infection period of an entry is the member's gossip period at its receipt
// (GossipState.infectionPeriod), so it never decreases along the ring: a round's sweep (period > infP + 2(spread+1))
// removes a prefix and the spread window (infP + spread >= period) is a suffix. The window bit row WB is rebuilt
// at each of the member's rounds from the ring entries whose status changed since its previous round (swept, left
// the window, re-entered it after the spread grew, or received since), so a round costs the entries it moves, not a
// scan of the slot table.
//
// Target-major sends. All senders of one target in a tick are evaluated by the same lane for each 64-slot group:
// the first receipts of the target are OR-ed in a register (no per-receipt atomics for deduplication), the sends are
// counted by popcount, and the target's held bits and receipt ring are updated by the lane that owns them. Loss is
// drawn per message only where the link is lossy (NetworkLinkSettings.evaluateLoss, SEMANTICS.md §2) and only for
// messages that can still be a first receipt.
//
// infectedFrom. The reference keeps a set per (holder, gossip); here `y ∈ infectedFrom_x(g)` is recomputed only for
// pairs with a logged contact (replay below). Slots are recycled at a bound after their latest creation or receipt
// by which every holder has swept them (slot_exp), so no holder count is kept.
#include "dev_util.h"

namespace swim {

// ------------------------------------------------------------------------------------------------------------
// infectedFrom without storing it. `y ∈ infectedFrom_x(g)` at x's round at tick tau holds iff y delivered g to x by
// a send in one of y's logged rounds t2 with c_x <= t2 + lat <= tau, where c_x is the creation tick of x's current
// state for g. Whether such a send was delivered depends, one level down, on whether x had delivered g to y earlier
// (then y skips x), and so on. The dependency only runs over the contact events between the pair (x's rounds that
// targeted y, y's rounds that targeted x). Those are replayed in tick order as a small dynamic program.
// pct: NetworkEmulator's loss percent of the send (link_loss at its tick: 100 for a dead receiver or a blocked link),
// rb: the sender's gossip rounds before its tick (rounds_before); both independent of the gossip, so they are evaluated
// once per pair (k_contact_cache) instead of once per replayed gossip
struct Contact {
  uint32_t tick, slot, spread, dir;  // dir 0: y -> x, 1: x -> y
  uint32_t pct, rb;
};

// the pair-level parts of a contact event: sender snd -> receiver rcv at tick t2
__device__ __forceinline__ Contact make_contact(const Dev& d, uint32_t t2, uint32_t s2, uint32_t spread, uint32_t dir,
                                                uint32_t snd, uint32_t rcv) {
  const int ep = epoch_at(d, t2);
  uint32_t pct = 100;
  if (ep < 0)
    set_err(d, E_EPOCH);  // (lost_gossip_ep's answer: the send fails)
  else
    pct = link_loss(d, ep, snd, rcv, t2);
  return Contact{t2, s2, spread, dir, pct, rounds_before(d, snd, t2)};
}

// lost_gossip_ep with the link's loss percent already known (Contact.pct)
__device__ __forceinline__ bool lost_gossip_pct(const Dev& d, uint32_t pct, uint32_t src, uint32_t k, uint32_t slot,
                                                uint64_t gid) {
  if (pct == 0) return false;
  if (pct >= 100) return true;
  const u32x4 r = philox(src, k ^ ((slot >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid, d.seed_lo ^ SALT_LOSS_GOSSIP,
                         d.seed_hi);
  return next_int(pick(r, slot & 3), 100) < pct;
}

// incarnation history of (gid, member): creation ticks of swept incarnations (rebirths are rare)
__device__ __forceinline__ uint64_t hist_tag(uint64_t gid, uint32_t member) {
  return mix64(gid ^ ((uint64_t)member * 0x9E3779B97F4A7C15ull)) | 1ull;
}

__device__ void hist_push(const Dev& d, uint64_t gid, uint32_t member, uint32_t cprev) {
  uint64_t tag = hist_tag(gid, member);
  uint32_t mask = d.HCAP - 1;
  for (uint32_t p = 0; p < d.HCAP; ++p) {
    unsigned long long* e = (unsigned long long*)(d.hist + (size_t)((tag + p) & mask) * HREC);
    unsigned long long old = atomicCAS(e, 0ull, (unsigned long long)tag);
    if (old != 0ull && old != tag) continue;
    if (old == 0ull) {
      e[1] = gid;
      e[2] = member;
      // entries in use, sampled: one entry in 8 counts 8 (grow_caps enlarges the table past half full; one counter
      // taking an atomic per rebirth would serialise the heal of a C4 storm)
      if (d.hist_n && (tag & 0x700ull) == 0) atomicAdd(d.hist_n, 8u);
    }
    uint32_t n = (uint32_t)(e[2] >> 32);  // total rebirths so far; the ring keeps the latest HKEEP
    uint32_t* c = (uint32_t*)(e + 3);
    c[n % HKEEP] = cprev;
    e[2] = (uint64_t)member | ((uint64_t)(n + 1) << 32);
    return;
  }
  if (atomicOr(d.err, E_REBORN) == 0) d.err[1] = 1;  // info 1: the history table is full (HCAP)
}

// creation tick of member's incarnation of g that existed at tick tau (NEVER if none)
__device__ uint32_t inc_at(const Dev& d, uint32_t member, uint32_t g, uint64_t gid, uint32_t tau, uint32_t ref) {
  uint32_t e = s_get(d, g, member, ref);
  if (!s_ever(e)) return NEVER;
  uint32_t c = s_ctick(e);
  if (c <= tau) return c;
  if (!(e & S_REBORN)) return NEVER;
  uint64_t tag = hist_tag(gid, member);
  uint32_t mask = d.HCAP - 1;
  for (uint32_t p = 0; p < d.HCAP; ++p) {
    const uint64_t* h = d.hist + (size_t)((tag + p) & mask) * HREC;
    if (h[0] == 0) break;
    if (h[0] != tag || h[1] != gid || (uint32_t)h[2] != member) continue;
    uint32_t n = (uint32_t)(h[2] >> 32), best = NEVER, oldest = NEVER;
    const uint32_t* cc = (const uint32_t*)(h + 3);
    uint32_t kept = n < HKEEP ? n : HKEEP;
    for (uint32_t i = 0; i < kept; ++i) {
      if (cc[i] < oldest) oldest = cc[i];
      if (cc[i] <= tau && (best == NEVER || cc[i] > best)) best = cc[i];
    }
    if (best == NEVER && n > HKEEP && tau < oldest && atomicOr(d.err, E_REBORN) == 0)
      d.err[1] = 2;  // info 2: an incarnation the ring dropped (more than HKEEP rebirths)
    return best;
  }
  return NEVER;
}

// Was x's incarnation of a gossip created at tick cs swept (sweepGossips :283-308) in one of x's rounds at ticks
// [cs, t)? The window check alone is not enough: the spread is recomputed from the gossip list every round, so a
// list that shrinks (members removed during a partition) and grows back reopens the window of a gossip already swept.
// The ring holds every round in that range: the window at t bounds t - cs to ~spread rounds, LOGW >= 4 (spread + 2).
// The ring is walked from the newest round back to cs (ring order is tick order), so the cost is the rounds since cs.
// While x's spread has not changed since cs (spchg: tick of x's latest round whose spread differs from the round
// before), the sweep condition is monotone in the round, so only the latest round before t needs a check.
__device__ bool swept_before(const Dev& d, uint32_t x, uint32_t cs, uint32_t t) {
  const uint32_t infP = rounds_before(d, x, cs);
  const uint32_t pos = d.log_pos[x], n = min(pos, d.LOGW);
  const bool steady = d.spchg[x] <= cs;
  for (uint32_t e = 1; e <= n; ++e) {
    const size_t li = (size_t)x * d.LOGW + ((pos - e) & (d.LOGW - 1u));  // LOGW is a power of two
    const uint32_t tr = d.log_tick[li];
    if (tr == NEVER || tr >= t) continue;
    if (tr < cs) break;
    if (rounds_before(d, x, tr) > infP + sweep_after(d.log_spread[li])) return true;
    if (steady) break;
  }
  return false;
}

// The replay over the sorted contact events of the pair (x, y) for gossip g (see the comment above Contact).
// oldest[0]: oldest tick in y's log, oldest[1]: in x's log (0 if that ring never wrapped).
template <uint32_t CM>
__device__ __forceinline__ bool replay_pair(const Dev& d, uint32_t x, uint32_t y, uint32_t g, uint64_t gid,
                                            uint32_t tau, uint32_t cx, const Contact* ev, uint32_t n,
                                            const uint32_t* oldest) {
  const uint32_t lat = d.lat;
  // Find which deliveries can matter: into x from cx on (the answer), and into a sender from its incarnation start
  // for every relevant event (its isInfected check). The fixpoint runs over at most CM events. The ring must cover
  // those ranges.
  uint32_t lo_in[2] = {cx, NEVER};  // [0]: deliveries into x, [1]: deliveries into y
  uint32_t cinc[CM];
  uint8_t swc[CM];  // swept_before of event i's sender: 0 not computed yet, 1 no, 2 yes (both loops ask)
  for (uint32_t i = 0; i < n; ++i) {
    cinc[i] = NEVER - 1;  // not computed yet
    swc[i] = 0;
  }
  auto swept = [&](uint32_t i, uint32_t snd, uint32_t cs) {
    if (!swc[i]) swc[i] = swept_before(d, snd, cs, ev[i].tick) ? 2 : 1;
    return swc[i] == 2;
  };
  for (int pass = 0; pass < 8; ++pass) {
    bool changed = false;
    for (int i = (int)n - 1; i >= 0; --i) {
      const Contact& c = ev[i];
      uint32_t rin = c.dir == 0 ? 0 : 1;  // receiver index into lo_in
      if (lo_in[rin] == NEVER || c.tick + lat + dmax(d) < lo_in[rin]) continue;
      if (d.dly_on && gossip_arrival(d, c.dir == 0 ? y : x, c.dir == 0 ? x : y, c.tick, c.slot, gid) < lo_in[rin]) continue;
      if (cinc[i] == NEVER - 1) cinc[i] = inc_at(d, c.dir == 0 ? y : x, g, gid, c.tick, tau + lat);
      uint32_t cs = cinc[i];
      uint32_t snd = c.dir == 0 ? y : x;
      if (cs == NEVER || rounds_before(d, snd, cs) + c.spread < c.rb) continue;
      if (swept((uint32_t)i, snd, cs)) continue;
      uint32_t sin = 1 - rin;
      if (lo_in[sin] == NEVER || cs < lo_in[sin]) {
        lo_in[sin] = cs;
        changed = true;
      }
    }
    if (!changed) break;
  }
  // deliveries into x come from y's log (oldest[0]); into y from x's log (oldest[1])
  // (oldest 0: that ring never wrapped, so it holds every round since tick 0; a delayed send arrives up to dmax
  // ticks later, so the log must reach that much further back)
  if ((lo_in[0] != NEVER && oldest[0] && lo_in[0] < oldest[0] + lat + dmax(d)) ||
      (lo_in[1] != NEVER && oldest[1] && lo_in[1] < oldest[1] + lat + dmax(d))) {
    if (atomicOr(d.err, E_LOGWIN) == 0) {
      d.err[1] = tau;
      d.err[2] = lo_in[0];
      d.err[3] = lo_in[1];
      d.err[4] = oldest[0];
      d.err[5] = oldest[1];
    }
  }
  uint32_t del[2][CM];  // arrival ticks of the delivered sends, per direction
  uint32_t nd[2] = {0, 0};
  // the answer reads only the deliveries y -> x; an x -> y delivery matters only by blocking a later y -> x send, so
  // the events after the last y -> x one change nothing
  uint32_t nlast = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (ev[i].dir == 0) nlast = i + 1;
  for (uint32_t i = 0; i < nlast; ++i) {
    const Contact& c = ev[i];
    uint32_t snd = c.dir == 0 ? y : x;
    // the sender held g at that round (its incarnation then), inside its spread window (selectGossipsToSend :246)
    uint32_t cs = cinc[i] != NEVER - 1 ? cinc[i] : inc_at(d, snd, g, gid, c.tick, tau + lat);
    if (cs == NEVER) continue;
    if (rounds_before(d, snd, cs) + c.spread < c.rb) continue;
    if (swept(i, snd, cs)) continue;  // x no longer held it
    // the receiver delivered g to the sender during that incarnation: infectedFrom (isInfected :247)
    uint32_t od = 1 - c.dir;  // opposite direction
    bool blocked = false;
    for (uint32_t q = 0; q < nd[od] && !blocked; ++q) blocked = del[od][q] >= cs && del[od][q] <= c.tick;
    if (blocked) continue;
    const uint32_t rcv = c.dir == 0 ? x : y;
    if (lost_gossip_pct(d, c.pct, snd, c.tick, c.slot, gid)) continue;
    const uint32_t at = d.dly_on ? gossip_arrival(d, snd, rcv, c.tick, c.slot, gid) : c.tick + lat;
    // a delivery depends only on earlier events: the first y -> x one inside [cx, tau] is the answer
    if (c.dir == 0 && at >= cx && at <= tau) return true;
    del[c.dir][nd[c.dir]++] = at;
  }
  for (uint32_t q = 0; q < nd[0]; ++q)
    if (del[0][q] >= cx && del[0][q] <= tau) return true;
  return false;
}

// contact events of the pair (x, y) in both logs up to tick tau - lat, in tick order; n = CM + 1 on overflow
template <uint32_t CM>
__device__ __forceinline__ uint32_t collect_contacts(const Dev& d, uint32_t x, uint32_t y, uint32_t tau, uint32_t born,
                                                     Contact* ev, uint32_t* oldest) {
  uint32_t n = 0;
  for (int side = 0; side < 2; ++side) {
    uint32_t from = side == 0 ? y : x, to = side == 0 ? x : y;
    bool wrapped = d.log_pos[from] > d.LOGW;
    uint32_t old = NEVER;
    for (uint32_t e = 0; e < d.LOGW; ++e) {
      size_t li = (size_t)from * d.LOGW + e;
      uint32_t t2 = d.log_tick[li];
      if (t2 == NEVER) continue;
      if (t2 < old) old = t2;
      if (t2 + d.lat > tau || t2 < born) continue;
      uint32_t cnt = d.log_cnt[li];
      for (uint32_t s2 = 0; s2 < cnt; ++s2)
        if (d.log_tg[li * d.F + s2] == to) {
          if (n == CM) return CM + 1;
          uint32_t j = n++;
          while (j > 0 && ev[j - 1].tick > t2) {
            ev[j] = ev[j - 1];
            --j;
          }
          ev[j] = make_contact(d, t2, s2, d.log_spread[li], (uint32_t)side, from, to);
        }
    }
    oldest[side] = wrapped ? old : 0;
  }
  return n;
}

// isInfected replay from a full scan of both logs (used when the cached contact list of the pair overflowed)
__device__ __noinline__ bool blocked_pair(const Dev& d, uint32_t x, uint32_t y, uint32_t g, uint64_t gid,
                                          uint32_t tau, uint32_t cx) {
  constexpr uint32_t CMAX = 512;  // contact events between one pair inside the log window (small clusters: many)
  Contact ev[CMAX];
  uint32_t oldest[2];
  const uint32_t n = collect_contacts<CMAX>(d, x, y, tau, d.slot_ctick[g], ev, oldest);
  if (n > CMAX) {
    atomicOr(d.err, E_CONTACTS);
    return false;
  }
  return replay_pair<CMAX>(d, x, y, g, gid, tau, cx, ev, n, oldest);
}

// isInfected replay from the pair's contact list cached by k_gossip_contacts (gossip-independent; the creation
// tick of g filters it: nobody could send g before it existed)
__device__ __forceinline__ bool blocked_pair_cached(const Dev& d, uint32_t x, uint32_t y, uint32_t g, uint64_t gid,
                                                    uint32_t tau, uint32_t cx, const uint32_t* rec) {
  const uint32_t nall = rec[0];  // <= CEV: overflowed pairs go to k_gossip_send_slow
  const uint32_t born = d.slot_ctick[g];
  // only a delivery y -> x at or after x's incarnation start cx can put y in infectedFrom_x (most cached contacts
  // are older than the gossip)
  bool relevant = false;
  for (uint32_t i = 0; i < nall; ++i) {
    const uint32_t t2 = rec[4 + 3 * i];
    relevant |= ((rec[5 + 3 * i] >> 8) & 1u) == 0 && t2 >= born && t2 + d.lat + dmax(d) >= cx;
  }
  if (!relevant) return false;
  // y never held g up to now: no send y -> x carried it (inc_at of every y -> x event is NEVER)
  if (!s_ever(s_get(d, g, y, tau + d.lat))) return false;
  Contact ev[CEV];
  uint32_t n = 0;
  for (uint32_t i = 0; i < nall; ++i) {
    const uint32_t t2 = rec[4 + 3 * i], w = rec[5 + 3 * i];
    if (t2 < born) continue;
    ev[n++] = Contact{t2, w & 0xFFu, w >> 16, (w >> 8) & 1u, (w >> 9) & 0x7Fu, rec[6 + 3 * i]};
  }
  const uint32_t oldest[2] = {rec[1], rec[2]};
  return replay_pair<CEV>(d, x, y, g, gid, tau, cx, ev, n, oldest);
}

// ------------------------------------------------------------------------------------------------------------
// 1. the active 64-slot groups of this tick in ascending order (one block: a block-wide scan over the group words),
// and the per-tick list counters
__global__ void __launch_bounds__(1024) k_gossip_groups(Dev d) {
  __shared__ uint32_t sh[1024];
  __shared__ uint32_t base;
  if (threadIdx.x == 0) {
    base = 0;
    *d.slow_n = *d.rp_n = *d.nrwl = *d.ntl = *d.xd_n = *d.nfexp = *d.nrx = *d.ncfl = *d.nsg = *d.nap = 0;
  }
  __syncthreads();
  for (uint32_t q0 = 0; q0 < d.QW; q0 += 1024) {
    const uint32_t q = q0 + threadIdx.x;
    const uint32_t f = q < d.QW && d.GU[q] != 0ull ? 1u : 0u;
    sh[threadIdx.x] = f;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
      const uint32_t v = threadIdx.x >= o ? sh[threadIdx.x - o] : 0u;
      __syncthreads();
      sh[threadIdx.x] += v;
      __syncthreads();
    }
    if (f) d.agroup[base + sh[threadIdx.x] - 1] = q;
    __syncthreads();
    if (threadIdx.x == 0) base += sh[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    d.nagroup[0] = base;
    d.nagroup[1] = base ? d.agroup[base - 1] + 1 : 0;  // span of the holder rows touched this tick
  }
}

// 2. per member with a gossip round this tick (every member on every shard: the holder state is replicated): where
// its sweep ends and its window starts in the ring (binary searches: the infection periods are sorted), and whether
// the round changes anything; the (sender, target) pairs of this shard's targets are counted per target
__global__ void __launch_bounds__(256) k_round_plan(Dev d, uint32_t k) {
  __shared__ uint32_t sh[5];
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  bool listed = false;
  if (m < d.N && d.tround[m]) {
    const uint32_t cnt = d.tcnt[m];
    for (uint32_t s = 0; s < cnt; ++s) {
      const uint32_t t = d.T[(size_t)m * d.F + s];
      if (t >= d.lo && t < d.hi) atomicAdd(&d.tin_cnt[t], 1u);
    }
    const uint32_t P = d.tperiod[m], sp = d.tspread[m];
    const int64_t slo = (int64_t)P - (int64_t)sweep_after(sp), wlo = (int64_t)P - (int64_t)sp;
    const uint32_t h = d.rhead[m], tl = d.rtail[m];
    const uint32_t* R = ring(d, m);
    const uint32_t mask = d.BCAP - 1;
    uint32_t lo = 0, hi = tl - h;  // offsets from h
    while (lo < hi) {  // first entry not swept: sweepGossips (:283-308) removes infP < P - 2 (spread + 1)
      const uint32_t mid = lo + (hi - lo) / 2;
      if (rg_period(R[(h + mid) & mask], P) < slo)
        lo = mid + 1;
      else
        hi = mid;
    }
    const uint32_t send = h + lo;
    hi = tl - h;
    while (lo < hi) {  // first entry inside the window: selectGossipsToSend (:246) keeps infP + spread >= P
      const uint32_t mid = lo + (hi - lo) / 2;
      if (rg_period(R[(h + mid) & mask], P) < wlo)
        lo = mid + 1;
      else
        hi = mid;
    }
    const uint32_t wnew = h + lo;
    listed = send != h || wnew != d.rwin[m] || d.rseen[m] != tl;
    if (listed) {
      d.rsend[m] = send;
      d.rwnew[m] = wnew;
    }
  }
  const uint32_t i = block_reserve(d.nrwl, listed ? 1u : 0u, sh);
  if (listed) d.rwl[i] = m;
}

// 3. senders of each target in one contiguous list (counting sort over this tick's pairs); the targets with senders;
// each target's ring end before this tick's receipts
__global__ void __launch_bounds__(256) k_tin_scatter(Dev d) {
  __shared__ uint32_t sh[5];
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t firsts = 0;  // bit s: this member's send s is its target's first this tick (the target is listed)
  if (m < d.N && d.tround[m]) {
    const uint32_t cnt = d.tcnt[m];
    for (uint32_t s = 0; s < cnt; ++s) {
      const uint32_t ms = m * d.F + s, t = d.T[ms];
      if (t < d.lo || t >= d.hi) continue;
      const uint32_t j = atomicAdd(&d.tin_fill[t], 1u);
      d.tin[d.tin_off[t] + j] = ms;
      if (j == 0) {
        d.rt0[t] = d.rtail[t];
        firsts |= 1u << s;  // gossip_fanout <= 8
      }
    }
  }
  uint32_t i = block_reserve(d.ntl, (uint32_t)__popc(firsts), sh);
  for (; firsts; firsts &= firsts - 1, ++i) d.tlist[i] = d.T[m * d.F + (uint32_t)(__ffs(firsts) - 1)];
}

// 4. the rounds' holder-state changes (sweepGossips :283-308 and the window of selectGossipsToSend :239-250), a
// wavefront (rows up to RCS words) or a workgroup (larger rows) per round member with work. Ring ranges (positions;
// see k_round_plan):
//   [h, send)                      swept: HB cleared, S marked SWEPT, the gossip count drops
//   [max(w0, h), min(seen, wnew))  out of the window: WB cleared (includes the swept entries that were in it)
//   [wnew, max(w0, h))             back in the window (the spread grew): WB set
//   [max(seen, wnew), tail)        received or created since the member's previous round: WB set
// Few changes (<= 64): one global atomic per entry. More: the member's HB / WB rows are staged through LDS in chunks
// of RCW words, so every word is read and written once per chunk and the bits change by LDS atomics.
constexpr uint32_t RCW = 4096;  // words per row chunk, block per member (large rows)
constexpr uint32_t RCS = 1024;  // words per row, wave per member (rows of up to 65 536 slots)

// a cooperative group of threads: one workgroup (BLOCK) or one wavefront
template <bool BLOCK>
__device__ __forceinline__ void grp_sync() {
  if (BLOCK) {
    __syncthreads();
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
}

// f(slot) for the ring entries at positions [a, b) of ring R, a group of nth threads (tid) taking every nth: four
// loads in flight per thread before their uses (a plain loop waited out each load: C2 walks ~10^4 entries per member)
template <typename F>
__device__ __forceinline__ void ring_walk(const uint32_t* R, uint32_t mask, uint32_t a, uint32_t b, uint32_t tid,
                                          uint32_t nth, F f) {
  const uint32_t n = b - a;
  uint32_t o = tid;
  for (; o + 3 * nth < n; o += 4 * nth) {
    const uint32_t g0 = R[(a + o) & mask], g1 = R[(a + o + nth) & mask], g2 = R[(a + o + 2 * nth) & mask],
                   g3 = R[(a + o + 3 * nth) & mask];
    f(g0 & RG_SLOT);
    f(g1 & RG_SLOT);
    f(g2 & RG_SLOT);
    f(g3 & RG_SLOT);
  }
  for (; o < n; o += nth) f(R[(a + o) & mask] & RG_SLOT);
}

__device__ __forceinline__ void rr_bits(const Dev& d, uint32_t m, uint32_t a, uint32_t b, uint32_t op,
                                        unsigned long long* lh, unsigned long long* lw, uint32_t c0, uint32_t c1,
                                        uint32_t tid, uint32_t nth) {
  ring_walk(ring(d, m), d.BCAP - 1, a, b, tid, nth, [&](uint32_t g) {
    const uint32_t q = g >> 6;
    const unsigned long long bit = 1ull << (g & 63u);
    if (lh) {  // LDS chunk [c0, c1) of the rows
      if (q < c0 || q >= c1) return;
      if (op == 0) atomicAnd(&lh[q - c0], ~bit);
      else if (op == 1) atomicAnd(&lw[q - c0], ~bit);
      else atomicOr(&lw[q - c0], bit);
    } else {
      if (op == 0) atomicAnd(&hrow(d, m)[q], ~bit);
      else if (op == 1) atomicAnd(&wrow(d, m)[q], ~bit);
      else atomicOr(&wrow(d, m)[q], bit);
    }
  });
}

// one round member's ring ranges (see above) by a group of nth threads; lh / lw: LDS rows of cw words
template <bool BLOCK>
__device__ void round_member(const Dev& d, uint32_t m, uint32_t k, unsigned long long* lh, unsigned long long* lw,
                             uint32_t cw, uint32_t span, uint32_t tid, uint32_t nth) {
  const uint32_t h = d.rhead[m], send = d.rsend[m], wnew = d.rwnew[m], tl = d.rtail[m], seen = d.rseen[m];
  const uint32_t w0 = (int32_t)(d.rwin[m] - h) > 0 ? d.rwin[m] : h;
  const uint32_t r2 = (int32_t)(seen - wnew) < 0 ? seen : wnew;  // min(seen, wnew)
  const uint32_t r4 = (int32_t)(seen - wnew) > 0 ? seen : wnew;  // max(seen, wnew)
  const uint32_t r3 = (int32_t)(w0 - wnew) > 0 ? w0 : wnew;      // end of the re-entry range
  // side effects of the sweeps (sweepGossips :283-308; on_sweep: a completed leave)
  ring_walk(ring(d, m), d.BCAP - 1, h, send, tid, nth, [&](uint32_t g) {
    d.S[s_idx(d, g, m)] |= S16_SWEPT;
    on_sweep(d, g, m, k);
  });
  const uint32_t nch = (send - h) + ((int32_t)(r2 - w0) > 0 ? r2 - w0 : 0u) + (r3 - wnew) + (tl - r4);
  if (nch <= d.rr_atomic || span == 0) {  // few changes: atomics on the rows
    rr_bits(d, m, h, send, 0, nullptr, nullptr, 0, 0, tid, nth);
    if ((int32_t)(r2 - w0) > 0) rr_bits(d, m, w0, r2, 1, nullptr, nullptr, 0, 0, tid, nth);
    rr_bits(d, m, wnew, r3, 2, nullptr, nullptr, 0, 0, tid, nth);
    rr_bits(d, m, r4, tl, 2, nullptr, nullptr, 0, 0, tid, nth);
  } else {
    for (uint32_t c0 = 0; c0 < span; c0 += cw) {
      const uint32_t c1 = min(span, c0 + cw);
      unsigned long long* H = hrow(d, m) + c0;
      unsigned long long* Wr = wrow(d, m) + c0;
      for (uint32_t j = tid; j < c1 - c0; j += nth) {
        lh[j] = H[j];
        lw[j] = Wr[j];
      }
      grp_sync<BLOCK>();
      rr_bits(d, m, h, send, 0, lh, lw, c0, c1, tid, nth);
      if ((int32_t)(r2 - w0) > 0) rr_bits(d, m, w0, r2, 1, lh, lw, c0, c1, tid, nth);
      rr_bits(d, m, wnew, r3, 2, lh, lw, c0, c1, tid, nth);
      rr_bits(d, m, r4, tl, 2, lh, lw, c0, c1, tid, nth);
      grp_sync<BLOCK>();
      for (uint32_t j = tid; j < c1 - c0; j += nth) {
        H[j] = lh[j];
        Wr[j] = lw[j];
      }
      grp_sync<BLOCK>();
    }
  }
  if (tid == 0) {
    d.rhead[m] = send;
    d.rwin[m] = wnew;
    d.rseen[m] = tl;
    if (send != h) {
      if (d.XW > 1)
        atomicSub(&d.held_delta[m], (int)(send - h));
      else
        atomicSub(&d.held[m], send - h);
    }
  }
}

// rows of up to cw = min(RCS, QW) words: one wavefront per round member (2 cw words of LDS each, four per workgroup,
// sized at launch: a slot table of 45 056 slots takes 11 KB per wave, so three workgroups fit a CU instead of two)
__global__ void __launch_bounds__(256) k_round_apply_w(const Dev* __restrict__ dp, uint32_t k, uint32_t cw) {
  const Dev& d = *dp;
  extern __shared__ unsigned long long lds_rows[];
  const uint32_t n = *d.nrwl, span = d.nagroup[1], wave = threadIdx.x >> 6;
  if (span > cw) return;  // k_round_apply_b
  unsigned long long* lh = lds_rows + (size_t)wave * 2 * cw;
  for (uint32_t i = blockIdx.x * 4 + wave; i < n; i += gridDim.x * 4)
    round_member<false>(d, d.rwl[i], k, lh, lh + cw, cw, span, threadIdx.x & 63u, 64u);
}

// larger rows: one workgroup per round member, the rows staged in chunks of RCW words
// (cb = min(RCW, QW): the chunk in LDS; cw: k_round_apply_w's row limit)
__global__ void __launch_bounds__(256) k_round_apply_b(const Dev* __restrict__ dp, uint32_t k, uint32_t cb, uint32_t cw) {
  const Dev& d = *dp;
  extern __shared__ unsigned long long lds_rows[];
  unsigned long long *lh = lds_rows, *lw = lds_rows + cb;
  const uint32_t n = *d.nrwl, span = d.nagroup[1];
  if (span <= cw) return;  // k_round_apply_w
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    round_member<true>(d, d.rwl[i], k, lh, lw, cb, span, threadIdx.x, blockDim.x);
    __syncthreads();
  }
}

// 5. contact lists: did target t = T[m][s] choose m in a logged round inside the look-back window? If so, cache the
// pair's contact events in both directions (independent of the gossip) for blocked_pair_cached. Eight lanes per
// (sender, target) pair of this shard's targets, eight pairs per wave: the lanes read consecutive entries of the
// target's round log for the sender (a wave per target walked its senders one after another, ~12 targets per wave at
// C3 with membership evolution; a lane per pair made every load touch 64 lines).
// The pair's contact events (collect_contacts for x = m, y = t), gathered by one wave: lanes test 64 log entries of
// one side at a time, a wave prefix sum places the hits, and lane 0 orders them by (tick, side, target slot) as the
// serial insertion does. n = CEV + 1 on overflow.
__device__ uint32_t collect_contacts_wave(const Dev& d, uint32_t m, uint32_t t, uint32_t k, uint32_t lane, Contact* ev,
                                          uint32_t* oldest) {
  uint32_t n = 0;
  for (uint32_t side = 0; side < 2; ++side) {
    const uint32_t from = side == 0 ? t : m, to = side == 0 ? m : t;
    uint32_t old = NEVER;
    for (uint32_t e0 = 0; e0 < d.LOGW; e0 += 64) {
      const uint32_t e = e0 + lane;
      uint32_t hits = 0, t2 = NEVER, sp = 0;
      if (e < d.LOGW) {
        const size_t li = (size_t)from * d.LOGW + e;
        t2 = d.log_tick[li];
        if (t2 != NEVER) {
          old = min(old, t2);
          if (t2 + d.lat <= k) {
            const uint32_t cnt = d.log_cnt[li];
            for (uint32_t s2 = 0; s2 < cnt; ++s2) hits |= (d.log_tg[li * d.F + s2] == to ? 1u : 0u) << s2;
            if (hits) sp = d.log_spread[li];
          }
        }
      }
      const uint32_t c = __popc(hits);
      uint32_t incl = c;
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      const uint32_t tot = __shfl(incl, 63);
      if (n <= CEV && n + tot <= CEV)
        for (uint32_t j = n + incl - c; hits; hits &= hits - 1, ++j)
          ev[j] = make_contact(d, t2, (uint32_t)(__ffs(hits) - 1), sp, side, from, to);
      n = min(n + tot, CEV + 1u);
    }
#pragma unroll
    for (uint32_t o = 32; o > 0; o >>= 1) old = min(old, (uint32_t)__shfl_xor(old, o));
    oldest[side] = d.log_pos[from] > d.LOGW ? old : 0u;
  }
  grp_sync<false>();  // the lanes' LDS writes, before lane 0 orders them
  if (lane == 0 && n <= CEV)
    for (uint32_t a = 1; a < n; ++a)  // insertion by (tick, side, slot): the order collect_contacts produces
      for (uint32_t b = a; b > 0; --b) {
        const Contact &p = ev[b - 1], &q = ev[b];
        if (p.tick < q.tick || (p.tick == q.tick && (p.dir < q.dir || (p.dir == q.dir && p.slot <= q.slot)))) break;
        const Contact tmp = ev[b];
        ev[b] = ev[b - 1];
        ev[b - 1] = tmp;
      }
  return n;
}

// lane 0 of the wave that gathered ev (collect_contacts_wave): the pair's cache record and its replay row
__device__ void contact_cache(const Dev& d, uint32_t i, uint32_t m, uint32_t t, uint32_t k, const Contact* ev,
                              uint32_t n, const uint32_t* oldest) {
  uint32_t* rec = d.cev + (size_t)i * CEVW;
  if (n > d.cev_cap) n = CEV + 1;  // SWIM_CAPS: a smaller cache overflows into k_gossip_send_slow
  rec[0] = n;
  rec[1] = oldest[0];
  rec[2] = oldest[1];
  uint32_t last_in = NEVER;  // latest t -> m contact (NEVER: none); overflow is flagged by n alone
  if (n <= CEV)
    for (uint32_t j = 0; j < n; ++j) {
      rec[4 + 3 * j] = ev[j].tick;
      rec[5 + 3 * j] = ev[j].slot | (ev[j].dir << 8) | (ev[j].pct << 9) | (ev[j].spread << 16);
      rec[6 + 3 * j] = ev[j].rb;
      if (ev[j].dir == 0) last_in = ev[j].tick;  // events are in tick order
    }
  rec[3] = last_in;
  // a gossip inside m's window this round was received after tick k - (spread + 1) * gossip_t, so a contact t -> m
  // that arrived at or before that tick (sent at most lat + dmax ticks earlier) can never put t in infectedFrom_m of
  // any gossip m sends now
  const int64_t horizon = (int64_t)k - (int64_t)(d.tspread[m] + 1u) * d.gossip_t;
  uint32_t ci;
  if (n > CEV)
    ci = CIN_SLOW;
  else
    ci = last_in == NEVER || (int64_t)last_in + d.lat + dmax(d) <= horizon ? NEVER : last_in;
  d.crow[i] = RX_ALL;
  if (ci != NEVER && ci != CIN_SLOW) {
    // Only gossips m received at or before the latest contact t -> m arrived (last_in + lat) can have t in
    // infectedFrom_m. Their infection periods are at most B1 = rounds_before(last_in + lat + 1); the window entries
    // of m's ring with a period above B1 were received later (sorted ring: a suffix) and are sent normally.
    const uint32_t P = d.tperiod[m], B1 = rounds_before(d, m, last_in + d.lat + dmax(d) + 1u);
    const uint32_t* R = ring(d, m);
    const uint32_t w0 = d.rwin[m], tl = d.rseen[m];  // the window as k_round_apply left it for this round
    uint32_t lo = 0, hi = tl - w0;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (rg_period(R[(w0 + mid) & (d.BCAP - 1)], P) <= (int64_t)B1)
        lo = mid + 1;
      else
        hi = mid;
    }
    if (lo == 0) {
      ci = NEVER;  // every window gossip arrived after the contact: no replay at all
    } else if (lo < tl - w0) {
      const uint32_t r = wave_append(d.nrx);
      if (r < d.CRCAP) {
        d.crow[i] = r;
        d.rxl[3 * r] = i;
        d.rxl[3 * r + 1] = w0;
        d.rxl[3 * r + 2] = w0 + lo;
      } else {
        fb_add(d, FB_RX_ALL);
      }
    }
  }
  d.cin[i] = ci;
}

// the RX rows of this tick's contact pairs: bit g set for the window gossips received no later than the contact (one
// workgroup per row, staged through LDS in chunks of at most RXW words)
constexpr uint32_t RXW = 8192;
// (cx = min(RXW, QW) words of LDS, sized at launch)
__global__ void __launch_bounds__(256) k_rx_build(const Dev* __restrict__ dp, uint32_t cx) {
  const Dev& d = *dp;
  extern __shared__ unsigned long long lr[];
  const uint32_t n = min(*d.nrx, d.CRCAP), span = d.nagroup[1];
  for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
    const uint32_t m = d.rxl[3 * r] / d.F, a = d.rxl[3 * r + 1], b = d.rxl[3 * r + 2];
    const uint32_t* R = ring(d, m);
    unsigned long long* row = d.RX + (size_t)r * d.QW;
    for (uint32_t c0 = 0; c0 < span; c0 += cx) {
      const uint32_t c1 = min(span, c0 + cx);
      for (uint32_t j = threadIdx.x; j < c1 - c0; j += blockDim.x) lr[j] = 0ull;
      __syncthreads();
      ring_walk(R, d.BCAP - 1, a, b, threadIdx.x, blockDim.x, [&](uint32_t g) {
        const uint32_t q = g >> 6;
        if (q >= c0 && q < c1) atomicOr(&lr[q - c0], 1ull << (g & 63u));
      });
      __syncthreads();
      for (uint32_t j = threadIdx.x; j < c1 - c0; j += blockDim.x) row[c0 + j] = lr[j];
      __syncthreads();
    }
  }
}

__global__ void __launch_bounds__(256) k_gossip_contacts(Dev d, uint32_t k) {
  __shared__ uint32_t sh[5];
  const uint32_t np = d.tin_off[d.N - 1] + d.tin_cnt[d.N - 1];  // this tick's (sender, target) pairs, by target
  const uint32_t sub = threadIdx.x & 7u;
  for (uint32_t j0 = blockIdx.x * 32; j0 < np; j0 += gridDim.x * 32) {  // block-uniform trip count (block_reserve)
    const uint32_t j = j0 + (threadIdx.x >> 3);
    uint32_t i = 0;
    bool hit = false;
    if (j < np) {
      i = d.tin[j];
      const uint32_t m = i / d.F, t = d.T[i];
      const uint32_t pos = d.log_pos[t], nlog = min(pos, d.LOGW);
      // Only a contact t -> m that arrived after m's window horizon can put t in infectedFrom_m (contact_cache): t's
      // rounds since then, newest first. t logs at most one round per gossip interval, so they are its last R entries.
      const int64_t cut = (int64_t)k - (int64_t)(d.tspread[m] + 1u) * d.gossip_t - d.lat - dmax(d);
      const uint32_t R = min(nlog, d.tspread[m] + 2u + (d.lat + dmax(d) + d.gossip_t - 1u) / d.gossip_t);
      for (uint32_t e = sub; e < R; e += 8) {
        const size_t lo = (size_t)t * d.LOGW + ((pos - 1u - e) & (d.LOGW - 1u));
        const uint32_t t2 = d.log_tick[lo];
        if (t2 == NEVER || t2 >= k || (int64_t)t2 <= cut) continue;
        const uint32_t n = d.log_cnt[lo];
        for (uint32_t s2 = 0; s2 < n; ++s2) hit |= d.log_tg[lo * d.F + s2] == m;
      }
    }
    // the pair's eight lanes
    uint32_t h = hit ? 1u : 0u;
    h |= __shfl_xor(h, 1);
    h |= __shfl_xor(h, 2);
    h |= __shfl_xor(h, 4);
    const bool lead = j < np && sub == 0;
    if (lead) {
      d.tcontact[i] = h;
      d.cin[i] = NEVER;
    }
    const uint32_t c = block_reserve(d.ncfl, lead && h ? 1u : 0u, sh);
    if (lead && h) d.cfl[c] = i;  // its contact events are cached by k_contact_cache
  }
}

// the flagged pairs' contact caches, one wave each: its lanes scan the two round logs 64 entries at a time
// (Dev through a pointer: the contacts' loss percents index its epoch table by a per-lane epoch, which a by-value Dev
// would copy to scratch, 2.3 KB per lane)
__global__ void __launch_bounds__(256, 8) k_contact_cache(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  __shared__ Contact sev[4][CEV];
  const uint32_t n = *d.ncfl, lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (uint32_t j = blockIdx.x * 4 + wave; j < n; j += gridDim.x * 4) {
    const uint32_t i = d.cfl[j], m = i / d.F, t = d.T[i];
    uint32_t oldest[2];
    const uint32_t ne = collect_contacts_wave(d, m, t, k, lane, sev[wave], oldest);
    if (lane == 0) contact_cache(d, i, m, t, k, sev[wave], ne, oldest);
    grp_sync<false>();  // lane 0 is done with sev before the next pair's lanes write it
  }
}

// a first receipt of (g, t) at this tick (one lane owns it): the receiver-side bookkeeping that does not depend on
// the other receipts of the tick happens at once (held bit, ring entry, DEAD-record stamp, exchange record)
__device__ __forceinline__ void receipt_mark(const Dev& d, uint32_t g, uint32_t t, uint32_t k, uint32_t pos) {
  ring(d, t)[pos & (d.BCAP - 1)] = rg_entry(g, rounds_before(d, t, k + d.lat));
  if (pos + 1u - d.rhead[t] > d.BCAP) set_err(d, E_RING);
}

// 6. target-major sends (the fast path). Work item = (target t, active group q); the lanes of a wave take 64
// consecutive items (64 groups of one target when there are that many). For each sender (m, s) of t: its window word
// (sends = popcount), and the first-receipt candidates WB & ~HB[t] (t does not hold them past this tick: the rounds'
// sweeps ran in k_round_apply), each surviving its loss draw (NetworkEmulator.tryFail, NetworkLinkSettings
// .evaluateLoss: SEMANTICS.md §2). A receipt needs one surviving send from any sender; draws of candidates another
// sender already delivered are skipped (they change nothing). Pairs with a cached contact go to k_gossip_replay and
// pairs whose contact list overflowed to k_gossip_send_slow (isInfected, :247).
__global__ void __launch_bounds__(256, 8) k_gossip_send(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  __shared__ unsigned long long red[4];
  const uint32_t nag = d.nagroup[0], ntl = *d.ntl;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t items = (uint64_t)ntl * nag;
  const int ep = epoch_at(d, k);
  if ((d.exp & 4) && blockIdx.x == 0 && threadIdx.x == 0) {  // work units: (target, group) items, their sender words
    uint64_t pairs = 0;
    for (uint32_t i = 0; i < ntl; ++i) pairs += d.tin_cnt[d.tlist[i]];
    atomicAdd(&d.ctr[C_XU], (unsigned long long)items);
    atomicAdd(&d.ctr[C_XU + 1], (unsigned long long)pairs * nag);
  }
  unsigned long long sends = 0;
  uint32_t st[4] = {0, 0, 0, 0};  // SWIM_EXP & 4: items with window bits, contact-path bits, -, candidates
  for (uint64_t i0 = ((uint64_t)blockIdx.x * 4 + wave) * 64; i0 < items; i0 += (uint64_t)gridDim.x * 256) {
    const uint64_t i = i0 + lane;
    const bool act = i < items;
    uint32_t t = NEVER, q = 0, o = 0, ns = 0;
    unsigned long long nb = 0, h = 0;
    if (act) {
      t = d.tlist[(uint32_t)(i / nag)];
      q = d.agroup[(uint32_t)(i % nag)];
      h = hrow(d, t)[q];
      o = d.tin_off[t];
      ns = d.tin_cnt[t];
    }
    // the senders loop is wave-uniform (lanes past their own target's senders idle), so the replay lists take one
    // atomic per wave
    uint32_t nsw = ns;
#pragma unroll
    for (uint32_t x = 32; x > 0; x >>= 1) nsw = max(nsw, (uint32_t)__shfl_xor(nsw, x));
    for (uint32_t p = 0; p < nsw; ++p) {
      uint32_t ms = 0, m = 0, s = 0, ci = NEVER;
      unsigned long long w = 0, wr = 0;
      if (p < ns) {
        ms = d.tin[o + p];
        m = ms / d.F;
        s = ms - m * d.F;
        w = wrow(d, m)[q];
        if (w) ci = d.cin[ms];
        if (ci != NEVER) {  // a logged contact: the gossips that can have t in infectedFrom are replayed
          const uint32_t r = ci == CIN_SLOW ? RX_ALL : d.crow[ms];
          wr = r == RX_ALL ? w : w & d.RX[(size_t)r * d.QW + q];
          w &= ~wr;
        }
      }
      if ((w | wr) && (d.exp & 4)) st[0]++;
      // (the slow path past the contact cache replays from a full scan of both round logs)
      const bool slow = ci == CIN_SLOW;
      if (__ballot(wr != 0ull)) {
        const uint32_t c = (uint32_t)__popcll(wr);
        if (d.exp & 4) st[1] += c;
        fb_add(d, slow ? FB_CEV_SLOW : FB_REPLAY, c);
        uint32_t jr = wave_reserve(d.rp_n, slow ? 0u : c), js = wave_reserve(d.slow_n, slow ? c : 0u);
        uint32_t j = slow ? js : jr;
        for (unsigned long long b = wr; b; b &= b - 1, ++j) {
          const uint64_t v = ((uint64_t)(q * 64u + (uint32_t)(__ffsll((long long)b) - 1)) << 32) | ms;
          if (j < (slow ? d.SLOWCAP : d.RPCAP))
            (slow ? d.slow : d.rp)[j] = v;
          else
            set_err(d, E_CONTACTS);
        }
      }
      if (!w) continue;
      sends += __popcll(w);
      if (d.dbg_send) {  // debugging aid: every counted send
        for (unsigned long long b = w; b; b &= b - 1) {
          const uint32_t di = atomicAdd(d.dbg_send_n, 1u);
          if (di >= d.dbg_send_cap) break;
          const uint64_t gid = d.slot_gid[q * 64u + (uint32_t)(__ffsll((long long)b) - 1)];
          uint32_t* r = d.dbg_send + (size_t)di * 5;
          r[0] = k, r[1] = m, r[2] = (uint32_t)gid, r[3] = (uint32_t)(gid >> 32), r[4] = t;
        }
      }
      const unsigned long long cand = w & ~h & ~nb;
      if (d.dly_on || d.em) {  // delays or emulator counters: the exact per-send path
        if (ep < 0) {
          set_err(d, E_EPOCH);
          continue;
        }
        if (dead_at(d, t, k)) continue;  // refused before the emulator: nothing delivered or counted
        const uint32_t ls = link_set(d, ep, m, t, k), pct = ls & 0xFFu, di = ls >> 8;
        // the counters need every send's loss outcome, and so does a delayed send to a holder: the target may sweep
        // the gossip before it arrives, and then it is a first receipt again (onGossipReq :171-183 at arrival)
        const unsigned long long drawn = (d.em || di) ? w : cand;
        unsigned long long lostm = 0;
        if (pct >= 100) {
          lostm = drawn;
        } else if (pct > 0) {
          for (unsigned long long b = drawn; b; b &= b - 1) {
            const uint32_t j = (uint32_t)(__ffsll((long long)b) - 1);
            if (next_int(gossip_loss_word(d, m, k, s, d.slot_gid[q * 64u + j]), 100) < pct) lostm |= 1ull << j;
          }
        }
        em_count(d, m, (uint32_t)__popcll(w), (uint32_t)__popcll(lostm & w));
        unsigned long long ok = cand & ~lostm;
        if (di)  // every delivered send that arrives after the next tick is queued (k_gossip_due decides at arrival)
          for (unsigned long long b = w & ~lostm; b; b &= b - 1) {
            const uint32_t j = (uint32_t)(__ffsll((long long)b) - 1), g = q * 64u + j;
            const uint32_t e = gossip_delay(d, di, m, k, s, d.slot_gid[g]);
            if (e) {
              ok &= ~(1ull << j);
              delay_push(d, g, t, k + d.lat + e);
            }
          }
        nb |= ok;
        continue;
      }
      if (!cand) continue;
      if (d.exp & 4) st[3] += (uint32_t)__popcll(cand);
      if (ep < 0) {
        set_err(d, E_EPOCH);
        continue;
      }
      const uint32_t pct = link_loss(d, ep, m, t, k);
      if (pct == 0) {
        nb |= cand;
      } else if (pct < 100) {
        for (unsigned long long b = cand; b; b &= b - 1) {
          const uint32_t j = (uint32_t)(__ffsll((long long)b) - 1);
          const uint64_t gid = d.slot_gid[q * 64u + j];
          const u32x4 r = philox(m, k ^ ((s >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid,
                                 d.seed_lo ^ SALT_LOSS_GOSSIP, d.seed_hi);  // lost_gossip_ep's draw
          if (!(next_int(pick(r, s & 3), 100) < pct)) nb |= 1ull << j;
        }
      }
    }
    // the target's receipt ring: one reservation per run of lanes with the same target
    const uint32_t c = (uint32_t)__popcll(nb);
    uint32_t incl = c;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const uint32_t tp = __shfl_up(t, 1);
    const unsigned long long heads = __ballot(lane == 0 || tp != t);
    const uint32_t head = 63u - (uint32_t)__clzll(heads & ((2ull << lane) - 1ull));  // this lane's run head
    const unsigned long long above = heads & ~((2ull << lane) - 1ull);
    const uint32_t last = above ? (uint32_t)(__ffsll((long long)above) - 2) : 63u;  // the run's last lane
    const uint32_t excl_head = __shfl(incl, (int)head) - __shfl(c, (int)head);
    const uint32_t run_total = __shfl(incl, (int)last) - excl_head;
    uint32_t base = 0;
    if (lane == head && act && run_total) base = atomicAdd(&d.rtail[t], run_total);
    base = __shfl(base, (int)head) + (incl - c - excl_head);
    if (act && nb) {
      hrow(d, t)[q] = h | nb;  // the lane owns (t, q) in this kernel: later receipts of the tick see it held
      if (nb & d.DM[q]) d.dead_rx[t] = k + d.lat;  // a DEAD membership record arrives in P4 of k + lat
      // the receipts' ring entries (receipt_mark, with the loop-invariant parts hoisted)
      const uint32_t tag = rounds_before(d, t, k + d.lat) << 22, mask = d.BCAP - 1;
      uint32_t* Rt = ring(d, t);
      if (base + c - d.rhead[t] > d.BCAP) set_err(d, E_RING);
      uint32_t pos = base;
      for (unsigned long long b = nb; b; b &= b - 1, ++pos) Rt[pos & mask] = (q * 64u + (uint32_t)(__ffsll((long long)b) - 1)) | tag;
      if (d.W > 1) {  // replicated on the other shards from exchange B
        uint32_t xi = atomicAdd(d.xd_n, c);
        for (unsigned long long b = nb; b; b &= b - 1, ++xi) {
          if (xi < d.DCAP)
            d.xd[xi] = ((uint64_t)(q * 64u + (uint32_t)(__ffsll((long long)b) - 1)) << 32) | t;
          else
            set_err(d, E_DELIV);
        }
      }
    }
  }
  if (d.exp & 4)
    for (int q2 = 0; q2 < 4; ++q2)
      if (st[q2]) atomicAdd(&d.ctr[8 + q2], (unsigned long long)st[q2]);
  for (uint32_t o = 32; o > 0; o >>= 1) sends += __shfl_xor(sends, o);
  if (lane == 0) red[wave] = sends;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long tot = red[0] + red[1] + red[2] + red[3];
    if (tot) atomicAdd(&d.ctr[C_G], tot);
  }
}

// one send of the replay / slow paths, after its isInfected check: a first receipt unless t holds g past this tick
// (or received it already this tick: the held bit), subject to the loss draw; the held bit deduplicates by atomics
__device__ __forceinline__ void deliver_one(const Dev& d, uint32_t g, uint32_t m, uint32_t s, uint32_t t, uint32_t k,
                                            uint64_t gid, int ep) {
  if (d.dbg_send) {
    uint32_t di = atomicAdd(d.dbg_send_n, 1u);
    if (di < d.dbg_send_cap) {
      uint32_t* r = d.dbg_send + (size_t)di * 5;
      r[0] = k, r[1] = m, r[2] = (uint32_t)gid, r[3] = (uint32_t)(gid >> 32), r[4] = t;
    }
  }
  unsigned long long* hw = hrow(d, t) + (g >> 6);
  const unsigned long long bit = 1ull << (g & 63u);
  if (d.dly_on || d.em) {  // the exact per-send path (see k_gossip_send)
    if (ep < 0) {
      set_err(d, E_EPOCH);
      return;
    }
    if (dead_at(d, t, k)) return;
    const uint32_t ls = link_set(d, ep, m, t, k), pct = ls & 0xFFu, di = ls >> 8;
    const bool held = (*hw & bit) != 0ull;
    if (held && !d.em && !di) return;
    const bool lost = pct >= 100 || (pct > 0 && next_int(gossip_loss_word(d, m, k, s, gid), 100) < pct);
    em_count(d, m, 1u, lost ? 1u : 0u);
    if (lost) return;
    const uint32_t e = gossip_delay(d, di, m, k, s, gid);
    if (e) {  // decided at arrival (a holder may have swept it by then): k_gossip_due
      delay_push(d, g, t, k + d.lat + e);
      return;
    }
    if (held) return;
  } else {
    if (*hw & bit) return;
    if (lost_gossip_ep(d, ep, m, t, k, s, gid)) return;
  }
  if (atomicOr(hw, bit) & bit) return;
  if (d.DM[g >> 6] & bit) d.dead_rx[t] = k + d.lat;
  receipt_mark(d, g, t, k, atomicAdd(&d.rtail[t], 1u));
  if (d.W > 1) {
    const uint32_t xi = atomicAdd(d.xd_n, 1u);
    if (xi < d.DCAP)
      d.xd[xi] = ((uint64_t)g << 32) | t;
    else
      set_err(d, E_DELIV);
  }
}

// 7a. sends of pairs with a cached contact, one thread per (slot, sender, target): the isInfected replay runs only
// where the contact can matter (t -> m at or after m's incarnation start and after the gossip existed), then the send
__global__ void __launch_bounds__(256, 8) k_gossip_replay(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  __shared__ unsigned long long red[4];
  const uint32_t n = min(*d.rp_n, d.RPCAP);
  const int ep = epoch_at(d, k);
  unsigned long long sends = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t v = d.rp[i];
    const uint32_t g = (uint32_t)(v >> 32), ms = (uint32_t)v, m = ms / d.F, s = ms % d.F;
    const uint32_t t = d.T[ms], c = s_ctick(s_get(d, g, m, k + d.lat)), ci = d.cin[ms];  // m holds g: a current entry
    const uint64_t gid = d.slot_gid[g];
    const bool maybe = ci >= d.slot_ctick[g] && ci + d.lat + dmax(d) >= c;
    if (d.exp & 4) {  // timing experiment: replay items that reach the contact replay, and those it blocks
      if (maybe) atomicAdd(&d.ctr[10], 1ull);
    }
    if (maybe && blocked_pair_cached(d, m, t, g, gid, k, c, d.cev + (size_t)ms * CEVW)) {
      if (d.exp & 4) atomicAdd(&d.ctr[12], 1ull);
      continue;
    }
    sends++;
    deliver_one(d, g, m, s, t, k, gid, ep);
  }
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (uint32_t o = 32; o > 0; o >>= 1) sends += __shfl_xor(sends, o);
  if (lane == 0) red[wave] = sends;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long tot = red[0] + red[1] + red[2] + red[3];
    if (tot) atomicAdd(&d.ctr[C_G], tot);
  }
}

// 7b. sends whose pair had more contact events than the cache holds (small clusters): full log scan + replay
__global__ void __launch_bounds__(64) k_gossip_send_slow(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  const uint32_t n = min(*d.slow_n, d.SLOWCAP);
  const int ep = epoch_at(d, k);
  unsigned long long sends = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t v = d.slow[i];
    const uint32_t g = (uint32_t)(v >> 32), ms = (uint32_t)v, m = ms / d.F, s = ms % d.F;
    const uint32_t t = d.T[ms], c = s_ctick(s_get(d, g, m, k + d.lat));
    const uint64_t gid = d.slot_gid[g];
    if (blocked_pair(d, m, t, g, gid, k, c)) continue;  // isInfected (:247)
    sends++;
    deliver_one(d, g, m, s, t, k, gid, ep);
  }
  if (sends) atomicAdd(&d.ctr[C_G], sends);
}

// 7c. delayed first-receipt candidates due in P4 of k + lat (delay_push). Targets without senders this tick join the
// target list first (their ring end before this tick's receipts: k_gossip_apply takes [rt0, rtail)), then each
// candidate is a first receipt unless the target holds the gossip by now or is dead then.
__global__ void k_gossip_due_mark(Dev d, uint32_t k) {
  const uint32_t b = (k + d.lat) % (d.EMAX + 2u), n = min(d.dq_n[b], d.DQCAP);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t t = (uint32_t)d.dq[(size_t)b * d.DQCAP + i];
    if (dead_at(d, t, k + d.lat) || d.tin_cnt[t]) continue;
    if (atomicExch(&d.dmark[t], k + 1u) != k + 1u) {
      d.rt0[t] = d.rtail[t];
      d.tlist[atomicAdd(d.ntl, 1u)] = t;
    }
  }
}
__global__ void k_gossip_due(Dev d, uint32_t k) {
  const uint32_t b = (k + d.lat) % (d.EMAX + 2u), n = min(d.dq_n[b], d.DQCAP);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t v = d.dq[(size_t)b * d.DQCAP + i];
    const uint32_t g = (uint32_t)(v >> 32), t = (uint32_t)v;
    if (dead_at(d, t, k + d.lat)) continue;
    const unsigned long long bit = 1ull << (g & 63u);
    if (atomicOr(hrow(d, t) + (g >> 6), bit) & bit) continue;  // held, or made a receipt by another delivery
    if (d.DM[g >> 6] & bit) d.dead_rx[t] = k + d.lat;
    receipt_mark(d, g, t, k, atomicAdd(&d.rtail[t], 1u));
    if (d.W > 1) {  // replicated on the other shards from exchange B
      const uint32_t xi = atomicAdd(d.xd_n, 1u);
      if (xi < d.DCAP)
        d.xd[xi] = ((uint64_t)g << 32) | t;
      else
        set_err(d, E_DELIV);
    }
  }
}
__global__ void k_dq_reset(Dev d, uint32_t k) { d.dq_n[(k + d.lat) % (d.EMAX + 2u)] = 0; }

// P4 pre-filter (onMembershipGossip -> updateMembership, MembershipProtocolImpl.java:401-408,475-485). A first
// receipt is routed to P4 of tick k4 unless it provably cannot change t's row there: its record does not override
// the row as it stands now (= at the start of tick k4), the row is present, and the row cannot be removed before the
// receipt in that tick. Present rows only move up the isOverrides order except through a removal, so a record that
// does not override the start row overrides no later one. A removal needs a DEAD record: in P4 another receipt
// (dead_rx[t] = k4, stamped by the delivering send), or in P1 a leaver's own record in SYNC data (leaving[subject]);
// after one the row is absent or re-added at any incarnation (an absent row accepts any ALIVE,
// MembershipRecord.java:67-69), so every receipt is kept then. An absent start row keeps every receipt (the row may
// become present earlier in the tick). User gossips are always routed (each one emits a GOSSIP event).
__device__ __forceinline__ bool receipt_matters(const Dev& d, uint32_t t, uint32_t g, uint32_t k4) {
  const uint32_t subj = d.slot_subj[g];
  if (subj == USER_SUBJ || (d.exp & 8)) return true;  // SWIM_EXP & 8: route every receipt (debugging aid)
  const uint64_t key = d.slot_key[g];
  const uint32_t r0 = d.rowk[lidx(d, t) * d.NS + subj], s1 = rec_status(key);
  if ((r0 & 3u) == ST_ABSENT || overrides(s1, rec_inc(key), r0 & 3u, r0 >> 2)) return true;
  return d.dead_rx[t] == k4 || d.leaving[subj];
}

// the holder-table entry of a first receipt (onGossipReq :176-180): the incarnation created at tick k + lat; a
// rebirth after a sweep keeps the swept incarnation's creation tick in the history (infectedFrom replay)
__device__ __forceinline__ void receipt_create(const Dev& d, uint32_t g, uint32_t t, uint32_t k) {
  const uint32_t e = s_get(d, g, t, k + d.lat);
  if (s_ever(e)) hist_push(d, d.slot_gid[g], t, s_ctick(e));
  s_put(d, g, t, k + d.lat, s_ever(e));
  if (d.dly_on)  // a delayed first receipt still queued may have pushed it further (delay_push)
    atomicMax(&d.slot_exp[g], k + d.lat + d.EXPB);
  else
    d.slot_exp[g] = k + d.lat + d.EXPB;  // every holder sweeps it by then (all receipts of a tick store the same value)
}

// 8. first receipts of this shard's targets: the entries each target's ring gained this tick. Holder table, expiry,
// gossip count, then membership: records that can change the row are queued for P4 of k + lat in gossip-id order
// (receipt routing), the others are counted as record compares; RUMOR mode hashes the GOSSIP events here (fastp4).
// The senders' lists are reset for the next tick. A wave takes 64 targets: those with at most APPLY_LANE new entries
// (C3 with membership evolution: one to three) on a lane each; the others (C2: a few hundred) are listed for
// k_gossip_apply_big, a wave each, so neither 63 idle lanes per target nor one lane walking hundreds of entries hold
// the launch.
constexpr uint32_t APPLY_LANE = 8;

// the target's bookkeeping once its entries are applied (one lane)
__device__ __forceinline__ void apply_target_end(const Dev& d, uint32_t t, uint32_t a, uint32_t b, uint32_t drops,
                                                 unsigned long long eh) {
  const uint32_t nr = b - a;
  // the host grows the rings before they can overflow (the atomic only when the fill beats the maximum so far:
  // one address taking an atomic from every target serialises, ~13 ns each)
  if (d.rfill && b - d.rhead[t] > __hip_atomic_load(d.rfill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(d.rfill, b - d.rhead[t]);
  if (nr) {
    if (d.XW > 1)
      atomicAdd(&d.held_delta[t], (int)nr);
    else
      atomicAdd(&d.held[t], nr);
  }
  if (drops) atomicAdd(&d.rc_ndrop[t], drops);
  if (d.fastp4 && nr) {
    atomicAdd(&d.evp_hash[t], eh);
    atomicAdd(&d.evp_n[t], nr);
  }
  d.tin_cnt[t] = 0;
  d.tin_fill[t] = 0;
}

// one entry at ring position p of target t: holder table and expiry; true if its record is routed to P4
__device__ __forceinline__ bool apply_entry(const Dev& d, uint32_t t, uint32_t g, uint32_t k, uint32_t& drops,
                                            unsigned long long& eh) {
  receipt_create(d, g, t, k);
  if (d.fastp4 && d.slot_subj[g] == USER_SUBJ) {  // RUMOR mode: the GOSSIP event of P4 (k + lat), hashed now
    const uint64_t gid = d.slot_gid[g], key = d.slot_key[g];
    const uint64_t ev = ((uint64_t)(k + d.lat) << 32) | (3ull << 30) | (uint32_t)(gid >> 32);
    const uint64_t meta = ((uint64_t)(uint32_t)key << 32) | (key >> 32);  // (oldMeta, newMeta) = payload (lo, hi)
    eh += hpair(hpair(ev, meta), (uint32_t)gid);
    return false;
  }
  if (!receipt_matters(d, t, g, k + d.lat)) {  // counted as a record compare in P4, nothing else
    drops++;
    return false;
  }
  return true;
}

__global__ void __launch_bounds__(256) k_gossip_apply(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  const uint32_t lane = threadIdx.x & 63u, ntl = *d.ntl, mask = d.BCAP - 1;
  const uint32_t nw = gridDim.x * 4;
  for (uint32_t t0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64; t0 < ntl; t0 += nw * 64) {
    const uint32_t ti = t0 + lane;
    uint32_t t = 0, a = 0, b = 0;
    if (ti < ntl) {
      t = d.tlist[ti];
      a = d.rt0[t];
      b = d.rtail[t];
    }
    const bool small = ti < ntl && b - a <= APPLY_LANE;
    // the small targets, a lane each: which entries are routed is kept as a bit per entry, then the wave reserves
    // their places in the routing list with one atomic (a per-entry append would serialise on rc_n)
    uint32_t routed = 0, drops = 0;
    unsigned long long eh = 0;
    if (small) {
      const uint32_t* R = ring(d, t);
      for (uint32_t i = 0; i < b - a; ++i)
        if (apply_entry(d, t, R[(a + i) & mask] & RG_SLOT, k, drops, eh)) routed |= 1u << i;
    }
    uint32_t ri = wave_reserve(d.rc_n, (uint32_t)__popc(routed));
    if (small) {
      const uint32_t* R = ring(d, t);
      for (uint32_t r = routed; r; r &= r - 1, ++ri) {
        const uint32_t p = a + (uint32_t)(__ffs(r) - 1);
        if (ri < d.RCAP)
          d.rc_raw[ri] = ((uint64_t)t << 32) | (R[p & mask] & RG_SLOT);
        else
          set_err(d, E_RECEIPTS);
      }
      apply_target_end(d, t, a, b, drops, eh);
    }
    // the large targets go to a list for k_gossip_apply_big (a wave each, all of them in parallel)
    const bool big = ti < ntl && !small;
    const uint32_t bi = wave_reserve(d.nap, big ? 1u : 0u);
    if (big) d.ap_list[bi] = t;
  }
}

__global__ void __launch_bounds__(256) k_gossip_apply_big(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  const uint32_t lane = threadIdx.x & 63u, n = *d.nap, mask = d.BCAP - 1;
  for (uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6); w < n; w += gridDim.x * 4) {
    const uint32_t t = d.ap_list[w], a = d.rt0[t], b = d.rtail[t];
    const uint32_t* R = ring(d, t);
    uint32_t dr = 0;
    unsigned long long h = 0;
    for (uint32_t p0 = a; p0 - a < b - a; p0 += 64u * 64u) {  // 64 entries per lane per batch
      unsigned long long rt = 0;
      // the next entry's ring load is issued before this one's holder-table and row accesses (their stores would
      // otherwise keep the compiler from hoisting it)
      uint32_t g = p0 + lane - a < b - a ? R[(p0 + lane) & mask] & RG_SLOT : 0u;
      for (uint32_t it = 0; it < 64; ++it) {
        const uint32_t p = p0 + it * 64u + lane;
        if (p - a >= b - a) break;
        const uint32_t pn = p + 64u;
        const uint32_t gn = it + 1 < 64 && pn - a < b - a ? R[pn & mask] & RG_SLOT : 0u;
        if (apply_entry(d, t, g, k, dr, h)) rt |= 1ull << it;
        g = gn;
      }
      uint32_t rj = wave_reserve(d.rc_n, (uint32_t)__popcll(rt));
      for (; rt; rt &= rt - 1, ++rj) {
        const uint32_t p = p0 + (uint32_t)(__ffsll((long long)rt) - 1) * 64u + lane;
        if (rj < d.RCAP)
          d.rc_raw[rj] = ((uint64_t)t << 32) | (R[p & mask] & RG_SLOT);
        else
          set_err(d, E_RECEIPTS);
      }
    }
    for (uint32_t o = 32; o > 0; o >>= 1) {
      dr += __shfl_xor(dr, o);
      const uint32_t lo = __shfl_xor((uint32_t)h, o), hi = __shfl_xor((uint32_t)(h >> 32), o);
      h += ((unsigned long long)hi << 32) | lo;
    }
    if (lane == 0) apply_target_end(d, t, a, b, dr, h);
  }
}

// 9. slots every holder has swept (slot_exp): nobody can send them again. Pass 1 lists them and clears their
// group bits; pass 2 returns each one to its owner shard's free list. Their holder-table entries stay: they predate
// the slot's next gossip, so s_get reads them as never held.
__global__ void k_gossip_expire(Dev d, uint32_t k) {
  const uint32_t nag = d.nagroup[0];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nag * 64u) return;
  const uint32_t q = d.agroup[i >> 6], g = q * 64u + (i & 63u);
  if (!((d.GU[q] >> (g & 63u)) & 1ull)) return;
  if (k - d.slot_ctick[g] > SLIFE) set_err(d, E_SLIFE);  // its 16-bit holder entries could alias (engine.h)
  if (d.slot_exp[g] > k) return;
  const unsigned long long bit = 1ull << (g & 63u);
  atomicAnd(&d.GU[q], ~bit);
  atomicAnd(&d.DM[q], ~bit);
  d.fexp[wave_append(d.nfexp)] = g;
}
__global__ void __launch_bounds__(256) k_gossip_free(Dev d) {
  const uint32_t n = *d.nfexp;
  for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < n; a += gridDim.x * blockDim.x) {
    const uint32_t g = d.fexp[a];
    d.slot_used[g] = 0;
    if (g / d.SPR == d.rank) d.free_list[atomicAdd(d.free_top, 1)] = g;  // back to the owning shard's free list
  }
}

// W > 1: peers' first receipts into this shard's replicated holder state (the owning shard did the membership part)
__global__ void k_unpack_b(Dev d, uint32_t k) {
  const uint32_t p = blockIdx.y;
  if (p == d.rank || (d.xb_rcnt[p] & XCNT_MASK) < 16) return;
  const uint8_t* R = d.xb_recv + (size_t)p * d.XB_PEER;
  const uint32_t nd = ((const uint32_t*)R)[0];
  const uint64_t* V = (const uint64_t*)(R + 16);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nd; i += gridDim.x * blockDim.x) {
    const uint32_t g = (uint32_t)(V[i] >> 32), t = (uint32_t)V[i];
    if (t & XD_EXT) {  // a peer's delayed send keeps the slot (delay_push)
      atomicMax(&d.slot_exp[g], (t & ~XD_EXT) + d.EXPB);
      continue;
    }
    atomicOr(&hrow(d, t)[g >> 6], 1ull << (g & 63u));
    const uint32_t pos = atomicAdd(&d.rtail[t], 1u);
    receipt_mark(d, g, t, k, pos);
    receipt_create(d, g, t, k);
    atomicAdd(&d.held[t], 1u);
    // the ring fill for grow_caps_shard (an atomic only on a new maximum)
    if (d.rfill && pos + 1u - d.rhead[t] > __hip_atomic_load(d.rfill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(d.rfill, pos + 1u - d.rhead[t]);
  }
}

// ------------------------------------------------------------------------------------------------------------
// host launchers
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
void launch_scan(const uint32_t* in, uint32_t* out, uint32_t* part, uint32_t n, hipStream_t st);  // kernels.hip
void launch_receipt_routing(const Dev& d, hipStream_t st);                                         // kernels.hip

constexpr uint32_t SEND_GRID = 4096;  // 16 blocks per CU, grid-stride

// the sends of this tick and the holder-state changes they need, up to the first receipts (the sharded tick
// exchanges them before launch_gossip_apply)
void launch_gossip_send(const Dev& d, uint32_t k, hipStream_t st, const TickEvents* prof) {
  hipLaunchKernelGGL(k_gossip_groups, dim3(1), dim3(1024), 0, st, d);
  hipLaunchKernelGGL(k_round_plan, dim3(cdiv(d.N, 256)), dim3(256), 0, st, d, k);
  launch_scan(d.tin_cnt, d.tin_off, d.scan_part, d.N, st);
  hipLaunchKernelGGL(k_tin_scatter, dim3(cdiv(d.N, 256)), dim3(256), 0, st, d);
  {  // LDS rows sized by the slot table (the active span never exceeds QW words)
    const uint32_t cw = std::min<uint32_t>(RCS, d.QW), cb = std::min<uint32_t>(RCW, d.QW);
    hipLaunchKernelGGL(k_round_apply_w, dim3(4096), dim3(256), 4 * 2 * 8 * cw, st, d.self, k, cw);
    hipLaunchKernelGGL(k_round_apply_b, dim3(2048), dim3(256), 2 * 8 * cb, st, d.self, k, cb, cw);
  }
  hipLaunchKernelGGL(k_gossip_contacts, dim3(2048), dim3(256), 0, st, d, k);
  hipLaunchKernelGGL(k_contact_cache, dim3(1024), dim3(256), 0, st, d.self, k);
  {
    const uint32_t cx = std::min<uint32_t>(RXW, d.QW);
    hipLaunchKernelGGL(k_rx_build, dim3(512), dim3(256), 8 * cx, st, d.self, cx);
  }
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[4], st);
  hipLaunchKernelGGL(k_gossip_send, dim3(SEND_GRID), dim3(256), 0, st, d.self, k);
  hipLaunchKernelGGL(k_gossip_send_slow, dim3(64), dim3(64), 0, st, d.self, k);  // rare; ~14 KB of stack per lane
  hipLaunchKernelGGL(k_gossip_replay, dim3(2048), dim3(256), 0, st, d.self, k);
  if (d.dly_on) {
    hipLaunchKernelGGL(k_gossip_due_mark, dim3(256), dim3(256), 0, st, d, k);
    hipLaunchKernelGGL(k_gossip_due, dim3(256), dim3(256), 0, st, d, k);
    hipLaunchKernelGGL(k_dq_reset, dim3(1), dim3(1), 0, st, d, k);
  }
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[5], st);
}

// the receivers' side of this tick's first receipts, P4 routing and slot recycling
void launch_gossip_apply(const Dev& d, uint32_t k, hipStream_t st) {
  hipLaunchKernelGGL(k_gossip_apply, dim3(2048), dim3(256), 0, st, d.self, k);
  hipLaunchKernelGGL(k_gossip_apply_big, dim3(2048), dim3(256), 0, st, d.self, k);
  launch_receipt_routing(d, st);
  hipLaunchKernelGGL(k_gossip_expire, dim3(cdiv((uint64_t)d.QW * 64, 256)), dim3(256), 0, st, d, k);
  hipLaunchKernelGGL(k_gossip_free, dim3(1024), dim3(256), 0, st, d);
}

void launch_unpack_b(const Dev& d, uint32_t k, hipStream_t st) {
  hipLaunchKernelGGL(k_unpack_b, dim3(64, d.W), dim3(256), 0, st, d, k);
}

}  // namespace swim

namespace swim {
// capacity growth (api.hip grow_caps): member m's held ring entries [rhead, rtail) at their positions in a ring of B2
// entries (positions are absolute; a ring of B entries keeps position p at p & (B - 1))
__global__ void __launch_bounds__(256) k_ring_move(const uint32_t* rg, uint32_t* rg2, const uint32_t* rhead,
                                                   const uint32_t* rtail, uint32_t N, uint32_t B, uint32_t B2) {
  for (uint32_t m = blockIdx.x; m < N; m += gridDim.x) {
    const uint32_t h = rhead[m], t = rtail[m];
    for (uint32_t p = h + threadIdx.x; p - h < t - h; p += blockDim.x)
      rg2[(size_t)m * B2 + (p & (B2 - 1))] = rg[(size_t)m * B + (p & (B - 1))];
  }
}
void launch_ring_move(const uint32_t* rg, uint32_t* rg2, const uint32_t* rhead, const uint32_t* rtail, uint32_t N,
                      uint32_t B, uint32_t B2, void* stream) {
  hipLaunchKernelGGL(k_ring_move, dim3(4096), dim3(256), 0, (hipStream_t)stream, rg, rg2, rhead, rtail, N, B, B2);
}

// capacity growth: every entry of the incarnation history re-inserted into a table of cap2 entries (same probing as
// hist_push: linear from its tag)
__global__ void __launch_bounds__(256) k_hist_rehash(const uint64_t* h1, uint32_t cap1, uint64_t* h2, uint32_t cap2) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < cap1; i += gridDim.x * blockDim.x) {
    const uint64_t* e = h1 + (size_t)i * HREC;
    const uint64_t tag = e[0];
    if (!tag) continue;
    for (uint32_t p = 0; p < cap2; ++p) {
      unsigned long long* o = (unsigned long long*)(h2 + (size_t)((tag + p) & (cap2 - 1)) * HREC);
      if (atomicCAS(o, 0ull, (unsigned long long)tag) != 0ull) continue;
      for (uint32_t j = 1; j < HREC; ++j) o[j] = e[j];
      break;
    }
  }
}
void launch_hist_rehash(const uint64_t* h1, uint32_t cap1, uint64_t* h2, uint32_t cap2, void* stream) {
  hipLaunchKernelGGL(k_hist_rehash, dim3(2048), dim3(256), 0, (hipStream_t)stream, h1, cap1, h2, cap2);
}

// test surface (swim_debug_holders): per member of [first, first + n): its gossip count, the receipt-ring positions of
// the first held entry and of the end, the popcount of its held-bit row, and the first receipts whose GOSSIP events the
// next P4 folds (RUMOR mode without recorded events)
__global__ void __launch_bounds__(256) k_dbg_holders(const Dev* __restrict__ dp, uint32_t first, uint32_t n, uint32_t* out) {
  const Dev& d = *dp;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t m = first + i;
    const unsigned long long* hb = d.HB + (size_t)m * d.QW;
    uint32_t pop = 0;
    for (uint32_t w = 0; w < d.QW; ++w) pop += (uint32_t)__popcll(hb[w]);
    uint32_t* o = out + 5ull * i;
    o[0] = d.held[m];
    o[1] = d.rhead[m];
    o[2] = d.rtail[m];
    o[3] = pop;
    o[4] = d.evp_n ? d.evp_n[m] : 0u;
  }
}
void launch_dbg_holders(const Dev& d, uint32_t first, uint32_t n, uint32_t* out, void* stream) {
  hipLaunchKernelGGL(k_dbg_holders, dim3(std::min<uint32_t>(4096, (n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     d.self, first, n, out);
}
}  // namespace swim
