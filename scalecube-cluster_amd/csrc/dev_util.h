// dev_util.h — device helpers shared by the member, SYNC and gossip kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"

namespace swim {

__device__ __forceinline__ void set_err(const Dev& d, uint32_t bit) { atomicOr(d.err, bit); }

// a capacity fallback fired (engine.h Fb), when the handle counts them
__device__ __forceinline__ void fb_add(const Dev& d, uint32_t i, unsigned long long n = 1) {
  if (d.fb && n) atomicAdd(&d.fb[i], n);
}

// The workgroup that finishes last on `ctr` (nblocks workgroups) sees every other workgroup's plain stores. The
// hand-off of MI355X_MICROARCH.md / cdna_hip_programming.md §6 Guideline 16 (counter form): every wave drains its
// stores, then one lane releases at agent scope (write-back of its XCD's L2) and draws a ticket; the last one acquires
// (invalidates its CU's L1) before any wave of it loads. Without the per-wave drain and the explicit waits, a
// producer on another XCD can still hold its stores in L2 when the last workgroup reads them (ROCm 7.2 may also drop
// the fence's own wait).
__device__ __forceinline__ bool last_block(uint32_t* ctr, uint32_t nblocks) {
  __shared__ bool last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return last;
}

// ticket only, no release / acquire: for a last block that reads nothing the other blocks stored with plain stores
// (k_member_tick: tick_flag reads free_top by an atomic load). A release per block writes back its XCD's L2, which
// the waves still running there then pay for.
__device__ __forceinline__ bool last_block_ticket(uint32_t* ctr, uint32_t nblocks) {
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblocks - 1u;
  __syncthreads();
  return last;
}

// 16-B row loads
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld_c4(const uint32_t* p) { return *(const uint4*)p; }

// settings epoch in force at tick k (the latest epoch that started at or before k)
__device__ __forceinline__ int epoch_at(const Dev& d, uint32_t k) {
  int best = -1;
  uint32_t bf = 0;
  for (int e = 0; e < (int)MAX_EPOCHS; ++e) {
    uint32_t f = d.ep_from[e];
    if (f != NEVER && f <= k && (best < 0 || f >= bf)) {
      best = e;
      bf = f;
    }
  }
  return best;
}

__device__ __forceinline__ bool dead_at(const Dev& d, uint32_t x, uint32_t k) { return k >= d.dead_tick[x]; }

// member m's own FailureDetectorConfig and syncGroup (swim_set_member_config), else the handle's
__device__ __forceinline__ uint32_t mc_ping_t(const Dev& d, uint32_t m) { return d.permember ? d.mcfg[4 * m] : d.ping_t; }
__device__ __forceinline__ uint32_t mc_timeout_t(const Dev& d, uint32_t m) {
  return d.permember ? d.mcfg[4 * m + 1] : d.pingTimeout_t;
}
__device__ __forceinline__ uint32_t mc_kreq(const Dev& d, uint32_t m) { return d.permember ? d.mcfg[4 * m + 2] : d.kreq; }
__device__ __forceinline__ uint32_t mc_group(const Dev& d, uint32_t m) { return d.permember ? d.mcfg[4 * m + 3] : 0u; }

// NetworkEmulator.getLinkSettings (:57-59): the custom setting of link src -> dst in force at tick k, or -1
__device__ __noinline__ int link_loss_at(const Dev& d, uint32_t src, uint32_t dst, uint32_t k) {
  const uint64_t key = (((uint64_t)src << 32) | dst) + 1ull;
  for (uint32_t p = 0, h = (uint32_t)mix64(key) & (LKCAP - 1); p < LKCAP; ++p, h = (h + 1) & (LKCAP - 1)) {
    const uint64_t kk = d.link_key[h];
    if (kk == 0) return -1;
    if (kk != key) continue;
    const uint32_t* e = d.link_hist + (size_t)h * LKH * 2;
    int best = -2;
    for (uint32_t i = 0; i < LKH; ++i) {
      const uint32_t from = (i == 0 ? e[0] & ~LK_TRUNC : e[2 * i]), v = e[2 * i + 1];
      if (from == LK_NONE || from > k) break;
      best = v == LK_NONE ? -1 : (int)v;
    }
    if (best == -2) {
      if (e[0] & LK_TRUNC) set_err(d, E_LINKHIST);
      return -1;
    }
    return best;
  }
  return -1;
}

// NetworkEmulator.getLinkSettings (:57-59) of link src -> dst at tick k: its custom setting if it has one (block =
// 100 %), else the partition block (DEAD_LINK_SETTINGS, no delay) and the default settings. Returns loss % | delay
// index << 8.
__device__ __forceinline__ uint32_t link_set(const Dev& d, int ep, uint32_t src, uint32_t dst, uint32_t k) {
  if (d.link_n) {
    const int lp = link_loss_at(d, src, dst, k);
    if (lp >= 0) return (uint32_t)lp;
  }
  if (d.ep_part[ep] && d.ep_group[(size_t)ep * d.N + src] != d.ep_group[(size_t)ep * d.N + dst]) return 100;
  return d.ep_loss[ep] | (d.ep_delay[ep] << 8);
}

// NetworkEmulator.tryFail (transport/.../NetworkEmulator.java:231-248) at the sender, evaluated for tick k: a dead
// destination fails the send; then the link's loss. Returns the loss percent to draw against, or 100 for a certain
// failure.
__device__ __forceinline__ uint32_t link_loss(const Dev& d, int ep, uint32_t src, uint32_t dst, uint32_t k) {
  if (dead_at(d, dst, k)) return 100;
  return link_set(d, ep, src, dst, k) & 0xFFu;
}

// the delay in ticks past lat of a message whose delay draw is x, on a link with delay index di (SEMANTICS.md §2)
__device__ __forceinline__ uint32_t delay_ticks(const Dev& d, uint32_t di, uint32_t x) {
  const uint32_t* t = d.dly_thr + (size_t)di * 256;
  uint32_t lo = 0, hi = d.dly_len[di];
  while (lo < hi) {  // thresholds ascend: count those <= x
    const uint32_t mid = (lo + hi) >> 1;
    if (t[mid] <= x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// this member's emulator counters (NetworkEmulator.java:200-222, 231-272): tryFail counts every send that reaches the
// emulator, tryDelay every one that survived it
__device__ __forceinline__ void em_count(const Dev& d, uint32_t src, uint32_t sent, uint32_t lost) {
  if (!d.em) return;
  if (sent) atomicAdd(&d.em[2 * src], 2ull * sent - lost);
  if (lost) atomicAdd(&d.em[2 * src + 1], (unsigned long long)lost);
}

// the delay draw of one non-gossip message on a link with delay index di > 0 (out of line: the member kernel inlines
// xmit_ep at every FD / SYNC / metadata send, and the delay path only runs with link delays set)
__device__ __noinline__ int xmit_delay(const Dev& d, uint32_t di, uint32_t kind, uint32_t src, uint32_t dst, uint32_t k,
                                       uint32_t aux, uint32_t id) {
  return (int)delay_ticks(d, di, delay_draw(d.seed_lo, d.seed_hi, kind, src, dst, k, aux, id));
}

// tryFail + tryDelay of one non-gossip message: -1 if the send fails, else its delay in ticks past lat. dd: whether
// dst is dead at k when the caller loaded it already (-1: look it up)
__device__ __forceinline__ int xmit_ep(const Dev& d, int ep, uint32_t kind, uint32_t src, uint32_t dst, uint32_t k,
                                       uint32_t aux, uint32_t id, int dd = -1) {
  if (ep < 0) {
    set_err(d, E_EPOCH);
    return -1;
  }
  if (dd < 0 ? dead_at(d, dst, k) : dd != 0) return -1;  // connection refused: fails before the emulator, not counted
  const uint32_t ls = link_set(d, ep, src, dst, k), loss = ls & 0xFFu, di = ls >> 8;
  const bool lost = loss >= 100 || (loss > 0 && loss_roll(d.seed_lo, d.seed_hi, kind, src, dst, k, aux, id) < loss);
  em_count(d, src, 1u, lost ? 1u : 0u);
  if (lost) return -1;
  if (di == 0) return 0;
  return xmit_delay(d, di, kind, src, dst, k, aux, id);
}

// the gossip-send draw words (LOSS_GOSSIP, DELAY_GOSSIP: SEMANTICS.md §2) of gossip gid sent by src to target slot s
__device__ __forceinline__ uint32_t gossip_loss_word(const Dev& d, uint32_t src, uint32_t k, uint32_t s, uint64_t gid) {
  return pick(philox(src, k ^ ((s >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid, d.seed_lo ^ SALT_LOSS_GOSSIP,
                     d.seed_hi), s & 3);
}
__device__ __forceinline__ uint32_t gossip_delay(const Dev& d, uint32_t di, uint32_t src, uint32_t k, uint32_t s,
                                                 uint64_t gid) {
  if (di == 0) return 0;
  return delay_ticks(d, di, pick(philox(src, k ^ ((s >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid,
                                        d.seed_lo ^ SALT_DELAY_GOSSIP, d.seed_hi), s & 3));
}

// the arrival tick of a gossip send (delay only, not loss): tick + lat + its delay under the settings of that tick
__device__ __forceinline__ uint32_t gossip_arrival(const Dev& d, uint32_t src, uint32_t dst, uint32_t tick, uint32_t s,
                                                   uint64_t gid) {
  const uint32_t a = tick + d.lat;
  if (!d.dly_on) return a;
  const int ep = epoch_at(d, tick);
  if (ep < 0) return a;
  return a + gossip_delay(d, link_set(d, ep, src, dst, tick) >> 8, src, tick, s, gid);
}
// the latest a send can arrive past tick + lat
__device__ __forceinline__ uint32_t dmax(const Dev& d) { return d.dly_on ? d.EMAX : 0u; }

// a first-receipt candidate delayed past the next tick: queued by its delivery tick (k_gossip_due delivers it then);
// its slot lives until every holder it makes has swept it
__device__ __forceinline__ void delay_push(const Dev& d, uint32_t g, uint32_t t, uint32_t due) {
  const uint32_t b = due % (d.EMAX + 2u), j = atomicAdd(&d.dq_n[b], 1u);
  if (j < d.DQCAP)
    d.dq[(size_t)b * d.DQCAP + j] = ((uint64_t)g << 32) | t;
  else
    set_err(d, E_DELAYQ);
  atomicMax(&d.slot_exp[g], due + d.EXPB);
  if (d.W > 1) {  // the other shards extend the slot's life the same way (exchange B: XD_EXT record, k_unpack_b)
    const uint32_t xi = atomicAdd(d.xd_n, 1u);
    if (xi < d.DCAP)
      d.xd[xi] = ((uint64_t)g << 32) | XD_EXT | due;
    else
      set_err(d, E_DELIV);
  }
}

// the same with the settings epoch of tick k already looked up (epoch_at once per thread, not per message)
__device__ __forceinline__ bool lost_msg_ep(const Dev& d, int ep, uint32_t kind, uint32_t src, uint32_t dst,
                                            uint32_t k, uint32_t aux, uint32_t id) {
  if (ep < 0) {
    set_err(d, E_EPOCH);
    return true;
  }
  uint32_t loss = link_loss(d, ep, src, dst, k);
  if (loss == 0) return false;
  if (loss >= 100) return true;
  return loss_roll(d.seed_lo, d.seed_hi, kind, src, dst, k, aux, id) < loss;
}
__device__ __forceinline__ bool lost_msg(const Dev& d, uint32_t kind, uint32_t src, uint32_t dst, uint32_t k,
                                         uint32_t aux, uint32_t id) {
  int ep = epoch_at(d, k);
  if (ep < 0) {
    set_err(d, E_EPOCH);
    return true;
  }
  uint32_t loss = link_loss(d, ep, src, dst, k);
  if (loss == 0) return false;
  if (loss >= 100) return true;
  return loss_roll(d.seed_lo, d.seed_hi, kind, src, dst, k, aux, id) < loss;
}

__device__ __forceinline__ bool lost_gossip_ep(const Dev& d, int ep, uint32_t src, uint32_t dst, uint32_t k,
                                               uint32_t slot, uint64_t gid) {
  if (ep < 0) {
    set_err(d, E_EPOCH);
    return true;
  }
  uint32_t loss = link_loss(d, ep, src, dst, k);
  if (loss == 0) return false;
  if (loss >= 100) return true;
  u32x4 r = philox(src, k ^ ((slot >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid, d.seed_lo ^ SALT_LOSS_GOSSIP,
                   d.seed_hi);
  return next_int(pick(r, slot & 3), 100) < loss;
}
__device__ __forceinline__ bool lost_gossip(const Dev& d, uint32_t src, uint32_t dst, uint32_t k, uint32_t slot,
                                            uint64_t gid) {
  return lost_gossip_ep(d, epoch_at(d, k), src, dst, k, slot, gid);
}

// wave-aggregated append: the active lanes that call it together reserve consecutive indices with ONE atomic on
// the shared counter (a hot single-address atomic per lane serialises at L2 under C2's receipt storms)
__device__ __forceinline__ uint32_t wave_append(uint32_t* ctr) {
  const uint64_t mask = __ballot(1);
  const uint32_t lane = __lane_id();
  const uint32_t leader = (uint32_t)__ffsll((unsigned long long)mask) - 1u;
  const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(mask));
  base = __shfl(base, (int)leader);
  return base + rank;
}

// reserve n entries per lane on a shared counter with ONE atomic per wave; every lane of the wave must call it
// (inactive work passes n = 0). Returns the lane's first index.
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* ctr, uint32_t n) {
  const uint32_t lane = __lane_id();
  uint32_t incl = n;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const uint32_t total = __shfl(incl, 63);
  uint32_t base = 0;
  if (lane == 0 && total) base = atomicAdd(ctr, total);
  return __shfl(base, 0) + incl - n;
}

// reserve n entries per thread with ONE atomic per workgroup of 256; every thread of the block must call it (sh: 5
// words of LDS). A list built by a per-member kernel over 10^5 members took one atomic per wave on one address,
// ~1 500 of them queued at its L2 channel (~13 ns each)
__device__ __forceinline__ uint32_t block_reserve(uint32_t* ctr, uint32_t n, uint32_t* sh) {
  const uint32_t lane = __lane_id(), wv = threadIdx.x >> 6;
  uint32_t incl = n;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) sh[wv] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t tot = sh[0] + sh[1] + sh[2] + sh[3];
    sh[4] = tot ? atomicAdd(ctr, tot) : 0u;
  }
  __syncthreads();
  uint32_t before = sh[4];
  for (uint32_t w = 0; w < wv; ++w) before += sh[w];
  __syncthreads();  // sh may be reused by the caller
  return before + incl - n;
}

// A receiver with several SYNC / SYNC_ACK payloads in one tick reads the later ones' records for the subjects an
// earlier one changed (member.hip, merge_payload), after their senders may have written their live rows again:
// such a live-row payload gets an arena row that k_sync_diff fills with its keys. A lost CAS race wastes a row.
__device__ __forceinline__ void pin_msg(const Dev& d, uint32_t b, uint32_t j) {
  uint32_t* p = &d.msgs[b][j].pin;
  if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != NEVER) return;
  const uint32_t r = atomicAdd(&d.arena_used[b], 1u);
  if (r >= d.ARENA_ROWS) {
    set_err(d, E_ARENA);
    return;
  }
  atomicCAS(p, NEVER, r);
}

// key32 of subject s in payload mm (messages of buffer b): its copy-on-write snapshot, its pinned copy, or a
// payload received from another shard (shipped chunk or baseline row). Only for payloads that are immutable now.
__device__ __forceinline__ uint32_t payload_key_at(const Dev& d, const SyncMsg& mm, uint32_t b, uint32_t s) {
  if (mm.payload == NEVER) {
    if (mm.pin == NEVER) {
      set_err(d, E_PIN);
      return 0;
    }
    return d.arena[b][(size_t)mm.pin * d.NS + s];
  }
  if (mm.payload & PAY_RX) {
    const uint32_t ri = mm.payload & ~PAY_RX, c = s / CH;
    const uint64_t* mk = d.rx_mask + (size_t)ri * d.MW;
    if (!((mk[c >> 6] >> (c & 63)) & 1ull)) return d.base_row[s];
    uint32_t rank = __popcll(mk[c >> 6] & ((1ull << (c & 63)) - 1ull));
    for (uint32_t q = 0; q < (c >> 6); ++q) rank += __popcll(mk[q]);
    return ((const uint32_t*)(d.xa_recv + d.rx_off[ri]))[(size_t)rank * CH + s % CH];
  }
  return d.arena[b][(size_t)mm.payload * d.NS + s];
}

// (c - f + gossip_t - 1) / gossip_t without an integer division (~35 instructions for a runtime divisor; the infectedFrom
// replay evaluates this several times per replayed gossip): q = umulhi(x, floor(2^32 / gt)) is floor(x / gt) or one less
__device__ __forceinline__ uint32_t div_gt(const Dev& d, uint32_t x) {
  uint32_t q = __umulhi(x, d.gt_mul);
  q += x - q * d.gossip_t >= d.gossip_t ? 1u : 0u;
  return q;
}
__device__ __forceinline__ uint32_t rounds_before(const Dev& d, uint32_t x, uint32_t c) {
  uint32_t f = d.firstGossip[x];
  if (f == NEVER || c <= f) return 0;
  return div_gt(d, c - f + d.gossip_t - 1);
}

// ClusterMath (ClusterMath.java:99-125): gossipPeriodsToSpread, gossipPeriodsToSweep (from the spread), and
// suspicionTimeout in ticks; swim_selftest_eval exposes these exact functions for the known-answer tests
__device__ __forceinline__ uint32_t spread_of(const Dev& d, uint32_t cluster) { return d.repeatMult * bitlen(cluster); }
__device__ __forceinline__ uint32_t sweep_after(uint32_t spread) { return 2u * (spread + 1u); }
__device__ __forceinline__ uint32_t suspicion_ticks(const Dev& d, uint32_t size, uint32_t ping_t) {
  return d.suspMult * bitlen(size) * ping_t;  // the member's own pingInterval (mc_ping_t)
}

// member m swept gossip slot g at tick k: if g is m's own leave notification, leaveCluster completes and
// ClusterImpl.doShutdown stops the member (ClusterImpl.java:305-313, GossipProtocolImpl.java:296-306): it is dead
// from tick k + 1
__device__ __forceinline__ void on_sweep(const Dev& d, uint32_t g, uint32_t m, uint32_t k) {
  if ((uint32_t)(d.slot_gid[g] >> 32) != m || d.slot_subj[g] != m || rec_status(d.slot_key[g]) != ST_DEAD) return;
  d.dead_tick[m] = k + 1u;
}

// S entries: creation tick + 1 (0 = never held), SWEPT, REBORN
__device__ __forceinline__ uint32_t s_ctick(uint32_t e) { return (e & S_TICK_MASK) - 1u; }
__device__ __forceinline__ bool s_ever(uint32_t e) { return (e & S_TICK_MASK) != 0; }
__device__ __forceinline__ bool s_held(uint32_t e) { return (e & S_TICK_MASK) != 0 && !(e & S_SWEPT); }
// S is member-major ([N][SLOTS]): one member's entries for the 64 slots of a group share two cache lines, so the
// receipts of one target (k_gossip_apply) and the sweeps of one member touch few lines
__device__ __forceinline__ size_t s_idx(const Dev& d, uint32_t g, uint32_t m) { return (size_t)m * d.SLOTS + g; }
// member m's entry for slot g in the 32-bit form (creation tick + 1 | SWEPT | REBORN; 0 = never held). A recycled
// slot's entries are not cleared at once (k_gossip_free, k_s_scrub): an entry created before the slot's current gossip
// existed (slot_ctick) belongs to an earlier gossip of the slot and reads as never held. (Every holder of the earlier
// gossip received it before its slot expired, EXPB > 0 ticks before the recycle.)
__device__ __forceinline__ uint32_t s_get(const Dev& d, uint32_t g, uint32_t m, uint32_t ref) {
  const uint16_t e = d.S[s_idx(d, g, m)];
  if (!(e & S16_EVER)) return 0u;
  const uint32_t c = s16_tick(e, ref);
  if (c < d.slot_ctick[g]) return 0u;
  return ((c + 1u) & S_TICK_MASK) | ((e & S16_SWEPT) ? S_SWEPT : 0u) | ((e & S16_REBORN) ? S_REBORN : 0u);
}
__device__ __forceinline__ void s_put(const Dev& d, uint32_t g, uint32_t m, uint32_t ctick, bool reborn) {
  d.S[s_idx(d, g, m)] = (uint16_t)(S16_EVER | (ctick & S16_TICK) | (reborn ? S16_REBORN : 0u));
}

// ---- gossip holder state (gossip.hip) ----
// ring entries: slot (22 bits) | infection period & 1023 << 22. At a round every entry's period lies in
// [P - 2 spreadMax - 3, P] (swim_create bounds spreadMax), so the low 10 bits identify it.
constexpr uint32_t RG_SLOT = (1u << 22) - 1u;
__device__ __forceinline__ uint32_t rg_entry(uint32_t g, uint32_t infp) { return g | ((infp & 1023u) << 22); }
__device__ __forceinline__ int64_t rg_period(uint32_t e, uint32_t P) {
  const int32_t rel = (int32_t)(((e >> 22) - (P & 1023u) + 512u) & 1023u) - 512;
  return (int64_t)P + rel;
}
__device__ __forceinline__ uint32_t* ring(const Dev& d, uint32_t m) { return d.rg + (size_t)m * d.BCAP; }
__device__ __forceinline__ unsigned long long* hrow(const Dev& d, uint32_t m) { return d.HB + (size_t)m * d.QW; }
__device__ __forceinline__ unsigned long long* wrow(const Dev& d, uint32_t m) { return d.WB + (size_t)m * d.QW; }

// createAndPutGossip (GossipProtocolImpl.java:163-169) at member m, tick k: the slot's table entries and the
// creator's holder state. The caller reserved ring position `pos` of m.
__device__ __forceinline__ void slot_create(const Dev& d, uint32_t g, uint32_t m, uint32_t k, uint64_t gid, uint32_t subj, uint64_t key,
                            uint32_t pos) {
  d.slot_gid[g] = gid;
  d.slot_subj[g] = subj;
  d.slot_ctick[g] = k;
  d.slot_key[g] = key;
  d.slot_exp[g] = k + d.EXPB;
  d.slot_used[g] = 1;
  const unsigned long long bit = 1ull << (g & 63u);
  atomicOr(&d.GU[g >> 6], bit);
  if (subj != USER_SUBJ && rec_status(key) == ST_DEAD) atomicOr(&d.DM[g >> 6], bit);
  s_put(d, g, m, k, false);
  atomicOr(&hrow(d, m)[g >> 6], bit);
  ring(d, m)[pos & (d.BCAP - 1)] = rg_entry(g, rounds_before(d, m, k));
  if (pos + 1u - d.rhead[m] > d.BCAP) set_err(d, E_RING);
}

// end of a sharded tick (W > 1): the same resets, plus the exchange counters (one block)
// a launch of a speculative batch that halted at an earlier tick (or at this one, for the kernels after the gate)
__device__ __forceinline__ bool spec_halted(const Dev& d, uint32_t spec) {
  return spec && *(volatile uint32_t*)d.halt != 0u;
}

__device__ __forceinline__ void tick_end(const Dev& d, uint32_t k) {
  uint32_t t = threadIdx.x;
  if (t < 8) d.xn[t] = 0;
  if (t < d.W) {
    d.xa_scnt[t] = 0;
    d.xb_scnt[t] = 0;
  }
  for (uint32_t i = t; i < 2 * d.W; i += blockDim.x) d.xdone[i] = 0;
  if (t == 0) {
    uint32_t nb = (k + 1) & 1;
    d.nmsg[nb] = 0;
    d.arena_used[nb] = 0;
    *d.pool_used = 0;
    *d.rc_n = 0;
    if (d.ackres) *d.ndl = *d.ndlw = 0;
  }
}

// start of a speculative k_member_tick (W == 1, block 0, one thread): the per-tick counters the SYNC diff and the
// member control of the next tick append to; this tick's member kernel uses only the other buffer's. (In a speculative
// batch no gossip slot is in use and no gossip plane runs, so the receipt lists and peaks stay as they are.)
// Slots already in use when the launch starts (the host's user gossips of this tick, k_ug_create) stop the batch after
// this tick like the ones its members take (flush_spreads).
__device__ __forceinline__ void tick_reset(const Dev& d, uint32_t k) {
  const uint32_t nb = (k + 1) & 1;
  d.nmsg[nb] = 0;
  d.arena_used[nb] = 0;
  *d.pool_used = 0;
  if (d.ackres) *d.ndl = *d.ndlw = 0;
  if (__hip_atomic_load(d.free_top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (int32_t)d.SPR)
    *(volatile uint32_t*)d.halt = k + 1u;
}

// end of k_member_tick (W == 1, the last block, one thread): reset the per-tick counters the gossip plane of this tick and the SYNC diff and
// member control of the next tick append to, and tell the host whether any gossip slot is in use (if none, the
// gossip data plane of this tick has nothing to send, deliver, route or recycle and is not launched)
// (A speculative launch never runs this: it resets the counters at its start, tick_reset, and the member taking a slot
// raises d.halt.)
__device__ __forceinline__ void tick_flag(const Dev& d, uint32_t k) {
  uint32_t nb = (k + 1) & 1;
  // every load first (in flight together), then the stores; the host-mapped words are written only when they change
  // (a write to host memory holds the end of the kernel for a round trip over the host link)
  const uint32_t used =
      (uint32_t)((int32_t)d.SPR - __hip_atomic_load(d.free_top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  uint32_t v[6] = {used, 0, 0, 0, 0, 0}, sh[6];
  if (d.rfill) {  // the previous gossip plane's peaks, for the host's capacity growth (api.hip grow_caps)
    v[1] = *d.rfill;
    v[2] = *d.rc_n;
    v[3] = *d.rp_n;
    v[4] = *d.slow_n;
    v[5] = *d.hist_n;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) sh[i] = d.hsh[i];
  d.nmsg[nb] = 0;
  d.arena_used[nb] = 0;
  *d.pool_used = 0;
  if (d.rfill) *d.rfill = 0;
  *d.rc_n = 0;
  if (d.ackres) *d.ndl = *d.ndlw = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i)
    if ((i == 0 || d.rfill) && v[i] != sh[i]) {
      d.hflag[i == 0 ? 0 : i + 1] = v[i];  // [0] slots in use, [2..6] the peaks
      d.hsh[i] = v[i];
    }
  __threadfence_system();
}

}  // namespace swim
