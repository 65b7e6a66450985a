// kernels.hip — initialisation, receipt routing, the SYNC-payload diff, state hashes and the tick launchers (the
// gossip data plane is in gossip.hip).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "dev_util.h"

namespace swim {

enum : uint32_t { BODY_FULL = 0, BODY_SPLIT = 1, BODY_RESUME = 2 };  // member.hip
template <uint32_t MODE>
__global__ void k_member_tick_t(const Dev* __restrict__ dp, uint32_t k, uint32_t flag);  // member.hip
// shard.hip
__global__ void k_pack_all(Dev d, uint32_t b, uint32_t spec);  // shard.hip
__global__ void k_unpack_a(Dev d, uint32_t k, uint32_t end, uint32_t spec);
__global__ void k_pack_b(Dev d);
__global__ void k_round_reset(Dev d);

// ------------------------------------------------------------------------------------------------------------
// init (SEMANTICS.md §3)
__device__ __forceinline__ uint32_t init_draw(const Dev& d, uint32_t m, uint32_t what, uint32_t i) {
  return philox(m, what, i, 0, d.seed_lo ^ SALT_INIT, d.seed_hi).x;
}

__global__ void k_init_members(Dev d) {
  uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= d.N) return;
  bool pre = d.init_mode == 1;
  d.ms[m].tsize = pre ? d.N : 1;
  d.ms[m].fdLen = pre ? d.N - 1 : 0;
  d.ms[m].gLen = pre ? d.N - 1 : 0;
  d.ms[m].fdPeriod = d.ms[m].gPeriod = d.ms[m].gCounter = 0;
  d.nextPing[m] = pre ? 1 + init_draw(d, m, 1, 0) % d.ping_t : d.ping_t;
  uint32_t ng = pre ? 1 + init_draw(d, m, 2, 0) % d.gossip_t : d.gossip_t;
  d.nextGossip[m] = ng;
  d.firstGossip[m] = ng;
  d.nextSync[m] = pre ? 1 + init_draw(d, m, 3, 0) % d.sync_t : NEVER;
  if (d.mode == 1u) d.nextPing[m] = d.nextSync[m] = NEVER;  // RUMOR: gossip layer only (SEMANTICS.md §9)
  const bool dormant = m >= d.N - d.n_dormant;  // not started until swim_join (k_join)
  d.start_tick[m] = (pre || dormant) ? NEVER : 0u;
  d.jseed_n[m] = NONE32;
  d.md_uidx[m] = NONE32;
  d.ms[m].cidCnt = d.ms[m].syncSeq = d.ms[m].evSeq = d.held[m] = 0;
  d.timerMin[m] = NEVER;
  d.initFlags[m] = d.ms[m].initDeadline = d.ms[m].initCidBase = d.ms[m].initN = 0;
  d.ms[m].nsub = d.ms[m].npath = d.ms[m].nfetch = 0;
  d.ms[m].fnext = NEVER;
  d.ms[m].pingIdx = 0;
  d.ms[m].remoteIdx = pre ? 0 : -1;
  for (int i = 0; i < 8; ++i) d.sel[(size_t)m * 8 + i] = 0;
  d.ms[m].evHash = 0;
  d.tround[m] = 0;
  d.log_pos[m] = 0;
  d.spchg[m] = 0;
  d.dead_tick[m] = dormant ? 0u : NEVER;  // a process not started yet refuses connections, like a dead one
  d.md_version[m] = 0;
  d.rc_cnt[m] = 0;
  d.rc_off[m] = 0;
  d.rc_fill[m] = 0;
  d.m_head[m] = d.m_head[d.N + m] = NEVER;
  d.next_evt[m] = NEVER;
  d.pending_inc[m] = 0;
  d.rhead[m] = d.rwin[m] = d.rseen[m] = d.rtail[m] = 0;  // empty receipt ring (gossip.hip)
  d.tin_cnt[m] = d.tin_fill[m] = 0;
  if (m >= d.lo && m < d.hi)
    for (uint32_t g = 0; g < d.GRCAP; ++g) d.groups[(lidx(d, m) * d.GRCAP + g) * GREC + 5] = 0;
  for (uint32_t e = 0; e < d.LOGW; ++e) d.log_tick[(size_t)m * d.LOGW + e] = NEVER;
}

// one block per observer row (grid-strided): both planes are written with coalesced 4-B stores
__global__ void k_init_rows(Dev d) {
  if (d.implicit) return;
  const uint64_t full = rec_key(ST_ALIVE, 0) | META_BIT;
  for (uint32_t li = blockIdx.x; li < d.NL; li += gridDim.x) {
    uint32_t m = d.lo + li;
    uint32_t* rk = d.rowk + (size_t)li * d.NS;
    uint32_t* ra = d.rowa + (size_t)li * d.NS;
    for (uint32_t s = threadIdx.x; s < d.NS; s += blockDim.x) {
      const uint64_t v = s >= d.N ? 0ull : (d.init_mode == 1 || m == s) ? full : 0ull;
      rk[s] = key32(v);
      ra[s] = aux32(v);
      if (d.rowk8) d.rowk8[(size_t)li * d.NS8 + s] = key8(key32(v));
    }
    if (d.rowk8)  // (the 8-bit plane's wider padding: zero, absent)
      for (uint32_t s = d.NS + threadIdx.x; s < d.NS8; s += blockDim.x) d.rowk8[(size_t)li * d.NS8 + s] = 0;
    if (d.W > 1)  // dirty chunks against base_row: none for a PRECONVERGED row, the own chunk for a cold join
      for (uint32_t w = threadIdx.x; w < d.MW; w += blockDim.x)
        d.rdirty[(size_t)li * d.MW + w] = (d.init_mode != 1 && (m / CH) >> 6 == w) ? 1ull << ((m / CH) & 63) : 0ull;
  }
}

// PRECONVERGED lists: position p of observer m holds the other member of rank feistel_m(p) (SEMANTICS.md §3)
__global__ void k_init_lists(Dev d) {
  if (d.init_mode != 1 || d.N < 2 || d.implicit) return;
  uint32_t n = d.N - 1;
  for (uint32_t m = d.lo + blockIdx.x; m < d.hi; m += gridDim.x) {
    for (uint32_t w = 0; w < 2; ++w) {
      FeistelPerm P = make_perm(n, init_draw(d, m, 16 + 4 * w + 0, 0), init_draw(d, m, 16 + 4 * w + 1, 0),
                                init_draw(d, m, 16 + 4 * w + 2, 0), init_draw(d, m, 16 + 4 * w + 3, 0));
      uint32_t* L = (w == 0 ? d.fdl : d.gl) + lidx(d, m) * d.LCAP;
      for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) {
        uint32_t j = feistel(P, p);
        L[p] = j < m ? j : j + 1;
      }
    }
  }
}

__global__ void k_init_slots(Dev d) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= d.SLOTS) return;
  d.slot_used[g] = 0;
  d.slot_exp[g] = NEVER;
  // each shard allocates only from its own slot range [rank SPR, (rank+1) SPR), so slot ids are global
  if (g < d.SPR) d.free_list[g] = d.rank * d.SPR + d.SPR - 1 - g;
}

// the SYNC baseline row (record keys): what a PRECONVERGED row starts as, an empty row for a cold join
// (and its 8-bit shadow, what a narrow item reads for a peer's payload chunk that was not shipped)
__global__ void k_init_base(Dev d) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t v = (s < d.N && d.init_mode == 1) ? key32(rec_key(ST_ALIVE, 0)) : 0u;
  if (s < d.NS) d.base_row[s] = v;
  if (d.base_row8 && s < d.NS8) d.base_row8[s] = key8(v);
}

// ------------------------------------------------------------------------------------------------------------
// receipt routing: counting sort of first receipts by member, then per-member sort by gossip id
__global__ void k_count_rc(const uint64_t* raw, const uint32_t* n_, uint32_t cap, uint32_t* cnt) {
  uint32_t n = *n_ < cap ? *n_ : cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    atomicAdd(&cnt[(uint32_t)(raw[i] >> 32)], 1u);
}
__global__ void k_scatter_rc(const Dev d, const uint64_t* raw, const uint32_t* n_, uint32_t cap, const uint32_t* off,
                             uint32_t* fill, uint32_t* idx, uint64_t* key) {
  uint32_t n = *n_ < cap ? *n_ : cap;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t t = (uint32_t)(raw[i] >> 32), g = (uint32_t)raw[i];
    const uint32_t f = atomicAdd(&fill[t], 1u);
    if (f == 1u) d.sg_list[wave_append(d.nsg)] = t;  // a segment with two receipts or more: k_seg_sort sorts it
    uint32_t p = off[t] + f;
    idx[p] = g;
    key[p] = d.slot_gid[g];
  }
}

// exclusive scan of n counts: per-1024 block scans, a scan of the block sums, then the add-back
__device__ __forceinline__ uint32_t block_excl_scan_256(uint32_t v, uint32_t* sh, uint32_t* total) {
  uint32_t t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {
    uint32_t a = t >= o ? sh[t - o] : 0;
    __syncthreads();
    sh[t] += a;
    __syncthreads();
  }
  uint32_t incl = sh[t];
  *total = sh[255];
  __syncthreads();
  return incl - v;
}
__global__ void __launch_bounds__(256) k_scan_blocks(const uint32_t* in, uint32_t* out, uint32_t* part, uint32_t n) {
  __shared__ uint32_t sh[256];
  uint32_t base = blockIdx.x * 1024 + threadIdx.x * 4;
  uint32_t v[4], s = 0;
  for (int j = 0; j < 4; ++j) {
    v[j] = base + j < n ? in[base + j] : 0;
    s += v[j];
  }
  uint32_t tot;
  uint32_t run = block_excl_scan_256(s, sh, &tot);
  for (int j = 0; j < 4; ++j) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(256) k_scan_top(uint32_t* part, uint32_t nb) {  // nb <= 1024
  __shared__ uint32_t sh[256];
  uint32_t base = threadIdx.x * 4;
  uint32_t v[4], s = 0;
  for (int j = 0; j < 4; ++j) {
    v[j] = base + j < nb ? part[base + j] : 0;
    s += v[j];
  }
  uint32_t tot;
  uint32_t run = block_excl_scan_256(s, sh, &tot);
  for (int j = 0; j < 4; ++j) {
    if (base + j < nb) part[base + j] = run;
    run += v[j];
  }
}
__global__ void k_scan_add(uint32_t* out, const uint32_t* part, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += part[i / 1024];
}

// per-segment sort of (key, val) by key (keys are unique within a segment): one block per segment. Segments of
// up to SORT_MAX entries are sorted bitonically in LDS; larger ones (a member receiving thousands of new gossips in
// one tick, C2-style storms) sort SORT_MAX runs in LDS and then merge run pairs through the scratch arrays, each
// element finding its output position by a binary search in the partner run (merge path, no atomics).
// (SORT_MAX: engine.h; the runtime run length is Dev::sort_cap <= SORT_MAX)
__device__ void lds_bitonic(uint64_t* K, uint32_t* V, const uint64_t* key, const uint32_t* val, uint32_t n,
                            uint64_t* okey, uint32_t* oval) {
  uint32_t p2 = 1;
  while (p2 < n) p2 <<= 1;
  for (uint32_t i = threadIdx.x; i < p2; i += blockDim.x) {
    K[i] = i < n ? key[i] : ~0ull;
    V[i] = i < n ? val[i] : 0;
  }
  __syncthreads();
  for (uint32_t size = 2; size <= p2; size <<= 1)
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = threadIdx.x; i < p2; i += blockDim.x) {
        uint32_t j = i ^ stride;
        if (j > i) {
          bool up = (i & size) == 0;
          if ((K[i] > K[j]) == up) {
            uint64_t tk = K[i];
            K[i] = K[j];
            K[j] = tk;
            uint32_t tv = V[i];
            V[i] = V[j];
            V[j] = tv;
          }
        }
      }
      __syncthreads();
    }
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    okey[i] = K[i];
    oval[i] = V[i];
  }
  __syncthreads();
}

// number of entries of the sorted run r[0..n) that are < x
__device__ __forceinline__ uint32_t lower_rank(const uint64_t* r, uint32_t n, uint64_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (r[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// the segments listed in sg (nsg of them: members with two receipts or more, k_scatter_rc), not all N
__global__ void __launch_bounds__(256) k_seg_sort(uint64_t* key, uint32_t* val, uint64_t* tkey, uint32_t* tval,
                                                  const uint32_t* off, const uint32_t* cnt, const uint32_t* sg,
                                                  const uint32_t* nsg, uint32_t run, unsigned long long* fb) {
  __shared__ uint64_t K[SORT_MAX];
  __shared__ uint32_t V[SORT_MAX];
  const uint32_t nseg = *nsg;
  for (uint32_t li = blockIdx.x; li < nseg; li += gridDim.x) {
    const uint32_t sgi = sg[li];
    const uint32_t n = cnt[sgi];
    if (n <= 1) continue;
    const uint32_t o = off[sgi];
    if (n <= run) {
      lds_bitonic(K, V, key + o, val + o, n, key + o, val + o);
      continue;
    }
    if (fb && threadIdx.x == 0) atomicAdd(&fb[FB_SORT_MERGE], 1ull);
    for (uint32_t c = 0; c < n; c += run)
      lds_bitonic(K, V, key + o + c, val + o + c, min(run, n - c), key + o + c, val + o + c);
    uint64_t *sk = key + o, *dk = tkey + o;
    uint32_t *sv = val + o, *dv = tval + o;
    for (uint32_t w = run; w < n; w <<= 1) {
      for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t base = i / (2 * w) * (2 * w), mid = min(base + w, n), end = min(base + 2 * w, n);
        const uint64_t x = sk[i];
        uint32_t pos;
        if (i < mid)  // run A element: its index in A plus the B entries below it
          pos = i + lower_rank(sk + mid, end - mid, x);
        else  // run B element: its index in B plus the A entries below it
          pos = base + (i - mid) + lower_rank(sk + base, mid - base, x);
        dk[pos] = x;
        dv[pos] = sv[i];
      }
      __syncthreads();
      uint64_t* tk = sk;
      sk = dk;
      dk = tk;
      uint32_t* tv = sv;
      sv = dv;
      dv = tv;
    }
    if (sk != key + o) {
      for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        key[o + i] = sk[i];
        val[o + i] = sv[i];
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------------------------------
// k_sync_diff: for every SYNC / SYNC_ACK sent in tick k-1, stream the payload's key plane (the sender's live row,
// or its copy-on-write snapshot) against the receiver's key plane and extract, per 2048-subject chunk and in
// subject order, the records that differ (the eager `!r1.equals(table.get(id))` filter of syncMembership,
// :456-467). This is the HBM-bound hot loop: 2 x 1 B read per subject per merge on one GPU (the keys' 8-bit
// shadows, key8; an escaped key is compared on its 4-B key32), 2 x 4 B for the rest. SHARDED adds payloads
// received from other shards (baseline row + shipped chunks); the single-GPU instance has only local rows and
// snapshots.
//
// an item's message as k_sync_diff reads it (the 16-B entries of Dev::dlist / dlist_w, written by k_ack_resolve;
// without a list, read from the message): x = the message index, y = sender, z = receiver, w = where the payload is
// (desc_pay)
__device__ __forceinline__ uint32_t desc_pay(const SyncMsg& mm) {
  if (mm.kind & KF_DEFER) return DESC_DEFER;  // merged in a later tick: nothing to compare now
  if (mm.payload != NEVER) return mm.payload;  // an arena snapshot, or (W > 1) PAY_RX | rx index
  return mm.pin == NEVER ? NEVER : DESC_PIN | mm.pin;  // the live row (pinned: copied into the arena as it streams)
}

// a peer's payload (PAY_RX | rx index): was chunk c shipped (it differs from the baseline row)?
__device__ __forceinline__ bool rx_shipped(const Dev& d, uint32_t pay, uint32_t c) {
  const uint64_t* mk = d.rx_mask + (size_t)(pay & ~PAY_RX) * d.MW;
  return (mk[c >> 6] >> (c & 63)) & 1ull;
}
// the 4-B payload keys from subject s on (within one chunk) of the entry's payload: the local sender's row, or a peer's
// shipped chunk, or the baseline row
template <bool SHARDED>
__device__ __forceinline__ const uint32_t* pay_keys(const Dev& d, const uint4& D, uint32_t s) {
  if (!SHARDED || D.w == NEVER) return d.rowk + lidx(d, D.y) * d.NS + s;
  const uint32_t ri = D.w & ~PAY_RX, c = s / CH;
  const uint64_t* mk = d.rx_mask + (size_t)ri * d.MW;
  if (!((mk[c >> 6] >> (c & 63)) & 1ull)) return d.base_row + s;
  uint32_t rank = __popcll(mk[c >> 6] & ((1ull << (c & 63)) - 1ull));
  for (uint32_t q = 0; q < (c >> 6); ++q) rank += __popcll(mk[q]);
  return (const uint32_t*)(d.xa_recv + d.rx_off[ri]) + (size_t)rank * CH + s % CH;
}

// this lane's keys of the item's chunk c: narrow (an entry of the narrow list: a local sender's unpinned live row, or
// on a row shard a peer's payload): the item is chunks c .. c + 3 of the message, lane i the 32 subjects c CH + 32 i
// ..., and x holds their 8-bit shadow keys (key8): payload x[0..1], receiver x[2..3], the same 64 B per lane in
// flight as one chunk of 4-B keys.
// Otherwise 8 payload keys and 8 receiver keys of chunk c: the payload is the sender's live row or its copy-on-write
// snapshot; for a payload received from another shard, the shipped chunk if it differs from the baseline, else the
// baseline. pinw: the arena row a live-row payload is copied into while it streams (pin_msg), else NEVER. Every lane
// of the block takes the same item, so the mode is uniform.
template <bool SHARDED>
__device__ __forceinline__ void diff_fetch(const Dev& d, uint32_t b, const uint4& D, uint32_t c, uint4 (&x)[4],
                                           uint32_t& pinw, bool& narrow, bool narrow_item) {
  pinw = NEVER;
  narrow = false;
  if (narrow_item) {
    narrow = true;
    const uint32_t n0 = c * CH + threadIdx.x * 32;  // NS8 is a multiple of 16: 16-subject groups wholly in or out
    // the payload: the local sender's row, or (a peer's payload) the baseline row's shadow for a chunk that was not
    // shipped; a shipped chunk has no shadow: its lanes read as escaped (0xFF) and diff_wave8 compares its u32 keys
    const uint8_t* p8 = nullptr;
    if (!SHARDED || D.w == NEVER) {
      p8 = d.rowk8 + lidx(d, D.y) * d.NS8 + n0;
    } else if (n0 < d.NS8 && !rx_shipped(d, D.w, n0 / CH)) {
      p8 = d.base_row8 + n0;
    }
    const uint8_t* r8 = d.rowk8 + lidx(d, D.z) * d.NS8 + n0;
    const uint4 z = make_uint4(0, 0, 0, 0), e = make_uint4(~0u, ~0u, ~0u, ~0u);
    x[0] = n0 < d.NS8 ? (p8 ? ld_c4((const uint32_t*)p8) : e) : z;
    x[1] = n0 + 16 < d.NS8 ? (p8 ? ld_c4((const uint32_t*)(p8 + 16)) : e) : z;
    x[2] = n0 < d.NS8 ? ld_c4((const uint32_t*)r8) : z;
    x[3] = n0 + 16 < d.NS8 ? ld_c4((const uint32_t*)(r8 + 16)) : z;
    return;
  }
  const uint32_t s0 = c * CH + threadIdx.x * 8;
  // NS is a multiple of 8: a 32-B group is wholly in or out; padding entries are 0 (absent)
  if (s0 >= d.NS || D.w == DESC_DEFER) {
    x[0] = x[1] = x[2] = x[3] = make_uint4(0, 0, 0, 0);
    return;
  }
  const uint32_t* p8;
  if (D.w == NEVER || (D.w & DESC_PIN)) {
    pinw = D.w == NEVER ? NEVER : D.w & ~DESC_PIN;
    p8 = d.rowk + lidx(d, D.y) * d.NS + s0;
  } else if (SHARDED && (D.w & PAY_RX)) {  // the shipped chunk, or the baseline row
    p8 = pay_keys<SHARDED>(d, D, s0);
  } else {
    p8 = d.arena[b] + (size_t)D.w * d.NS + s0;
  }
  const uint32_t* r8 = d.rowk + lidx(d, D.z) * d.NS + s0;
  // (non-temporal loads measured 1.5x slower here on gfx950)
  x[0] = ld_c4(p8);
  x[1] = ld_c4(p8 + 4);
  x[2] = ld_c4(r8);
  x[3] = ld_c4(r8 + 4);
}

// chunk c of message mi against this lane's 8 payload keys p and receiver keys r (s0: its first subject): the
// differing records in subject order into the candidate pool, the chunk's (offset, count) into chunk_meta
__device__ __forceinline__ void diff_chunk(const Dev& d, uint32_t b, uint32_t mi, uint32_t c, uint32_t s0,
                                           const uint32_t (&p)[8], const uint32_t (&r)[8], uint32_t* scan,
                                           uint32_t& base) {
  const bool dl = d.ackres != 0;
  uint32_t mask = 0, ab = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if ((p[j] & 3u) != ST_ABSENT && p[j] != r[j]) mask |= 1u << j;
    ab |= (uint32_t)((p[j] & 3u) == ST_ABSENT && (r[j] & 3u) != ST_ABSENT);
  }
  uint32_t nc = __popc(mask);
  const bool two = 2 * c + 1 < d.NMETA;  // the chunk's second candidate segment (lanes 128-255)
  if (!__syncthreads_or(nc | ab)) {  // steady state: the whole 2048-subject chunk matches
    if (threadIdx.x == 0) {
      uint32_t* cm = d.chunk_meta + ((size_t)mi * d.NMETA + 2 * c) * 2;
      cm[0] = cm[1] = 0;
      if (two) cm[2] = cm[3] = 0;
    }
    return;
  }
  if (dl && ab) atomicOr(&d.msgs[b][mi].kind, KF_ABS);  // (rare: a record the payload lacks)
  scan[threadIdx.x] = nc;
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {
    uint32_t v = threadIdx.x >= o ? scan[threadIdx.x - o] : 0;
    __syncthreads();
    scan[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t incl = scan[threadIdx.x];
  uint32_t totc = scan[255];
  if (threadIdx.x == 0) {
    const uint32_t first = scan[127];  // the first segment's candidates (lanes 0-127)
    uint32_t bo = atomicAdd(d.pool_used, totc);
    if (bo + totc > d.POOLCAP) {  // no room: nothing of this chunk is written (the error aborts the step)
      atomicOr(d.err, E_POOL);
      totc = 0;
      bo = NEVER;
    }
    base = bo;
    uint32_t* cm = d.chunk_meta + ((size_t)mi * d.NMETA + 2 * c) * 2;
    cm[0] = bo;
    cm[1] = bo == NEVER ? 0u : first;
    if (two) {
      cm[2] = bo == NEVER ? NEVER : bo + first;
      cm[3] = bo == NEVER ? 0u : totc - first;
    }
    if (totc) atomicAdd(&d.msgs[b][mi].ncand, totc);
  }
  __syncthreads();
  uint32_t o = base + incl - nc;
  if (base != NEVER)  // (an overflowed chunk must not overwrite other chunks' candidates)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (mask & (1u << j)) d.pool[o++] = ((uint64_t)(s0 + j) << 34) | key34(p[j]);
  __syncthreads();
}

// a narrow item: chunks c .. c + 3 of message mi, each wave two 1024-subject candidate segments (wave w: segments
// 2c + 2w (lanes 0-31) and 2c + 2w + 1 (lanes 32-63), 32 subjects per lane from x), tested, scanned and written by the
// wave alone: no block barrier. A lane with an escaped shadow (0xFF: an incarnation past 62 among its subjects)
// compares its 32 full keys of both rows.
template <bool SHARDED>
__device__ __forceinline__ void diff_wave8(const Dev& d, uint32_t b, const uint4& D, uint32_t c, const uint4 (&x)[4]) {
  const uint32_t mi = D.x;
  const bool dl = d.ackres != 0;
  const uint32_t lane = threadIdx.x & 63u, seg = 2 * c + 2 * (threadIdx.x >> 6) + (lane >> 5);
  const uint32_t n0 = c * CH + threadIdx.x * 32;  // = seg * MCH + (lane & 31) * 32
  const uint32_t pw[8] = {x[0].x, x[0].y, x[0].z, x[0].w, x[1].x, x[1].y, x[1].z, x[1].w};
  const uint32_t rw[8] = {x[2].x, x[2].y, x[2].z, x[2].w, x[3].x, x[3].y, x[3].z, x[3].w};
  uint32_t esc = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q)  // a 0xFF byte in either word (a zero byte of the complement)
    esc |= ((~pw[q] - 0x01010101u) & pw[q] & 0x80808080u) | ((~rw[q] - 0x01010101u) & rw[q] & 0x80808080u);
  uint32_t mask = 0, ab = 0;
  const uint32_t *pk = nullptr, *rk = nullptr;
  if (esc) {  // (rare) the 32 subjects' 4-B keys, one at a time
    pk = pay_keys<SHARDED>(d, D, n0);  // (32 subjects: within one chunk)
    rk = d.rowk + lidx(d, D.z) * d.NS + n0;
#pragma unroll 1
    for (uint32_t j = 0; j < 32; ++j) {
      const uint32_t p = n0 + j < d.NS ? pk[j] : 0u, r = n0 + j < d.NS ? rk[j] : 0u;
      if ((p & 3u) != ST_ABSENT && p != r) mask |= 1u << j;
      ab |= (uint32_t)((p & 3u) == ST_ABSENT && (r & 3u) != ST_ABSENT);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint32_t p = (pw[j >> 2] >> (8 * (j & 3))) & 0xFFu, r = (rw[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      if ((p & 3u) != ST_ABSENT && p != r) mask |= 1u << j;
      ab |= (uint32_t)((p & 3u) == ST_ABSENT && (r & 3u) != ST_ABSENT);
    }
  }
  const uint32_t nc = __popc(mask);
  uint32_t* cm = d.chunk_meta + ((size_t)mi * d.NMETA + seg) * 2;
  const bool live = seg < d.NMETA, head = (lane & 31u) == 0;
  if (!__ballot(nc | ab)) {  // steady state: the wave's 2048 subjects match
    if (head && live) cm[0] = cm[1] = 0;
    return;
  }
  if (dl && __ballot(ab) && lane == 0) atomicOr(&d.msgs[b][mi].kind, KF_ABS);  // (rare: a record the payload lacks)
  uint32_t incl = nc;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const uint32_t totc = __shfl(incl, 63), first = __shfl(incl, 31);  // both segments, the first one
  uint32_t bo = 0;
  if (lane == 0 && totc) {
    bo = atomicAdd(d.pool_used, totc);
    if (bo + totc > d.POOLCAP) {  // no room: nothing of these segments is written (the error aborts the step)
      atomicOr(d.err, E_POOL);
      bo = NEVER;
    }
    if (bo != NEVER) atomicAdd(&d.msgs[b][mi].ncand, totc);
  }
  bo = __shfl(bo, 0);
  if (head && live) {
    const uint32_t off = lane ? first : 0u, cnt = lane ? totc - first : first;
    cm[0] = bo == NEVER ? NEVER : bo + off;
    cm[1] = bo == NEVER ? 0u : cnt;
  }
  if (bo == NEVER) return;  // (an overflowed segment must not overwrite other segments' candidates)
  uint32_t o = bo + incl - nc;
  if (esc) {
    for (uint32_t m = mask; m; m &= m - 1, ++o) {
      const uint32_t j = (uint32_t)(__ffs(m) - 1);
      d.pool[o] = ((uint64_t)(n0 + j) << 34) | key34(pk[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (mask & (1u << j)) d.pool[o++] = ((uint64_t)(n0 + j) << 34) | key34((pw[j >> 2] >> (8 * (j & 3))) & 0xFFu);
  }
}

// k_sync_diff's work, two lists of 16-B entries (message, sender, receiver, payload place; desc_pay) over the blocks
// blk of nblk, grid-stride, each with the next item's keys in flight while the current one is tested and the entry of
// the item after that in flight too, so that an item's key loads never wait for its message:
// * stream_wide: payloads compared on 4-B keys (snapshots, pinned live rows, payloads from other shards, or no 8-bit
//   plane), one 2048-subject chunk per item, block barriers per chunk (diff_chunk);
// * stream_narrow: unpinned live-row payloads (on a row shard: of local senders) on the 8-bit plane, four chunks per
//   item, one wave per two 1024-subject candidate segments and no block barrier (diff_wave8).
// Two loops rather than one with both kinds of item: the narrow loop's registers are then not sized by the wide
// path's (with both in one loop it spilled, and a scratch reload made every iteration wait for the prefetched keys).
// A list entry is block-uniform: held in scalar registers once loaded (uni), so that the addresses, modes and
// branches derived from it are scalar.
__device__ __forceinline__ uint4 uni(const uint4& v) {
  return make_uint4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                    __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}
// list entry j (without a list: message j itself, read from the message buffer)
__device__ __forceinline__ uint4 diff_entry(const Dev& d, uint32_t b, const uint4* lst, uint32_t j) {
  if (lst) return lst[j];
  const SyncMsg& mm = d.msgs[b][j];
  return make_uint4(j, mm.src, mm.dst, desc_pay(mm));
}

template <bool SHARDED>
__device__ __forceinline__ void stream_wide(const Dev& d, uint32_t b, const uint4* lst, uint32_t n, uint32_t blk,
                                            uint32_t nblk, uint32_t* scan, uint32_t& base, uint32_t timed) {
  const uint32_t nch = d.NCHUNK, total = n * nch;
  uint4 cur[4], dc = make_uint4(0, 0, 0, 0), dn = dc;
  uint32_t pcur = NEVER;
  bool nw;
  if (blk < total) {
    dc = uni(diff_entry(d, b, lst, blk / nch));
    diff_fetch<SHARDED>(d, b, dc, blk % nch, cur, pcur, nw, false);
  }
  if (blk + nblk < total) dn = diff_entry(d, b, lst, (blk + nblk) / nch);
  for (uint32_t w = blk; w < total; w += nblk) {
    uint4 nxt[4], dnn = make_uint4(0, 0, 0, 0);
    uint32_t pnxt = NEVER;
    const uint4 du = uni(dn);
    if (w + nblk < total) diff_fetch<SHARDED>(d, b, du, (w + nblk) % nch, nxt, pnxt, nw, false);
    if (w + 2 * nblk < total) dnn = diff_entry(d, b, lst, (w + 2 * nblk) / nch);
    const uint32_t mi = dc.x, c = w % nch, s0 = c * CH + threadIdx.x * 8;
    if (!SHARDED && c == 0 && threadIdx.x == 0) {  // priced at 8 B per subject (swim_counters)
      atomicAdd(&d.ctr[C_DIFFWIDE_ALL], 1ull);
      if (timed) atomicAdd(&d.ctr[C_DIFFWIDE], 1ull);
    }
    if (pcur != NEVER && s0 < d.NS) {  // a live-row payload read again later (pin_msg)
      uint4* dst = (uint4*)(d.arena[b] + (size_t)pcur * d.NS + s0);
      dst[0] = cur[0];
      dst[1] = cur[1];
    }
    const uint32_t p[8] = {cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y, cur[1].z, cur[1].w};
    const uint32_t r[8] = {cur[2].x, cur[2].y, cur[2].z, cur[2].w, cur[3].x, cur[3].y, cur[3].z, cur[3].w};
    diff_chunk(d, b, mi, c, s0, p, r, scan, base);
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    dc = du;
    dn = dnn;
    pcur = pnxt;
  }
}

// e0 (uniform), e1: the entries of items blk and blk + nblk, loaded by the caller before the list's length was known
// (indices clamped to the list's capacity: an entry past the length is never used)
template <bool SHARDED>
__device__ __forceinline__ void stream_narrow(const Dev& d, uint32_t b, const uint4* lst, uint32_t n, uint32_t blk,
                                              uint32_t nblk, const uint4& e0, const uint4& e1) {
  constexpr uint32_t PER = 4;
  const uint32_t nit = (d.NCHUNK + PER - 1) / PER, total = n * nit;
  uint4 cur[4], dc = make_uint4(0, 0, 0, 0), dn = e1;
  uint32_t pw;
  bool nr;
  if (blk < total) {
    dc = e0;
    diff_fetch<SHARDED>(d, b, dc, (blk % nit) * PER, cur, pw, nr, true);
  }
  for (uint32_t w = blk; w < total; w += nblk) {
    uint4 nxt[4], dnn = make_uint4(0, 0, 0, 0);
    const uint4 du = uni(dn);
    if (w + nblk < total) diff_fetch<SHARDED>(d, b, du, ((w + nblk) % nit) * PER, nxt, pw, nr, true);
    if (w + 2 * nblk < total) dnn = lst[(w + 2 * nblk) / nit];
    diff_wave8<SHARDED>(d, b, dc, (w % nit) * PER, cur);
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    dc = du;
    dn = dnn;
  }
}

// k_sync_diff: the diff of every payload streamed this tick (see diff_fetch and the stream loops above). The narrow
// items go first, on blocks 0, 1, ... (so a block's first entries are loaded together with the lists' lengths, not
// after them); the wide ones continue from the block after the last narrow one.
// DIFF_WAVES waves per SIMD; the grid is DIFF_WAVES blocks per CU, all resident (diff_grid)
constexpr uint32_t DIFF_WAVES = 7;
template <bool SHARDED>
__global__ void __launch_bounds__(256, DIFF_WAVES) k_sync_diff(const Dev* __restrict__ dp, uint32_t b, uint32_t timed, uint32_t spec) {
  const Dev& d = *dp;  // global, not kernarg (as k_member_tick): a by-value Dev of this size was copied to scratch
  if (spec && *(volatile uint32_t*)d.halt) return;  // a speculative batch halted at an earlier tick
  __shared__ uint32_t scan[256];
  __shared__ uint32_t base;
  // (timed launches are bracketed by HIP events on the stream. A self-timing variant, first block start to last block
  // end by wall clock and atomics, made every launch of this kernel 30 % slower by its mere presence in the code:
  // 85 -> 112 us per launch at C3, profiles/r03_*)
  // with SYNC_ACK resolution, only the messages k_ack_resolve listed (and counted); without it every message, on
  // 4-B keys
  const bool dl = d.ackres != 0;
  // this block's first two narrow entries, issued before the lengths arrive
  uint4 e0 = make_uint4(0, 0, 0, 0), e1 = e0;
  if (dl) {
    const uint32_t nit = (d.NCHUNK + 3) / 4, cap = d.MSGCAP - 1;
    e0 = ((const uint4*)d.dlist)[min(blockIdx.x / nit, cap)];
    e1 = ((const uint4*)d.dlist)[min((blockIdx.x + gridDim.x) / nit, cap)];
  }
  const uint32_t nmsg = d.nmsg[b] < d.MSGCAP ? d.nmsg[b] : d.MSGCAP;
  const uint32_t nwide = dl ? *(volatile uint32_t*)d.ndlw : nmsg;
  const uint32_t nnar = dl ? *(volatile uint32_t*)d.ndl : 0u;
  if (!dl && blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&d.ctr[C_DIFFMSG_ALL], (unsigned long long)nmsg);
    if (timed) atomicAdd(&d.ctr[C_DIFFMSG], (unsigned long long)nmsg);
    if (SHARDED) {  // (one GPU: stream_wide counts its messages)
      atomicAdd(&d.ctr[C_DIFFWIDE_ALL], (unsigned long long)nmsg);
      if (timed) atomicAdd(&d.ctr[C_DIFFWIDE], (unsigned long long)nmsg);
    }
  }
  const uint32_t nblk = gridDim.x, ntot = nnar * ((d.NCHUNK + 3) / 4);
  if (nnar) stream_narrow<SHARDED>(d, b, (const uint4*)d.dlist, nnar, blockIdx.x, nblk, uni(e0), e1);
  stream_wide<SHARDED>(d, b, dl ? (const uint4*)d.dlist_w : nullptr, nwide, (blockIdx.x + nblk - ntot % nblk) % nblk,
                       nblk, scan, base, timed);
}

// ------------------------------------------------------------------------------------------------------------
// k_ack_resolve (W == 1): the SYNC_ACKs of tick k-1 whose diff follows from logs instead of a stream.
// Member A's SYNC of tick k-2 carried A's row as of its send; B's diff at tick k-1 extracted D = {s : payload[s] !=
// B's row[s]} (no record the payload lacked, else KF_ABS), B merged D and answered in the same tick with its row at
// that moment. For any subject outside D, outside what B wrote in tick k-1 before the answer and outside what A
// wrote in ticks k-2 and k-1, B's answer and A's row now both equal A's payload. So only the subjects of those three
// logs (tl_add: every key change and every merged candidate) can differ; they are tested here, in subject order,
// into the same pool / chunk_meta form k_sync_diff writes. A message that cannot be resolved this way (no KF_RES, a
// log past TL, a pinned live-row payload, a delayed one) goes to dlist for k_sync_diff. One wave per message.
// the fields k_ack_resolve reads, passed as kernel arguments: through Dev* every one of them was a dependent load of
// its own before the loads that use it (the kernel is a chain of short dependent loads)
struct ResArgs {
  const uint32_t *halt, *nmsg, *tl_tick, *tl_n, *tlog, *rowk, *arena;
  SyncMsg* msgs;
  uint32_t *dlist, *ndl, *dlist_w, *ndlw, *chunk_meta, *pool_used, *err;
  uint64_t* pool;
  unsigned long long* ctr;
  uint32_t NL, NS, MSGCAP, NCHUNK, POOLCAP, NMETA;
  uint32_t k8;  // the 8-bit key plane exists (k_sync_diff streams live-row payloads narrow)
  // W > 1: this shard's first observer, the senders' log prefixes by message (Dev::mlog), and the received payloads
  // (baseline row + shipped chunks, as diff_fetch reads them)
  uint32_t lo, W, MW;
  const uint32_t *mlog, *base_row;
  const uint64_t *rx_mask, *rx_off;
  const uint8_t* xa_recv;
};

// subject v of a message's payload: the sender's live row, its arena snapshot, or (W > 1) a payload received from
// another shard (the shipped chunk if the chunk mask has it, else the baseline row)
__device__ __forceinline__ uint32_t res_payload_key(const ResArgs& d, uint32_t pay, uint32_t src, uint32_t v) {
  if (pay == NEVER) return d.rowk[(size_t)(src - d.lo) * d.NS + v];
  if (!(pay & PAY_RX) || d.W == 1) return d.arena[(size_t)pay * d.NS + v];
  const uint32_t ri = pay & ~PAY_RX, c = v / CH;
  const uint64_t* mk = d.rx_mask + (size_t)ri * d.MW;
  if (!((mk[c >> 6] >> (c & 63)) & 1ull)) return d.base_row[v];
  uint32_t rank = __popcll(mk[c >> 6] & ((1ull << (c & 63)) - 1ull));
  for (uint32_t q = 0; q < (c >> 6); ++q) rank += __popcll(mk[q]);
  return ((const uint32_t*)(d.xa_recv + d.rx_off[ri]))[(size_t)rank * CH + v % CH];
}
// one SYNC_ACK (message i of buffer d.msgs) by one wave: true if it was resolved from the write logs (its candidates
// written), false if k_sync_diff must stream it
__device__ __forceinline__ bool res_wave(const ResArgs& d, uint32_t i, uint32_t k, uint32_t lane, volatile uint32_t* sv,
                                         volatile uint32_t* sc) {
  const SyncMsg& mm = d.msgs[i];
  const uint32_t kind = mm.kind, src = mm.src, dst = mm.dst, tln = mm.tln, pay = mm.payload;
  bool res = k >= 2 && (kind & KF_RES) && !(kind & KF_DEFER) && mm.pin == NEVER && tln <= TL;
  uint32_t n0 = 0, n1 = 0;  // A's log entries of ticks k-2 and k-1
  const uint32_t ld = dst - d.lo;  // the requester: an observer of this shard
  if (res) {
    const size_t a0 = (size_t)(k & 1) * d.NL + ld, a1 = (size_t)((k - 1) & 1) * d.NL + ld;
    n0 = d.tl_tick[a0] == k - 2 ? d.tl_n[a0] : 0u;
    n1 = d.tl_tick[a1] == k - 1 ? d.tl_n[a1] : 0u;
    res = n0 <= TL && n1 <= TL;
  }
  const uint32_t nall = tln + n0 + n1;
  if (!res) return false;
  if (nall == 0) {  // nothing written on either side and nothing merged: nothing can differ
    if (lane == 0) d.msgs[i].ncand = 0;
    return true;
  }
  // gather: B's prefix, then A's two ticks (at most 3 TL <= 64 subjects, one per lane)
  uint32_t v = NEVER;
  if (lane < tln)  // W > 1: the prefix came with the message (the responder may live on another shard)
    v = d.W > 1 ? d.mlog[(size_t)i * TL + lane] : d.tlog[((size_t)((k - 1) & 1) * d.NL + src) * TL + lane];
  else if (lane < tln + n0) v = d.tlog[((size_t)(k & 1) * d.NL + ld) * TL + (lane - tln)];
  else if (lane < tln + n0 + n1) v = d.tlog[((size_t)((k - 1) & 1) * d.NL + ld) * TL + (lane - tln - n0)];
  sv[lane] = v;
  __builtin_amdgcn_wave_barrier();
  bool first = v != NEVER;
  for (uint32_t j = 0; j < min(lane, nall); ++j) first &= sv[j] != v;
  uint32_t key = 0;
  bool cand = false;
  if (first) {
    key = res_payload_key(d, pay, src, v);
    cand = (key & 3u) != ST_ABSENT && key != d.rowk[(size_t)ld * d.NS + v];
  }
  sc[lane] = cand ? v : NEVER;
  __builtin_amdgcn_wave_barrier();
  const uint64_t cb = __ballot(cand);
  const uint32_t total = (uint32_t)__popcll(cb);
  uint32_t off = 0;
  if (total) {  // (wave-uniform; none in the C3 steady state)
    uint32_t pos = 0;
    for (uint32_t j = 0; j < nall; ++j) pos += sc[j] < v;
    if (lane == 0) {
      off = atomicAdd(d.pool_used, total);
      if (off + total > d.POOLCAP) {
        atomicOr(d.err, E_POOL);
        off = NEVER;
      }
    }
    off = __shfl(off, 0);
    if (cand && off != NEVER) d.pool[(size_t)off + pos] = ((uint64_t)v << 34) | key34(key);
  }
  // per chunk: first candidate and count (the chunk walk of merge_payload, which reads none of it when ncand is 0)
  if (total && off != NEVER)
    for (uint32_t c = lane; c < d.NMETA; c += 64) {
      uint32_t before = 0, in = 0;
      for (uint32_t j = 0; j < nall; ++j) {
        const uint32_t t = sc[j];
        before += t < c * MCH;
        in += t != NEVER && t / MCH == c;
      }
      uint32_t* cm = d.chunk_meta + ((size_t)i * d.NMETA + c) * 2;
      cm[0] = off + before;
      cm[1] = in;
    }
  if (lane == 0) d.msgs[i].ncand = off == NEVER ? 0u : total;
  return true;
}

// sharded handles: every message of the tick, one wave each; the unresolved ones go to the list k_sync_diff streams
__global__ void __launch_bounds__(512) k_ack_resolve(ResArgs d, uint32_t k, uint32_t spec, uint32_t timed) {
  if (spec && *(volatile uint32_t*)d.halt) return;
  __shared__ uint32_t sv_[8][64], sc_[8][64];
  __shared__ uint4 slist[8], wlist[8];
  __shared__ uint32_t nstream, nwide, nres, sbase, wbase;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  volatile uint32_t* sv = sv_[wv];  // this wave's lists (volatile: read across lanes)
  volatile uint32_t* sc = sc_[wv];
  const uint32_t nmsg = min(*d.nmsg, d.MSGCAP);
  // block-uniform loop, one message per wave; the stream list and the counters take one atomic per block (a few
  // hundred waves adding to one address one by one took ~17 us per tick at C3)
  for (uint32_t base = blockIdx.x * 8; base < nmsg; base += gridDim.x * 8) {
    if (threadIdx.x == 0) nstream = nwide = nres = 0;
    __syncthreads();
    const uint32_t i = base + wv;
    if (i < nmsg) {  // wave-uniform
      if (res_wave(d, i, k, lane, sv, sc)) {
        if (lane == 0) atomicAdd(&nres, 1u);
      } else if (lane == 0) {  // its entry in the narrow list (one GPU, unpinned live row) or the wide one
        const SyncMsg& mm = d.msgs[i];
        const uint32_t pw = desc_pay(mm);
        const uint4 e = make_uint4(i, mm.src, mm.dst, pw);
        if (d.k8 && (pw == NEVER || (d.W > 1 && pw != DESC_DEFER && (pw & PAY_RX) && !(pw & DESC_PIN))))
          slist[atomicAdd(&nstream, 1u)] = e;
        else
          wlist[atomicAdd(&nwide, 1u)] = e;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (nstream) sbase = atomicAdd(d.ndl, nstream);
      if (nwide) wbase = atomicAdd(d.ndlw, nwide);
      if (nstream + nwide) {  // the messages k_sync_diff streams (the wide ones: 8 B per subject)
        atomicAdd(&d.ctr[C_DIFFMSG_ALL], (unsigned long long)(nstream + nwide));
        if (timed) atomicAdd(&d.ctr[C_DIFFMSG], (unsigned long long)(nstream + nwide));
      }
      if (nwide && d.W > 1) {  // (one GPU: k_sync_diff counts its wide messages)
        atomicAdd(&d.ctr[C_DIFFWIDE_ALL], (unsigned long long)nwide);
        if (timed) atomicAdd(&d.ctr[C_DIFFWIDE], (unsigned long long)nwide);
      }
      if (nres) {
        atomicAdd(&d.ctr[C_ACKRES_ALL], (unsigned long long)nres);
        if (timed) atomicAdd(&d.ctr[C_ACKRES], (unsigned long long)nres);
      }
    }
    __syncthreads();
    if (threadIdx.x < nstream) ((uint4*)d.dlist)[sbase + threadIdx.x] = slist[threadIdx.x];
    if (threadIdx.x >= 64 && threadIdx.x - 64 < nwide) ((uint4*)d.dlist_w)[wbase + threadIdx.x - 64] = wlist[threadIdx.x - 64];
    __syncthreads();  // (slist and the counts are reused)
  }
}

// ------------------------------------------------------------------------------------------------------------
// state hashes (SEMANTICS.md §8), one block per member
__global__ void __launch_bounds__(256) k_hash(Dev d, uint64_t* out, uint32_t now) {
  __shared__ unsigned long long red[4][256];
  uint32_t m = d.lo + blockIdx.x;
  if (m >= d.hi) return;
  unsigned long long hr = 0, hf = 0, hg = 0, hgs = 0;
  const uint32_t* rk = d.rowk + lidx(d, m) * d.NS;
  const uint32_t* ra = d.rowa + lidx(d, m) * d.NS;
  uint32_t fl = d.ms[m].fdLen, gl = d.ms[m].gLen;
  if (d.implicit) {  // the PRECONVERGED row and lists, computed (engine.h list_at)
    const FeistelPerm P0 = list_perm(d, m, 0), P1 = list_perm(d, m, 1);
    for (uint32_t s = threadIdx.x; s < d.N; s += blockDim.x) hr += hpair(s, PRE_REC);
    for (uint32_t p = threadIdx.x; p < fl; p += blockDim.x) hf += hpair((uint64_t)p | (1ull << 40), list_at(P0, m, p));
    for (uint32_t p = threadIdx.x; p < gl; p += blockDim.x) hg += hpair((uint64_t)p | (2ull << 40), list_at(P1, m, p));
  } else {
    for (uint32_t s = threadIdx.x; s < d.N; s += blockDim.x) {
      const uint32_t k = rk[s];
      if ((k & 3u) != ST_ABSENT) hr += hpair(s, rec_join(k, ra[s]));
    }
    for (uint32_t p = threadIdx.x; p < fl; p += blockDim.x) hf += hpair((uint64_t)p | (1ull << 40), d.fdl[lidx(d, m) * d.LCAP + p]);
    for (uint32_t p = threadIdx.x; p < gl; p += blockDim.x) hg += hpair((uint64_t)p | (2ull << 40), d.gl[lidx(d, m) * d.LCAP + p]);
  }
  const bool dead = d.dead_tick[m] != NEVER;  // a crashed member keeps no gossips (SEMANTICS.md §1)
  for (uint32_t g = threadIdx.x; g < d.SLOTS && !dead; g += blockDim.x) {
    if (!d.slot_used[g]) continue;
    uint32_t e = s_get(d, g, m, now + d.lat);
    // receipts applied at the end of tick now-1 belong to P4 of tick `now`: not yet visible
    if (s_held(e) && s_ctick(e) < now) hgs += hpair(d.slot_gid[g], rounds_before(d, m, s_ctick(e)));
  }
  red[0][threadIdx.x] = hr;
  red[1][threadIdx.x] = hf;
  red[2][threadIdx.x] = hg;
  red[3][threadIdx.x] = hgs;
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    uint64_t* o6 = out + (size_t)m * 6;
    o6[0] = red[0][0];
    o6[1] = red[1][0] + mix64((uint64_t)(int64_t)d.ms[m].pingIdx ^ 0xF00Dull) + fl;
    o6[2] = red[2][0] + mix64((uint64_t)(int64_t)d.ms[m].remoteIdx ^ 0xBEEFull) + gl;
    o6[3] = d.ms[m].evHash;
    o6[4] = red[3][0];
    uint64_t ns = d.nextSync[m] == NEVER ? ~0ull : (uint64_t)d.nextSync[m];
    o6[5] = hpair(hpair(hpair(d.ms[m].cidCnt, d.ms[m].syncSeq), d.ms[m].gCounter), ns) +
            mix64((uint64_t)d.ms[m].fdPeriod * 3 + (uint64_t)d.ms[m].gPeriod * 7);
  }
}


__global__ void k_tick_end(Dev d, uint32_t k) { tick_end(d, k); }

// slot sharding: the all-reduced gossip-count deltas of this tick
__global__ void k_held_add(Dev d, const int32_t* sum) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= d.N) return;
  d.held[m] = (uint32_t)((int32_t)d.held[m] + sum[m]);
  d.held_delta[m] = 0;
}
void launch_held_add(const Dev& d, const int32_t* sum, void* stream) {
  hipLaunchKernelGGL(k_held_add, dim3((d.N + 255) / 256), dim3(256), 0, (hipStream_t)stream, d, sum);
}

// every SCRUB ticks (engine.h): the holder entries of recycled slots are cleared, 8 entries (16 B) per lane, so that
// no stale entry outlives the 13-bit tick window of s_get. SLOTS is a multiple of 64: a lane's 8 entries share a member.
__global__ void __launch_bounds__(256) k_s_scrub(Dev d, uint32_t now) {
  const uint64_t nq = (uint64_t)d.N * d.SLOTS / 8;
  const uint32_t ref = now + d.lat;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4* p = (uint4*)d.S + i;
    uint4 v = *p;
    if ((v.x | v.y | v.z | v.w) == 0u) continue;
    const uint32_t g0 = (uint32_t)((i * 8) % d.SLOTS);
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    bool changed = false;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint16_t e = (uint16_t)(w[j >> 1] >> ((j & 1) * 16));
      if (!(e & S16_EVER)) continue;
      const uint32_t g = g0 + j;
      if (!d.slot_used[g] || s16_tick(e, ref) < d.slot_ctick[g]) {
        w[j >> 1] &= ~(0xFFFFu << ((j & 1) * 16));
        changed = true;
      }
    }
    if (changed) *p = make_uint4(w[0], w[1], w[2], w[3]);
  }
}
void launch_s_scrub(const Dev& d, uint32_t now, void* stream) {
  hipLaunchKernelGGL(k_s_scrub, dim3(8192), dim3(256), 0, (hipStream_t)stream, d, now);
}

// ------------------------------------------------------------------------------------------------------------
// host launchers
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

void launch_init(const Dev& d, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_init_members, dim3(cdiv(d.N, 256)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_init_rows, dim3(4096), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_init_lists, dim3(4096), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_init_slots, dim3(cdiv(d.SLOTS, 256)), dim3(256), 0, st, d);
  if (d.W > 1) hipLaunchKernelGGL(k_init_base, dim3(cdiv(d.NS8, 256)), dim3(256), 0, st, d);
}

// timed: this launch is bracketed by profiling events; it adds its message count to ctr[C_DIFFMSG]
// DIFF_WAVES resident blocks per CU (the launch bounds), all of them resident; SWIM_DIFF_GRID overrides it
// (measurements; a value that does not parse, or 0, keeps the default)
static uint32_t diff_grid() {
  const char* e = getenv("SWIM_DIFF_GRID");
  const unsigned long v = e ? strtoul(e, nullptr, 0) : 0ul;
  if (v >= 1 && v <= (1ul << 20)) return (uint32_t)v;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  return DIFF_WAVES * (uint32_t)cus;
}

// a timed launch carries its start / stop events in its own dispatch (hipExtLaunchKernelGGL): the interval is the
// kernel's, not that of two marker packets around it (those read ~4 us per launch longer than rocprofv3)
static void launch_sync_diff(const Dev& d, uint32_t b, hipStream_t st, uint32_t timed, uint32_t spec = 0,
                             const TickEvents* prof = nullptr) {
  static const uint32_t grid = diff_grid();
  if (prof) {
    hipEvent_t e0 = (hipEvent_t)prof->ev[0], e1 = (hipEvent_t)prof->ev[1];
    if (d.W > 1)
      hipExtLaunchKernelGGL(k_sync_diff<true>, dim3(grid), dim3(256), 0, st, e0, e1, 0, d.self, b, timed, spec);
    else
      hipExtLaunchKernelGGL(k_sync_diff<false>, dim3(grid), dim3(256), 0, st, e0, e1, 0, d.self, b, timed, spec);
  } else if (d.W > 1) {
    hipLaunchKernelGGL(k_sync_diff<true>, dim3(grid), dim3(256), 0, st, d.self, b, timed, spec);
  } else {
    hipLaunchKernelGGL(k_sync_diff<false>, dim3(grid), dim3(256), 0, st, d.self, b, timed, spec);
  }
}

// single GPU: the tick is cut in three so that the host can hold back the gossip data plane when no slot is in
// use; the SYNC diff of tick k+1 does not depend on the gossip plane of tick k and is queued in between
// SYNC_ACKs of tick k - 1 resolved from write logs (the rest go to the list k_sync_diff streams)
static void launch_ack_resolve(const Dev& d, uint32_t k, hipStream_t st, bool spec, bool timed) {
  if (k == 0 || !d.ackres) return;
  const uint32_t b = (k - 1) & 1;
  const ResArgs ra{d.halt, d.nmsg + b, d.tl_tick, d.tl_n, d.tlog, d.rowk, d.arena[b], d.msgs[b], d.dlist, d.ndl,
                   d.dlist_w, d.ndlw, d.chunk_meta, d.pool_used, d.err, d.pool, d.ctr, d.NL, d.NS, d.MSGCAP, d.NCHUNK, d.POOLCAP, d.NMETA,
                   d.rowk8 ? 1u : 0u, d.lo, d.W, d.MW, d.mlog, d.base_row, d.rx_mask, d.rx_off, d.xa_recv};
  hipLaunchKernelGGL(k_ack_resolve, dim3(128), dim3(512), 0, st, ra, k, spec ? 1u : 0u, timed ? 1u : 0u);
}

void launch_diff(const Dev& d, uint32_t k, void* stream, const TickEvents* prof, bool spec) {
  hipStream_t st = (hipStream_t)stream;
  launch_ack_resolve(d, k, st, spec, prof != nullptr);
  if (k > 0) launch_sync_diff(d, (k - 1) & 1, st, prof ? 1u : 0u, spec ? 1u : 0u, prof);
}

// link delays: SYNC / SYNC_ACK messages due in the next tick back into this tick's buffer, then the delayed messages
// of this tick into the store (k_sync_diff of the next tick skips them)
__global__ void __launch_bounds__(256) k_sync_redeliver(Dev d, uint32_t k, uint32_t spec) {
  // a speculative batch halted at an earlier tick (halt = k + 1: this tick's member kernel ran and raised it, and its
  // delayed messages still move)
  if (spec) {
    const uint32_t hk = *(volatile uint32_t*)d.halt;
    if (hk != 0 && hk <= k) return;
  }
  __shared__ uint32_t slot[2];
  const uint32_t b = k & 1;
  for (uint32_t e = blockIdx.x; e < d.DSCAP; e += gridDim.x) {
    if (!d.ds_used[e] || d.ds_msg[e].due != k + 1u) continue;
    if (threadIdx.x == 0) {
      slot[0] = atomicAdd(&d.nmsg[b], 1u);
      slot[1] = atomicAdd(&d.arena_used[b], 1u);
      if (slot[0] >= d.MSGCAP) set_err(d, E_MSGS);
      if (slot[1] >= d.ARENA_ROWS) set_err(d, E_ARENA);
    }
    __syncthreads();
    const uint32_t i = slot[0], r = slot[1];
    if (i < d.MSGCAP && r < d.ARENA_ROWS) {
      const uint32_t* src = d.ds_row + (size_t)e * d.NS;
      uint32_t* dst = d.arena[b] + (size_t)r * d.NS;
      for (uint32_t s = threadIdx.x; s < d.NS; s += blockDim.x) dst[s] = src[s];
      __syncthreads();
      if (threadIdx.x == 0) {
        SyncMsg m = d.ds_msg[e];
        m.kind = (m.kind & ~KF_DEFER) | KF_LATE;
        m.payload = r;
        m.ncand = 0;
        m.pad = NEVER;
        m.pin = NEVER;
        d.msgs[b][i] = m;
        const uint32_t old = atomicExch(&d.m_head[(size_t)b * d.N + m.dst], i);
        d.m_next[(size_t)b * d.MSGCAP + i] = old;
        if (old != NEVER) {
          pin_msg(d, b, i);
          pin_msg(d, b, old);
        }
      }
    }
    if (threadIdx.x == 0) {
      d.ds_used[e] = 0;
      d.ds_free[atomicAdd(d.ds_top, 1)] = e;
    }
    __syncthreads();
  }
}
__global__ void __launch_bounds__(256) k_sync_defer(Dev d, uint32_t k, uint32_t spec) {
  // a speculative batch halted at an earlier tick (halt = k + 1: this tick's member kernel ran and raised it, and its
  // delayed messages still move)
  if (spec) {
    const uint32_t hk = *(volatile uint32_t*)d.halt;
    if (hk != 0 && hk <= k) return;
  }
  __shared__ int32_t slot;
  const uint32_t b = k & 1, n = min(d.nmsg[b], d.MSGCAP);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const SyncMsg mm = d.msgs[b][i];
    if (!(mm.kind & KF_DEFER)) continue;
    if (threadIdx.x == 0) {
      const int32_t top = atomicSub(d.ds_top, 1) - 1;
      slot = top >= 0 ? (int32_t)d.ds_free[top] : -1;
      if (top < 0) set_err(d, E_SYNCQ);
    }
    __syncthreads();
    const int32_t e = slot;
    if (e >= 0) {  // the payload as sent: the sender's row at the end of the tick, or its copy-on-write snapshot
      const uint32_t* src = mm.payload == NEVER ? d.rowk + lidx(d, mm.src) * d.NS : d.arena[b] + (size_t)mm.payload * d.NS;
      uint32_t* dst = d.ds_row + (size_t)e * d.NS;
      for (uint32_t s = threadIdx.x; s < d.NS; s += blockDim.x) dst[s] = src[s];
      if (threadIdx.x == 0) {
        d.ds_msg[e] = mm;
        d.ds_used[e] = 1;
      }
    }
    __syncthreads();
  }
}

// Row-sharded handles (W > 1): a delayed SYNC / SYNC_ACK travels to its receiver's shard in the tick it is sent (the
// route and exchange A carry it like any other message, flagged KF_DEFER, and msgs_commit leaves it out of the inbound
// lists); the receiver's shard stores it with its payload as sent at the end of that tick (k_sync_defer_x), and puts
// it back into the inbound list of the tick before its delivery (k_sync_redeliver_x, before the list is committed).
__global__ void __launch_bounds__(256) k_sync_redeliver_x(Dev d, uint32_t k, uint32_t spec) {
  if (spec) {  // a speculative batch halted at an earlier tick
    const uint32_t hk = *(volatile uint32_t*)d.halt;
    if (hk != 0 && hk <= k) return;
  }
  __shared__ uint32_t slot[2];
  const uint32_t b = k & 1;
  for (uint32_t e = blockIdx.x; e < d.DSCAP; e += gridDim.x) {
    if (!d.ds_used[e] || d.ds_msg[e].due != k + 1u) continue;
    if (threadIdx.x == 0) {
      slot[0] = atomicAdd(&d.xn[4], 1u);
      slot[1] = atomicAdd(&d.arena_used[b], 1u);
      if (slot[0] >= d.MSGCAP) set_err(d, E_MSGS);
      if (slot[1] >= d.ARENA_ROWS) set_err(d, E_ARENA);
    }
    __syncthreads();
    const uint32_t j = slot[0], r = slot[1];
    if (j < d.MSGCAP && r < d.ARENA_ROWS) {
      const uint32_t* src = d.ds_row + (size_t)e * d.NS;
      uint32_t* dst = d.arena[b] + (size_t)r * d.NS;
      for (uint32_t s = threadIdx.x; s < d.NS; s += blockDim.x) dst[s] = src[s];
      if (threadIdx.x == 0) {
        SyncMsg m = d.ds_msg[e];
        m.kind = (m.kind & ~KF_DEFER) | KF_LATE;
        m.payload = r;
        m.ncand = 0;
        m.pad = NEVER;
        m.pin = NEVER;
        d.mtmp[j] = m;
      }
    }
    if (threadIdx.x == 0) {
      d.ds_used[e] = 0;
      d.ds_free[atomicAdd(d.ds_top, 1)] = e;
    }
    __syncthreads();
  }
}
__global__ void __launch_bounds__(256) k_sync_defer_x(Dev d, uint32_t k, uint32_t spec) {
  if (spec) {  // this tick's list was not committed (the batch halted at it or earlier)
    const uint32_t hk = *(volatile uint32_t*)d.halt;
    if (hk != 0 && hk <= k + 1u) return;
  }
  __shared__ int32_t slot;
  const uint32_t b = k & 1, n = min(d.nmsg[b], d.MSGCAP);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const SyncMsg mm = d.msgs[b][i];
    if (!(mm.kind & KF_DEFER)) continue;
    if (threadIdx.x == 0) {
      const int32_t top = atomicSub(d.ds_top, 1) - 1;
      slot = top >= 0 ? (int32_t)d.ds_free[top] : -1;
      if (top < 0) set_err(d, E_SYNCQ);
    }
    __syncthreads();
    const int32_t e = slot;
    if (e >= 0) {  // the payload as sent: this shard's sender's row or snapshot, or the chunks a peer shipped
      uint32_t* dst = d.ds_row + (size_t)e * d.NS;
      if (mm.payload & PAY_RX && mm.payload != NEVER) {
        const uint32_t ri = mm.payload & ~PAY_RX;
        const uint64_t* mk = d.rx_mask + (size_t)ri * d.MW;
        const uint32_t* data = (const uint32_t*)(d.xa_recv + d.rx_off[ri]);
        for (uint32_t s = threadIdx.x; s < d.NS; s += blockDim.x) {
          const uint32_t c = s / CH;
          uint32_t v = d.base_row[s];
          if ((mk[c >> 6] >> (c & 63)) & 1ull) {
            uint32_t rank = __popcll(mk[c >> 6] & ((1ull << (c & 63)) - 1ull));
            for (uint32_t q = 0; q < (c >> 6); ++q) rank += __popcll(mk[q]);
            v = data[(size_t)rank * CH + s % CH];
          }
          dst[s] = v;
        }
      } else {
        const uint32_t* src = mm.payload == NEVER ? d.rowk + lidx(d, mm.src) * d.NS : d.arena[b] + (size_t)mm.payload * d.NS;
        for (uint32_t s = threadIdx.x; s < d.NS; s += blockDim.x) dst[s] = src[s];
      }
      if (threadIdx.x == 0) {
        d.ds_msg[e] = mm;
        d.ds_used[e] = 1;
      }
    }
    __syncthreads();
  }
}

__global__ void k_inbox_apply(const Dev* __restrict__ dp, uint32_t k);  // member.hip
void launch_member(const Dev& d, uint32_t k, void* stream, const TickEvents* prof, bool spec, bool split) {
  hipStream_t st = (hipStream_t)stream;
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[2], st);
  if (split) {  // a gossip plane ran last tick: members with many routed receipts run P4 a wave each (k_inbox_apply)
    hipLaunchKernelGGL(k_member_tick_t<BODY_SPLIT>, dim3(cdiv(d.NL, 256)), dim3(256), 0, st, d.self, k, 0u);
    hipLaunchKernelGGL(k_inbox_apply, dim3(2048), dim3(256), 0, st, d.self, k);
    hipLaunchKernelGGL(k_member_tick_t<BODY_RESUME>, dim3(cdiv(d.NL, 256)), dim3(256), 0, st, d.self, k, 1u);  // + tick_flag
  } else {
    hipLaunchKernelGGL(k_member_tick_t<BODY_FULL>, dim3(cdiv(d.NL, 256)), dim3(256), 0, st, d.self, k, spec ? 3u : 1u);  // + tick_flag
  }
  if (d.dly_on) {
    hipLaunchKernelGGL(k_sync_redeliver, dim3(256), dim3(256), 0, st, d, k, spec ? 1u : 0u);
    hipLaunchKernelGGL(k_sync_defer, dim3(256), dim3(256), 0, st, d, k, spec ? 1u : 0u);
  }
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[3], st);
}

// gossip.hip
void launch_gossip_send(const Dev& d, uint32_t k, hipStream_t st, const TickEvents* prof);
void launch_gossip_apply(const Dev& d, uint32_t k, hipStream_t st);
void launch_unpack_b(const Dev& d, uint32_t k, hipStream_t st);

void launch_gossip(const Dev& d, uint32_t k, void* stream, const TickEvents* prof) {
  hipStream_t st = (hipStream_t)stream;
  launch_gossip_send(d, k, st, prof);
  launch_gossip_apply(d, k, st);
}

// exclusive scan of n counts (n <= 2^20)
void launch_scan(const uint32_t* in, uint32_t* out, uint32_t* part, uint32_t n, hipStream_t st) {
  uint32_t nb = cdiv(n, 1024);
  hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, st, in, out, part, n);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, st, part, nb);
  hipLaunchKernelGGL(k_scan_add, dim3(cdiv(n, 256)), dim3(256), 0, st, out, part, n);
}

// receipts routed to P4: counting sort by member, then each member's receipts by gossip id
void launch_receipt_routing(const Dev& d, hipStream_t st) {
  hipLaunchKernelGGL(k_count_rc, dim3(256), dim3(256), 0, st, d.rc_raw, d.rc_n, d.RCAP, d.rc_cnt);
  launch_scan(d.rc_cnt, d.rc_off, d.scan_part, d.N, st);
  hipLaunchKernelGGL(k_scatter_rc, dim3(256), dim3(256), 0, st, d, d.rc_raw, d.rc_n, d.RCAP, d.rc_off, d.rc_fill,
                     d.rc_slot, d.rc_key);
  hipLaunchKernelGGL(k_seg_sort, dim3(1024), dim3(256), 0, st, d.rc_key, d.rc_slot, d.rc_key2, d.rc_slot2, d.rc_off,
                     d.rc_cnt, d.sg_list, d.nsg, d.sort_cap, d.fb);
}

// sharded tick (W > 1): A = SYNC diff + member control + pack exchange A; B = unpack A, the rounds' holder-state
// changes and this shard's targets' sends, pack exchange B (their first receipts); C = peers' first receipts into the
// replicated holder state, this shard's receipts, routing, slot recycling
void launch_tick_a(const Dev& d, uint32_t k, void* stream, const TickEvents* prof, bool spec) {
  hipStream_t st = (hipStream_t)stream;
  uint32_t b = k & 1;
  const uint32_t sp = spec ? 1u : 0u;
  launch_ack_resolve(d, k, st, spec, prof != nullptr);
  if (k > 0) launch_sync_diff(d, (k - 1) & 1, st, prof ? 1u : 0u, sp, prof);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[2], st);
  hipLaunchKernelGGL(k_member_tick_t<BODY_FULL>, dim3(cdiv(d.NL, 256)), dim3(256), 0, st, d.self, k, spec ? 2u : 0u);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[3], st);
  if (d.dly_on) hipLaunchKernelGGL(k_sync_redeliver_x, dim3(256), dim3(256), 0, st, d, k, sp);
  hipLaunchKernelGGL(k_pack_all, dim3(16, d.W), dim3(256), 0, st, d, b, sp);  // route + exchange-A regions
}

void launch_tick_b(const Dev& d, uint32_t k, void* stream, const TickEvents* prof, bool gossip, bool spec) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_unpack_a, dim3(32, d.W), dim3(256), 0, st, d, k, gossip ? 0u : 1u, spec ? 1u : 0u);
  if (d.dly_on) hipLaunchKernelGGL(k_sync_defer_x, dim3(256), dim3(256), 0, st, d, k, spec ? 1u : 0u);
  if (!gossip) {  // no gossip slot in use on any shard: nothing to send, deliver or recycle; no exchange B
    if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[4], st);
    if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[5], st);
    return;
  }
  launch_gossip_send(d, k, st, prof);
  hipLaunchKernelGGL(k_pack_b, dim3(64, d.W), dim3(256), 0, st, d);
}

void launch_tick_c(const Dev& d, uint32_t k, void* stream, bool gossip) {
  hipStream_t st = (hipStream_t)stream;
  if (!gossip) return;  // k_unpack_a closed the tick
  launch_unpack_b(d, k, st);
  launch_gossip_apply(d, k, st);
  hipLaunchKernelGGL(k_round_reset, dim3(16, d.W), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_tick_end, dim3(1), dim3(64), 0, st, d, k);
}

// swim_update_metadata of a member with no column yet: column u; every local observer stores version 0 (the only
// version it could have fetched so far)
__global__ void k_md_column(Dev d, uint32_t m, uint32_t u) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) d.md_uidx[m] = u;
  if (i < d.NL) d.md_ver[(size_t)i * MDU + u] = 0;
}

void launch_md_column(const Dev& d, uint32_t m, uint32_t u, void* stream) {
  hipLaunchKernelGGL(k_md_column, dim3((d.NL + 255) / 256), dim3(256), 0, (hipStream_t)stream, d, m, u);
}

// swim_join: a dormant member starts at tick k as a fresh process (ClusterImpl.join0, schedules from k) with its seeds
struct JoinSeeds {
  uint32_t s[16];
};
__global__ void k_join(Dev d, uint32_t m, uint32_t k, JoinSeeds js, uint32_t n) {
  if (threadIdx.x != 0) return;
  d.dead_tick[m] = NEVER;
  d.start_tick[m] = k;
  d.nextPing[m] = k + mc_ping_t(d, m);
  d.nextGossip[m] = d.firstGossip[m] = k + d.gossip_t;
  d.jseed_n[m] = n;
  for (uint32_t i = 0; i < n; ++i) d.jseeds[(size_t)m * 16 + i] = js.s[i];
}

void launch_join(const Dev& d, uint32_t m, uint32_t k, const uint32_t* seeds, uint32_t n, void* stream) {
  JoinSeeds js{};
  for (uint32_t i = 0; i < n && i < 16; ++i) js.s[i] = seeds[i];
  hipLaunchKernelGGL(k_join, dim3(1), dim3(64), 0, (hipStream_t)stream, d, m, k, js, n);
}


void launch_hash(const Dev& d, uint64_t* out, uint32_t now, void* stream) {
  hipLaunchKernelGGL(k_hash, dim3(d.NL), dim3(256), 0, (hipStream_t)stream, d, out, now);
}

}  // namespace swim
