// kernels.hip — initialisation, message routing, the SYNC-payload diff, the gossip data plane, kill and state hashes.
#include <hip/hip_runtime.h>

#include "dev_util.h"

namespace swim {

__global__ void k_member_tick(const Dev* __restrict__ dp, uint32_t k, uint32_t flag);  // member.hip
// shard.hip
__global__ void k_sync_route(Dev d, uint32_t b);
__global__ void k_pack_a(Dev d, uint32_t b);
__global__ void k_pack_a_chunks(Dev d, uint32_t b);
__global__ void k_unpack_a(Dev d, uint32_t k, uint32_t end);
__global__ void k_pack_b(Dev d);
__global__ void k_unpack_b_sweeps(Dev d, uint32_t k);
__global__ void k_unpack_b_deliv(Dev d, uint32_t k);
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
  d.tsize[m] = pre ? d.N : 1;
  d.fdLen[m] = pre ? d.N - 1 : 0;
  d.gLen[m] = pre ? d.N - 1 : 0;
  d.fdPeriod[m] = d.gPeriod[m] = d.gCounter[m] = 0;
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
  d.cidCnt[m] = d.syncSeq[m] = d.evSeq[m] = d.held[m] = 0;
  d.timerMin[m] = NEVER;
  d.initFlags[m] = d.initDeadline[m] = d.initCidBase[m] = d.initN[m] = 0;
  d.nsub[m] = d.npath[m] = d.nfetch[m] = 0;
  d.fnext[m] = NEVER;
  d.pingIdx[m] = 0;
  d.remoteIdx[m] = pre ? 0 : -1;
  for (int i = 0; i < 8; ++i) d.sel[(size_t)m * 8 + i] = 0;
  d.evHash[m] = 0;
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
    }
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
  d.slot_holders[g] = 0;
  // each shard allocates only from its own slot range [rank SPR, (rank+1) SPR), so slot ids are global
  if (g < d.SPR) d.free_list[g] = d.rank * d.SPR + d.SPR - 1 - g;
}

// the SYNC baseline row (record keys): what a PRECONVERGED row starts as, an empty row for a cold join
__global__ void k_init_base(Dev d) {
  uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < d.NS) d.base_row[s] = (s < d.N && d.init_mode == 1) ? key32(rec_key(ST_ALIVE, 0)) : 0u;
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
    uint32_t p = off[t] + atomicAdd(&fill[t], 1u);
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

__global__ void __launch_bounds__(256) k_seg_sort(uint64_t* key, uint32_t* val, uint64_t* tkey, uint32_t* tval,
                                                  const uint32_t* off, const uint32_t* cnt, uint32_t nseg,
                                                  const uint32_t* nitems, uint32_t run, unsigned long long* fb) {
  __shared__ uint64_t K[SORT_MAX];
  __shared__ uint32_t V[SORT_MAX];
  if (*nitems == 0) return;  // nothing was routed this tick
  for (uint32_t sgi = blockIdx.x; sgi < nseg; sgi += gridDim.x) {
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
// :456-467). This is the HBM-bound hot loop: 2 x 4 B read per subject per merge (key32, swim_common.h). SHARDED adds
// payloads received from other shards (baseline row + shipped chunks); the single-GPU instance has only local rows
// and snapshots.
// this lane's 8 payload keys and 8 receiver keys of work item w (message w / NCHUNK, chunk w % NCHUNK): the payload
// is the sender's live row or its copy-on-write snapshot; for a payload received from another shard, the shipped
// chunk if it differs from the baseline, else the baseline
template <bool SHARDED>
__device__ __forceinline__ void diff_fetch(const Dev& d, uint32_t b, uint32_t w, uint4 (&x)[4]) {
  const uint32_t mi = w / d.NCHUNK, c = w % d.NCHUNK;
  const SyncMsg& mm = d.msgs[b][mi];
  const uint32_t s0 = c * CH + threadIdx.x * 8;
  if (s0 >= d.NS) {  // NS is a multiple of 8: a 32-B group is wholly in or out; padding entries are 0 (absent)
    x[0] = x[1] = x[2] = x[3] = make_uint4(0, 0, 0, 0);
    return;
  }
  const uint32_t* p8;
  if (mm.payload == NEVER) {
    p8 = d.rowk + lidx(d, mm.src) * d.NS + s0;
  } else if (SHARDED && (mm.payload & PAY_RX)) {
    const uint32_t ri = mm.payload & ~PAY_RX;
    const uint64_t* mk = d.rx_mask + (size_t)ri * d.MW;
    if ((mk[c >> 6] >> (c & 63)) & 1ull) {
      uint32_t rank = __popcll(mk[c >> 6] & ((1ull << (c & 63)) - 1ull));
      for (uint32_t q = 0; q < (c >> 6); ++q) rank += __popcll(mk[q]);
      p8 = (const uint32_t*)(d.xa_recv + d.rx_off[ri]) + (size_t)rank * CH + threadIdx.x * 8;
    } else {
      p8 = d.base_row + s0;
    }
  } else {
    p8 = d.arena[b] + (size_t)mm.payload * d.NS + s0;
  }
  const uint32_t* r8 = d.rowk + lidx(d, mm.dst) * d.NS + s0;
  // (non-temporal loads measured 1.5x slower here on gfx950)
  x[0] = ld_c4(p8);
  x[1] = ld_c4(p8 + 4);
  x[2] = ld_c4(r8);
  x[3] = ld_c4(r8 + 4);
}

// k_sync_diff: for every SYNC / SYNC_ACK sent in tick k-1, stream the payload's key plane (the sender's live row,
// or its copy-on-write snapshot) against the receiver's key plane and extract, per 2048-subject chunk and in
// subject order, the records that differ (the eager `!r1.equals(table.get(id))` filter of syncMembership,
// :456-467). This is the HBM-bound hot loop: 2 x 4 B read per subject per merge (key32, swim_common.h). Each block
// walks its work items grid-strided with the next item's loads in flight while it tests the current one. SHARDED
// adds payloads received from other shards (baseline row + shipped chunks); the single-GPU instance has only local
// rows and snapshots.
template <bool SHARDED>
__global__ void __launch_bounds__(256) k_sync_diff(Dev d, uint32_t b, uint32_t timed) {
  __shared__ uint32_t scan[256];
  __shared__ uint32_t base;
  uint32_t nmsg = d.nmsg[b] < d.MSGCAP ? d.nmsg[b] : d.MSGCAP;
  if (timed && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&d.ctr[C_DIFFMSG], (unsigned long long)nmsg);
  uint32_t total = nmsg * d.NCHUNK;
  uint4 cur[4];
  if (blockIdx.x < total) diff_fetch<SHARDED>(d, b, blockIdx.x, cur);
  for (uint32_t w = blockIdx.x; w < total; w += gridDim.x) {
    uint4 nxt[4];
    if (w + gridDim.x < total) diff_fetch<SHARDED>(d, b, w + gridDim.x, nxt);
    const uint32_t mi = w / d.NCHUNK, c = w % d.NCHUNK;
    const uint32_t s0 = c * CH + threadIdx.x * 8;
    const uint32_t pin = d.msgs[b][mi].pin;
    if (pin != NEVER && d.msgs[b][mi].payload == NEVER && s0 < d.NS) {  // a live-row payload read again later (pin_msg)
      uint4* dst = (uint4*)(d.arena[b] + (size_t)pin * d.NS + s0);
      dst[0] = cur[0];
      dst[1] = cur[1];
    }
    const uint32_t p[8] = {cur[0].x, cur[0].y, cur[0].z, cur[0].w, cur[1].x, cur[1].y, cur[1].z, cur[1].w};
    const uint32_t r[8] = {cur[2].x, cur[2].y, cur[2].z, cur[2].w, cur[3].x, cur[3].y, cur[3].z, cur[3].w};
    uint32_t mask = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if ((p[j] & 3u) != ST_ABSENT && p[j] != r[j]) mask |= 1u << j;
    uint32_t nc = __popc(mask);
    if (!__syncthreads_or(nc)) {  // steady state: the whole 2048-subject item matches
      if (threadIdx.x == 0) {
        uint32_t* cm = d.chunk_meta + ((size_t)mi * d.NCHUNK + c) * 2;
        cm[0] = 0;
        cm[1] = 0;
      }
    } else {
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
        uint32_t bo = atomicAdd(d.pool_used, totc);
        if (bo + totc > d.POOLCAP) {  // no room: nothing of this item is written (the error aborts the step)
          atomicOr(d.err, E_POOL);
          totc = 0;
          bo = NEVER;
        }
        base = bo;
        uint32_t* cm = d.chunk_meta + ((size_t)mi * d.NCHUNK + c) * 2;
        cm[0] = bo;
        cm[1] = totc;
        if (totc) atomicAdd(&d.msgs[b][mi].ncand, totc);
      }
      __syncthreads();
      uint32_t o = base + incl - nc;
      if (base != NEVER)  // (an overflowed item must not overwrite other items' candidates)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (mask & (1u << j)) d.pool[o++] = ((uint64_t)(s0 + j) << 34) | key34(p[j]);
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
  }
}

// ------------------------------------------------------------------------------------------------------------
// gossip data plane (GossipProtocolImpl.java:139-308 for all members at once)
//
// infectedFrom is never stored. `y ∈ infectedFrom_x(g)` at x's round at tick tau holds iff y delivered g to x by a
// send in one of y's logged rounds t2 with c_x <= t2 + lat <= tau, where c_x is the creation tick of x's current
// state for g. Whether such a send was delivered depends, one level down, on whether x had delivered g to y
// earlier (then y skips x), and so on. The dependency only runs over the contact events between the pair
// (x's rounds that targeted y, y's rounds that targeted x). Those are replayed in tick order as a small dynamic
// program, so there is no recursion.
struct Contact {
  uint32_t tick, slot, spread, dir;  // dir 0: y -> x, 1: x -> y
};

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
    }
    uint32_t n = (uint32_t)(e[2] >> 32);  // total rebirths so far; the ring keeps the latest 6
    uint32_t* c = (uint32_t*)(e + 3);
    c[n % HKEEP] = cprev;
    e[2] = (uint64_t)member | ((uint64_t)(n + 1) << 32);
    return;
  }
  if (atomicOr(d.err, E_REBORN) == 0) d.err[1] = 1;  // info 1: the history table is full (HCAP)
}

// creation tick of member's incarnation of g that existed at tick tau (NEVER if none)
__device__ uint32_t inc_at(const Dev& d, uint32_t member, uint32_t g, uint64_t gid, uint32_t tau) {
  uint32_t e = d.S[(size_t)g * d.N + member];
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
    const size_t li = (size_t)x * d.LOGW + (pos - e) % d.LOGW;
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
  for (uint32_t i = 0; i < n; ++i) cinc[i] = NEVER - 1;  // not computed yet
  for (int pass = 0; pass < 8; ++pass) {
    bool changed = false;
    for (int i = (int)n - 1; i >= 0; --i) {
      const Contact& c = ev[i];
      uint32_t rin = c.dir == 0 ? 0 : 1;  // receiver index into lo_in
      if (lo_in[rin] == NEVER || c.tick + lat < lo_in[rin]) continue;
      if (cinc[i] == NEVER - 1) cinc[i] = inc_at(d, c.dir == 0 ? y : x, g, gid, c.tick);
      uint32_t cs = cinc[i];
      uint32_t snd = c.dir == 0 ? y : x;
      if (cs == NEVER || rounds_before(d, snd, cs) + c.spread < rounds_before(d, snd, c.tick)) continue;
      if (swept_before(d, snd, cs, c.tick)) continue;
      uint32_t sin = 1 - rin;
      if (lo_in[sin] == NEVER || cs < lo_in[sin]) {
        lo_in[sin] = cs;
        changed = true;
      }
    }
    if (!changed) break;
  }
  // deliveries into x come from y's log (oldest[0]); into y from x's log (oldest[1])
  // (oldest 0: that ring never wrapped, so it holds every round since tick 0)
  if ((lo_in[0] != NEVER && oldest[0] && lo_in[0] < oldest[0] + lat) ||
      (lo_in[1] != NEVER && oldest[1] && lo_in[1] < oldest[1] + lat)) {
    if (atomicOr(d.err, E_LOGWIN) == 0) {
      d.err[1] = tau;
      d.err[2] = lo_in[0];
      d.err[3] = lo_in[1];
      d.err[4] = oldest[0];
      d.err[5] = oldest[1];
    }
  }
  uint32_t del[2][CM];
  uint32_t nd[2] = {0, 0};
  for (uint32_t i = 0; i < n; ++i) {
    const Contact& c = ev[i];
    uint32_t snd = c.dir == 0 ? y : x;
    // the sender held g at that round (its incarnation then), inside its spread window (selectGossipsToSend :246)
    uint32_t cs = cinc[i] != NEVER - 1 ? cinc[i] : inc_at(d, snd, g, gid, c.tick);
    if (cs == NEVER) continue;
    if (rounds_before(d, snd, cs) + c.spread < rounds_before(d, snd, c.tick)) continue;
    if (swept_before(d, snd, cs, c.tick)) continue;  // x no longer held it
    // the receiver delivered g to the sender during that incarnation: infectedFrom (isInfected :247)
    uint32_t od = 1 - c.dir;  // opposite direction
    bool blocked = false;
    for (uint32_t q = 0; q < nd[od] && !blocked; ++q) blocked = del[od][q] + lat >= cs && del[od][q] + lat <= c.tick;
    if (blocked) continue;
    if (lost_gossip(d, snd, c.dir == 0 ? x : y, c.tick, c.slot, gid)) continue;
    del[c.dir][nd[c.dir]++] = c.tick;
  }
  for (uint32_t q = 0; q < nd[0]; ++q)
    if (del[0][q] + lat >= cx) return true;
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
          ev[j] = Contact{t2, s2, d.log_spread[li], (uint32_t)side};
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
    const uint32_t t2 = rec[4 + 2 * i];
    relevant |= ((rec[5 + 2 * i] >> 8) & 1u) == 0 && t2 >= born && t2 + d.lat >= cx;
  }
  if (!relevant) return false;
  Contact ev[CEV];
  uint32_t n = 0;
  for (uint32_t i = 0; i < nall; ++i) {
    const uint32_t t2 = rec[4 + 2 * i], w = rec[5 + 2 * i];
    if (t2 < born) continue;
    ev[n++] = Contact{t2, w & 0xFFu, w >> 16, (w >> 8) & 1u};
  }
  const uint32_t oldest[2] = {rec[1], rec[2]};
  return replay_pair<CEV>(d, x, y, g, gid, tau, cx, ev, n, oldest);
}

__global__ void k_gossip_active(Dev d, uint32_t k, uint32_t* active, uint32_t* nactive) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g == 0) *d.slow_n = *d.rn = *d.rp_n = 0;  // deferred sends, round members and replays of this tick
  if (g >= d.SLOTS || !d.slot_used[g]) return;
  // members stopped after their leave completed at tick k - 1 hold nothing any more (as k_kill)
  const uint32_t pb = (k - 1) & 1u, nd = k > 0 ? min(d.deaths_n[pb], DEATHCAP) : 0u;
  for (uint32_t i = 0; i < nd; ++i)
    if (s_held(d.S[(size_t)g * d.N + d.deaths[(size_t)pb * DEATHCAP + i]])) atomicSub(&d.slot_holders[g], 1);
  active[atomicAdd(nactive, 1u)] = g;
}

// per member (all N, every shard): swthr = creation-tick bound of the gossips it sweeps in its round this tick
// (sweepGossips :283-308): sweeps g iff rounds_before(c) < P = period - 2 (spread + 1) iff c < swthr; 0 = sweeps none
__global__ void k_round_info(Dev d) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= d.N) return;
  uint32_t thr = 0;
  if (d.tround[m]) {
    const int64_t P = (int64_t)d.tperiod[m] - (int64_t)sweep_after(d.tspread[m]);
    const uint32_t f = d.firstGossip[m];
    if (P >= 1) thr = f == NEVER ? NEVER : (uint32_t)min<int64_t>((int64_t)NEVER, (int64_t)f + (P - 1) * d.gossip_t + 1);
  }
  d.swthr[m] = thr;
}

// contact lists: did target t = T[m][s] choose m in a logged round inside the look-back window? If so, cache the
// pair's contact events in both directions (independent of the gossip) for blocked_pair_cached
__global__ void k_gossip_contacts(Dev d, uint32_t k) {
  uint32_t i = d.lo * d.F + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.hi * d.F) return;
  uint32_t m = i / d.F, s = i % d.F;
  uint32_t flag = 0;
  if (d.tround[m] && s < d.tcnt[m]) {
    uint32_t t = d.T[i];
    for (uint32_t e = 0; e < d.LOGW && !flag; ++e) {
      size_t lo = (size_t)t * d.LOGW + e;
      uint32_t t2 = d.log_tick[lo];
      if (t2 == NEVER || t2 >= k) continue;
      uint32_t n = d.log_cnt[lo];
      for (uint32_t s2 = 0; s2 < n; ++s2)
        if (d.log_tg[lo * d.F + s2] == m) flag = 1;
    }
    if (flag) {
      Contact ev[CEV];
      uint32_t oldest[2];
      uint32_t* rec = d.cev + (size_t)i * CEVW;
      uint32_t n = collect_contacts<CEV>(d, m, t, k, 0, ev, oldest);
      if (n > d.cev_cap) n = CEV + 1;  // SWIM_CAPS: a smaller cache overflows into k_gossip_send_slow
      rec[0] = n;
      rec[1] = oldest[0];
      rec[2] = oldest[1];
      uint32_t last_in = NEVER;  // latest y -> x contact (NEVER: none); overflow is flagged by n alone
      if (n <= CEV)
        for (uint32_t j = 0; j < n; ++j) {
          rec[4 + 2 * j] = ev[j].tick;
          rec[5 + 2 * j] = ev[j].slot | (ev[j].dir << 8) | (ev[j].spread << 16);
          if (ev[j].dir == 0) last_in = ev[j].tick;  // events are in tick order
        }
      rec[3] = last_in;
      // a gossip inside m's window this round was created after tick k - (spread + 1) * gossip_t, so a contact
      // t -> m at or before that tick - lat can never put t in infectedFrom_m of any gossip m sends now
      const int64_t horizon = (int64_t)k - (int64_t)(d.tspread[m] + 1u) * d.gossip_t;
      if (n > CEV)
        d.cin[i] = CIN_SLOW;
      else
        d.cin[i] = last_in == NEVER || (int64_t)last_in + d.lat <= horizon ? NEVER : last_in;
    }
  }
  d.tcontact[i] = flag;
  if (!flag) d.cin[i] = NEVER;
  if (s == 0 && d.tround[m]) {  // compact list of this tick's round members (k_gossip_send iterates over it)
    uint32_t r = wave_append(d.rn);
    d.rlist[r] = m;
  }
}

// one counted send of gossip g from m to its round target t = T[m][s] (isInfected already checked): the receipt is
// potential unless t holds g past this tick; a loss draw, then the first sender of (g, t) queues the delivery
// potential: the caller already knows t does not hold g past this tick (k_gossip_send's candidates come from
// WB & ~HB[t], and HB is exactly that test: nothing changes S between k_gossip_scan and the sends but PENDING bits)
__device__ __forceinline__ void send_tail(const Dev& d, uint32_t g, uint32_t m, uint32_t s, uint32_t t, uint32_t k,
                                          uint64_t gid, uint32_t* Sg, int ep, bool potential = false) {
  if (d.dbg_send) {
    uint32_t di = atomicAdd(d.dbg_send_n, 1u);
    if (di < d.dbg_send_cap) {
      uint32_t* r = d.dbg_send + (size_t)di * 5;
      r[0] = k;
      r[1] = m;
      r[2] = (uint32_t)gid;
      r[3] = (uint32_t)(gid >> 32);
      r[4] = t;
    }
  }
  if (!potential) {
    const uint32_t et = Sg[t];
    // potential unless t holds g and does not sweep it in its own round this tick (a delivery would re-create it)
    if (s_held(et) && !(s_ctick(et) < d.swthr[t])) return;
  }
  if (lost_gossip_ep(d, ep, m, t, k, s, gid)) return;
  uint32_t old = atomicOr(&Sg[t], S_PENDING);
  if (!(old & S_PENDING)) {
    uint32_t di = wave_append(d.deliv_n);
    if (di < d.DCAP)
      d.deliv[di] = ((uint64_t)g << 32) | t;
    else
      atomicOr(d.err, E_DELIV);
  }
}

// The gossip round is bit-parallel over groups of 64 active slots (active[64 q .. 64 q + 63] = group q). Both masks
// are member-major, [member][QW] words, so a sender reads its window mask and its target's held mask as contiguous
// rows:
//   k_gossip_scan  streams the holder table once per tick, coalesced (lane = member), and writes per (member, group)
//                  two 64-bit masks: HB = slots the member holds past this tick (held and not sweeping them in its
//                  round: swthr), WB = slots a round member holds inside its spread window (selectGossipsToSend
//                  :239-250). It also performs the round members' sweeps (sweepGossips :283-308). A block covers 256
//                  members x QT groups and transposes the masks through LDS, so every row segment is one 128-B store.
//   k_gossip_send  one wave per (round member m, target slot s), lanes over the groups: each load of WB[m][q] and
//                  HB[t][q] is a 512-B contiguous segment. t gets WB minus the slots t is in infectedFrom of
//                  (isInfected, cached contact replay, only where a contact can matter); the count is a popcount,
//                  and the first-receipt candidates are WB & ~HB[t].
// A pair whose contact list overflowed is deferred to k_gossip_send_slow (the full replay needs a large stack).
__global__ void __launch_bounds__(256) k_gossip_scan(const Dev* __restrict__ dp, uint32_t k, const uint32_t* active,
                                                     const uint32_t* nactive) {
  const Dev& d = *dp;
  const uint32_t na = *nactive, ngroups = (na + 63) / 64;
  const uint32_t mchunks = (d.N + 255) / 256;
  for (uint32_t w = blockIdx.x; w < ngroups * mchunks; w += gridDim.x) {
    const uint32_t q = w / mchunks, m0 = (w % mchunks) * 256 + threadIdx.x;
    const bool act = m0 < d.N;  // lanes past N take part in the wave OR below with nothing to sweep
    const uint32_t m = act ? m0 : d.N - 1;
    const uint32_t gn = act ? min(64u, na - q * 64) : 0u;
    const uint32_t thr = d.swthr[m];
    const bool rnd = act && d.tround[m] && m >= d.lo && m < d.hi;  // this shard's round members send and sweep
    uint32_t per = 0, sp = 0, fg = NEVER;
    if (rnd) {
      per = d.tperiod[m];
      sp = d.tspread[m];
      fg = d.firstGossip[m];
    }
    // pass 1 has no side effects, so the 64 holder-word loads pipeline; the sweeps (rare) run after it, per slot
    // that any lane of the wave sweeps
    unsigned long long hb = 0, wb = 0, swm = 0;
#pragma unroll 8
    for (uint32_t j = 0; j < gn; ++j) {
      const uint32_t e = d.S[(size_t)active[q * 64 + j] * d.N + m];
      if (s_held(e)) {
        const uint32_t c = s_ctick(e);
        if (!(c < thr)) hb |= 1ull << j;
        if (rnd) {
          const uint32_t infP = (fg == NEVER || c <= fg) ? 0u : (c - fg + d.gossip_t - 1) / d.gossip_t;  // rounds_before
          if (infP + sp >= per) wb |= 1ull << j;               // selectGossipsToSend window (:246)
          if (per > infP + sweep_after(sp)) swm |= 1ull << j;  // sweepGossips (:283-308)
        }
      }
    }
    unsigned long long any = swm;  // the slots any lane of this wave sweeps (wave-uniform loop below)
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t lo = __shfl_xor((uint32_t)any, o), hi = __shfl_xor((uint32_t)(any >> 32), o);
      any |= ((unsigned long long)hi << 32) | lo;
    }
    for (; any; any &= any - 1) {
      const uint32_t j = (uint32_t)(__ffsll((long long)any) - 1), g = active[q * 64 + j];
      const bool sweep = (swm >> j) & 1ull;
      if (sweep) {
        atomicOr(&d.S[(size_t)g * d.N + m], S_SWEPT);
        if (d.XW > 1)
          atomicSub(&d.held_delta[m], 1);
        else
          atomicSub(&d.held[m], 1u);
        on_sweep(d, g, m, k);
        if (d.W > 1) {  // applied on the other shards from exchange B
          uint32_t i = wave_append(&d.xn[2]);
          if (i < d.SWCAP)
            d.sw_rec[i] = ((uint64_t)g << 32) | m;
          else
            atomicOr(d.err, E_XCAP);
        }
      }
      // the slot's holder count, once per wave (64 lanes of one slot would serialise on its address)
      const unsigned long long sm = __ballot(sweep);
      if (sm && __lane_id() == (uint32_t)(__ffsll((long long)sm) - 1)) atomicSub(&d.slot_holders[g], (int)__popcll(sm));
    }
    if (!act) continue;
    d.HBq[(size_t)q * d.N + m] = hb;  // group-major here (coalesced); k_mask_transpose makes the member-major rows
    d.WBq[(size_t)q * d.N + m] = wb;
  }
}

// [q][N] -> [N][QW] for both masks, 64 x 64 word tiles through LDS (512-B contiguous reads and writes)
__global__ void __launch_bounds__(256) k_mask_transpose(const Dev* __restrict__ dp, const uint32_t* nactive) {
  const Dev& d = *dp;
  __shared__ unsigned long long tile[2][64][65];
  const uint32_t ngroups = (*nactive + 63) / 64, qt = (ngroups + 63) / 64, mt = (d.N + 63) / 64;
  const uint32_t lane = threadIdx.x & 63, row0 = threadIdx.x >> 6;  // 4 rows per pass
  for (uint32_t w = blockIdx.x; w < qt * mt; w += gridDim.x) {
    const uint32_t q0 = (w / mt) * 64, m0 = (w % mt) * 64;
    for (uint32_t r = row0; r < 64; r += 4) {  // rows q0 + r, columns m0 + lane
      const uint32_t q = q0 + r, m = m0 + lane;
      const bool in = q < ngroups && m < d.N;
      tile[0][r][lane] = in ? d.HBq[(size_t)q * d.N + m] : 0ull;
      tile[1][r][lane] = in ? d.WBq[(size_t)q * d.N + m] : 0ull;
    }
    __syncthreads();
    for (uint32_t r = row0; r < 64; r += 4) {  // rows m0 + r, columns q0 + lane
      const uint32_t m = m0 + r, q = q0 + lane;
      if (m < d.N && q < ngroups) {
        d.HB[(size_t)m * d.QW + q] = tile[0][lane][r];
        d.WB[(size_t)m * d.QW + q] = tile[1][lane][r];
      }
    }
    __syncthreads();
  }
}

// the r-th (from 0) set bit of w
__device__ __forceinline__ uint32_t nth_bit(unsigned long long w, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t half = 32; half > 0; half >>= 1) {
    const uint32_t c = (uint32_t)__popcll(w & ((1ull << half) - 1ull));
    if (r >= c) {
      r -= c;
      w >>= half;
      pos += half;
    }
  }
  return pos;
}

// reserve n entries per lane on a wave-shared counter with one atomic (every lane of the wave must call it)
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

__global__ void __launch_bounds__(256) k_gossip_send(const Dev* __restrict__ dp, uint32_t k, const uint32_t* active,
                                                     const uint32_t* nactive) {
  const Dev& d = *dp;
  __shared__ unsigned long long red[4];
  const uint32_t na = *nactive, nr = *d.rn, ngroups = (na + 63) / 64;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const int ep = epoch_at(d, k);
  unsigned long long sends = 0;
  uint32_t st[4] = {0, 0, 0, 0};  // SWIM_EXP & 4: items with window bits, contact-loop bits, replays, first-receipt candidates
  // wave-uniform work unit = (round member, target slot, chunk of 64 slot groups): a pair with many gossips in its
  // window is spread over several waves instead of holding one wave for all its chunks (the kernel waits for the
  // longest wave)
  const uint32_t nch = (ngroups + 63) / 64;
  const uint64_t units = (uint64_t)nr * d.F * nch;
  for (uint64_t w = blockIdx.x * 4 + wave; w < units; w += gridDim.x * 4) {
    const uint32_t item = (uint32_t)(w / nch), ch = (uint32_t)(w % nch);
    const uint32_t ri = item / d.F, s = item % d.F;
    const uint32_t m = d.rlist[ri];
    if (s >= d.tcnt[m]) continue;
    const size_t ms = (size_t)m * d.F + s;
    const uint32_t t = d.T[ms], ci = d.cin[ms];
    const unsigned long long* wrow = d.WB + (size_t)m * d.QW;
    const unsigned long long* hrow = d.HB + (size_t)t * d.QW;
    for (uint32_t q0 = ch * 64; q0 < ngroups && q0 < ch * 64 + 64; q0 += 64) {  // one chunk
      const uint32_t q = q0 + lane;
      const unsigned long long wb = q < ngroups ? wrow[q] : 0ull;
      if (__ballot(wb != 0ull) == 0ull) continue;
      if (d.exp & 4) st[0] += wb != 0ull;
      const uint32_t* ga = active + (size_t)q * 64;
      if (ci == CIN_SLOW) {  // overflowed contact list: the full replay runs in k_gossip_send_slow
        fb_add(d, FB_CEV_SLOW, __popcll(wb));  // each lane its own group's slots
        uint32_t i = wave_reserve(d.slow_n, (uint32_t)__popcll(wb));
        for (unsigned long long b = wb; b; b &= b - 1, ++i) {
          if (i < d.SLOWCAP)
            d.slow[i] = ((uint64_t)ga[__ffsll(b) - 1] << 32) | (uint32_t)ms;
          else
            atomicOr(d.err, E_CONTACTS);
        }
        continue;
      }
      if (ci != NEVER) {  // a cached contact t -> m: every slot of the pair goes to k_gossip_replay (isInfected :247)
        const uint32_t nb = (uint32_t)__popcll(wb);
        if (d.exp & 4) st[1] += nb;
        fb_add(d, FB_REPLAY, nb);  // each lane its own group's slots
        uint32_t i = wave_reserve(d.rp_n, nb);
        for (unsigned long long b = wb; b; b &= b - 1, ++i) {
          if (i < d.RPCAP)
            d.rp[i] = ((uint64_t)ga[__ffsll(b) - 1] << 32) | (uint32_t)ms;
          else
            atomicOr(d.err, E_CONTACTS);
        }
        continue;
      }
      sends += __popcll(wb);
      const unsigned long long cand = d.dbg_send ? wb : wb & ~(q < ngroups ? hrow[q] : 0ull);
      // the wave's candidates are spread over its lanes (a few groups hold most of them: new gossips take recently
      // freed slots): lane p takes candidates p, p + 64, ... of the wave's list in (group, slot) order
      const uint32_t c = (uint32_t)__popcll(cand);
      uint32_t incl = c;
#pragma unroll
      for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      const uint32_t total = __shfl(incl, 63);
      for (uint32_t b0 = 0; b0 < total; b0 += 64) {  // wave-uniform: every lane takes part in the shuffles
        const uint32_t j = b0 + lane;
        uint32_t own = 0;  // the lane whose word holds candidate j: the number of lanes with incl <= j
#pragma unroll
        for (uint32_t step = 32; step > 0; step >>= 1)
          if (__shfl(incl, (int)(own + step - 1)) <= j) own += step;
        const unsigned long long word = __shfl(cand, (int)own);
        const uint32_t r = j - (__shfl(incl, (int)own) - (uint32_t)__popcll(word));
        if (j < total) {
          const uint32_t g = active[(size_t)(q0 + own) * 64 + nth_bit(word, r)];
          if (d.exp & 4) st[3]++;
          send_tail(d, g, m, s, t, k, d.slot_gid[g], d.S + (size_t)g * d.N, ep, d.dbg_send == nullptr);
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

// sends of pairs with a cached contact, one thread per (slot, sender, target): the isInfected replay runs only where
// the contact can matter (t -> m at or after m's incarnation start and after the gossip existed), then the send
__global__ void __launch_bounds__(256) k_gossip_replay(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  __shared__ unsigned long long red[4];
  const uint32_t n = min(*d.rp_n, d.RPCAP);
  const int ep = epoch_at(d, k);
  unsigned long long sends = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t v = d.rp[i];
    const uint32_t g = (uint32_t)(v >> 32), ms = (uint32_t)v, m = ms / d.F, s = ms % d.F;
    uint32_t* Sg = d.S + (size_t)g * d.N;
    const uint32_t t = d.T[ms], c = s_ctick(Sg[m]), ci = d.cin[ms];
    const uint64_t gid = d.slot_gid[g];
    if (ci >= d.slot_ctick[g] && ci + d.lat >= c && blocked_pair_cached(d, m, t, g, gid, k, c, d.cev + (size_t)ms * CEVW))
      continue;
    sends++;
    send_tail(d, g, m, s, t, k, gid, Sg, ep);
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

// deferred sends whose pair had more contact events than the cache holds (small clusters): full log scan + replay
__global__ void __launch_bounds__(64) k_gossip_send_slow(const Dev* __restrict__ dp, uint32_t k) {
  const Dev& d = *dp;
  const uint32_t n = min(*d.slow_n, d.SLOWCAP);
  const int ep = epoch_at(d, k);
  unsigned long long sends = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t v = d.slow[i];
    const uint32_t g = (uint32_t)(v >> 32), ms = (uint32_t)v, m = ms / d.F, s = ms % d.F;
    uint32_t* Sg = d.S + (size_t)g * d.N;
    const uint32_t t = d.T[ms], c = s_ctick(Sg[m]);
    const uint64_t gid = d.slot_gid[g];
    if (blocked_pair(d, m, t, g, gid, k, c)) continue;  // isInfected (:247)
    sends++;
    send_tail(d, g, m, s, t, k, gid, Sg, ep);
  }
  if (sends) atomicAdd(&d.ctr[C_G], sends);
}

// P4 pre-filter (onMembershipGossip -> updateMembership, MembershipProtocolImpl.java:401-408,475-485). A first
// receipt is routed to P4 of tick k4 unless it provably cannot change t's row there: its record does not override
// the row as it stands now (= at the start of tick k4), the row is present, and the row cannot be removed before the
// receipt in that tick. Present rows only move up the isOverrides order except through a removal, so a record that
// does not override the start row overrides no later one. A removal needs a DEAD record: in P4 another receipt
// (k_stamp_dead set dead_rx[t] = k4), or in P1 a leaver's own record in SYNC data (leaving[subject]); after one the
// row is absent or re-added at any incarnation (an absent row accepts any ALIVE, MembershipRecord.java:67-69), so
// every receipt is kept then. An absent start row keeps every receipt (the row may become present earlier in the
// tick). User gossips are always routed (each one emits a GOSSIP event).
__device__ __forceinline__ bool receipt_matters(const Dev& d, uint32_t t, uint32_t g, uint32_t k4) {
  const uint32_t subj = d.slot_subj[g];
  if (subj == USER_SUBJ || (d.exp & 8)) return true;  // SWIM_EXP & 8: route every receipt (debugging aid)
  const uint64_t key = d.slot_key[g];
  const uint32_t r0 = d.rowk[lidx(d, t) * d.NS + subj], s1 = rec_status(key);
  if ((r0 & 3u) == ST_ABSENT || overrides(s1, rec_inc(key), r0 & 3u, r0 >> 2)) return true;
  return d.dead_rx[t] == k4 || d.leaving[subj];
}

// the deliveries of DEAD membership records: their targets receive one in P4 of tick k + lat (receipt_matters)
__global__ void k_stamp_dead(Dev d, uint32_t k) {
  const uint32_t n = *d.deliv_n < d.DCAP ? *d.deliv_n : d.DCAP;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t v = d.deliv[i];
    const uint32_t g = (uint32_t)(v >> 32), t = (uint32_t)v;
    if (rec_status(d.slot_key[g]) == ST_DEAD && d.slot_subj[g] != USER_SUBJ) d.dead_rx[t] = k + d.lat;
  }
}

// first receipts (onGossipReq :176-180): create the holder state at tick k + lat and queue the record for P4.
// Deliveries come in runs of one target (a send-kernel wave appends one (sender, target) pair's receipts together), so
// the target's counters are added once per run of equal targets in the wave instead of once per lane (one address
// per wave serialised at L2). The loop is wave-uniform so that every lane reaches the run reduction.
__global__ void k_gossip_apply(Dev d, uint32_t k) {
  const uint32_t n = *d.deliv_n < d.DCAP ? *d.deliv_n : d.DCAP;
  const uint32_t lane = __lane_id(), stride = gridDim.x * blockDim.x;
  for (uint32_t i0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < n; i0 += stride) {
    const uint32_t i = i0 + lane;
    const bool act = i < n;
    uint32_t g = 0, t = NEVER, created = 0, dropped = 0;
    if (act) {
      const uint64_t v = d.deliv[i];
      g = (uint32_t)(v >> 32);
      t = (uint32_t)v;
      uint32_t* p = d.S + (size_t)g * d.N + t;
      const uint32_t e = *p & ~S_PENDING;
      if (s_held(e)) {
        *p = e;
      } else {
        if (s_ever(e)) hist_push(d, d.slot_gid[g], t, s_ctick(e));  // rebirth after a sweep (:176-180)
        *p = ((k + d.lat + 1u) & S_TICK_MASK) | (s_ever(e) ? S_REBORN : 0u);
        created = 1;
        atomicAdd(&d.slot_holders[g], 1);
        if (t >= d.lo && t < d.hi) {  // else P4 of another shard's member
          if (d.fastp4 && d.slot_subj[g] == USER_SUBJ) {  // RUMOR mode: the GOSSIP event of P4 (k + lat), hashed now
            const uint64_t gid = d.slot_gid[g], key = d.slot_key[g];
            const uint64_t ev = ((uint64_t)(k + d.lat) << 32) | (3ull << 30) | (uint32_t)(gid >> 32);
            const uint64_t meta = ((uint64_t)(uint32_t)key << 32) | (key >> 32);  // (oldMeta, newMeta) = payload (lo, hi)
            atomicAdd(&d.evp_hash[t], (unsigned long long)hpair(hpair(ev, meta), (uint32_t)gid));
            atomicAdd(&d.evp_n[t], 1u);
          } else if (!receipt_matters(d, t, g, k + d.lat)) {  // counted as a record compare in P4, nothing else
            dropped = 1;
          } else {
            uint32_t ri = wave_append(d.rc_n);
            if (ri < d.RCAP)
              d.rc_raw[ri] = ((uint64_t)t << 32) | g;
            else
              atomicOr(d.err, E_RECEIPTS);
          }
        }
      }
    }
    // runs of equal targets among the wave's lanes (lanes past n carry NEVER and nothing)
    const uint32_t tp = __shfl_up(t, 1);
    const unsigned long long heads = __ballot(lane == 0 || tp != t);
    const unsigned long long cm = __ballot(created != 0), dm = __ballot(dropped != 0);
    if (act && ((heads >> lane) & 1ull)) {
      const unsigned long long above = heads & ~((2ull << lane) - 1ull);  // heads after this lane (lane < 63)
      const uint32_t end = lane == 63 || !above ? 64u : (uint32_t)(__ffsll((long long)above) - 1);
      const unsigned long long run = (end == 64 ? ~0ull : ((1ull << end) - 1ull)) & ~((1ull << lane) - 1ull);
      const uint32_t nc = (uint32_t)__popcll(cm & run), nd = (uint32_t)__popcll(dm & run);
      if (nc) {
        if (d.XW > 1)
          atomicAdd(&d.held_delta[t], (int)nc);
        else
          atomicAdd(&d.held[t], nc);
      }
      if (nd) atomicAdd(&d.rc_ndrop[t], nd);
    }
  }
}

// a slot nobody holds can never be sent again: clear its holder row and recycle it
__global__ void __launch_bounds__(256) k_gossip_free(Dev d, const uint32_t* active, const uint32_t* nactive) {
  uint32_t na = *nactive;
  for (uint32_t a = blockIdx.x; a < na; a += gridDim.x) {
    uint32_t g = active[a];
    if (d.slot_holders[g] > 0) continue;
    uint32_t* Sg = d.S + (size_t)g * d.N;
    for (uint32_t s = threadIdx.x; s < d.N; s += blockDim.x) Sg[s] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
      d.slot_used[g] = 0;
      if (g / d.SPR == d.rank) {  // back to the owning shard's free list
        int pos = atomicAdd(d.free_top, 1);
        d.free_list[pos] = g;
      }
    }
  }
}

// swim_kill: the member stops holding gossips (it can never send them again)
__global__ void k_kill(Dev d, uint32_t m) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= d.SLOTS || !d.slot_used[g]) return;
  if (s_held(d.S[(size_t)g * d.N + m])) atomicSub(&d.slot_holders[g], 1);
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
  uint32_t fl = d.fdLen[m], gl = d.gLen[m];
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
    uint32_t e = d.S[(size_t)g * d.N + m];
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
    o6[1] = red[1][0] + mix64((uint64_t)(int64_t)d.pingIdx[m] ^ 0xF00Dull) + fl;
    o6[2] = red[2][0] + mix64((uint64_t)(int64_t)d.remoteIdx[m] ^ 0xBEEFull) + gl;
    o6[3] = d.evHash[m];
    o6[4] = red[3][0];
    uint64_t ns = d.nextSync[m] == NEVER ? ~0ull : (uint64_t)d.nextSync[m];
    o6[5] = hpair(hpair(hpair(d.cidCnt[m], d.syncSeq[m]), d.gCounter[m]), ns) +
            mix64((uint64_t)d.fdPeriod[m] * 3 + (uint64_t)d.gPeriod[m] * 7);
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

// ------------------------------------------------------------------------------------------------------------
// host launchers
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

void launch_init(const Dev& d, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_init_members, dim3(cdiv(d.N, 256)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_init_rows, dim3(4096), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_init_lists, dim3(4096), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_init_slots, dim3(cdiv(d.SLOTS, 256)), dim3(256), 0, st, d);
  if (d.W > 1) hipLaunchKernelGGL(k_init_base, dim3(cdiv(d.NS, 256)), dim3(256), 0, st, d);
}

// timed: this launch is bracketed by profiling events; it adds its message count to ctr[C_DIFFMSG]
static void launch_sync_diff(const Dev& d, uint32_t b, hipStream_t st, uint32_t timed) {
  if (d.W > 1)
    hipLaunchKernelGGL(k_sync_diff<true>, dim3(2048), dim3(256), 0, st, d, b, timed);
  else
    hipLaunchKernelGGL(k_sync_diff<false>, dim3(2048), dim3(256), 0, st, d, b, timed);
}

// single GPU: the tick is cut in three so that the host can hold back the gossip data plane when no slot is in
// use; the SYNC diff of tick k+1 does not depend on the gossip plane of tick k and is queued in between
void launch_diff(const Dev& d, uint32_t k, void* stream, const TickEvents* prof) {
  hipStream_t st = (hipStream_t)stream;
  if (prof) hipEventRecord((hipEvent_t)prof->ev[0], st);
  if (k > 0) launch_sync_diff(d, (k - 1) & 1, st, prof ? 1u : 0u);
  if (prof) hipEventRecord((hipEvent_t)prof->ev[1], st);
}

void launch_member(const Dev& d, uint32_t k, void* stream, const TickEvents* prof) {
  hipStream_t st = (hipStream_t)stream;
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[2], st);
  hipLaunchKernelGGL(k_member_tick, dim3(cdiv(d.NL, 256)), dim3(256), 0, st, d.self, k, 1u);  // + k_tick_flag's work
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[3], st);
}

static void launch_receipt_routing(const Dev& d, hipStream_t st);

constexpr uint32_t SEND_GRID = 4096;  // 16 blocks per CU, grid-stride

void launch_gossip(const Dev& d, uint32_t k, void* stream, const TickEvents* prof) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_gossip_active, dim3(cdiv(d.SLOTS, 256)), dim3(256), 0, st, d, k, d.active, d.nactive);
  hipLaunchKernelGGL(k_round_info, dim3(cdiv(d.N, 256)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_gossip_contacts, dim3(cdiv((uint64_t)d.NL * d.F, 256)), dim3(256), 0, st, d, k);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[4], st);
  hipLaunchKernelGGL(k_gossip_scan, dim3(SEND_GRID), dim3(256), 0, st, d.self, k, d.active, d.nactive);
  hipLaunchKernelGGL(k_mask_transpose, dim3(SEND_GRID), dim3(256), 0, st, d.self, d.nactive);
  hipLaunchKernelGGL(k_gossip_send, dim3(SEND_GRID), dim3(256), 0, st, d.self, k, d.active, d.nactive);
  hipLaunchKernelGGL(k_gossip_send_slow, dim3(64), dim3(64), 0, st, d.self, k);  // rare; ~14 KB of stack per lane
  hipLaunchKernelGGL(k_gossip_replay, dim3(2048), dim3(256), 0, st, d.self, k);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[5], st);
  hipLaunchKernelGGL(k_stamp_dead, dim3(1024), dim3(256), 0, st, d, k);
  hipLaunchKernelGGL(k_gossip_apply, dim3(1024), dim3(256), 0, st, d, k);
  launch_receipt_routing(d, st);
  hipLaunchKernelGGL(k_gossip_free, dim3(1024), dim3(256), 0, st, d, d.active, d.nactive);
}

// ---- sharded tick (W > 1): the same kernel sequence as launch_tick, cut at the two exchange points ----
static void launch_receipt_routing(const Dev& d, hipStream_t st) {
  hipLaunchKernelGGL(k_count_rc, dim3(256), dim3(256), 0, st, d.rc_raw, d.rc_n, d.RCAP, d.rc_cnt);
  uint32_t nb = cdiv(d.N, 1024);
  hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, st, d.rc_cnt, d.rc_off, d.scan_part, d.N);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, st, d.scan_part, nb);
  hipLaunchKernelGGL(k_scan_add, dim3(cdiv(d.N, 256)), dim3(256), 0, st, d.rc_off, d.scan_part, d.N);
  hipLaunchKernelGGL(k_scatter_rc, dim3(256), dim3(256), 0, st, d, d.rc_raw, d.rc_n, d.RCAP, d.rc_off, d.rc_fill,
                     d.rc_slot, d.rc_key);
  hipLaunchKernelGGL(k_seg_sort, dim3(1024), dim3(256), 0, st, d.rc_key, d.rc_slot, d.rc_key2, d.rc_slot2, d.rc_off,
                     d.rc_cnt, d.N, d.rc_n, d.sort_cap, d.fb);
}

void launch_tick_a(const Dev& d, uint32_t k, void* stream, const TickEvents* prof) {
  hipStream_t st = (hipStream_t)stream;
  uint32_t b = k & 1, pb = (k - 1) & 1;
  if (prof) hipEventRecord((hipEvent_t)prof->ev[0], st);
  if (k > 0) launch_sync_diff(d, pb, st, prof ? 1u : 0u);
  if (prof) hipEventRecord((hipEvent_t)prof->ev[1], st);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[2], st);
  hipLaunchKernelGGL(k_member_tick, dim3(cdiv(d.NL, 256)), dim3(256), 0, st, d.self, k, 0u);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[3], st);
  hipLaunchKernelGGL(k_sync_route, dim3(cdiv(d.MSGCAP, 256)), dim3(256), 0, st, d, b);
  hipLaunchKernelGGL(k_pack_a, dim3(d.W), dim3(256), 0, st, d, b);
  hipLaunchKernelGGL(k_pack_a_chunks, dim3(64, d.W), dim3(256), 0, st, d, b);
}

void launch_tick_b(const Dev& d, uint32_t k, void* stream, const TickEvents* prof, bool gossip) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_unpack_a, dim3(32, d.W), dim3(256), 0, st, d, k, gossip ? 0u : 1u);
  if (!gossip) {  // no gossip slot in use on any shard: nothing to send, deliver or recycle; no exchange B
    if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[4], st);
    if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[5], st);
    return;
  }
  hipLaunchKernelGGL(k_gossip_active, dim3(cdiv(d.SLOTS, 256)), dim3(256), 0, st, d, k, d.active, d.nactive);
  hipLaunchKernelGGL(k_round_info, dim3(cdiv(d.N, 256)), dim3(256), 0, st, d);
  hipLaunchKernelGGL(k_gossip_contacts, dim3(cdiv((uint64_t)d.NL * d.F, 256)), dim3(256), 0, st, d, k);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[4], st);
  hipLaunchKernelGGL(k_gossip_scan, dim3(SEND_GRID), dim3(256), 0, st, d.self, k, d.active, d.nactive);
  hipLaunchKernelGGL(k_mask_transpose, dim3(SEND_GRID), dim3(256), 0, st, d.self, d.nactive);
  hipLaunchKernelGGL(k_gossip_send, dim3(SEND_GRID), dim3(256), 0, st, d.self, k, d.active, d.nactive);
  hipLaunchKernelGGL(k_gossip_send_slow, dim3(64), dim3(64), 0, st, d.self, k);  // rare; ~14 KB of stack per lane
  hipLaunchKernelGGL(k_gossip_replay, dim3(2048), dim3(256), 0, st, d.self, k);
  if (prof && prof->all) hipEventRecord((hipEvent_t)prof->ev[5], st);
  hipLaunchKernelGGL(k_pack_b, dim3(64, d.W), dim3(256), 0, st, d);
}

void launch_tick_c(const Dev& d, uint32_t k, void* stream, bool gossip) {
  hipStream_t st = (hipStream_t)stream;
  if (!gossip) return;  // k_unpack_a closed the tick
  hipLaunchKernelGGL(k_unpack_b_sweeps, dim3(64, d.W), dim3(256), 0, st, d, k);
  hipLaunchKernelGGL(k_unpack_b_deliv, dim3(64, d.W), dim3(256), 0, st, d, k);
  hipLaunchKernelGGL(k_stamp_dead, dim3(1024), dim3(256), 0, st, d, k);
  hipLaunchKernelGGL(k_gossip_apply, dim3(1024), dim3(256), 0, st, d, k);
  launch_receipt_routing(d, st);
  hipLaunchKernelGGL(k_gossip_free, dim3(1024), dim3(256), 0, st, d, d.active, d.nactive);
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

void launch_kill(const Dev& d, uint32_t member, void* stream) {
  hipLaunchKernelGGL(k_kill, dim3(cdiv(d.SLOTS, 256)), dim3(256), 0, (hipStream_t)stream, d, member);
}

void launch_hash(const Dev& d, uint64_t* out, uint32_t now, void* stream) {
  hipLaunchKernelGGL(k_hash, dim3(d.NL), dim3(256), 0, (hipStream_t)stream, d, out, now);
}

}  // namespace swim
