// shard.hip — row-sharded observers: packing and unpacking of the two per-tick exchanges.
//
// Each shard owns the observers [lo, hi) and runs their protocol control (k_member_tick) and their SYNC merges.
// The gossip plane stays replicated: every shard keeps the whole slot table, holder state (S, HB / WB, receipt rings),
// the round logs and the incarnation history, and applies the union of every shard's gossip records, so the
// data-plane kernels read any member's gossip state locally. The sends of a tick are split by target shard.
//
//   exchange A (after k_member_tick): gossips created this tick, gossip rounds this tick (targets, spread, period),
//     and the SYNC / SYNC_ACK messages addressed to the peer's observers. A SYNC payload (the sender's row at send
//     time, MembershipProtocolImpl.prepareSyncDataMsg :446-454) ships as a 2048-record chunk mask against the
//     replicated baseline row plus the chunks that differ, so a converged row costs a few bytes on xGMI.
//   exchange B (after the sends): first receipts (slot, target) of this shard's targets. Every shard runs every
//     member's round (sweeps and windows) on its replicated holder state, so sweeps need no exchange.
//
// Peer regions have a fixed capacity; a region that would overflow raises E_XCAP instead of being truncated.
// Region A: u32 hdr[8] = {nslot, nround, nsync, nchunk, data_off, 0, 0, 0}; slot records; round records;
//           sync entries {SyncMsg, u32 chunk base, u32 pad, u64 mask[MW], u32 log[TL]}; chunk data at data_off
//           (256-B aligned). log: a resolvable SYNC_ACK's responder write-log prefix (k_ack_resolve).
// Region B: u32 hdr[4] = {nreceipt, 0, 0, 0}; u64 receipts.
#include "dev_util.h"

namespace swim {


__device__ __forceinline__ uint64_t sync_entry_bytes(const Dev& d) { return sync_entry_size(d.MW); }

// SYNC_ACK resolution (k_ack_resolve): a resolvable SYNC_ACK's sender's write-log prefix of this tick (tick parity b),
// the SyncMsg.tln subjects it wrote before answering; nothing for the other messages
__device__ __forceinline__ void copy_log_prefix(const Dev& d, const SyncMsg& mm, uint32_t b, uint32_t* out) {
  const uint32_t n = (mm.kind & KF_RES) && mm.tln <= TL ? mm.tln : 0u;
  const uint32_t* src = d.tlog + ((size_t)b * d.NL + lidx(d, mm.src)) * TL;
  for (uint32_t j = 0; j < n; ++j) out[j] = src[j];
}

// a payload's key plane: the sender's live row or its copy-on-write snapshot
__device__ __forceinline__ const uint32_t* payload_row(const Dev& d, const SyncMsg& mm, uint32_t b) {
  return mm.payload == NEVER ? d.rowk + lidx(d, mm.src) * d.NS : d.arena[b] + (size_t)mm.payload * d.NS;
}

// block-wide exclusive prefix sum of v over the 256 threads (sh: 8 words of LDS); *tot = the block's sum
__device__ __forceinline__ uint32_t block_excl_256(uint32_t v, uint32_t* sh, uint32_t* tot) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  __syncthreads();
  if (lane == 63) sh[wv] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < wv; ++w) before += sh[w];
  *tot = sh[0] + sh[1] + sh[2] + sh[3];
  return before + incl - v;
}

// k_pack_all: routing, packing and chunk copy of exchange A in one launch (grid 16 x W): every block of peer column q walks this
// tick's messages in index order and finds the ones to shard q (the same list in every block of the column, so no
// block waits for another); block 0 writes the region's header, records and SYNC entries, every block copies its share
// of the payloads' differing chunks, and the last block of the column writes q's inline all-to-all block. Column
// `rank` queues the local messages for the next tick's inbound list. (A steady-state sharded tick was member kernel,
// route, pack, chunk launches back to back: two launches and their drains fewer.)
__global__ void __launch_bounds__(256) k_pack_all(Dev d, uint32_t b, uint32_t spec) {
  if (spec_halted(d, spec)) return;
  const uint32_t q = blockIdx.y, x = blockIdx.x, t = threadIdx.x;
  __shared__ uint32_t sh[8], tot_sh[2];
  const uint32_t n = min(d.nmsg[b], d.MSGCAP);
  if (q == d.rank) {  // local destinations: straight to the next tick's inbound list
    if (d.inl && x == 0 && t == 0) *(uint64_t*)(d.xi_send + (size_t)q * d.XI) = 0ull;  // the block to itself: empty
    for (uint32_t base = 0; x == 0 && base < n; base += 256) {
      const uint32_t i = base + t;
      const bool sel = i < n && shard_of(d.N, d.W, d.msgs[b][i].dst) == q;
      uint32_t tot;
      const uint32_t ex = block_excl_256(sel ? 1u : 0u, sh, &tot);
      if (t == 0 && tot) tot_sh[0] = atomicAdd(&d.xn[4], tot);
      __syncthreads();
      if (sel) {
        const uint32_t j = tot_sh[0] + ex;
        if (j < d.MSGCAP) {
          const SyncMsg& mm = d.msgs[b][i];
          d.mtmp[j] = mm;
          if (d.ackres) copy_log_prefix(d, mm, b, d.mlog + (size_t)j * TL);
        } else if (j == d.MSGCAP) {
          set_err(d, E_MSGS);
        }
      }
      __syncthreads();
    }
  } else {
  uint8_t* R = d.xa_send + (size_t)q * d.XA_PEER;
  const uint64_t SE = sync_entry_bytes(d);
  // pass 1: how many messages go to q and how many payload chunks they ship
  uint32_t nsync = 0, nchunk = 0;
  for (uint32_t base = 0; base < n; base += 256) {
    const uint32_t i = base + t;
    uint32_t sel = 0, nc = 0;
    if (i < n) {
      const SyncMsg& mm = d.msgs[b][i];
      if (shard_of(d.N, d.W, mm.dst) == q) {
        sel = 1;
        const uint64_t* dm = mm.payload == NEVER ? d.rdirty + lidx(d, mm.src) * d.MW : d.arena_dirty[b] + (size_t)mm.payload * d.MW;
        for (uint32_t w = 0; w < d.MW; ++w) nc += (uint32_t)__popcll(dm[w]);
      }
    }
    uint32_t ts, tc;
    block_excl_256(sel, sh, &ts);
    __syncthreads();
    block_excl_256(nc, sh, &tc);
    nsync += ts;
    nchunk += tc;
  }
  const uint32_t nslot = min(d.xn[0], d.NSCAP), nround = min(d.xn[1], d.RRCAP);
  const uint64_t off_sync = 32 + 4ull * NSW * nslot + 4ull * RRW * nround;
  uint64_t data_off = (off_sync + SE * nsync + 255) & ~255ull;
  const bool fits = nsync <= d.RQCAP && data_off + (uint64_t)nchunk * CH * 4 <= d.XA_PEER && nchunk <= d.CHCAP;
  if (x == 0 && t == 0) {
    uint32_t* H = (uint32_t*)R;
    uint64_t total = data_off + (uint64_t)nchunk * CH * 4;
    if (!fits) {
      atomicOr(d.err, E_XCAP);
      data_off = 256;
      total = 32;
    }
    H[0] = fits ? nslot : 0u;
    H[1] = fits ? nround : 0u;
    H[2] = fits ? nsync : 0u;
    H[3] = fits ? nchunk : 0u;
    H[4] = (uint32_t)data_off;
    H[5] = H[6] = H[7] = 0;
    // the flag rides on the byte count: every shard learns whether any shard has a gossip slot in use
    d.xa_scnt[q] = total | ((int32_t)d.SPR - *d.free_top > 0 ? XFLAG_GOSSIP : 0ull);
  }
  if (fits) {
    if (x == 0) {  // gossip records (replicated on every shard)
      uint32_t* S = (uint32_t*)(R + 32);
      for (uint32_t i = t; i < nslot * NSW; i += blockDim.x) S[i] = d.ns_rec[i];
      uint32_t* RR = S + (size_t)nslot * NSW;
      for (uint32_t i = t; i < nround * RRW; i += blockDim.x) RR[i] = d.rr_rec[i];
    }
    uint8_t* E = R + off_sync;
    uint32_t* dst0 = (uint32_t*)(R + data_off);
    // pass 2: the entries (block 0) and the chunks (chunk r of the column's payloads by block r % gridDim.x)
    uint32_t j0 = 0, c0 = 0;
    for (uint32_t base = 0; base < n; base += 256) {
      const uint32_t i = base + t;
      uint32_t sel = 0, nc = 0;
      const uint64_t* dm = nullptr;
      if (i < n) {
        const SyncMsg& mm = d.msgs[b][i];
        if (shard_of(d.N, d.W, mm.dst) == q) {
          sel = 1;
          dm = mm.payload == NEVER ? d.rdirty + lidx(d, mm.src) * d.MW : d.arena_dirty[b] + (size_t)mm.payload * d.MW;
          for (uint32_t w = 0; w < d.MW; ++w) nc += (uint32_t)__popcll(dm[w]);
        }
      }
      uint32_t ts, tc;
      const uint32_t ej = block_excl_256(sel, sh, &ts);
      __syncthreads();
      const uint32_t ec = block_excl_256(nc, sh, &tc);
      if (sel && x == 0) {
        uint8_t* p = E + SE * (j0 + ej);
        *(SyncMsg*)p = d.msgs[b][i];
        ((uint32_t*)(p + sizeof(SyncMsg)))[0] = c0 + ec;
        ((uint32_t*)(p + sizeof(SyncMsg)))[1] = 0;
        uint64_t* mk = (uint64_t*)(p + sizeof(SyncMsg) + 8);
        for (uint32_t w = 0; w < d.MW; ++w) mk[w] = dm[w];
        if (d.ackres) copy_log_prefix(d, d.msgs[b][i], b, (uint32_t*)(mk + d.MW));
      }
      if (tc) {  // this batch's payload chunks: the block's share, 8 keys per thread with 16-B loads and stores
        __shared__ uint32_t cmsg[256], cbase[256];
        __syncthreads();
        cmsg[t] = nc ? i : NEVER;
        cbase[t] = c0 + ec;
        __syncthreads();
        for (uint32_t l = 0; l < 256; ++l) {
          const uint32_t mi = cmsg[l];
          if (mi == NEVER) continue;
          const SyncMsg& mm = d.msgs[b][mi];
          const uint64_t* mk = mm.payload == NEVER ? d.rdirty + lidx(d, mm.src) * d.MW : d.arena_dirty[b] + (size_t)mm.payload * d.MW;
          uint32_t r = cbase[l];
          for (uint32_t c = 0; c < d.NCHUNK; ++c) {
            if (!((mk[c >> 6] >> (c & 63)) & 1ull)) continue;
            if (r % gridDim.x == x) {
              const uint32_t s0 = c * CH + t * 8;
              if (s0 < d.NS) {
                const uint4* src = (const uint4*)(payload_row(d, mm, b) + s0);
                uint4* dst = (uint4*)(dst0 + (size_t)r * CH + t * 8);
                dst[0] = src[0];
                dst[1] = src[1];
              }
            }
            ++r;
          }
        }
      }
      j0 += ts;
      c0 += tc;
      __syncthreads();
    }
  }
  }  // q != rank
  // the last block of each peer column writes that peer's inline all-to-all block (count word, then the region's first
  // XI - 8 bytes: every lane's loads before its stores); the last peer column to finish then marks every count word
  // if any of this shard's regions is past its inline block (a send/recv group follows), so every peer of a
  // speculative batch halts at the same tick. (One block of the whole grid writing every peer's block one after the
  // other grew with W.)
  if (!d.inl || q == d.rank || !last_block(&d.xdone[1 + q], gridDim.x)) return;
  {
    const unsigned long long w = d.xa_scnt[q];
    uint64_t* idst = (uint64_t*)(d.xi_send + (size_t)q * d.XI);
    const uint64_t nw = min((uint64_t)(w & XCNT_MASK), (uint64_t)d.XI - 8) / 8;  // regions are multiples of 8 B
    const uint64_t* isrc = (const uint64_t*)(d.xa_send + (size_t)q * d.XA_PEER);
    for (uint64_t i0 = 0; i0 < nw; i0 += 8 * blockDim.x) {
      uint64_t v[8];
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const uint64_t i = i0 + t + (uint64_t)j * blockDim.x;
        v[j] = i < nw ? isrc[i] : 0ull;
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        const uint64_t i = i0 + t + (uint64_t)j * blockDim.x;
        if (i < nw) idst[1 + i] = v[j];
      }
    }
    if (t == 0) idst[0] = w;
  }
  if (!last_block(&d.xdone[0], d.W - 1)) return;
  bool over = false;
  for (uint32_t r = 0; r < d.W; ++r) over |= r != d.rank && (d.xa_scnt[r] & XCNT_MASK) > d.XI - 8;
  if (over && t < d.W && t != d.rank) *(uint64_t*)(d.xi_send + (size_t)t * d.XI) |= XFLAG_OVER;
}

// the assembled inbound list becomes msgs[b], which the next tick sorts and merges (one block)
// (one block). A receiver with several payloads gets its live-row payloads pinned (pin_msg, dev_util.h).
__device__ void msgs_commit(const Dev& d, uint32_t b) {
  uint32_t n = min(d.xn[4], d.MSGCAP);
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    d.msgs[b][i] = d.mtmp[i];
    d.msgs[b][i].pin = NEVER;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    if (d.mtmp[i].kind & KF_DEFER) continue;  // delivered later: stored by k_sync_defer_x at the end of this tick
    const uint32_t old = atomicExch(&d.m_head[(size_t)b * d.N + d.mtmp[i].dst], i);
    d.m_next[(size_t)b * d.MSGCAP + i] = old;
    if (old != NEVER) {
      if (d.msgs[b][i].payload == NEVER) pin_msg(d, b, i);
      if (d.msgs[b][old].payload == NEVER) pin_msg(d, b, old);
    }
  }
  if (threadIdx.x == 0) d.nmsg[b] = n;
}

// replay peer p's gossip creations and rounds into the replicated gossip plane; queue its SYNC messages. The block
// that finishes last commits the inbound list, and, when no shard has a gossip slot in use (`end`), closes the tick
// (k_tick_end): the steady-state tick after exchange A is this one launch.
__device__ __forceinline__ bool spec_gate(const Dev& d);
__global__ void __launch_bounds__(256) k_unpack_a(Dev d, uint32_t k, uint32_t end, uint32_t spec) {
  if (spec_halted(d, spec)) return;
  // the gate of a speculative batch, evaluated by every block from the same count words: all of them see the same
  // answer, and one raises d.halt for the host
  if (spec && spec_gate(d)) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *d.halt = k + 1u;
    return;
  }
  const uint32_t p = blockIdx.y;
  if (p != d.rank && (d.xa_rcnt[p] & XCNT_MASK) >= 32) {
    const uint8_t* R = d.xa_recv + (size_t)p * d.XA_PEER;
    const uint32_t* H = (const uint32_t*)R;
    const uint32_t nslot = H[0], nround = H[1], nsync = H[2], data_off = H[4];
    const uint32_t* S = (const uint32_t*)(R + 32);
    const uint32_t* RR = S + (size_t)nslot * NSW;
    const uint8_t* E = (const uint8_t*)(RR + (size_t)nround * RRW);
    const uint64_t SE = sync_entry_bytes(d);
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    for (uint32_t i = tid; i < nslot; i += nth) {  // spread -> createAndPutGossip at the origin (member.hip)
      const uint32_t* r = S + (size_t)i * NSW;
      const uint32_t g = r[0], origin = r[7];
      slot_create(d, g, origin, r[4], (uint64_t)r[1] | ((uint64_t)r[2] << 32), r[3], (uint64_t)r[5] | ((uint64_t)r[6] << 32),
                  atomicAdd(&d.rtail[origin], 1u));
      atomicAdd(&d.held[origin], 1u);
    }
    for (uint32_t i = tid; i < nround; i += nth) {  // do_spread_gossip at the sender (member.hip)
      const uint32_t* r = RR + (size_t)i * RRW;
      uint32_t m = r[0], cnt = r[1];
      d.tround[m] = 1;
      d.tcnt[m] = cnt;
      d.tspread[m] = r[2];
      d.tperiod[m] = r[3];
      uint32_t pos = d.log_pos[m] % d.LOGW;
      size_t lo = (size_t)m * d.LOGW + pos;
      if (d.log_pos[m] > 0 && d.log_spread[(size_t)m * d.LOGW + (d.log_pos[m] - 1) % d.LOGW] != r[2]) d.spchg[m] = k;
      d.log_tick[lo] = k;
      d.log_spread[lo] = r[2];
      d.log_cnt[lo] = cnt;
      for (uint32_t j = 0; j < cnt; ++j) {
        d.T[(size_t)m * d.F + j] = r[4 + j];
        d.log_tg[lo * d.F + j] = r[4 + j];
      }
      d.log_pos[m]++;
    }
    for (uint32_t i = tid; i < nsync; i += nth) {
      const uint8_t* e = E + SE * i;
      SyncMsg mm = *(const SyncMsg*)e;
      uint32_t base = ((const uint32_t*)(e + sizeof(SyncMsg)))[0];
      const uint64_t* mk = (const uint64_t*)(e + sizeof(SyncMsg) + 8);
      uint32_t ri = atomicAdd(&d.xn[5], 1u);
      uint32_t j = atomicAdd(&d.xn[4], 1u);
      if (ri >= d.RXCAP || j >= d.MSGCAP) {
        atomicOr(d.err, E_XCAP);
        continue;
      }
      for (uint32_t w = 0; w < d.MW; ++w) d.rx_mask[(size_t)ri * d.MW + w] = mk[w];
      if (d.ackres && (mm.kind & KF_RES) && mm.tln <= TL)  // the responder's log prefix (k_ack_resolve)
        for (uint32_t q = 0; q < mm.tln; ++q) d.mlog[(size_t)j * TL + q] = ((const uint32_t*)(mk + d.MW))[q];
      d.rx_off[ri] = (uint64_t)p * d.XA_PEER + data_off + (uint64_t)base * CH * 4;
      mm.payload = PAY_RX | ri;
      mm.ncand = 0;
      d.mtmp[j] = mm;
    }
  }
  if (!last_block(&d.xn[6], gridDim.x * gridDim.y)) return;
  msgs_commit(d, k & 1);
  if (end) {
    __syncthreads();
    tick_end(d, k);
  }
}

// this shard's first receipts of the tick (its targets' senders ran here): every peer applies them to its replicated
// holder state (gossip.hip k_unpack_b)
__global__ void __launch_bounds__(256) k_pack_b(Dev d) {
  const uint32_t q = blockIdx.y;
  if (q == d.rank) return;
  uint8_t* R = d.xb_send + (size_t)q * d.XB_PEER;
  uint32_t nd = min(*d.xd_n, d.DCAP);
  if (16 + 8ull * nd > d.XB_PEER) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(d.err, E_XCAP);
    nd = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t* H = (uint32_t*)R;
    H[0] = nd;
    H[1] = H[2] = H[3] = 0;
    d.xb_scnt[q] = 16 + 8ull * nd;
  }
  uint64_t* V = (uint64_t*)(R + 16);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nd; i += gridDim.x * blockDim.x) V[i] = d.xd[i];
}

// the peers' members are out of their gossip round again
__global__ void k_round_reset(Dev d) {
  const uint32_t p = blockIdx.y;
  if (p == d.rank || (d.xa_rcnt[p] & XCNT_MASK) < 32) return;
  const uint8_t* R = d.xa_recv + (size_t)p * d.XA_PEER;
  const uint32_t* H = (const uint32_t*)R;
  const uint32_t* RR = (const uint32_t*)(R + 32) + (size_t)H[0] * NSW;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < H[1]; i += gridDim.x * blockDim.x) d.tround[RR[(size_t)i * RRW]] = 0;
}

// RCCL exchange, fixed-size part: block q = the count word of region q followed by its first XINL - 8 bytes. The
// all-to-all of these blocks needs no sizes on the host, and in the steady state carries the whole exchange.
__global__ void __launch_bounds__(256) k_inline_out(const uint8_t* send, uint64_t cap, const unsigned long long* scnt,
                                                    uint8_t* isend, uint32_t XI) {
  const uint32_t q = blockIdx.x;
  const unsigned long long w = scnt[q];
  uint64_t* dst = (uint64_t*)(isend + (size_t)q * XI);
  if (threadIdx.x == 0) dst[0] = w;
  const uint64_t n = min((uint64_t)(w & XCNT_MASK), (uint64_t)XI - 8) / 8;  // regions are multiples of 8 B
  const uint64_t* src = (const uint64_t*)(send + (size_t)q * cap);
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) dst[1 + i] = src[i];
}

__global__ void __launch_bounds__(256) k_inline_in(const uint8_t* irecv, uint8_t* recv, uint64_t cap,
                                                   const unsigned long long* scnt, unsigned long long* rcnt,
                                                   unsigned long long* host, uint32_t W, const uint32_t* halt,
                                                   uint32_t XI) {
  if (halt && *(volatile const uint32_t*)halt) return;  // speculative batch: halted at an earlier tick
  const uint32_t p = blockIdx.x;
  const uint64_t* src = (const uint64_t*)(irecv + (size_t)p * XI);
  const unsigned long long w = src[0];
  const uint64_t n = min((uint64_t)(w & XCNT_MASK), (uint64_t)XI - 8) / 8;
  uint64_t* dst = (uint64_t*)(recv + (size_t)p * cap);
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[1 + i];
  if (threadIdx.x == 0) {
    rcnt[p] = w;
    host[p] = scnt[p];
    host[W + p] = w;
    __threadfence_system();
  }
}

void launch_inline_out(const Dev& d, const uint8_t* send, uint64_t cap, const unsigned long long* scnt, void* stream) {
  hipLaunchKernelGGL(k_inline_out, dim3(d.W), dim3(256), 0, (hipStream_t)stream, send, cap, scnt, d.xi_send, d.XI);
}

void launch_inline_in(const Dev& d, uint8_t* recv, uint64_t cap, const unsigned long long* scnt, unsigned long long* rcnt,
                      void* stream, bool spec) {
  hipLaunchKernelGGL(k_inline_in, dim3(d.W), dim3(256), 0, (hipStream_t)stream, d.xi_recv, recv, cap, scnt, rcnt,
                     d.xi_host, d.W, spec ? (const uint32_t*)d.halt : nullptr, d.XI);
}

// speculative sharded batch, after exchange A's inline all-to-all of a tick (k_unpack_a): halt if any shard has a
// gossip slot in use or a region past its inline block. Every shard reads the same flags (its own and every peer's
// count words), so all of them halt at the same tick and run its rest on the host path
__device__ __forceinline__ bool spec_gate(const Dev& d) {
  unsigned long long f = 0;
  for (uint32_t p = 0; p < d.W; ++p) {
    f |= d.xa_rcnt[p] | d.xa_scnt[p];
    if ((d.xa_scnt[p] & XCNT_MASK) > d.XI - 8) f |= XFLAG_OVER;
  }
  return (f & (XFLAG_GOSSIP | XFLAG_OVER)) != 0;
}

}  // namespace swim
