// dev_util.h — device helpers shared by the member, SYNC and gossip kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"

namespace swim {

__device__ __forceinline__ void set_err(const Dev& d, uint32_t bit) { atomicOr(d.err, bit); }

// 16-B row loads
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u64x2 ld_c(const uint64_t* p) { return *(const u64x2*)p; }

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

// NetworkEmulator.tryFail (transport/.../NetworkEmulator.java:231-248) at the sender, evaluated for tick k:
// a dead destination or a partition block fails the send; otherwise a loss draw unless loss is 0 or >= 100.
__device__ __forceinline__ bool blocked_at(const Dev& d, int ep, uint32_t src, uint32_t dst, uint32_t k) {
  if (dead_at(d, dst, k)) return true;
  if (d.ep_part[ep] && d.ep_group[(size_t)ep * d.N + src] != d.ep_group[(size_t)ep * d.N + dst]) return true;
  return false;
}

__device__ __forceinline__ bool lost_msg(const Dev& d, uint32_t kind, uint32_t src, uint32_t dst, uint32_t k,
                                         uint32_t aux, uint32_t id) {
  int ep = epoch_at(d, k);
  if (ep < 0) {
    set_err(d, E_EPOCH);
    return true;
  }
  if (blocked_at(d, ep, src, dst, k)) return true;
  uint32_t loss = d.ep_loss[ep];
  if (loss == 0) return false;
  if (loss >= 100) return true;
  u32x4 r = philox(src, dst, k, id, d.seed_lo ^ (SALT_LOSS_BASE + kind), d.seed_hi ^ (aux * 0x9E3779B9u));
  return next_int(r.x, 100) < loss;
}

__device__ __forceinline__ bool lost_gossip(const Dev& d, uint32_t src, uint32_t dst, uint32_t k, uint32_t slot,
                                            uint64_t gid) {
  int ep = epoch_at(d, k);
  if (ep < 0) {
    set_err(d, E_EPOCH);
    return true;
  }
  if (blocked_at(d, ep, src, dst, k)) return true;
  uint32_t loss = d.ep_loss[ep];
  if (loss == 0) return false;
  if (loss >= 100) return true;
  u32x4 r = philox(src, k ^ ((slot >> 2) << 31), (uint32_t)(gid >> 32), (uint32_t)gid, d.seed_lo ^ SALT_LOSS_GOSSIP,
                   d.seed_hi);
  return next_int(pick(r, slot & 3), 100) < loss;
}

// gPeriod of member x before its gossip task at tick c = number of its gossip rounds at ticks < c
__device__ __forceinline__ uint32_t rounds_before(const Dev& d, uint32_t x, uint32_t c) {
  uint32_t f = d.firstGossip[x];
  if (f == NEVER || c <= f) return 0;
  return (c - f + d.gossip_t - 1) / d.gossip_t;
}

__device__ __forceinline__ uint32_t spread_of(const Dev& d, uint32_t cluster) { return d.repeatMult * bitlen(cluster); }

__device__ __forceinline__ uint32_t s_ctick(uint32_t e) { return (e & S_TICK_MASK) - 1u; }
__device__ __forceinline__ bool s_ever(uint32_t e) { return (e & S_TICK_MASK) != 0; }
__device__ __forceinline__ bool s_held(uint32_t e) { return (e & S_TICK_MASK) != 0 && !(e & S_SWEPT); }

}  // namespace swim
