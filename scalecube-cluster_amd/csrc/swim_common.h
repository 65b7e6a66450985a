// swim_common.h — primitives shared by the host and gfx950 sides of libswimhip.
//
// Packed record layout in a membership-table row (one u64 per (observer, subject)); SEMANTICS.md §8:
//   bits  0..31  incarnation            MembershipRecord.incarnation (membership/MembershipRecord.java:12-84)
//   bits 32..33  status                 0 = no row, 1 = ALIVE, 2 = SUSPECT (DEAD is never stored, :512-513)
//   bit  34      metadata known         MetadataStoreImpl.membersMetadata contains the subject
//   bits 35..63  suspicion deadline     scheduleSuspicionTimeoutTask deadline tick, 0 = no timer (:597-606)
// The record key (inc | status<<32) is what SYNC payloads carry and what isOverrides compares.
//
// Physical layout: a row is two u32 planes. The key plane holds key32 = inc << 2 | status, the only
// part of a record that SYNC payloads carry and k_sync_diff compares (4 B per record instead of 8); the aux plane
// holds bits 34..63 of the logical record (metadata known, suspicion deadline). Incarnations therefore must stay
// below 2^30 in a stored row; a larger one raises E_INC instead of being truncated.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SW_HD __host__ __device__ __forceinline__
#else
#define SW_HD inline
#endif

namespace swim {

constexpr uint32_t NONE32 = 0xFFFFFFFFu;
constexpr uint32_t USER_SUBJ = 0xFFFFFFFFu;  // slot subject of a user gossip (Cluster.spreadGossip): payload in the key
constexpr uint32_t ST_ABSENT = 0, ST_ALIVE = 1, ST_SUSPECT = 2, ST_DEAD = 3;

constexpr uint64_t KEY_MASK = (1ull << 34) - 1;  // inc | status
constexpr uint64_t META_BIT = 1ull << 34;
constexpr int TIMER_SHIFT = 35;
constexpr uint64_t TIMER_MASK29 = (1ull << 29) - 1;

SW_HD uint32_t rec_status(uint64_t v) { return (uint32_t)(v >> 32) & 3u; }
SW_HD uint32_t rec_inc(uint64_t v) { return (uint32_t)v; }
SW_HD uint64_t rec_key(uint32_t st, uint32_t inc) { return (uint64_t)inc | ((uint64_t)st << 32); }
constexpr uint32_t INC_LIMIT = 1u << 30;
SW_HD uint32_t key32(uint64_t v) { return ((uint32_t)v << 2) | rec_status(v); }
// the 8-bit shadow of a key (Dev::rowk8, k_sync_diff): the key itself below 0xFF (incarnations up to 62, or 63 for a
// record that is not DEAD), else the escape 0xFF, whose subjects the diff compares on the full keys. Two keys below
// 0xFF are equal iff their shadows are, so the shadow compare is exact wherever neither side escapes
SW_HD uint8_t key8(uint32_t k) { return k < 0xFFu ? (uint8_t)k : (uint8_t)0xFFu; }
SW_HD uint64_t key34(uint32_t k) { return (uint64_t)(k >> 2) | ((uint64_t)(k & 3u) << 32); }
SW_HD uint32_t aux32(uint64_t v) { return (uint32_t)(v >> 34); }
SW_HD uint64_t rec_join(uint32_t k, uint32_t a) { return key34(k) | ((uint64_t)a << 34); }
SW_HD uint32_t rec_timer(uint64_t v) { return (uint32_t)(v >> TIMER_SHIFT); }
SW_HD uint64_t rec_with_timer(uint64_t v, uint32_t dl) {
  return (v & ((1ull << TIMER_SHIFT) - 1)) | ((uint64_t)(dl & TIMER_MASK29) << TIMER_SHIFT);
}

// MembershipRecord.isOverrides (membership/MembershipRecord.java:66-84). r0 status 0 is the `r0 == null` case.
SW_HD bool overrides(uint32_t s1, uint32_t i1, uint32_t s0, uint32_t i0) {
  if (s0 == ST_ABSENT) return s1 == ST_ALIVE;
  if (s0 == ST_DEAD) return false;
  if (s1 == ST_DEAD) return true;
  if (i1 == i0) return s1 != s0 && s1 == ST_SUSPECT;
  return i1 > i0;
}

// ClusterMath.ceilLog2 (ClusterMath.java:133-135): bit length
SW_HD uint32_t bitlen(uint32_t n) {
#if defined(__HIP_DEVICE_COMPILE__)
  return n ? 32u - (uint32_t)__clz((int)n) : 0u;
#else
  return n ? 32u - (uint32_t)__builtin_clz(n) : 0u;
#endif
}

// ---- Philox4x32-10 (Salmon et al., SC'11): the injected selector of SEMANTICS.md §2 ----
struct u32x4 {
  uint32_t x, y, z, w;
};
SW_HD void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
#if defined(__HIP_DEVICE_COMPILE__)
  lo = a * b;
  hi = __umulhi(a, b);
#else
  uint64_t p = (uint64_t)a * b;
  lo = (uint32_t)p;
  hi = (uint32_t)(p >> 32);
#endif
}
SW_HD u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo(0xD2511F53u, c0, hi0, lo0);
    mulhilo(0xCD9E8D57u, c2, hi1, lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return u32x4{c0, c1, c2, c3};
}
SW_HD uint32_t pick(const u32x4& r, uint32_t i) { return i == 0 ? r.x : i == 1 ? r.y : i == 2 ? r.z : r.w; }

constexpr uint32_t SALT_SEL = 0x53454C31u, SALT_INIT = 0x494E4954u, SALT_LOSS_BASE = 0x4C4F5300u,
                   SALT_LOSS_GOSSIP = 0x474F5353u, SALT_CHURN = 0x43485552u, SALT_DELAY_BASE = 0x444C5900u,
                   SALT_DELAY_GOSSIP = 0x444C5947u;
// message kinds (loss-key salts; SEMANTICS.md §2)
constexpr uint32_t K_SYNC = 1, K_SYNC_ACK = 2, K_PING = 3, K_PING_REQ = 4, K_PING_ACK = 5, K_GMD_REQ = 6,
                   K_GMD_RESP = 7;
// selector streams
constexpr uint32_t S_FD_SHUFFLE = 1, S_FD_INSERT = 2, S_PINGREQ = 3, S_GOSSIP_SHUFFLE = 4, S_SYNC_PICK = 5;

SW_HD uint32_t next_int(uint32_t x, uint32_t bound) { return (uint32_t)(((uint64_t)x * bound) >> 32); }

// NetworkLinkSettings.evaluateLoss (:54-57): `nextInt(100) < loss` on the LOSS_<kind> draw of one message
// (SEMANTICS.md §2); the roll in [0, 100) of message `id` sent by src to dst at tick k, aux = the id's issuer
SW_HD uint32_t loss_roll(uint32_t seed_lo, uint32_t seed_hi, uint32_t kind, uint32_t src, uint32_t dst, uint32_t k,
                         uint32_t aux, uint32_t id) {
  const u32x4 r = philox(src, dst, k, id, seed_lo ^ (SALT_LOSS_BASE + kind), seed_hi ^ (aux * 0x9E3779B9u));
  return next_int(r.x, 100);
}

// NetworkLinkSettings.evaluateDelay (:64-74): the DELAY_<kind> draw of one message, same counter words as its loss draw
SW_HD uint32_t delay_draw(uint32_t seed_lo, uint32_t seed_hi, uint32_t kind, uint32_t src, uint32_t dst, uint32_t k,
                          uint32_t aux, uint32_t id) {
  return philox(src, dst, k, id, seed_lo ^ (SALT_DELAY_BASE + kind), seed_hi ^ (aux * 0x9E3779B9u)).x;
}

SW_HD uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
SW_HD uint64_t hpair(uint64_t a, uint64_t b) { return mix64(mix64(a) ^ b); }
SW_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// PRECONVERGED list order: 4-round Feistel bijection on [0,n), cycle-walked (SEMANTICS.md §3)
struct FeistelPerm {
  uint32_t n, half, mask, rk0, rk1, rk2, rk3;
};
SW_HD FeistelPerm make_perm(uint32_t n, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  FeistelPerm p;
  p.n = n ? n : 1;
  uint32_t b = 2;
  while (b < 32 && (1ull << b) < p.n) b += 2;
  p.half = b / 2;
  p.mask = (1u << p.half) - 1u;
  p.rk0 = k0;
  p.rk1 = k1;
  p.rk2 = k2;
  p.rk3 = k3;
  return p;
}
SW_HD uint32_t feistel_once(const FeistelPerm& p, uint32_t x) {
  uint32_t L = x >> p.half, R = x & p.mask;
  uint32_t t;
  t = L ^ (fmix32(R ^ p.rk0) & p.mask); L = R; R = t;
  t = L ^ (fmix32(R ^ p.rk1) & p.mask); L = R; R = t;
  t = L ^ (fmix32(R ^ p.rk2) & p.mask); L = R; R = t;
  t = L ^ (fmix32(R ^ p.rk3) & p.mask); L = R; R = t;
  return (L << p.half) | R;
}
SW_HD uint32_t feistel(const FeistelPerm& p, uint32_t x) {
  uint32_t y = feistel_once(p, x);
  while (y >= p.n) y = feistel_once(p, y);
  return y;
}

}  // namespace swim
