// oracle/rng.h — TEST INFRASTRUCTURE (oracle). The injected selector of SEMANTICS.md §2, restated on the CPU.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use anything under oracle/.
//
// Philox4x32-10: Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3" (SC'11).
// It replaces ThreadLocalRandom / Collections.shuffle at the reference's randomness seams:
// FailureDetectorImpl.java:329,344,358; GossipProtocolImpl.java:259; MembershipProtocolImpl.java:414,418;
// NetworkLinkSettings.java:56.
#pragma once
#include <cstdint>

namespace swimref {

struct P4 {
  uint32_t v[4];
};

inline P4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
  }
  return P4{{c0, c1, c2, c3}};
}

// purpose salts (SEMANTICS.md §2)
enum Salt : uint32_t {
  SALT_SEL = 0x53454C31u,
  SALT_INIT = 0x494E4954u,
  SALT_LOSS_BASE = 0x4C4F5300u,  // + message kind
  SALT_LOSS_GOSSIP = 0x474F5353u,
  SALT_CHURN = 0x43485552u,  // RUMOR mode churn draws (SEMANTICS.md §9)
  SALT_DELAY_BASE = 0x444C5900u,  // + message kind: NetworkLinkSettings.evaluateDelay draws (SEMANTICS.md §2)
  SALT_DELAY_GOSSIP = 0x444C5947u,
};

inline uint32_t next_int(uint32_t x, uint32_t bound) { return (uint32_t)(((uint64_t)x * bound) >> 32); }

inline uint64_t mix64(uint64_t z) {  // splitmix64 finalizer
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t hpair(uint64_t a, uint64_t b) { return mix64(mix64(a) ^ b); }

inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Bijection on [0,n) used for PRECONVERGED list orders (SEMANTICS.md §3):
// a 4-round Feistel network on the smallest even bit width b with 2^b >= n, cycle-walked into [0,n).
struct Feistel {
  uint32_t n, half, mask;
  uint32_t rk[4];
  Feistel(uint32_t n_, const uint32_t keys[4]) : n(n_) {
    uint32_t b = 2;
    while (b < 32 && (1ull << b) < n) b += 2;
    half = b / 2;
    mask = (1u << half) - 1u;
    for (int i = 0; i < 4; ++i) rk[i] = keys[i];
  }
  uint32_t once(uint32_t x) const {
    uint32_t L = x >> half, R = x & mask;
    for (int r = 0; r < 4; ++r) {
      uint32_t nl = R;
      uint32_t nr = L ^ (fmix32(R ^ rk[r]) & mask);
      L = nl;
      R = nr;
    }
    return (L << half) | R;
  }
  uint32_t operator()(uint32_t x) const {
    uint32_t y = once(x);
    while (y >= n) y = once(y);
    return y;
  }
};

}  // namespace swimref
