/*
 * swimhip_selftest.h — known-answer surface of libswimhip (and of the CPU oracle, which exports the same entry point).
 *
 * swim_selftest_eval runs the engine's own device primitives — the functions the simulation kernels call — on caller
 * inputs, in a gfx950 kernel, so the reference's known answers pin the device code itself, not a host copy of it:
 *   SWIM_SELFTEST_OVERRIDES      MembershipRecord.isOverrides (cluster/.../membership/MembershipRecord.java:66-84),
 *                                pinned by MembershipRecordTest.java:34-108
 *   SWIM_SELFTEST_PHILOX         Philox4x32-10, the injected selector (SEMANTICS.md §2), pinned by the Random123
 *                                known-answer vectors
 *   SWIM_SELFTEST_CLUSTER_MATH   ClusterMath.ceilLog2 / gossipPeriodsToSpread / gossipPeriodsToSweep / suspicionTimeout
 *                                (ClusterMath.java:99-135) as the engine evaluates them
 *   SWIM_SELFTEST_LOSS_ROLL      the per-message loss draw of the NetworkEmulator (TransportTest.testNetworkSettings,
 *                                transport/src/test/.../TransportTest.java:130-153, checks its statistics)
 * Not part of the simulation API; the oracle evaluates the same functions on the CPU.
 */
#ifndef SWIMHIP_SELFTEST_H
#define SWIMHIP_SELFTEST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SWIM_SELFTEST_OVERRIDES 0u    /* in[4i..4i+3] = r1 status, r1 inc, r0 status, r0 inc (status 0 = null, 3 = DEAD)
                                         -> out[i] = 1 if r1 overrides r0 */
#define SWIM_SELFTEST_PHILOX 1u       /* in[6i..6i+5] = ctr0..ctr3, key0, key1 -> out[4i..4i+3] */
#define SWIM_SELFTEST_CLUSTER_MATH 2u /* in[4i..4i+3] = cluster size, repeatMult, suspicionMult, pingInterval ticks
                                         -> out[4i..4i+3] = ceilLog2, periods to spread, periods to sweep, suspicion ticks */
#define SWIM_SELFTEST_LOSS_ROLL 3u    /* in[8i..8i+7] = message kind, src, dst, tick, issuer, id, seed lo, seed hi
                                         -> out[i] = the roll in [0,100) a send is lost below (NetworkLinkSettings
                                         .evaluateLoss, transport/.../NetworkLinkSettings.java:54-57) */

/* evaluates n cases of `op` on HIP device `device` (libswimhip) or on the host (oracle); 0 or a negative SWIM_E* code */
int swim_selftest_eval(uint32_t op, const uint32_t* in, uint32_t* out, size_t n, uint32_t device);

#ifdef __cplusplus
}
#endif
#endif
