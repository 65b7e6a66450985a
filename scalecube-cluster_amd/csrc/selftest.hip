// selftest.hip — swim_selftest_eval (include/swimhip_selftest.h): the device primitives the simulation kernels call,
// evaluated on caller inputs in a gfx950 kernel, so the reference's known answers pin the device code itself.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/swimhip.h"
#include "../../include/swimhip_selftest.h"
#include "dev_util.h"

namespace swim {

__global__ void k_selftest(uint32_t op, const uint32_t* in, uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (op == SWIM_SELFTEST_OVERRIDES) {
    const uint32_t* a = in + 4ull * i;
    out[i] = overrides(a[0], a[1], a[2], a[3]) ? 1u : 0u;  // swim_common.h, as update_membership calls it
  } else if (op == SWIM_SELFTEST_PHILOX) {
    const uint32_t* a = in + 6ull * i;
    const u32x4 r = philox(a[0], a[1], a[2], a[3], a[4], a[5]);
    out[4ull * i] = r.x;
    out[4ull * i + 1] = r.y;
    out[4ull * i + 2] = r.z;
    out[4ull * i + 3] = r.w;
  } else if (op == SWIM_SELFTEST_LOSS_ROLL) {
    const uint32_t* a = in + 8ull * i;  // the roll lost_msg compares with the link's loss percent (dev_util.h)
    out[i] = loss_roll(a[6], a[7], a[0], a[1], a[2], a[3], a[4], a[5]);
  } else {
    const uint32_t* a = in + 4ull * i;
    Dev d;  // only the fields the ClusterMath helpers read (dev_util.h)
    d.repeatMult = a[1];
    d.suspMult = a[2];
    d.ping_t = a[3];
    const uint32_t sp = spread_of(d, a[0]);
    out[4ull * i] = bitlen(a[0]);
    out[4ull * i + 1] = sp;
    out[4ull * i + 2] = sweep_after(sp);
    out[4ull * i + 3] = suspicion_ticks(d, a[0], a[3]);
  }
}

}  // namespace swim

extern "C" int swim_selftest_eval(uint32_t op, const uint32_t* in, uint32_t* out, size_t n, uint32_t device) {
  if (op > SWIM_SELFTEST_LOSS_ROLL || (n && (!in || !out)) || n > (1u << 24)) return SWIM_EINVAL;
  if (n == 0) return SWIM_OK;
  const size_t win = op == SWIM_SELFTEST_PHILOX ? 6 : op == SWIM_SELFTEST_LOSS_ROLL ? 8 : 4;
  const size_t wout = (op == SWIM_SELFTEST_OVERRIDES || op == SWIM_SELFTEST_LOSS_ROLL) ? 1 : 4;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= (int)device || hipSetDevice((int)device) != hipSuccess)
    return SWIM_EDEVICE;
  uint32_t *din = nullptr, *dout = nullptr;
  int rc = SWIM_OK;
  if (hipMalloc(&din, 4 * win * n) != hipSuccess || hipMalloc(&dout, 4 * wout * n) != hipSuccess) {
    rc = SWIM_ENOMEM;
  } else if (hipMemcpy(din, in, 4 * win * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = SWIM_EDEVICE;
  } else {
    hipLaunchKernelGGL(swim::k_selftest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, op, din, dout, (uint32_t)n);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, dout, 4 * wout * n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = SWIM_EDEVICE;
  }
  if (din) hipFree(din);
  if (dout) hipFree(dout);
  return rc;
}
