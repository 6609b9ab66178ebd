// Exhaustive check of drt::rcp_rn (drt_device.hpp) against the correctly rounded 1.0f / a over
// all 2^32 float bit patterns on gfx950.  Prints one JSON line; "mismatches" must be 0.
// The short path alone (v_rcp_f32 + one FMA Newton step, no range guard) is counted too, split by
// whether |a| lies in the guarded range [2^-125, 2^125].
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../distributionraytracer_amd/csrc/hip/drt_device.hpp"

__global__ void check(uint32_t hi, unsigned long long* cnt) {
  const uint32_t bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
  const float a = __uint_as_float(bits);
  const float ref = 1.0f / a;
  auto same = [&](float y) { return __float_as_uint(ref) == __float_as_uint(y) || (ref != ref && y != y); };
  if (!same(drt::rcp_rn(a))) atomicAdd(&cnt[0], 1ull);
  const float r = __builtin_amdgcn_rcpf(a);
  const float y = __builtin_fmaf(__builtin_fmaf(-a, r, 1.0f), r, r);
  if (!same(y)) {
    const float m = __builtin_fabsf(a);
    atomicAdd(&cnt[(m >= 0x1p-125f && m <= 0x1p125f) ? 1 : 2], 1ull);
  }
}

int main() {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 3 * sizeof(unsigned long long)) != hipSuccess) return 1;
  if (hipMemset(d, 0, 3 * sizeof(unsigned long long)) != hipSuccess) return 1;
  for (uint32_t hi = 0; hi < 256; hi++) hipLaunchKernelGGL(check, dim3(1 << 16), dim3(256), 0, 0, hi, d);
  unsigned long long c[3] = {0, 0, 0};
  if (hipMemcpy(c, d, sizeof(c), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  printf("{\"inputs\": 4294967296, \"mismatches\": %llu, \"short_path_mismatches_in_range\": %llu, "
         "\"short_path_mismatches_outside_range\": %llu}\n", c[0], c[1], c[2]);
  return c[0] == 0 ? 0 : 2;
}
