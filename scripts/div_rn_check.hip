// div_rn (hn_common.h) against the IEEE f32 division over random operands
// in the trilinear weights' range: numerators |n| <= 2^8 (with exact zeros
// and tiny ones), denominators in [2^-12, 2^2]; prints the mismatches.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/div_rn_check.hip -o /tmp/div_rn_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../hashnerf-pytorch_amd/csrc/hn_common.h"

__device__ uint32_t hmix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}
__global__ void check(uint64_t base, unsigned long long* bad, float* ex) {
  const uint64_t i = base + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint32_t a = hmix(2 * i), b = hmix(2 * i + 1);
  // n: sign, exponent in [-40, 8], random mantissa; 1/16 exact zeros
  const int en = (int)(a >> 24) % 49 - 40;
  float n = ldexpf(1.f + (float)(a & 0x7fffff) * 0x1p-23f, en) * ((a >> 23) & 1 ? -1.f : 1.f);
  if ((b & 15) == 0) n = 0.f;
  const int ed = (int)((b >> 24) % 15) - 12;
  const float d = ldexpf(1.f + (float)((b >> 1) & 0x7fffff) * 0x1p-23f, ed);
  const float q0 = n / d, q1 = hn::div_rn(n, d);
  if (__float_as_uint(q0) != __float_as_uint(q1)) {
    const unsigned long long k = atomicAdd(bad, 1ull);
    if (k < 4) { ex[4 * k] = n; ex[4 * k + 1] = d; ex[4 * k + 2] = q0; ex[4 * k + 3] = q1; }
  }
}
int main() {
  unsigned long long* bad; float* ex;
  hipMalloc(&bad, 8); hipMalloc(&ex, 64); hipMemset(bad, 0, 8);
  const uint64_t per = 1ull << 28;   // operands per launch
  const int launches = 16;           // 4.3e9 pairs
  for (int l = 0; l < launches; ++l) hipLaunchKernelGGL(check, dim3(per / 256), dim3(256), 0, 0, l * per, bad, ex);
  unsigned long long nb = 0; float e[16];
  hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(e, ex, 64, hipMemcpyDeviceToHost);
  printf("div_rn vs IEEE division: %llu mismatches in %llu pairs\n", nb, (unsigned long long)per * launches);
  for (int k = 0; k < 4 && k < (int)nb; ++k) printf("  n=%a d=%a ieee=%a div_rn=%a\n", e[4*k], e[4*k+1], e[4*k+2], e[4*k+3]);
  return nb != 0;
}
