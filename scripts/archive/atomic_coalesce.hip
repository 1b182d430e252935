// Diagnostic microbenchmark (not part of the library): how many memory-side
// float-atomic requests (TCC_EA0_ATOMIC) does one wave-instruction cost for a
// given lane -> address pattern?  Each kernel launch issues `iters`
// instructions per wave; patterns differ only in how 64 lanes map onto
// 16 distinct 64-B segments (4 dwords each) of a large random-row table.
//   build: hipcc -O3 --offload-arch=gfx950 scripts/atomic_coalesce.hip -o /tmp/ac
//   run:   rocprofv3 --kernel-trace --pmc TCC_EA0_ATOMIC_sum -- /tmp/ac
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// pattern: 0 = lane/4 -> segment (4 consecutive lanes per segment)
//          1 = lane%16 -> segment (segment-mates 16 lanes apart)
//          2 = lanes (l, l^32) pairs: segment = (l & 31)/2, dword by (l>>5, l&1)
//          3 = all 64 lanes distinct segments (one dword each)
//          4 = lane/8 -> segment, 8 lanes per segment hitting 2 dwords each (duplicates)
//          5 = lane%16 segments, but duplicates: dword = (lane>>4)&1 (2 lanes per dword)
__global__ void scatter(float* table, uint32_t n_seg_mask, int pattern, int iters) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  for (int it = 0; it < iters; ++it) {
    const uint32_t base = mix(wave * 7919u + (uint32_t)it * 104729u);
    int s, d;
    switch (pattern) {
      case 0: s = lane >> 2; d = lane & 3; break;
      case 1: s = lane & 15; d = lane >> 4; break;
      case 2: s = (lane & 31) >> 1; d = ((lane >> 5) << 1) | (lane & 1); break;
      case 3: s = lane; d = 0; break;
      case 4: s = lane >> 3; d = (lane >> 1) & 3; break;
      default: s = lane & 15; d = (lane >> 4) & 1; break;
    }
    const uint32_t seg = (mix(base + (uint32_t)s * 31u) & n_seg_mask);
    atomicAdd(table + (size_t)seg * 16 + d, 1.0f);
  }
}

int main() {
  const size_t n_seg = 1u << 20;          // 64 MiB of 64-B segments
  float* t;
  hipMalloc(&t, n_seg * 64);
  hipMemset(t, 0, n_seg * 64);
  const int blocks = 1024, threads = 256, iters = 64;
  const double instr = (double)blocks * (threads / 64) * iters;
  for (int p = 0; p <= 5; ++p) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(scatter, dim3(blocks), dim3(threads), 0, 0, t, (uint32_t)(n_seg - 1), p, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL(scatter, dim3(blocks), dim3(threads), 0, 0, t, (uint32_t)(n_seg - 1), p, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("pattern %d: %.3f ms, %.2f G instr/s, %.1f ns/instr-chip\n", p, ms, instr / ms / 1e6,
           ms * 1e6 / instr);
  }
  hipFree(t);
  return 0;
}
