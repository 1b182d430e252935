// Diagnostic (not part of the library): do VGPR spills to scratch ever come
// back with another wave's data?  The round-3 forward nondeterminism hit one
// ray's colour net on lanes 16-31 and 48-63 -- in a swizzled dwordx4 spill slot
// (lane l's dword at byte 4 l of a 256-B row) exactly the second 64-B half of
// each 128-B line -- for every tile of the ray, with its operand (the per-ray
// SH split) spilled once per ray and reloaded per tile.  Here every wave keeps
// 16 per-lane values that are unique to the wave live across a loop whose
// asm clobbers v0-v111, so the compiler spills them to scratch once and
// reloads them every iteration (check the .s), with gathers and MFMAs around
// it, 4 waves per SIMD and many more waves than slots (each slot's scratch
// holds the previous wave's values); every reload is checked.
//   hipcc --offload-arch=gfx950 -O3 scratch_probe.hip -o scratch_probe && ./scratch_probe [launches]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pattern(uint32_t w, uint32_t lane, uint32_t j) {
  uint32_t x = w * 0x9E3779B1u ^ (lane * 0x85EBCA77u) ^ (j * 0xC2B2AE3Du);
  x ^= x >> 15;
  x *= 0x2C1B3C6Du;
  return x ^ (x >> 12);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))
void probe(const float2* __restrict__ table, uint32_t mask, const f32x4* __restrict__ wsrc, unsigned* bad,
           float* sink, int iters) {
  const int lane = threadIdx.x & 63;
  const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
  uint32_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = pattern(w, lane, j);
  f32x16 acc = {};
  float g = 0.f;
  uint32_t h = w * 2654435761u + lane;
  unsigned errs = 0;
  for (int it = 0; it < iters; ++it) {
    // gathers
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      h = h * 1664525u + 1013904223u;
      const float2 t = table[h & mask];
      g += t.x * t.y;
    }
    // MFMAs on fresh operands
    const f32x4 a = wsrc[(it & 63) * 64 + lane], b = wsrc[((it + 7) & 63) * 64 + lane];
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
    // every live VGPR must be saved around this: the 16 values go to scratch
    asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13",
                 "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27",
                 "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41",
                 "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                 "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69",
                 "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83",
                 "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97",
                 "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109",
                 "v110", "v111");
#pragma unroll
    for (int j = 0; j < 16; ++j) errs += v[j] != pattern(w, lane, j) ? 1u : 0u;
  }
  if (errs) atomicAdd(&bad[((lane & 31) < 16 ? 0 : 1)], errs);
  sink[(size_t)w * 64 + lane] = g + acc[0] + acc[15];
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 10, iters = 64;
  const int blocks = 1024 * 8, waves = blocks * 4;   // 8 waves per wave slot over a launch
  const uint32_t T = 1u << 22;
  float2* table;
  f32x4* wsrc;
  unsigned* bad;
  float* sink;
  if (hipMalloc(&table, (size_t)T * 8) || hipMalloc(&wsrc, 64 * 64 * 16) || hipMalloc(&bad, 8) ||
      hipMalloc(&sink, (size_t)waves * 64 * 4))
    return 1;
  hipMemset(table, 0, (size_t)T * 8);
  hipMemset(wsrc, 0, 64 * 64 * 16);
  unsigned tot[2] = {0, 0};
  for (int l = 0; l < launches; ++l) {
    unsigned hb[2] = {0, 0};
    hipMemcpy(bad, hb, 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, table, T - 1, wsrc, bad, sink, iters);
    if (hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost)) return 1;
    if (hb[0] || hb[1]) printf("launch %d: %u bad reloads on lanes %%32 < 16, %u on lanes %%32 >= 16\n", l, hb[0], hb[1]);
    tot[0] += hb[0];
    tot[1] += hb[1];
  }
  printf("%d launches x %d waves x %d reloads of 16 values: %u bad on lanes 0-15/32-47, %u on lanes 16-31/48-63\n",
         launches, waves, iters, tot[0], tot[1]);
  return 0;
}
