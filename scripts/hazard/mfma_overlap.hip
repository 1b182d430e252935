// Diagnostic (not part of the library): does v_mfma_f32_32x32x16_bf16 whose
// VGPR destination partially overlaps its own SrcA (the first MFMA of a chain,
// C = inline 0, A dead afterwards -- the register allocator then puts D on A's
// registers) give the same result as the same product with A kept alive
// (D disjoint from A)?  Each wave runs a loop of chains on fresh operands
// from LDS under full MFMA load (4 waves per SIMD); the output is compared
// bitwise between the two builds of the loop and between repeated launches.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 mfma_overlap.hip -o mfma_overlap
//   ./mfma_overlap [launches]   (the library's flags: MFMA results in VGPRs)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KEEP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))
void chains(const f32x4* __restrict__ src, float* __restrict__ out, int iters) {
  __shared__ f32x4 lds[4][2][64 * 8];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + wave;
  for (int i = 0; i < 8; ++i) {
    lds[wave][0][i * 64 + lane] = src[(size_t)(gw * 16 + 2 * i) * 64 + lane];
    lds[wave][1][i * 64 + lane] = src[(size_t)(gw * 16 + 2 * i + 1) * 64 + lane];
  }
  __syncthreads();
  f32x16 tot = {};
  for (int it = 0; it < iters; ++it) {
    const int s = it & 7;
    // fresh A and B from LDS each iteration (dead after their MFMAs)
    bf16x8 a = __builtin_bit_cast(bf16x8, lds[wave][0][s * 64 + lane]);
    bf16x8 b = __builtin_bit_cast(bf16x8, lds[wave][1][s * 64 + lane]);
    bf16x8 a2 = __builtin_bit_cast(bf16x8, lds[wave][0][((s + 3) & 7) * 64 + lane]);
    f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, f32x16{}, 0, 0, 0);
    if (KEEP) asm volatile("" ::"v"(a));   // A stays live past the MFMA: D cannot overlap it
    d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b, d, 0, 0, 0);
    tot += d;
  }
  for (int r = 0; r < 16; ++r) out[((size_t)gw * 16 + r) * 64 + lane] = tot[r];
}

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 20, iters = 4096;
  const int blocks = 256 * 4, waves = blocks * 4;
  // bf16 operands: small integers / 16 (exact in bf16; every product and sum is
  // exact in fp32, so the result does not depend on the accumulation order)
  std::vector<uint16_t> h((size_t)waves * 16 * 64 * 8);
  srand(1);
  for (auto& x : h) {
    const float f = (float)((rand() % 129) - 64) / 16.f;
    uint32_t u;
    memcpy(&u, &f, 4);
    x = (uint16_t)(u >> 16);
  }
  f32x4* src;
  float *o0, *o1;
  const size_t nout = (size_t)waves * 16 * 64;
  hipMalloc(&src, h.size() * 2);
  hipMalloc(&o0, nout * 4);
  hipMalloc(&o1, nout * 4);
  hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  std::vector<float> ref(nout), got(nout);
  hipLaunchKernelGGL(chains<1>, dim3(blocks), dim3(256), 0, 0, src, o1, iters);
  hipMemcpy(ref.data(), o1, nout * 4, hipMemcpyDeviceToHost);
  long bad_launches = 0, bad_vals = 0, bad_lo = 0, bad_hi = 0;
  for (int l = 0; l < launches; ++l) {
    for (int keep = 0; keep < 2; ++keep) {
      float* o = keep ? o1 : o0;
      if (keep) hipLaunchKernelGGL(chains<1>, dim3(blocks), dim3(256), 0, 0, src, o, iters);
      else hipLaunchKernelGGL(chains<0>, dim3(blocks), dim3(256), 0, 0, src, o, iters);
      hipMemcpy(got.data(), o, nout * 4, hipMemcpyDeviceToHost);
      long bv = 0;
      for (size_t i = 0; i < nout; ++i)
        if (memcmp(&got[i], &ref[i], 4) != 0) {
          ++bv;
          ((i & 63) % 32 < 16 ? bad_lo : bad_hi)++;
        }
      if (bv) {
        ++bad_launches;
        bad_vals += bv;
        printf("launch %d keep=%d: %ld values differ\n", l, keep, bv);
      }
    }
  }
  printf("launches %d x 2: %ld with differences, %ld values (columns 0-15: %ld, 16-31: %ld)\n", launches,
         bad_launches, bad_vals, bad_lo, bad_hi);
  return 0;
}
