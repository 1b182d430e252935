// hn_optim.hip -- the rest of the training step on the device:
//   * hash-table total variation (loss.py:11-43): all 16 levels' cubes in one
//     forward launch and one backward launch (the reference issues ~70 eager
//     ops per level, including a sort-based embedding backward);
//   * RAdam (radam.py:28-94): every parameter tensor in one launch, dense,
//     in the reference's per-element op order.
#include "hn_tv.h"

namespace hn {

HN_DEV float block_sum_256(float v) {
  __shared__ float red[4];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void tv_fwd_kernel(TvK k, float* __restrict__ tv) {
  const int l = tv_level(k, k.boff, blockIdx.x);
  const int c = k.cube[l], n1 = c + 1;
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < kTvFwdV; ++q) {
    const int t = ((blockIdx.x - k.boff[l]) * kTvFwdV + q) * 256 + threadIdx.x;
    if (t < n1 * n1 * n1) {
      // x fastest across the lanes: h(x..x+7) of one (y, z) fill one 64-B
      // segment, so neighbouring lanes' gathers share cache lines (the TV sum is
      // order-free up to fp32 rounding; the reference's 'ij' order is only its
      // summation order)
      const int i = t % n1, j = (t / n1) % n1, kk = t / (n1 * n1);
      const uint32_t x = (uint32_t)(k.mv[3 * l] + i), y = (uint32_t)(k.mv[3 * l + 1] + j),
                     z = (uint32_t)(k.mv[3 * l + 2] + kk);
      const float2 e = tv_row(k, l, x, y, z);
      if (i < c) { const float2 n = tv_row(k, l, x + 1, y, z); const float a = n.x - e.x, b = n.y - e.y; acc += a * a + b * b; }
      if (j < c) { const float2 n = tv_row(k, l, x, y + 1, z); const float a = n.x - e.x, b = n.y - e.y; acc += a * a + b * b; }
      if (kk < c) { const float2 n = tv_row(k, l, x, y, z + 1); const float a = n.x - e.x, b = n.y - e.y; acc += a * a + b * b; }
    }
  }
  const float s = block_sum_256(acc);
  if (threadIdx.x == 0 && s != 0.f) atomic_add_f32(tv + l, s / (float)c);
}

// One thread per (vertex, feature), x fastest: the two features of a row
// are adjacent lanes and 8 consecutive x of one (y, z) share a 64-B segment,
// so one wave-instruction of atomics is ~8 memory requests instead of 64.
__global__ __launch_bounds__(256) void tv_bwd_kernel(TvK k, const float* __restrict__ g_tv,
                                                     float* __restrict__ dtable) {
  const int l = tv_level(k, k.bofb, blockIdx.x);
  const int c = k.cube[l], n1 = c + 1;
  const int t = (blockIdx.x - k.bofb[l]) * 256 + threadIdx.x;
  const int v = t >> 1, f = t & 1;
  if (v >= n1 * n1 * n1) return;
  const int i = v % n1, j = (v / n1) % n1, kk = v / (n1 * n1);
  const uint32_t x = (uint32_t)(k.mv[3 * l] + i), y = (uint32_t)(k.mv[3 * l + 1] + j),
                 z = (uint32_t)(k.mv[3 * l + 2] + kk);
  const float g = tv_grad(k, l, c, i, j, kk, x, y, z, f);
  const float scale = g_tv[l] / (float)c;
  const uint32_t mask = (1u << k.log2T) - 1u;
  const uint32_t h = (x ^ (y * kPrimeY) ^ (z * kPrimeZ)) & mask;
  atomic_add_f32(dtable + ((((size_t)l << k.log2T) + h) << 1) + f, scale * g);
}

struct RadamK {
  int32_t n;
  hn_radam_tensor t[HN_RADAM_MAX_TENSORS];
};

__global__ __launch_bounds__(256) void radam_kernel(RadamK k) {
  const hn_radam_tensor& d = k.t[blockIdx.y];
  const int64_t n = d.n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool vec = ((n & 3) == 0) && ((((uintptr_t)d.p) | ((uintptr_t)d.g) | ((uintptr_t)d.m) |
                                       ((uintptr_t)d.v)) & 15) == 0;
  if (vec) {
    const int64_t n4 = n >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      float4 p = reinterpret_cast<float4*>(d.p)[i];
      const float4 g = reinterpret_cast<const float4*>(d.g)[i];
      float4 m = reinterpret_cast<float4*>(d.m)[i];
      float4 v = reinterpret_cast<float4*>(d.v)[i];
      radam_elem(d, p.x, g.x, m.x, v.x);
      radam_elem(d, p.y, g.y, m.y, v.y);
      radam_elem(d, p.z, g.z, m.z, v.z);
      radam_elem(d, p.w, g.w, m.w, v.w);
      reinterpret_cast<float4*>(d.m)[i] = m;
      reinterpret_cast<float4*>(d.v)[i] = v;
      if (d.mode != 0) reinterpret_cast<float4*>(d.p)[i] = p;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      float p = d.p[i], m = d.m[i], v = d.v[i];
      radam_elem(d, p, d.g[i], m, v);
      d.m[i] = m;
      d.v[i] = v;
      if (d.mode != 0) d.p[i] = p;
    }
  }
}

}  // namespace hn

using namespace hn;

extern "C" int32_t hn_tv_fwd(const hn_tv_args* a, float* tv, void* stream) {
  TvK k;
  int nb, nbb;
  int32_t st = make_tv(a, k, nb, nbb);
  if (st) return st;
  if (!tv) return HN_E_NULL;
  hipStream_t s = (hipStream_t)stream;
  if ((st = hip_status(hipMemsetAsync(tv, 0, sizeof(float) * a->n_levels, s)))) return st;
  hipLaunchKernelGGL(tv_fwd_kernel, dim3(nb), dim3(256), 0, s, k, tv);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_tv_bwd(const hn_tv_args* a, const float* g_tv, float* dtable, void* stream) {
  TvK k;
  int nb, nbb;
  int32_t st = make_tv(a, k, nb, nbb);
  if (st) return st;
  if (!g_tv || !dtable) return HN_E_NULL;
  hipLaunchKernelGGL(tv_bwd_kernel, dim3(nbb), dim3(256), 0, (hipStream_t)stream, k, g_tv,
                     dtable);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_radam_step(const hn_radam_tensor* ts, int32_t n_tensors, void* stream) {
  if (n_tensors < 0 || n_tensors > HN_RADAM_MAX_TENSORS) return HN_E_SHAPE;
  if (n_tensors == 0) return HN_OK;
  if (!ts) return HN_E_NULL;
  RadamK k;
  k.n = n_tensors;
  int64_t max_n = 0;
  for (int i = 0; i < n_tensors; ++i) {
    if (!ts[i].p || !ts[i].g || !ts[i].m || !ts[i].v) return HN_E_NULL;
    if (ts[i].n < 0) return HN_E_SHAPE;
    k.t[i] = ts[i];
    max_n = ts[i].n > max_n ? ts[i].n : max_n;
  }
  int64_t blocks = (max_n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(radam_kernel, dim3((unsigned)blocks, n_tensors), dim3(256), 0, (hipStream_t)stream, k);
  return hip_status(hipGetLastError());
}
