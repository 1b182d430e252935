// hn_optim.hip -- the rest of the training step on the device:
//   * hash-table total variation (loss.py:11-43): all 16 levels' cubes in one
//     forward launch and one backward launch (the reference issues ~70 eager
//     ops per level, including a sort-based embedding backward);
//   * RAdam (radam.py:28-94): every parameter tensor in one launch, dense,
//     in the reference's per-element op order.
#include "hn_common.h"

namespace hn {

struct TvK {
  int32_t L, log2T;
  int32_t cube[HN_MAX_LEVELS];
  // packed 1-D grids: level l owns blocks [boff[l], boff[l+1]) of the
  // forward (kTvFwdV vertices per thread) and [bofb[l], bofb[l+1]) of the
  // backward (one thread per (vertex, feature)), instead of a (max blocks) x L
  // grid that is mostly idle blocks
  int32_t boff[HN_MAX_LEVELS + 1], bofb[HN_MAX_LEVELS + 1];
  const int32_t* mv;
  const float* table;
};

// Entry of grid vertex (x, y, z) of level l (hash_encoding.py:112-128).
HN_DEV float2 tv_row(const TvK& k, int l, uint32_t x, uint32_t y, uint32_t z) {
  const uint32_t mask = (1u << k.log2T) - 1u;
  const uint32_t h = (x ^ (y * kPrimeY) ^ (z * kPrimeZ)) & mask;
  return ld_row(k.table, (((uint32_t)l << k.log2T) + h) * 8u);
}

HN_DEV float block_sum_256(float v) {
  __shared__ float red[4];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// level of packed block b (wave-uniform; at most 16 scalar compares)
HN_DEV int tv_level(const TvK& k, const int32_t* off, int b) {
  int l = 0;
  while (l + 1 < k.L && b >= off[l + 1]) ++l;
  return l;
}

// vertices per forward thread: fewer blocks, so fewer same-address atomics
// on the 16 level sums
#ifndef HN_TV_FWD_V
#define HN_TV_FWD_V 4
#endif
constexpr int kTvFwdV = HN_TV_FWD_V;

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
HN_DEV float tv_val(const TvK& k, int l, uint32_t x, uint32_t y, uint32_t z, int f) {
  const uint32_t mask = (1u << k.log2T) - 1u;
  const uint32_t h = (x ^ (y * kPrimeY) ^ (z * kPrimeZ)) & mask;
  return k.table[((((size_t)l << k.log2T) + h) << 1) + f];
}

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
  const float e = tv_val(k, l, x, y, z, f);
  float g = 0.f;   // sum over incident edges of d(d^2)/de = -+2d
  const int idx[3] = {i, j, kk};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (idx[a] < c) g -= 2.f * (tv_val(k, l, x + (a == 0), y + (a == 1), z + (a == 2), f) - e);
    if (idx[a] > 0) g += 2.f * (e - tv_val(k, l, x - (a == 0), y - (a == 1), z - (a == 2), f));
  }
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

static int32_t make_tv(const hn_tv_args* a, TvK& k, int& fwd_blocks, int& bwd_blocks) {
  if (!a || !a->min_vertex || !a->table) return HN_E_NULL;
  if (a->n_levels < 1 || a->n_levels > HN_MAX_LEVELS) return HN_E_SHAPE;
  if (a->log2_hashmap_size < 1 || a->log2_hashmap_size > 24) return HN_E_SHAPE;
  k.L = a->n_levels;
  k.log2T = a->log2_hashmap_size;
  k.mv = a->min_vertex;
  k.table = a->table;
  for (int l = 0; l < HN_MAX_LEVELS; ++l) k.cube[l] = l < a->n_levels ? a->cube[l] : 1;
  k.boff[0] = k.bofb[0] = 0;
  for (int l = 0; l < HN_MAX_LEVELS; ++l) {
    int nv = 0;
    if (l < a->n_levels) {
      const int c = a->cube[l];
      if (c < 1 || c > 1000) return HN_E_SHAPE;
      nv = (c + 1) * (c + 1) * (c + 1);
    }
    k.boff[l + 1] = k.boff[l] + (nv + 256 * kTvFwdV - 1) / (256 * kTvFwdV);
    k.bofb[l + 1] = k.bofb[l] + (2 * nv + 255) / 256;
  }
  fwd_blocks = k.boff[a->n_levels];
  bwd_blocks = k.bofb[a->n_levels];
  return HN_OK;
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
