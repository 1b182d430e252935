// hn_loss.h -- the training loss value (run_nerf.py:612-636 under
// train.dp_loss's data-parallel rule) reduced by one workgroup of NT threads:
// hn_loss_fwd's kernel (NT = 1024) and the render backward's composite
// pre-pass when it forms the loss itself (NT = 256, ABI 13).
#pragma once
#include "hn_common.h"

namespace hn {

// Forward: one workgroup, fp64 accumulation of the reductions (the value is
// reported, its gradient does not depend on the summation order).
template <int NT>
HN_DEV void loss_fwd_block(
    const float* __restrict__ rgb, const float* __restrict__ rgb0, const float* __restrict__ target,
    const float* __restrict__ sp, const float* __restrict__ sp0, int64_t n, const float* __restrict__ tv,
    int n_tv, float world, float sparse_w, float tv_w, float* __restrict__ out) {
  __shared__ double red[4][NT / 64];
  double a[4] = {0.0, 0.0, 0.0, 0.0};   // sse, sse0, entropy, tv
  // float4 loads where the arrays are 16-B aligned (torch allocations are),
  // every load of a thread in flight at once: one workgroup is launch-bound
  const bool vec = ((reinterpret_cast<uintptr_t>(rgb) | reinterpret_cast<uintptr_t>(target) |
                     reinterpret_cast<uintptr_t>(rgb0) | reinterpret_cast<uintptr_t>(sp) |
                     reinterpret_cast<uintptr_t>(sp0)) & 15u) == 0;
  const int64_t m3 = vec ? (3 * n) / 4 : 0, m1 = vec ? n / 4 : 0;
  for (int64_t j = threadIdx.x; j < m3; j += NT) {
    const float4 x = reinterpret_cast<const float4*>(rgb)[j], t = reinterpret_cast<const float4*>(target)[j];
    const float e[4] = {x.x - t.x, x.y - t.y, x.z - t.z, x.w - t.w};
    for (int q = 0; q < 4; ++q) a[0] += (double)(e[q] * e[q]);
    if (rgb0) {
      const float4 y = reinterpret_cast<const float4*>(rgb0)[j];
      const float f[4] = {y.x - t.x, y.y - t.y, y.z - t.z, y.w - t.w};
      for (int q = 0; q < 4; ++q) a[1] += (double)(f[q] * f[q]);
    }
  }
  for (int64_t j = 4 * m3 + threadIdx.x; j < 3 * n; j += NT) {
    const float e = rgb[j] - target[j];
    a[0] += (double)(e * e);
    if (rgb0) {
      const float e0 = rgb0[j] - target[j];
      a[1] += (double)(e0 * e0);
    }
  }
  for (int64_t j = threadIdx.x; j < m1; j += NT) {
    const float4 x = reinterpret_cast<const float4*>(sp)[j];
    a[2] += ((double)x.x + (double)x.y) + ((double)x.z + (double)x.w);
    if (sp0) {
      const float4 y = reinterpret_cast<const float4*>(sp0)[j];
      a[2] += ((double)y.x + (double)y.y) + ((double)y.z + (double)y.w);
    }
  }
  for (int64_t j = 4 * m1 + threadIdx.x; j < n; j += NT)
    a[2] += (double)sp[j] + (sp0 ? (double)sp0[j] : 0.0);
  if (tv)
    for (int j = threadIdx.x; j < n_tv; j += NT) a[3] += (double)tv[j];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double v = wave_sum(a[q]);
    if ((threadIdx.x & 63) == 0) red[q][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < 4; ++q)
      for (int w = 0; w < NT / 64; ++w) t[q] += red[q][w];
    const double N = 3.0 * (double)n;
    const float mse = (float)(t[0] / N), mse0 = rgb0 ? (float)(t[1] / N) : 0.f;
    const float ent = (float)t[2];
    out[0] = (mse + mse0) / world + sparse_w * ent + (tv ? tv_w * (float)t[3] : 0.f);
    out[1] = mse;
    out[2] = mse0;
    out[3] = ent;
  }
}

}  // namespace hn
