// hn_composite.hip -- standalone raw2outputs fwd/bwd (run_nerf_helpers.py:577-628)
// and sample_pdf (run_nerf_helpers.py:264-307): one wave64 per ray.
#include "hn_render.h"

namespace hn {

constexpr int kWaves = 4;   // waves (rays) per 256-thread block

template <int N>
__global__ __launch_bounds__(256) void composite_fwd_kernel(
    const float* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rays_d,
    const float* __restrict__ noise, int64_t n_rays, int S, int white, float* __restrict__ rgb,
    float* __restrict__ disp, float* __restrict__ acc, float* __restrict__ weights,
    float* __restrict__ depth, float* __restrict__ entropy) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (ray >= n_rays) return;
  const float* d = rays_d + 3 * ray;
  const float dnorm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  CompOut o;
  composite_fwd<N>(raw + ray * S * 4, z + ray * S, noise ? noise + ray * S : nullptr, S, dnorm,
                   white != 0, weights ? weights + ray * S : nullptr, o, lane);
  if (lane == 0) {
    if (rgb) { rgb[3 * ray] = o.rgb[0]; rgb[3 * ray + 1] = o.rgb[1]; rgb[3 * ray + 2] = o.rgb[2]; }
    if (disp) disp[ray] = o.disp;
    if (acc) acc[ray] = o.acc;
    if (depth) depth[ray] = o.depth;
    if (entropy) entropy[ray] = o.entropy;
  }
}

template <int N>
__global__ __launch_bounds__(256) void composite_bwd_kernel(
    const float* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rays_d,
    const float* __restrict__ noise, int64_t n_rays, int S, int white, const float* __restrict__ g_rgb,
    const float* __restrict__ g_acc, const float* __restrict__ g_depth,
    const float* __restrict__ g_entropy, const float* __restrict__ g_weights,
    float* __restrict__ d_raw) {
  const int lane = threadIdx.x & 63;
  const int64_t ray = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (ray >= n_rays) return;
  const float* d = rays_d + 3 * ray;
  const float dnorm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  CompGrad g;
  g.has_rgb = g_rgb != nullptr;
  g.has_acc = g_acc != nullptr;
  g.has_depth = g_depth != nullptr;
  g.has_entropy = g_entropy != nullptr;
  g.rgb[0] = g.has_rgb ? g_rgb[3 * ray] : 0.f;
  g.rgb[1] = g.has_rgb ? g_rgb[3 * ray + 1] : 0.f;
  g.rgb[2] = g.has_rgb ? g_rgb[3 * ray + 2] : 0.f;
  g.acc = g.has_acc ? g_acc[ray] : 0.f;
  g.depth = g.has_depth ? g_depth[ray] : 0.f;
  g.entropy = g.has_entropy ? g_entropy[ray] : 0.f;
  composite_bwd<N>(raw + ray * S * 4, z + ray * S, noise ? noise + ray * S : nullptr, S, dnorm,
                   white != 0, g, g_weights ? g_weights + ray * S : nullptr, nullptr,
                   d_raw + ray * S * 4, lane);
}

__global__ __launch_bounds__(256) void sample_pdf_kernel(const float* __restrict__ bins,
                                                         const float* __restrict__ weights,
                                                         const float* __restrict__ u, int64_t n_rays,
                                                         int nb, int ns, float* __restrict__ out) {
  __shared__ float cdf[kWaves][256];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t ray = (int64_t)blockIdx.x * kWaves + wave;
  if (ray >= n_rays) return;
  sample_pdf_wave(bins + ray * nb, weights + ray * (nb - 1), nb - 1, cdf[wave], u + ray * ns, ns,
                  out + ray * ns, lane);
}

}  // namespace hn

using namespace hn;

#define HN_DISPATCH_N(S, KER, ...)                                             \
  do {                                                                         \
    const int n_ = ((S) + 63) / 64;                                            \
    if (n_ == 1) hipLaunchKernelGGL(KER<1>, __VA_ARGS__);                      \
    else if (n_ == 2) hipLaunchKernelGGL(KER<2>, __VA_ARGS__);                 \
    else if (n_ == 3) hipLaunchKernelGGL(KER<3>, __VA_ARGS__);                 \
    else hipLaunchKernelGGL(KER<4>, __VA_ARGS__);                              \
  } while (0)

extern "C" int32_t hn_composite_fwd(const float* raw, const float* z, const float* rays_d,
                                    const float* noise, int64_t n_rays, int32_t n_samples,
                                    int32_t white_bkgd, float* rgb, float* disp, float* acc,
                                    float* weights, float* depth, float* entropy, void* stream) {
  if (n_rays < 0 || n_samples < 1 || n_samples > 256) return HN_E_SHAPE;
  if (n_rays == 0) return HN_OK;
  if (!raw || !z || !rays_d) return HN_E_NULL;
  const dim3 grid((unsigned)((n_rays + kWaves - 1) / kWaves));
  HN_DISPATCH_N(n_samples, composite_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, raw, z,
                rays_d, noise, n_rays, n_samples, white_bkgd, rgb, disp, acc, weights, depth, entropy);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_composite_bwd(const float* raw, const float* z, const float* rays_d,
                                    const float* noise, int64_t n_rays, int32_t n_samples,
                                    int32_t white_bkgd, const float* g_rgb, const float* g_acc,
                                    const float* g_depth, const float* g_entropy,
                                    const float* g_weights, float* d_raw, void* stream) {
  if (n_rays < 0 || n_samples < 1 || n_samples > 256) return HN_E_SHAPE;
  if (n_rays == 0) return HN_OK;
  if (!raw || !z || !rays_d || !d_raw) return HN_E_NULL;
  const dim3 grid((unsigned)((n_rays + kWaves - 1) / kWaves));
  HN_DISPATCH_N(n_samples, composite_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, raw, z,
                rays_d, noise, n_rays, n_samples, white_bkgd, g_rgb, g_acc, g_depth, g_entropy,
                g_weights, d_raw);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_sample_pdf(const float* bins, const float* weights, const float* u,
                                 int64_t n_rays, int32_t n_bins, int32_t n_samples, float* out,
                                 void* stream) {
  if (n_rays < 0 || n_bins < 2 || n_bins > 256 || n_samples < 0) return HN_E_SHAPE;
  if (n_rays == 0 || n_samples == 0) return HN_OK;
  if (!bins || !weights || !u || !out) return HN_E_NULL;
  hipLaunchKernelGGL(sample_pdf_kernel, dim3((unsigned)((n_rays + kWaves - 1) / kWaves)), dim3(256), 0,
                     (hipStream_t)stream, bins, weights, u, n_rays, n_bins, n_samples, out);
  return hip_status(hipGetLastError());
}
