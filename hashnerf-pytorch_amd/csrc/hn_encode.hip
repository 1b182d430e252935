// hn_encode.hip -- standalone hash-grid encoding (fwd/bwd) and SH encoding.
//
// Replaces HashEmbedder.forward (embedding/hash_encoding.py:84-110), its
// autograd (embedding_dense_backward per level) and SHEncoder.forward
// (embedding/spherical_harmonic.py:65-103).  One thread per (point, level):
// the 8 corner gathers of a level are independent 8-byte loads, consecutive
// threads write consecutive 8-byte feature pairs (coalesced [N][L*2] rows).
#include "hn_common.h"

namespace hn {

__global__ __launch_bounds__(256) void encode_fwd_kernel(GridArgs g, const float* __restrict__ x,
                                                         int64_t n, const float* __restrict__ table,
                                                         float* __restrict__ feat,
                                                         uint8_t* __restrict__ keep) {
  const int L = g.n_levels;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n * L) return;
  const int64_t p = tid / L;
  const int l = (int)(tid - p * L);
  const float xp[3] = {x[3 * p], x[3 * p + 1], x[3 * p + 2]};
  float xc[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) xc[a] = clamp_t(xp[a], g.bmin[a], g.bmax[a]);
  const uint32_t mask = (1u << g.log2T) - 1u;
  Voxel v;
  voxel_level(xp, xc, g.gs[l], g.bmin, mask, v);
  float f0, f1;
  encode_level(table + ((size_t)l << g.log2T) * 2, v, f0, f1);
  *reinterpret_cast<float2*>(feat + (size_t)p * (2 * L) + 2 * l) = make_float2(f0, f1);
  if (keep != nullptr && l == 0) {
    // hash_encoding.py:66,109: the mask of the LAST level, taken after the
    // level-0 clamp => only NaN coordinates fail when L > 1.
    bool k = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const float ref = (L > 1) ? xc[a] : xp[a];
      k = k && (ref == clamp_t(ref, g.bmin[a], g.bmax[a]));
    }
    keep[p] = k ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void encode_bwd_kernel(GridArgs g, const float* __restrict__ x,
                                                         int64_t n, const float* __restrict__ dfeat,
                                                         float* __restrict__ dtable) {
  const int L = g.n_levels;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n * L) return;
  const int64_t p = tid / L;
  const int l = (int)(tid - p * L);
  const float xp[3] = {x[3 * p], x[3 * p + 1], x[3 * p + 2]};
  float xc[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) xc[a] = clamp_t(xp[a], g.bmin[a], g.bmax[a]);
  const uint32_t mask = (1u << g.log2T) - 1u;
  Voxel v;
  voxel_level(xp, xc, g.gs[l], g.bmin, mask, v);
  const float2 gd = *reinterpret_cast<const float2*>(dfeat + (size_t)p * (2 * L) + 2 * l);
  float c0[8], c1[8];
  trilerp_bwd(gd.x, v.w, c0);
  trilerp_bwd(gd.y, v.w, c1);
  float* base = dtable + ((size_t)l << g.log2T) * 2;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    atomic_add_f32(base + 2 * (size_t)v.h[c], c0[c]);
    atomic_add_f32(base + 2 * (size_t)v.h[c] + 1, c1[c]);
  }
}

__global__ __launch_bounds__(256) void sh_fwd_kernel(const float* __restrict__ d, int64_t n,
                                                     float* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  float o[16];
  sh16(d[3 * p], d[3 * p + 1], d[3 * p + 2], o);
  float4* dst = reinterpret_cast<float4*>(out + 16 * p);
#pragma unroll
  for (int i = 0; i < 4; ++i) dst[i] = make_float4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

static int32_t check_grid(const hn_grid* g) {
  if (!g) return HN_E_NULL;
  if (g->n_levels < 1 || g->n_levels > HN_MAX_LEVELS) return HN_E_SHAPE;
  if (g->n_features != 2) return HN_E_SHAPE;
  if (g->log2_hashmap_size < 1 || g->log2_hashmap_size > 24) return HN_E_SHAPE;
  return HN_OK;
}

}  // namespace hn

using namespace hn;

extern "C" int32_t hn_encode_fwd(const hn_grid* g, const float* x, int64_t n, const float* table,
                                 float* feat, uint8_t* keep_mask, void* stream) {
  int32_t st = check_grid(g);
  if (st) return st;
  if (n < 0) return HN_E_SHAPE;
  if (n == 0) return HN_OK;
  if (!x || !table || !feat) return HN_E_NULL;
  const int64_t total = n * g->n_levels;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(encode_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     make_grid_args(*g), x, n, table, feat, keep_mask);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_encode_bwd(const hn_grid* g, const float* x, int64_t n, const float* dfeat,
                                 float* dtable, void* stream) {
  int32_t st = check_grid(g);
  if (st) return st;
  if (n < 0) return HN_E_SHAPE;
  if (n == 0) return HN_OK;
  if (!x || !dfeat || !dtable) return HN_E_NULL;
  const int64_t total = n * g->n_levels;
  const int64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(encode_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     make_grid_args(*g), x, n, dfeat, dtable);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_sh_fwd(const float* dirs, int64_t n, float* out, void* stream) {
  if (n < 0) return HN_E_SHAPE;
  if (n == 0) return HN_OK;
  if (!dirs || !out) return HN_E_NULL;
  hipLaunchKernelGGL(sh_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, dirs, n, out);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_abi_version(void) { return HN_ABI_VERSION; }

extern "C" const char* hn_status_string(int32_t s) {
  switch (s) {
    case HN_OK: return "ok";
    case HN_E_NULL: return "required pointer is NULL";
    case HN_E_SHAPE: return "unsupported shape/configuration";
    case HN_E_WORKSPACE: return "workspace too small";
    default: break;
  }
  if (s >= HN_E_HIP) return hipGetErrorString((hipError_t)(s - HN_E_HIP));
  return "unknown status";
}
