// hn_mlp.hip -- standalone NeRFSmall forward/backward (models.py:151-174)
// on f32 MFMA.  The fused render kernels use the same device code (hn_mlp.h).
#include "hn_mlp.h"

namespace hn {

__global__ __launch_bounds__(256) void mlp_pack_kernel(hn_mlp w, float* __restrict__ packed) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < G_END) packed[idx] = pack_value(w, idx);
}

// Load one point's inputs in tile layout from x[n][48] = [feat32 | sh16].
HN_DEV void load_x_tile(const float* __restrict__ x, int64_t q, bool valid, int lane, f32x16& feat,
                        float sh8[8], float sh_pt[16]) {
  const int h = lane >> 5;
  const float* row = x + q * 48;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float4 v = valid ? *reinterpret_cast<const float4*>(row + 8 * t + 4 * h) : make_float4(0, 0, 0, 0);
    feat[4 * t] = v.x; feat[4 * t + 1] = v.y; feat[4 * t + 2] = v.z; feat[4 * t + 3] = v.w;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float4 v = valid ? *reinterpret_cast<const float4*>(row + 32 + 4 * t) : make_float4(0, 0, 0, 0);
    sh_pt[4 * t] = v.x; sh_pt[4 * t + 1] = v.y; sh_pt[4 * t + 2] = v.z; sh_pt[4 * t + 3] = v.w;
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) sh8[s] = h ? sh_pt[2 * s + 1] : sh_pt[2 * s];
}

__global__ __launch_bounds__(256) void mlp_fwd_kernel(const float* __restrict__ P,
                                                      const float* __restrict__ x, int64_t n,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t q = tile * 32 + (lane & 31);
  const bool valid = q < n;
  f32x16 feat;
  float sh8[8], sh_pt[16];
  load_x_tile(x, q, valid, lane, feat, sh8, sh_pt);
  MlpAct a;
  f32x16 c2;
  mlp_fwd_tile(P, feat, sh8, a, c2, lane);
  if (valid && lane < 32)
    *reinterpret_cast<float4*>(out + 4 * q) = make_float4(c2[0], c2[1], c2[2], a.s1[0]);
}

constexpr int kBwdWaves = 4;

__global__ __launch_bounds__(256, 2) void mlp_bwd_kernel(const float* __restrict__ P,
                                                      const float* __restrict__ x,
                                                      const float* __restrict__ dout, int64_t n,
                                                      float* __restrict__ dx, hn_mlp_grad dw) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Wacc = smem;                                   // [9344]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float* T = smem + W_END + wave * 2 * kTBuf;
  for (int i = threadIdx.x; i < W_END; i += blockDim.x) Wacc[i] = 0.f;
  __syncthreads();
  const int h = lane >> 5, p = lane & 31;
  const int64_t n_tiles = (n + 31) / 32;
  for (int64_t tile = (int64_t)blockIdx.x * kBwdWaves + wave; tile < n_tiles;
       tile += (int64_t)gridDim.x * kBwdWaves) {
    const int64_t q = tile * 32 + p;
    const bool valid = q < n;
    const float* Pt = opaque_ptr(P);
    f32x16 feat;
    float sh8[8], sh_pt[16];
    load_x_tile(x, q, valid, lane, feat, sh8, sh_pt);
    MlpAct a;
    f32x16 c2;
    mlp_fwd_tile(Pt, feat, sh8, a, c2, lane);
    const float4 g = valid ? *reinterpret_cast<const float4*>(dout + 4 * q) : make_float4(0, 0, 0, 0);
    const float dy2[2] = {h ? g.y : g.x, h ? 0.f : g.z};
    const float rgbg[3] = {g.x, g.y, g.z};
    float shx8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) shx8[j] = h ? sh_pt[8 + j] : sh_pt[j];
    f32x16 dfeat, dsh;
    mlp_bwd_tile(Pt, feat, shx8, a, dy2, g.w, rgbg, T, Wacc, dfeat,
                 dx != nullptr ? &dsh : nullptr, lane);
    if (dx != nullptr && valid) {
      float* row = dx + q * 48;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        *reinterpret_cast<float4*>(row + 8 * t + 4 * h) =
            make_float4(dfeat[4 * t], dfeat[4 * t + 1], dfeat[4 * t + 2], dfeat[4 * t + 3]);
#pragma unroll
      for (int t = 0; t < 2; ++t)   // regs 0..7 hold sh rows row_of(r,h) < 16
        *reinterpret_cast<float4*>(row + 32 + 8 * t + 4 * h) =
            make_float4(dsh[4 * t], dsh[4 * t + 1], dsh[4 * t + 2], dsh[4 * t + 3]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < W_END; i += blockDim.x) {
    const float v = Wacc[i];
    float* dst;
    if (i < W_S1) dst = dw.sigma0 + i;
    else if (i < W_C0) dst = dw.sigma1 + (i - W_S1);
    else if (i < W_C1) dst = dw.color0 + (i - W_C0);
    else if (i < W_C2) dst = dw.color1 + (i - W_C1);
    else dst = dw.color2 + (i - W_C2);
    atomic_add_f32(dst, v);
  }
}

}  // namespace hn

using namespace hn;

static bool mlp_ok(const hn_mlp* w) {
  return w && w->sigma0 && w->sigma1 && w->color0 && w->color1 && w->color2;
}

extern "C" size_t hn_mlp_workspace_bytes(void) { return (size_t)G_END * sizeof(float); }

// Both networks of the renderer in one launch (blockIdx.y = network).
__global__ __launch_bounds__(256) void mlp_pack2_kernel(hn_mlp w0, float* __restrict__ p0, hn_mlp w1,
                                                        float* __restrict__ p1) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < G_END) {
    if (blockIdx.y == 0) p0[idx] = pack_value(w0, idx);
    else p1[idx] = pack_value(w1, idx);
  }
}

int32_t hn::mlp_pack2_launch(const hn_mlp* w0, float* p0, const hn_mlp* w1, float* p1, hipStream_t s) {
  hipLaunchKernelGGL(mlp_pack2_kernel, dim3((G_END + 255) / 256, 2), dim3(256), 0, s, *w0, p0, *w1, p1);
  return hip_status(hipGetLastError());
}

int32_t hn::mlp_pack_launch(const hn_mlp* w, float* packed, hipStream_t s) {
  hipLaunchKernelGGL(mlp_pack_kernel, dim3((G_END + 255) / 256), dim3(256), 0, s, *w, packed);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_mlp_fwd(const hn_mlp* w, const float* x, int64_t n, float* out,
                              void* workspace, size_t ws_bytes, void* stream) {
  if (!mlp_ok(w)) return HN_E_NULL;
  if (n < 0) return HN_E_SHAPE;
  if (n == 0) return HN_OK;
  if (!x || !out || !workspace) return HN_E_NULL;
  if (ws_bytes < hn_mlp_workspace_bytes()) return HN_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* P = (float*)workspace;
  int32_t st = mlp_pack_launch(w, P, s);
  if (st) return st;
  const int64_t tiles = (n + 31) / 32;
  const int64_t blocks = (tiles + 3) / 4;
  hipLaunchKernelGGL(mlp_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, P, x, n, out);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_mlp_bwd(const hn_mlp* w, const float* x, const float* dout, int64_t n,
                              float* dx, const hn_mlp_grad* dw, void* workspace, size_t ws_bytes,
                              void* stream) {
  if (!mlp_ok(w) || !dw) return HN_E_NULL;
  if (!dw->sigma0 || !dw->sigma1 || !dw->color0 || !dw->color1 || !dw->color2) return HN_E_NULL;
  if (n < 0) return HN_E_SHAPE;
  if (n == 0) return HN_OK;
  if (!x || !dout || !workspace) return HN_E_NULL;
  if (ws_bytes < hn_mlp_workspace_bytes()) return HN_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* P = (float*)workspace;
  int32_t st = mlp_pack_launch(w, P, s);
  if (st) return st;
  const int64_t tiles = (n + 31) / 32;
  int64_t blocks = (tiles + kBwdWaves - 1) / kBwdWaves;
  if (blocks > 512) blocks = 512;
  const size_t lds = (size_t)(W_END + kBwdWaves * 2 * kTBuf) * sizeof(float);
  hipLaunchKernelGGL(mlp_bwd_kernel, dim3((unsigned)blocks), dim3(256), lds, s, P, x, dout, n, dx, *dw);
  return hip_status(hipGetLastError());
}
