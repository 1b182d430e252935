// hn_train.hip -- the training-step driver pieces around the fused renderer
// (run_nerf.py:576-636), so one step is a handful of launches:
//   * hn_sample_rays: N_rand distinct pixels of one image (without
//     replacement), their rays (ray_util.py:62-80) packed as the ray batch
//     render() builds (run_nerf_helpers.py:355-368), and their target colours;
//   * hn_loss_fwd / hn_loss_bwd: the loss of run_nerf.py:612-636 (with the
//     data-parallel scaling of train.dp_loss) and its input gradients in
//     torch autograd's op order, instead of ~25 tiny eager kernels.
#include "hn_common.h"
#include "hn_loss.h"

namespace hn {

// ---------------------------------------------------------------------------
// Pixel sampling without replacement: a keyed 4-round Feistel permutation of
// [0, 2^k) (k even, 2^k >= window size M), restricted to [0, M) by cycle
// walking, is a bijection of [0, M); sample i is perm(i), so the n samples
// are distinct for any seed.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sample_rays_kernel(hn_ray_sampler s, const float* __restrict__ image,
                                                          const float* __restrict__ c2w, int64_t n,
                                                          int half, float* __restrict__ rays,
                                                          float* __restrict__ target) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t M = (uint32_t)s.crop_h * (uint32_t)s.crop_w;
  uint32_t x = (uint32_t)i;
  do {
    x = feistel(x, half, s.seed);
  } while (x >= M);
  const int py = s.crop_y0 + (int)(x / (uint32_t)s.crop_w);
  const int px = s.crop_x0 + (int)(x % (uint32_t)s.crop_w);
  // dirs = [(i - cx) / fx, -(j - cy) / fy, -1]; rays_d = sum(dirs * c2w[:3,:3], -1)
  const float d0 = ((float)px - s.cx) / s.fx;
  const float d1 = -(((float)py - s.cy) / s.fy);
  const float d2 = -1.f;
  float* out = rays + 11 * i;
  float d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    d[a] = d0 * c2w[4 * a] + d1 * c2w[4 * a + 1] + d2 * c2w[4 * a + 2];
    out[a] = c2w[4 * a + 3];
    out[3 + a] = d[a];
  }
  out[6] = s.near;
  out[7] = s.far;
  const float nrm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
#pragma unroll
  for (int a = 0; a < 3; ++a) out[8 + a] = d[a] / nrm;
  const float* px3 = image + 3 * ((size_t)py * s.W + px);
#pragma unroll
  for (int a = 0; a < 3; ++a) target[3 * i + a] = px3[a];
}

// ---------------------------------------------------------------------------
// The same draw in Morton order of its pixels (window-relative row, column):
// pixel x is drawn iff perm^-1(x) < n, so walking the Morton indices of the
// window and compacting the drawn ones lists the draw's set in that order with
// no sort.  Two launches: per-block counts, then prefix + block scan + emit.
// ---------------------------------------------------------------------------
constexpr int kMortonThreads = 1024;
HN_DEV uint32_t compact_bits16(uint32_t v) {
  v &= 0x55555555u;
  v = (v | (v >> 1)) & 0x33333333u;
  v = (v | (v >> 2)) & 0x0f0f0f0fu;
  v = (v | (v >> 4)) & 0x00ff00ffu;
  v = (v | (v >> 8)) & 0x0000ffffu;
  return v;
}
// Morton index m -> drawn pixel (window-relative linear index) or ~0u
HN_DEV uint32_t morton_drawn(const hn_ray_sampler& s, int half, int64_t n, uint32_t m) {
  const uint32_t row = compact_bits16(m >> 1), col = compact_bits16(m);
  if (row >= (uint32_t)s.crop_h || col >= (uint32_t)s.crop_w) return ~0u;
  const uint32_t M = (uint32_t)s.crop_h * (uint32_t)s.crop_w;
  const uint32_t x = row * (uint32_t)s.crop_w + col;
  uint32_t y = x;
  do {   // inverse of the cycle-walked permutation
    y = feistel_inv(y, half, s.seed);
  } while (y >= M);
  return (int64_t)y < n ? x : ~0u;
}

// torch.rand on the CUDA/HIP default generator, restated (ATen's
// distribution_elementwise_grid_stride_kernel with hiprand's Philox4x32-10,
// unroll 4): element li of a draw comes from thread idx = li % T of torch's
// launch (T threads), its call it = li / (4T) and component (li / T) % 4 --
// Philox of counter (offset / 4 + it, subsequence idx) under key = seed,
// mapped by rocrand's 2^-32 + v * 2^-32 to (0, 1], and 1 -> 0 (uniform_'s
// bound reversal).
struct UniK {
  uint32_t key[2];
  int n;
  int64_t start[HN_UNIFORM_MAX_DRAWS + 1];   // element prefix of the draws
  hn_uniform_draw d[HN_UNIFORM_MAX_DRAWS];
};
HN_DEV uint32_t philox_component(uint64_t ctr, uint64_t sub, uint32_t k0, uint32_t k1, int comp) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = (uint32_t)sub, c3 = (uint32_t)(sub >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return comp == 0 ? c0 : comp == 1 ? c1 : comp == 2 ? c2 : c3;
}
// global element g of the UniK's draws
HN_DEV void uniform_elem(const UniK& u, int64_t g) {
  int j = 0;
  while (j + 1 < u.n && g >= u.start[j + 1]) ++j;
  const hn_uniform_draw& d = u.d[j];
  const int64_t li = g - u.start[j];
  const uint64_t T = (uint64_t)d.threads, idx = (uint64_t)li % T, rem = (uint64_t)li / T;
  const uint32_t v = philox_component(d.offset / 4 + (rem >> 2), idx, u.key[0], u.key[1], (int)(rem & 3));
  const float x = 0x1p-32f + (float)v * 0x1p-32f;
  d.out[li] = x == 1.f ? 0.f : x;
}
__global__ __launch_bounds__(1024) void uniform_kernel(UniK u) {
  const int64_t g = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  if (g < u.start[u.n]) uniform_elem(u, g);
}

__global__ __launch_bounds__(kMortonThreads) void morton_count_kernel(hn_ray_sampler s, int half, int64_t n,
                                                                      uint32_t n_idx, int* __restrict__ counts,
                                                                      UniK u, unsigned count_blocks) {
  if (blockIdx.x >= count_blocks) {   // the batch's uniform draws, beside the counts
    const int64_t g = (int64_t)(blockIdx.x - count_blocks) * kMortonThreads + threadIdx.x;
    if (g < u.start[u.n]) uniform_elem(u, g);
    return;
  }
  const uint32_t m = blockIdx.x * kMortonThreads + threadIdx.x;
  const bool sel = m < n_idx && morton_drawn(s, half, n, m) != ~0u;
  const int c = __syncthreads_count(sel);
  if (threadIdx.x == 0) counts[blockIdx.x] = c;
}

HN_DEV void emit_ray(const hn_ray_sampler& s, const float* __restrict__ image, const float* __restrict__ c2w,
                     uint32_t x, int64_t r, float* __restrict__ rays, float* __restrict__ target) {
  const int py = s.crop_y0 + (int)(x / (uint32_t)s.crop_w);
  const int px = s.crop_x0 + (int)(x % (uint32_t)s.crop_w);
  // dirs = [(i - cx) / fx, -(j - cy) / fy, -1]; rays_d = sum(dirs * c2w[:3,:3], -1)
  const float d0 = ((float)px - s.cx) / s.fx;
  const float d1 = -(((float)py - s.cy) / s.fy);
  const float d2 = -1.f;
  float* out = rays + 11 * r;
  float d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    d[a] = d0 * c2w[4 * a] + d1 * c2w[4 * a + 1] + d2 * c2w[4 * a + 2];
    out[a] = c2w[4 * a + 3];
    out[3 + a] = d[a];
  }
  out[6] = s.near;
  out[7] = s.far;
  const float nrm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
#pragma unroll
  for (int a = 0; a < 3; ++a) out[8 + a] = d[a] / nrm;
  const float* px3 = image + 3 * ((size_t)py * s.W + px);
#pragma unroll
  for (int a = 0; a < 3; ++a) target[3 * r + a] = px3[a];
}

__global__ __launch_bounds__(kMortonThreads) void morton_emit_kernel(hn_ray_sampler s, const float* __restrict__ image,
                                                                     const float* __restrict__ c2w, int half,
                                                                     int64_t n, uint32_t n_idx,
                                                                     const int* __restrict__ counts,
                                                                     float* __restrict__ rays,
                                                                     float* __restrict__ target) {
  __shared__ int part[kMortonThreads / 64 + 1];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // rays drawn by the earlier blocks
  uint32_t pre = 0;
  for (uint32_t b = tid; b < blockIdx.x; b += kMortonThreads) pre += (uint32_t)counts[b];
  pre = wave_sum(pre);
  if (lane == 0) part[wave] = (int)pre;
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int w = 0; w < kMortonThreads / 64; ++w) base += part[w];
  __syncthreads();
  const uint32_t m = blockIdx.x * kMortonThreads + tid;
  const uint32_t x = m < n_idx ? morton_drawn(s, half, n, m) : ~0u;
  const bool sel = x != ~0u;
  const uint64_t bal = __ballot(sel);
  if (lane == 0) part[wave] = __popcll(bal);
  __syncthreads();
  int off = base;
  for (int w = 0; w < wave; ++w) off += part[w];
  if (!sel) return;
  const int64_t r = off + __popcll(bal & ((1ull << lane) - 1ull));
  emit_ray(s, image, c2w, x, r, rays, target);
}

// ---------------------------------------------------------------------------
// use_batching ray pool (run_nerf.py:505-521, 544-555).  The reference
// materialises rays_rgb = [every training pixel][ro, rd, rgb] (rays from
// get_rays_np, ray_util.py:82-93: float64 arithmetic under numpy 2, then
// .astype(float32)), shuffles it once and again after every epoch, and takes
// consecutive N_rand slices.  Here the shuffle is a keyed bijection of the
// pool index (cycle-walked Feistel, as the per-image sampler), so nothing is
// materialised: pool position q -> pixel perm(q) = (image, row, column) ->
// its ray, computed in float64 and rounded once, and its target colour.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sample_pool_kernel(hn_ray_pool p, const float* __restrict__ images,
                                                          const float* __restrict__ poses,
                                                          const int32_t* __restrict__ ids, int64_t start, int64_t n,
                                                          int half, float* __restrict__ rays,
                                                          float* __restrict__ target) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t hw = (uint32_t)p.H * (uint32_t)p.W;
  const uint32_t N = (uint32_t)p.n_images * hw;
  uint32_t x = (uint32_t)(start + i);
  do {
    x = feistel(x, half, p.seed);
  } while (x >= N);
  const int img = ids[x / hw];
  const uint32_t pix = x % hw;
  const int py = (int)(pix / (uint32_t)p.W), px = (int)(pix % (uint32_t)p.W);
  const float* c = poses + (size_t)img * p.pose_stride;
  // dirs = [(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -1] (float64: K is)
  const double d0 = ((double)px - p.cx) / p.fx;
  const double d1 = -((double)py - p.cy) / p.fy;
  const double d2 = -1.0;
  float* out = rays + 11 * i;
  float d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {   // np.sum(dirs[..., None, :] * c2w[:3, :3], -1): ((p0 + p1) + p2)
    d[a] = (float)((d0 * (double)c[4 * a] + d1 * (double)c[4 * a + 1]) + d2 * (double)c[4 * a + 2]);
    out[a] = c[4 * a + 3];
    out[3 + a] = d[a];
  }
  out[6] = p.near;
  out[7] = p.far;
  const float nrm = sqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);   // render(): viewdirs (:350)
#pragma unroll
  for (int a = 0; a < 3; ++a) out[8 + a] = d[a] / nrm;
  const float* px3 = images + 3 * (((size_t)img * p.H + py) * p.W + px);
#pragma unroll
  for (int a = 0; a < 3; ++a) target[3 * i + a] = px3[a];
}

// ---------------------------------------------------------------------------
// Blender image preparation: load/load_blender.py:63 (uint8 PNG / 255. in
// float64, .astype(float32)), :78-86 (half_res: cv2.resize INTER_AREA to H/2 x
// W/2, stored into a float64 array) and run_nerf.py:259-262 (white_bkgd:
// rgb * a + (1 - a), float32 arithmetic at full resolution, float64 after
// half_res; the trainer's torch.Tensor rounds to float32).  INTER_AREA at an
// exact factor 2 is the 2 x 2 box mean; OpenCV's float path sums
// ((top-left + top-right) + (bottom-left + bottom-right)) * 0.25 (cv2 is not in
// the image: that order is restated).  One thread per output pixel.
// ---------------------------------------------------------------------------
HN_DEV float u8_unit(uint8_t v) { return (float)((double)v / 255.0); }

__global__ __launch_bounds__(256) void blender_images_kernel(const uint8_t* __restrict__ rgba, int64_t n_px, int H,
                                                             int W, int half, int mode, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_px) return;
  const int Ho = half ? H / 2 : H, Wo = half ? W / 2 : W;
  const int64_t img = t / ((int64_t)Ho * Wo);
  const int r = (int)(t / Wo % Ho), col = (int)(t % Wo);
  float v[4];
  if (!half) {
    const uint8_t* s = rgba + 4 * ((img * H + r) * (int64_t)W + col);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = u8_unit(s[c]);
  } else {
    const uint8_t* s0 = rgba + 4 * ((img * H + 2 * r) * (int64_t)W + 2 * col);
    const uint8_t* s1 = s0 + 4 * (int64_t)W;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      v[c] = ((u8_unit(s0[c]) + u8_unit(s0[4 + c])) + (u8_unit(s1[c]) + u8_unit(s1[4 + c]))) * 0.25f;
  }
  if (mode == 0) {   // RGBA as load_blender_data returns it
#pragma unroll
    for (int c = 0; c < 4; ++c) out[4 * t + c] = v[c];
    return;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float o = v[c];
    if (mode == 1) {
      o = half ? (float)((double)v[c] * (double)v[3] + (1.0 - (double)v[3])) : v[c] * v[3] + (1.f - v[3]);
    }
    out[3 * t + c] = o;
  }
}

// ---------------------------------------------------------------------------
// Loss.  Forward: one workgroup, fp64 accumulation of the reductions (the
// value is reported, its gradient does not depend on the summation order).
// ---------------------------------------------------------------------------
constexpr int kLossThreads = 1024;

__global__ __launch_bounds__(kLossThreads) void loss_fwd_kernel(
    const float* __restrict__ rgb, const float* __restrict__ rgb0, const float* __restrict__ target,
    const float* __restrict__ sp, const float* __restrict__ sp0, int64_t n, const float* __restrict__ tv,
    int n_tv, float world, float sparse_w, float tv_w, float* __restrict__ out) {
  loss_fwd_block<kLossThreads>(rgb, rgb0, target, sp, sp0, n, tv, n_tv, world, sparse_w, tv_w, out);
}

// Backward, op for op as autograd evaluates the eager expression:
//   (mse + mse0) / world   -> g / world (DivBackward)
//   mean over 3n            -> (.) / 3n  (MeanBackward: expand, divide by numel)
//   (x - t) ** 2            -> (.) * (2 * (x - t))  (PowBackward)
//   sparse_w * sum(sp)      -> g * sparse_w;   tv_w * sum(tv) -> g * tv_w
HN_DEV void loss_bwd_elem(
    int64_t j, const float* __restrict__ rgb, const float* __restrict__ rgb0, const float* __restrict__ target,
    int64_t n, int n_tv, float world, float sparse_w, float tv_w, const float* __restrict__ g_loss,
    float* __restrict__ g_rgb, float* __restrict__ g_rgb0, float* __restrict__ g_sp, float* __restrict__ g_sp0,
    float* __restrict__ g_tv) {
  const float g = *g_loss;
  const float gm = (g / world) / (float)(3 * n);
  if (j < 3 * n) {
    g_rgb[j] = gm * (2.f * (rgb[j] - target[j]));
    if (rgb0) g_rgb0[j] = gm * (2.f * (rgb0[j] - target[j]));
  }
  if (j < n) {
    if (g_sp) g_sp[j] = g * sparse_w;
    if (g_sp0) g_sp0[j] = g * sparse_w;
  }
  if (g_tv && j < n_tv) g_tv[j] = g * tv_w;
}
__global__ __launch_bounds__(256) void loss_bwd_kernel(
    const float* __restrict__ rgb, const float* __restrict__ rgb0, const float* __restrict__ target, int64_t n,
    int n_tv, float world, float sparse_w, float tv_w, const float* __restrict__ g_loss,
    float* __restrict__ g_rgb, float* __restrict__ g_rgb0, float* __restrict__ g_sp, float* __restrict__ g_sp0,
    float* __restrict__ g_tv) {
  loss_bwd_elem((int64_t)blockIdx.x * blockDim.x + threadIdx.x, rgb, rgb0, target, n, n_tv, world, sparse_w, tv_w,
                g_loss, g_rgb, g_rgb0, g_sp, g_sp0, g_tv);
}
// Both in one launch (the trainer's step): workgroup 0 reduces the loss, the
// others write the gradients -- the backward does not depend on the loss
// value, so the two run side by side; results bitwise those of the two kernels.
__global__ __launch_bounds__(kLossThreads) void loss_fwd_bwd_kernel(
    const float* __restrict__ rgb, const float* __restrict__ rgb0, const float* __restrict__ target,
    const float* __restrict__ sp, const float* __restrict__ sp0, int64_t n, const float* __restrict__ tv,
    int n_tv, float world, float sparse_w, float tv_w, float* __restrict__ out, const float* __restrict__ g_loss,
    float* __restrict__ g_rgb, float* __restrict__ g_rgb0, float* __restrict__ g_sp, float* __restrict__ g_sp0,
    float* __restrict__ g_tv) {
  if (blockIdx.x == 0)
    loss_fwd_block<kLossThreads>(rgb, rgb0, target, sp, sp0, n, tv, n_tv, world, sparse_w, tv_w, out);
  else
    loss_bwd_elem((int64_t)(blockIdx.x - 1) * kLossThreads + threadIdx.x, rgb, rgb0, target, n, n_tv, world,
                  sparse_w, tv_w, g_loss, g_rgb, g_rgb0, g_sp, g_sp0, g_tv);
}

}  // namespace hn

using namespace hn;

extern "C" int32_t hn_sample_rays(const hn_ray_sampler* s, const float* image, const float* c2w, int64_t n_rays,
                                  float* rays, float* target, void* stream) {
  if (!s) return HN_E_NULL;
  if (n_rays < 0) return HN_E_SHAPE;
  if (n_rays == 0) return HN_OK;
  if (!image || !c2w || !rays || !target) return HN_E_NULL;
  if (s->H <= 0 || s->W <= 0 || s->crop_h <= 0 || s->crop_w <= 0 || s->crop_y0 < 0 || s->crop_x0 < 0 ||
      s->crop_y0 + s->crop_h > s->H || s->crop_x0 + s->crop_w > s->W)
    return HN_E_SHAPE;
  const uint64_t M = (uint64_t)s->crop_h * (uint64_t)s->crop_w;
  if ((uint64_t)n_rays > M || M > (1ull << 30)) return HN_E_SHAPE;   // without replacement
  int bits = 2;
  while ((1ull << bits) < M) bits += 2;
  const unsigned blocks = (unsigned)((n_rays + 255) / 256);
  hipLaunchKernelGGL(sample_rays_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *s, image, c2w, n_rays,
                     bits / 2, rays, target);
  return hip_status(hipGetLastError());
}

// Morton-window geometry: 4^k indices cover the window, 1024 per block.
static bool morton_geometry(const hn_ray_sampler* s, uint32_t& n_idx, unsigned& blocks) {
  if (s->crop_h <= 0 || s->crop_w <= 0 || s->crop_h > HN_SAMPLER_MORTON_MAX || s->crop_w > HN_SAMPLER_MORTON_MAX)
    return false;
  int k = 0;
  while ((1 << k) < s->crop_h || (1 << k) < s->crop_w) ++k;
  n_idx = 1u << (2 * k);
  blocks = (unsigned)((n_idx + kMortonThreads - 1) / kMortonThreads);
  return true;
}

extern "C" size_t hn_sample_rays_morton_workspace_bytes(const hn_ray_sampler* s) {
  uint32_t n_idx;
  unsigned blocks;
  if (!s || !morton_geometry(s, n_idx, blocks)) return 0;
  return (size_t)blocks * sizeof(int);
}

static int32_t make_uni(uint64_t seed, const hn_uniform_draw* draws, int32_t n_draws, UniK& u) {
  if (n_draws < 0 || n_draws > HN_UNIFORM_MAX_DRAWS) return HN_E_SHAPE;
  if (n_draws && !draws) return HN_E_NULL;
  u.key[0] = (uint32_t)seed;
  u.key[1] = (uint32_t)(seed >> 32);
  u.n = n_draws;
  u.start[0] = 0;
  for (int j = 0; j < n_draws; ++j) {
    const hn_uniform_draw& d = draws[j];
    if (d.numel < 0 || (d.numel && d.threads <= 0) || (d.offset & 3)) return HN_E_SHAPE;
    if (d.numel && !d.out) return HN_E_NULL;
    u.d[j] = d;
    u.start[j + 1] = u.start[j] + d.numel;
  }
  return HN_OK;
}

extern "C" int32_t hn_uniform_philox(uint64_t seed, const hn_uniform_draw* draws, int32_t n_draws, void* stream) {
  UniK u;
  const int32_t st = make_uni(seed, draws, n_draws, u);
  if (st) return st;
  const int64_t total = u.start[u.n];
  if (total == 0) return HN_OK;
  hipLaunchKernelGGL(uniform_kernel, dim3((unsigned)((total + 1023) / 1024)), dim3(1024), 0, (hipStream_t)stream, u);
  return hip_status(hipGetLastError());
}

static int32_t sample_morton(const hn_ray_sampler* s, const float* image, const float* c2w, int64_t n_rays,
                             float* rays, float* target, void* workspace, size_t ws_bytes, const UniK& u,
                             hipStream_t stream);

extern "C" int32_t hn_sample_rays_morton(const hn_ray_sampler* s, const float* image, const float* c2w,
                                         int64_t n_rays, float* rays, float* target, void* workspace,
                                         size_t ws_bytes, void* stream) {
  UniK u;
  make_uni(0, nullptr, 0, u);
  return sample_morton(s, image, c2w, n_rays, rays, target, workspace, ws_bytes, u, (hipStream_t)stream);
}

extern "C" int32_t hn_sample_batch_morton(const hn_ray_sampler* s, const float* image, const float* c2w,
                                          int64_t n_rays, float* rays, float* target, void* workspace,
                                          size_t ws_bytes, uint64_t seed, const hn_uniform_draw* draws,
                                          int32_t n_draws, void* stream) {
  UniK u;
  const int32_t st = make_uni(seed, draws, n_draws, u);
  if (st) return st;
  return sample_morton(s, image, c2w, n_rays, rays, target, workspace, ws_bytes, u, (hipStream_t)stream);
}

static int32_t sample_morton(const hn_ray_sampler* s, const float* image, const float* c2w, int64_t n_rays,
                             float* rays, float* target, void* workspace, size_t ws_bytes, const UniK& u,
                             hipStream_t stream) {
  if (!s) return HN_E_NULL;
  if (n_rays < 0) return HN_E_SHAPE;
  if (n_rays == 0) return HN_OK;
  if (!image || !c2w || !rays || !target) return HN_E_NULL;
  if (s->H <= 0 || s->W <= 0 || s->crop_h <= 0 || s->crop_w <= 0 || s->crop_y0 < 0 || s->crop_x0 < 0 ||
      s->crop_y0 + s->crop_h > s->H || s->crop_x0 + s->crop_w > s->W)
    return HN_E_SHAPE;
  uint32_t n_idx;
  unsigned blocks;
  if (!morton_geometry(s, n_idx, blocks)) return HN_E_SHAPE;
  const uint64_t M = (uint64_t)s->crop_h * (uint64_t)s->crop_w;
  if ((uint64_t)n_rays > M) return HN_E_SHAPE;   // without replacement
  if (!workspace) return HN_E_NULL;
  if (ws_bytes < (size_t)blocks * sizeof(int)) return HN_E_WORKSPACE;
  int bits = 2;
  while ((1ull << bits) < M) bits += 2;
  int* counts = static_cast<int*>(workspace);
  const unsigned ublocks = (unsigned)((u.start[u.n] + kMortonThreads - 1) / kMortonThreads);
  hipLaunchKernelGGL(morton_count_kernel, dim3(blocks + ublocks), dim3(kMortonThreads), 0, (hipStream_t)stream, *s,
                     bits / 2, n_rays, n_idx, counts, u, blocks);
  hipLaunchKernelGGL(morton_emit_kernel, dim3(blocks), dim3(kMortonThreads), 0, (hipStream_t)stream, *s, image, c2w,
                     bits / 2, n_rays, n_idx, counts, rays, target);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_loss_fwd(const float* rgb, const float* rgb0, const float* target, const float* sp,
                               const float* sp0, int64_t n_rays, const float* tv, int32_t n_tv, float world,
                               float sparse_w, float tv_w, float* out, void* stream) {
  if (n_rays <= 0 || n_tv < 0) return HN_E_SHAPE;
  if (!rgb || !target || !sp || !out) return HN_E_NULL;
  if ((rgb0 == nullptr) != (sp0 == nullptr)) return HN_E_NULL;
  hipLaunchKernelGGL(loss_fwd_kernel, dim3(1), dim3(kLossThreads), 0, (hipStream_t)stream, rgb, rgb0, target, sp,
                     sp0, n_rays, tv, n_tv, world, sparse_w, tv_w, out);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_loss_bwd(const float* rgb, const float* rgb0, const float* target, int64_t n_rays,
                               int32_t n_tv, float world, float sparse_w, float tv_w, const float* g_loss,
                               float* g_rgb, float* g_rgb0, float* g_sp, float* g_sp0, float* g_tv,
                               void* stream) {
  if (n_rays <= 0 || n_tv < 0) return HN_E_SHAPE;
  if (!rgb || !target || !g_loss || !g_rgb) return HN_E_NULL;
  if ((rgb0 == nullptr) != (g_rgb0 == nullptr)) return HN_E_NULL;
  const int64_t m = 3 * n_rays > n_tv ? 3 * n_rays : n_tv;
  const unsigned blocks = (unsigned)((m + 255) / 256);
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, rgb, rgb0, target, n_rays,
                     n_tv, world, sparse_w, tv_w, g_loss, g_rgb, g_rgb0, g_sp, g_sp0, g_tv);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_loss_fwd_bwd(const float* rgb, const float* rgb0, const float* target, const float* sp,
                                   const float* sp0, int64_t n_rays, const float* tv, int32_t n_tv, float world,
                                   float sparse_w, float tv_w, float* out, const float* g_loss, float* g_rgb,
                                   float* g_rgb0, float* g_sp, float* g_sp0, float* g_tv, void* stream) {
  if (n_rays <= 0 || n_tv < 0) return HN_E_SHAPE;
  if (!rgb || !target || !sp || !out || !g_loss || !g_rgb) return HN_E_NULL;
  if ((rgb0 == nullptr) != (sp0 == nullptr) || (rgb0 == nullptr) != (g_rgb0 == nullptr)) return HN_E_NULL;
  const int64_t m = 3 * n_rays > n_tv ? 3 * n_rays : n_tv;
  const unsigned blocks = 1u + (unsigned)((m + kLossThreads - 1) / kLossThreads);
  hipLaunchKernelGGL(loss_fwd_bwd_kernel, dim3(blocks), dim3(kLossThreads), 0, (hipStream_t)stream, rgb, rgb0,
                     target, sp, sp0, n_rays, tv, n_tv, world, sparse_w, tv_w, out, g_loss, g_rgb, g_rgb0, g_sp,
                     g_sp0, g_tv);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_sample_pool(const hn_ray_pool* p, const float* images, const float* poses,
                                  const int32_t* image_ids, int64_t start, int64_t n_rays, float* rays, float* target,
                                  void* stream) {
  if (!p) return HN_E_NULL;
  if (n_rays < 0 || start < 0) return HN_E_SHAPE;
  if (n_rays == 0) return HN_OK;
  if (!images || !poses || !image_ids || !rays || !target) return HN_E_NULL;
  if (p->n_images <= 0 || p->H <= 0 || p->W <= 0 || p->pose_stride < 12) return HN_E_SHAPE;
  const uint64_t N = (uint64_t)p->n_images * (uint64_t)p->H * (uint64_t)p->W;
  if (N > (1ull << 30) || (uint64_t)start + (uint64_t)n_rays > N) return HN_E_SHAPE;   // one epoch's positions
  int bits = 2;
  while ((1ull << bits) < N) bits += 2;
  const unsigned blocks = (unsigned)((n_rays + 255) / 256);
  hipLaunchKernelGGL(sample_pool_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p, images, poses,
                     image_ids, start, n_rays, bits / 2, rays, target);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_blender_images(const uint8_t* rgba, int64_t n_images, int32_t H, int32_t W, int32_t half_res,
                                     int32_t mode, float* out, void* stream) {
  if (n_images < 0 || H <= 0 || W <= 0 || mode < 0 || mode > 2) return HN_E_SHAPE;
  if (half_res && ((H | W) & 1)) return HN_E_SHAPE;   // INTER_AREA at exactly half
  if (n_images == 0) return HN_OK;
  if (!rgba || !out) return HN_E_NULL;
  const int64_t n_px = n_images * (int64_t)(half_res ? H / 2 : H) * (half_res ? W / 2 : W);
  hipLaunchKernelGGL(blender_images_kernel, dim3((unsigned)((n_px + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     rgba, n_px, H, W, half_res ? 1 : 0, mode, out);
  return hip_status(hipGetLastError());
}
