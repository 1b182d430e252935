// hn_render.hip -- fused render_rays (run_nerf_helpers.py:464-574) for one
// training ray batch: ONE forward kernel and ONE backward kernel (+ a tiny
// packing kernel in front and a deterministic weight-grad slab reduction behind).
//
// Forward, one wave64 per ray:
//   coarse z (linspace + stratified jitter, :514-536) -> 2 tiles of 32 points:
//   hash-encode (16 levels, 8 corner gathers each) + NeRFSmall on MFMA ->
//   composite (:541) -> sample_pdf 128 (:548) -> rank-sort 192 (:551) ->
//   6 fine tiles (encode + MLP) -> composite (:558).
// Backward, one wave64 per ray, workgroups specialised per network (coarse
// blocks / fine blocks, so each keeps ONE network's dW accumulator in LDS):
//   composite backward (wave suffix scan) -> per tile: re-encode, recompute the
//   MLP, MLP backward on MFMA (dW through LDS transposes, accumulated in LDS),
//   trilinear backward + float atomics into the hash-table gradient.
#include "hn_mlp.h"
#include "hn_render.h"

// Diagnostic ablations (never set in the product build): 1 = no scatter
// atomics, 2 = no MLP in the backward (gather + scatter only).
#ifndef HN_ABLATE
#define HN_ABLATE 0
#endif

namespace hn {

constexpr int kSc = 64, kNi = 128, kSf = 192;
constexpr int kFwdWaves = 4;
constexpr int kBwdWaves = 8;
constexpr int kBwdBlocks = 256;          // persistent: one 512-thread block per CU
constexpr int kBwdCoarseBlocks = 64;     // coarse work is 2 tiles/ray, fine 6

struct RenderK {
  GridArgs g;
  int white, lindisp, perturb;
  int64_t B;
  const float* rays;
  const float* tvals;
  const float* t_rand;
  const float* u;
  const float* noise_c;
  const float* noise_f;
  const float* table;
  const float* Pc;
  const float* Pf;
  float *rgb, *depth, *acc, *sparsity, *rgb0, *depth0, *acc0, *sparsity0, *z_std;
  float *z_coarse, *z_fine, *raw_c, *raw_f;
  uint8_t* fine_src;
};

struct RenderBK {
  GridArgs g;
  int white;
  int64_t B;
  const float* rays;
  const float* noise_c;
  const float* noise_f;
  const float* table;
  const float* Pc;
  const float* Pf;
  const float *z_coarse, *z_fine, *raw_c, *raw_f;
  const uint8_t* fine_src;
  const float *g_rgb, *g_depth, *g_acc, *g_sparsity, *g_rgb0, *g_depth0, *g_acc0, *g_sparsity0;
  const float* g_raw_f;
  float* d_table;
  float* slab;    // [kBwdBlocks][W_END]
  float* dfeat;   // [B][64 + 192][32]: d loss / d feature per evaluated point
};

struct Ray {
  float o[3], d[3], vd[3], near, far, dnorm;
};

HN_DEV void load_ray(const float* __restrict__ rays, int64_t ray, Ray& r) {
  const float* rb = rays + 11 * ray;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    r.o[a] = rb[a];
    r.d[a] = rb[3 + a];
    r.vd[a] = rb[8 + a];
  }
  r.near = rb[6];
  r.far = rb[7];
  r.dnorm = sqrtf(r.d[0] * r.d[0] + r.d[1] * r.d[1] + r.d[2] * r.d[2]);   // torch.norm (:595)
}

// pts = rays_o + rays_d * z (:538, :552)
HN_DEV void ray_point(const Ray& r, float z, float pt[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) pt[a] = r.o[a] + r.d[a] * z;
}

// Hash-encode one point into the 32-feature tile layout (lane half h owns
// levels tile_level(m, h), m = 0..7).  hash_encoding.py:84-110.
HN_DEV void encode_tile(const GridArgs& g, const float* gsl, const float* __restrict__ table, const float pt[3], int h,
                        f32x16& feat) {
  float xc[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) xc[a] = clamp_t(pt[a], g.bmin[a], g.bmax[a]);
  const uint32_t mask = (1u << g.log2T) - 1u;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int l0 = tile_level(m, 0), l1 = tile_level(m, 1);
    const uint32_t l = h ? l1 : l0;
    const float gs[3] = {gsl[3 * l], gsl[3 * l + 1], gsl[3 * l + 2]};
    Voxel v;
    voxel_level(pt, xc, gs, g.bmin, mask, v);
    float f0, f1;
    encode_level_off(table, l << g.log2T, v, f0, f1);
    feat[2 * m] = f0;
    feat[2 * m + 1] = f1;
    if (m & 1) __builtin_amdgcn_sched_barrier(0);   // <= 16 gathers in flight
  }
}

// One level of the scatter for the 32 points of a tile (lane half h adds
// feature h; both halves see the same point and level, so the f0/f1 atomics
// of an entry are two adjacent dwords of ONE wave-instruction = one memory
// request).  Consecutive lanes are consecutive samples along the ray; a run
// of samples inside one voxel shares all 8 corners, so the run is summed in
// registers first (segmented suffix sum over the half-wave) and only its head
// lane issues the 8 atomics.  The reduction is skipped when the level has no
// run (fine levels, sparse samples).
HN_DEV void scatter_level(const GridArgs& g, const float* gsl, float* __restrict__ dtable,
                          const float pt[3], const float xc[3], uint32_t l, float gf, int p, int h) {
  const float gs[3] = {gsl[3 * l], gsl[3 * l + 1], gsl[3 * l + 2]};
  const uint32_t mask = (1u << g.log2T) - 1u;
  Voxel v;
  uint32_t cell[3];
  voxel_level_cell(pt, xc, gs, g.bmin, mask, v, cell);
  float cv[8];
  trilerp_bwd(gf, v.w, cv);
  const uint32_t q0 = __shfl_up(cell[0], 1, 32), q1 = __shfl_up(cell[1], 1, 32),
                 q2 = __shfl_up(cell[2], 1, 32);
  const bool head = p == 0 || q0 != cell[0] || q1 != cell[1] || q2 != cell[2];
  const uint32_t hm = (uint32_t)(__ballot(head) >> (32 * h));   // heads of this half
#pragma unroll
  for (int d = 1; d < 32; d <<= 1) {
    // lane p absorbs lane p+d iff no run starts in (p, p+d]
    const bool same = p + d < 32 && ((hm >> (p + 1)) & ((1u << d) - 1u)) == 0u;
    if (!__any(same)) break;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float o = __shfl_down(cv[c], d, 32);
      if (same) cv[c] += o;
    }
  }
  if (head) {
    const uint32_t row0 = l << g.log2T;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float* dst = reinterpret_cast<float*>(reinterpret_cast<char*>(dtable) +
                                            (row0 + v.h[c]) * 8u + 4u * h);
      atomic_add_f32(dst, cv[c]);
    }
  }
}

// Trilinear backward + scatter-add of one tile's feature grads into the table
// gradient (embedding_dense_backward of hash_encoding.py:106).
HN_DEV void scatter_tile(const GridArgs& g, const float* gsl, float* __restrict__ dtable, const float pt[3], int h,
                         const f32x16& dfeat) {
  const int p = lane_id() & 31;
  float xc[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) xc[a] = clamp_t(pt[a], g.bmin[a], g.bmax[a]);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    // lane half h holds (f0, f1) of level tile_level(m, h); trade so that
    // half h holds feature h of both levels tile_level(m, 0/1)
    const float g0 = dfeat[2 * m], g1 = dfeat[2 * m + 1];
    const float recv = __shfl_xor(h ? g0 : g1, 32, 64);
    const float ga = h ? recv : g0;     // feature h of level tile_level(m, 0)
    const float gb = h ? g1 : recv;     // feature h of level tile_level(m, 1)
    scatter_level(g, gsl, dtable, pt, xc, tile_level(m, 0), ga, p, h);
    __builtin_amdgcn_sched_barrier(0);
    scatter_level(g, gsl, dtable, pt, xc, tile_level(m, 1), gb, p, h);
    __builtin_amdgcn_sched_barrier(0);
  }
}

HN_DEV void ray_sh(const Ray& r, int h, float sh8[8], float shx8[8]) {
  float sh[16];
  sh16(r.vd[0], r.vd[1], r.vd[2], sh);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    sh8[s] = h ? sh[2 * s + 1] : sh[2 * s];
    shx8[s] = h ? sh[8 + s] : sh[s];
  }
}

constexpr int kGsLds = 48;   // grid sizes [16][3] staged in LDS (saves 48 SGPRs)

HN_DEV void stage_grid_sizes(const GridArgs& g, float* gsl) {
  if (threadIdx.x < 48) gsl[threadIdx.x] = g.gs[threadIdx.x / 3][threadIdx.x % 3];
}

// LDS per forward wave (floats).
constexpr int kFZc = 0, kFZsrc = 64, kFZs = 256, kFRaw = 448, kFW = 1216, kFBins = 1280,
              kFCdf = 1344, kFLds = 1408;

__global__ __launch_bounds__(256) void render_fwd_kernel(RenderK k) {
  __shared__ __attribute__((aligned(16))) float smem[kFwdWaves * kFLds + kGsLds];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int p = lane & 31, h = lane >> 5;
  float* gsl = smem + kFwdWaves * kFLds;
  stage_grid_sizes(k.g, gsl);
  __syncthreads();
  const int64_t ray = (int64_t)blockIdx.x * kFwdWaves + wave;
  if (ray >= k.B) return;
  float* L = smem + wave * kFLds;
  float* zc = L + kFZc;
  float* zsrc = L + kFZsrc;
  float* zs = L + kFZs;
  float* rawb = L + kFRaw;
  float* wts = L + kFW;
  float* bins = L + kFBins;
  float* cdf = L + kFCdf;
  Ray r;
  load_ray(k.rays, ray, r);

  // ---- coarse z_vals (:514-536) ----
  auto zlin = [&](int i) {
    const float t = k.tvals[i];
    return k.lindisp ? 1.f / (1.f / r.near * (1.f - t) + 1.f / r.far * t)
                     : r.near * (1.f - t) + r.far * t;
  };
  float z = zlin(lane);
  if (k.perturb) {
    const float zm = lane > 0 ? zlin(lane - 1) : z;
    const float zp = lane < kSc - 1 ? zlin(lane + 1) : z;
    const float lower = lane > 0 ? .5f * (z + zm) : z;
    const float upper = lane < kSc - 1 ? .5f * (zp + z) : z;
    z = lower + (upper - lower) * k.t_rand[ray * kSc + lane];
  }
  zc[lane] = z;
  zsrc[lane] = z;
  k.z_coarse[ray * kSc + lane] = z;
  float sh8[8], shx8[8];
  ray_sh(r, h, sh8, shx8);
  lds_fence_wave();

  // ---- coarse network (:540) ----
  for (int tau = 0; tau < kSc / 32; ++tau) {
    const float* P = opaque_ptr(k.Pc);
    const int q = 32 * tau + p;
    float pt[3];
    ray_point(r, zc[q], pt);
    f32x16 feat;
    encode_tile(k.g, gsl, k.table, pt, h, feat);
    MlpAct a;
    f32x16 c2;
    mlp_fwd_tile(P, feat, sh8, a, c2, lane);
    if (h == 0) {
      const float4 o4 = make_float4(c2[0], c2[1], c2[2], a.s1[0]);
      *reinterpret_cast<float4*>(rawb + 4 * q) = o4;
      *reinterpret_cast<float4*>(k.raw_c + (ray * kSc + q) * 4) = o4;
    }
  }
  lds_fence_wave();
  CompOut co;
  composite_fwd<1>(rawb, zc, k.noise_c ? k.noise_c + ray * kSc : nullptr, kSc, r.dnorm, k.white != 0,
                   wts, co, lane);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) k.rgb0[3 * ray + c] = co.rgb[c];
    k.depth0[ray] = co.depth;
    k.acc0[ray] = co.acc;
    k.sparsity0[ray] = co.entropy;
  }

  // ---- importance sampling (:547-551) ----
  if (lane < kSc - 1) bins[lane] = .5f * (zc[lane + 1] + zc[lane]);
  lds_fence_wave();
  sample_pdf_wave(bins, wts + 1, kSc - 2, cdf, k.u + ray * kNi, kNi, zsrc + kSc, lane);
  lds_fence_wave();
  {
    const float s0 = zsrc[kSc + lane], s1 = zsrc[kSc + 64 + lane];
    const double mean = wave_sum((double)s0 + (double)s1) / kNi;
    const double d0 = (double)s0 - mean, d1 = (double)s1 - mean;
    const double var = wave_sum(d0 * d0 + d1 * d1) / kNi;
    if (lane == 0) k.z_std[ray] = (float)sqrt(var);
  }
  rank_sort_wave(zsrc, zs, kSf, lane, k.fine_src + ray * kSf, kSc);
  for (int i = lane; i < kSf; i += 64) k.z_fine[ray * kSf + i] = zs[i];

  // ---- fine network (:556) ----
  for (int tau = 0; tau < kSf / 32; ++tau) {
    const float* P = opaque_ptr(k.Pf);
    const int q = 32 * tau + p;
    float pt[3];
    ray_point(r, zs[q], pt);
    f32x16 feat;
    encode_tile(k.g, gsl, k.table, pt, h, feat);
    MlpAct a;
    f32x16 c2;
    mlp_fwd_tile(P, feat, sh8, a, c2, lane);
    if (h == 0) {
      const float4 o4 = make_float4(c2[0], c2[1], c2[2], a.s1[0]);
      *reinterpret_cast<float4*>(rawb + 4 * q) = o4;
      *reinterpret_cast<float4*>(k.raw_f + (ray * kSf + q) * 4) = o4;
    }
  }
  lds_fence_wave();
  CompOut fo;
  composite_fwd<3>(rawb, zs, k.noise_f ? k.noise_f + ray * kSf : nullptr, kSf, r.dnorm, k.white != 0,
                   nullptr, fo, lane);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) k.rgb[3 * ray + c] = fo.rgb[c];
    k.depth[ray] = fo.depth;
    k.acc[ray] = fo.acc;
    k.sparsity[ray] = fo.entropy;
  }
}

// LDS per backward wave (floats) after the workgroup's dW accumulator.
constexpr int kBT = 0, kBZ = 2 * kTBuf, kBRaw = kBZ + kSf, kBLds = kBRaw + 4 * kSf;
static_assert((W_END + kBRaw) % 4 == 0, "float4 alignment of the raw buffer");

template <int S>
HN_DEV void bwd_ray(const RenderBK& k, int64_t ray, bool fine, float* Wacc, float* L, const float* gsl,
                    int lane) {
  constexpr int N = S / 64;
  const int p = lane & 31, h = lane >> 5;
  float* T = L + kBT;
  float* zb = L + kBZ;
  float* rawb = L + kBRaw;
  Ray r;
  load_ray(k.rays, ray, r);
  const float* zsrc = (fine ? k.z_fine : k.z_coarse) + ray * S;
  const float* rsrc = (fine ? k.raw_f : k.raw_c) + ray * S * 4;
  for (int i = lane; i < S; i += 64) {
    zb[i] = zsrc[i];
    *reinterpret_cast<float4*>(rawb + 4 * i) = *reinterpret_cast<const float4*>(rsrc + 4 * i);
  }
  lds_fence_wave();
  CompGrad g;
  const float* grgb = fine ? k.g_rgb : k.g_rgb0;
  const float* gacc = fine ? k.g_acc : k.g_acc0;
  const float* gdep = fine ? k.g_depth : k.g_depth0;
  const float* gent = fine ? k.g_sparsity : k.g_sparsity0;
  g.has_rgb = grgb != nullptr;
  g.has_acc = gacc != nullptr;
  g.has_depth = gdep != nullptr;
  g.has_entropy = gent != nullptr;
#pragma unroll
  for (int c = 0; c < 3; ++c) g.rgb[c] = g.has_rgb ? grgb[3 * ray + c] : 0.f;
  g.acc = g.has_acc ? gacc[ray] : 0.f;
  g.depth = g.has_depth ? gdep[ray] : 0.f;
  g.entropy = g.has_entropy ? gent[ray] : 0.f;
  const float* noise = fine ? (k.noise_f ? k.noise_f + ray * S : nullptr)
                            : (k.noise_c ? k.noise_c + ray * S : nullptr);
  const float* graw = (fine && k.g_raw_f) ? k.g_raw_f + ray * S * 4 : nullptr;
  composite_bwd<N>(rawb, zb, noise, S, r.dnorm, k.white != 0, g, nullptr, graw, rawb, lane);
  lds_fence_wave();
  float sh8[8], shx8[8];
  ray_sh(r, h, sh8, shx8);
  for (int tau = 0; tau < S / 32; ++tau) {
    const float* P = opaque_ptr(fine ? k.Pf : k.Pc);
    const int q = 32 * tau + p;
    float pt[3];
    ray_point(r, zb[q], pt);
    f32x16 feat;
    encode_tile(k.g, gsl, k.table, pt, h, feat);
    f32x16 dfeat;
#if HN_ABLATE == 2   // diagnostic build: gather + scatter only (no MLP)
    dfeat = feat;
#else
    MlpAct a;
    f32x16 c2;
    mlp_fwd_tile(P, feat, sh8, a, c2, lane);
    const float4 dr = *reinterpret_cast<const float4*>(rawb + 4 * q);
    const float dy2[2] = {h ? dr.y : dr.x, h ? 0.f : dr.z};
    const float rgbg[3] = {dr.x, dr.y, dr.z};
    mlp_bwd_tile(P, feat, shx8, a, dy2, dr.w, rgbg, T, Wacc, dfeat, nullptr, lane);
#endif
    // per-point feature gradient stored [point][feature f][level] for the
    // scatter kernel (lane half h holds levels tile_level(m, h))
    float* dst = k.dfeat + ((size_t)ray * (kSc + kSf) + (fine ? kSc : 0) + q) * 32;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int l = h ? tile_level(m, 1) : tile_level(m, 0);
      dst[l] = dfeat[2 * m];
      dst[16 + l] = dfeat[2 * m + 1];
    }
  }
}

// Scatter of the table gradient, one wave per ray over its 192 UNIQUE points:
// a fine sample that is one of the 64 coarse samples (fine_src < 64) is the
// same point in both passes, so its coarse-pass and fine-pass feature grads
// are summed before the trilinear backward + atomics (25 % fewer atomics).
// Few registers -> high occupancy to keep many atomics in flight; kept out of
// the MFMA kernel so the atomics never stall its gathers on vmcnt.
//
// Lane layout: 16 points per pass, 4 lanes per point = (x offset i, feature f).
// One atomic wave-instruction then covers corners (0,j,k) and (1,j,k) of both
// features of 16 points: h(x+1) differs from h(x) only in low bits (prime 1
// on x), so 7/8 of the x-pairs fall in one 64-byte segment and the four dwords
// of a point go out as ~1 memory request instead of 2 (the float-atomic path
// is request-rate bound for random rows).  Consecutive points are consecutive
// samples along the ray; runs inside one voxel are summed first (segmented
// suffix sum over points) and only the run head issues atomics.
HN_DEV void scatter_level_x(const GridArgs& g, const float* gsl, float* __restrict__ dtable,
                            const float pt[3], const float xc[3], uint32_t l, float gl, int pp,
                            int xi, int f) {
  const float gs[3] = {gsl[3 * l], gsl[3 * l + 1], gsl[3 * l + 2]};
  uint32_t cell[3];
  float w[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float q = (xc[a] - g.bmin[a]) / gs[a];
    const int32_t i = (int32_t)floorf(q);
    const float vmin = (float)i * gs[a] + g.bmin[a];
    const float vmax = vmin + gs[a];
    w[a] = (pt[a] - vmin) / (vmax - vmin);
    cell[a] = (uint32_t)i;
  }
  const uint32_t mask = (1u << g.log2T) - 1u;
  const uint32_t hx = cell[0] + (uint32_t)xi;
  const uint32_t y0 = cell[1] * kPrimeY, y1 = (cell[1] + 1u) * kPrimeY;
  const uint32_t z0 = cell[2] * kPrimeZ, z1 = (cell[2] + 1u) * kPrimeZ;
  // d feat / d e_c = ((g * fz) * fy) * fx  (trilerp_bwd order), c = 4*xi + jk
  const float fx = xi ? w[0] : 1.f - w[0];
  const float gz0 = gl * (1.f - w[2]), gz1 = gl * w[2];
  float cv[4];
  cv[0] = (gz0 * (1.f - w[1])) * fx;   // j=0 k=0
  cv[1] = (gz1 * (1.f - w[1])) * fx;   // j=0 k=1
  cv[2] = (gz0 * w[1]) * fx;           // j=1 k=0
  cv[3] = (gz1 * w[1]) * fx;           // j=1 k=1
  const uint32_t q0 = __shfl_up(cell[0], 4, 64), q1 = __shfl_up(cell[1], 4, 64),
                 q2 = __shfl_up(cell[2], 4, 64);
  const bool head = pp == 0 || q0 != cell[0] || q1 != cell[1] || q2 != cell[2];
  const uint64_t hm = __ballot(head);
  uint32_t pm = 0;                                  // one head bit per point
#pragma unroll
  for (int j = 0; j < 16; ++j) pm |= (uint32_t)((hm >> (4 * j)) & 1u) << j;
#pragma unroll
  for (int d = 1; d < 16; d <<= 1) {
    const bool same = pp + d < 16 && ((pm >> (pp + 1)) & ((1u << d) - 1u)) == 0u;
    if (!__any(same)) break;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float o = __shfl_down(cv[c], 4 * d, 64);
      if (same) cv[c] += o;
    }
  }
  if (head) {
    const uint32_t row0 = l << g.log2T;
    const uint32_t hh[4] = {(hx ^ y0 ^ z0) & mask, (hx ^ y0 ^ z1) & mask, (hx ^ y1 ^ z0) & mask,
                            (hx ^ y1 ^ z1) & mask};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float* dst = reinterpret_cast<float*>(reinterpret_cast<char*>(dtable) +
                                            (row0 + hh[c]) * 8u + 4u * f);
      atomic_add_f32(dst, cv[c]);
    }
  }
}

__global__ __launch_bounds__(256) void render_scatter_kernel(RenderBK k) {
  __shared__ float gsl[kGsLds];
  stage_grid_sizes(k.g, gsl);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int pp = lane >> 2, xi = (lane >> 1) & 1, f = lane & 1;
  const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (ray >= k.B) return;
  Ray r;
  load_ray(k.rays, ray, r);
  const float* base = k.dfeat + (size_t)ray * (kSc + kSf) * 32;
  for (int grp = 0; grp < kSf / 16; ++grp) {
    const int q = 16 * grp + pp;
    float pt[3], xc[3];
    ray_point(r, k.z_fine[ray * kSf + q], pt);
#pragma unroll
    for (int a = 0; a < 3; ++a) xc[a] = clamp_t(pt[a], k.g.bmin[a], k.g.bmax[a]);
    const int src = k.fine_src[ray * kSf + q];
    float gl[16];
    const float* df = base + (size_t)(kSc + q) * 32 + 16 * f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 v = *reinterpret_cast<const float4*>(df + 4 * t);
      gl[4 * t] = v.x; gl[4 * t + 1] = v.y; gl[4 * t + 2] = v.z; gl[4 * t + 3] = v.w;
    }
    if (src < kSc) {
      const float* dc = base + (size_t)src * 32 + 16 * f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float4 v = *reinterpret_cast<const float4*>(dc + 4 * t);
        gl[4 * t] += v.x; gl[4 * t + 1] += v.y; gl[4 * t + 2] += v.z; gl[4 * t + 3] += v.w;
      }
    }
#if HN_ABLATE == 1   // diagnostic build: everything but the scatter atomics
    if (gl[0] == 1234.5f && gl[1] == -1234.5f) k.d_table[lane] = gl[2];
#else
#pragma unroll
    for (int l = 0; l < 16; ++l) {
      scatter_level_x(k.g, gsl, k.d_table, pt, xc, l, gl[l], pp, xi, f);
      __builtin_amdgcn_sched_barrier(0);
    }
#endif
  }
}

__global__ __launch_bounds__(512, 2) void render_bwd_kernel(RenderBK k) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Wacc = smem;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float* L = smem + W_END + wave * kBLds;
  float* gsl = smem + W_END + kBwdWaves * kBLds;
  stage_grid_sizes(k.g, gsl);
  for (int i = threadIdx.x; i < W_END; i += blockDim.x) Wacc[i] = 0.f;
  __syncthreads();
  const bool fine = blockIdx.x >= kBwdCoarseBlocks;
  const int blk = fine ? blockIdx.x - kBwdCoarseBlocks : blockIdx.x;
  const int nblk = fine ? kBwdBlocks - kBwdCoarseBlocks : kBwdCoarseBlocks;
  for (int64_t ray = (int64_t)blk * kBwdWaves + wave; ray < k.B; ray += (int64_t)nblk * kBwdWaves) {
    if (fine) bwd_ray<kSf>(k, ray, true, Wacc, L, gsl, lane);
    else bwd_ray<kSc>(k, ray, false, Wacc, L, gsl, lane);
  }
  __syncthreads();
  float* dst = k.slab + (size_t)blockIdx.x * W_END;
  for (int i = threadIdx.x; i < W_END; i += blockDim.x) dst[i] = Wacc[i];
}

// dW(coarse) += sum of coarse-block slabs, dW(fine) += sum of fine-block slabs.
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab,
                                                          hn_mlp_grad dc, hn_mlp_grad df) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * W_END) return;
  const bool fine = t >= W_END;
  const int i = fine ? t - W_END : t;
  const int b0 = fine ? kBwdCoarseBlocks : 0, b1 = fine ? kBwdBlocks : kBwdCoarseBlocks;
  float s = 0.f;
  for (int b = b0; b < b1; ++b) s += slab[(size_t)b * W_END + i];
  const hn_mlp_grad& d = fine ? df : dc;
  float* dst;
  if (i < W_S1) dst = d.sigma0 + i;
  else if (i < W_C0) dst = d.sigma1 + (i - W_S1);
  else if (i < W_C1) dst = d.color0 + (i - W_C0);
  else if (i < W_C2) dst = d.color1 + (i - W_C1);
  else dst = d.color2 + (i - W_C2);
  *dst += s;
}

static int32_t check_cfg(const hn_render_cfg* c) {
  if (!c) return HN_E_NULL;
  const hn_grid& g = c->grid;
  if (g.n_levels != 16 || g.n_features != 2) return HN_E_SHAPE;
  if (g.log2_hashmap_size < 1 || g.log2_hashmap_size > 24) return HN_E_SHAPE;
  if (c->n_samples != kSc || c->n_importance != kNi) return HN_E_SHAPE;
  return HN_OK;
}

static bool mlp_ok(const hn_mlp& w) { return w.sigma0 && w.sigma1 && w.color0 && w.color1 && w.color2; }
static bool grad_ok(const hn_mlp_grad& w) {
  return w.sigma0 && w.sigma1 && w.color0 && w.color1 && w.color2;
}

}  // namespace hn

using namespace hn;

// Workspace: packed coarse + fine weights | dW slabs [256][9344] |
// per-point feature grads [n_rays][256][32].
extern "C" size_t hn_render_workspace_bytes(const hn_render_cfg* cfg, int64_t n_rays) {
  (void)cfg;
  const size_t n = n_rays > 0 ? (size_t)n_rays : 0;
  return ((size_t)2 * G_END + (size_t)kBwdBlocks * W_END + n * (kSc + kSf) * 32) * sizeof(float);
}

extern "C" int32_t hn_render_fwd(const hn_render_cfg* cfg, const hn_render_fwd_args* a,
                                 void* workspace, size_t ws_bytes, void* stream) {
  int32_t st = check_cfg(cfg);
  if (st) return st;
  if (!a) return HN_E_NULL;
  if (a->n_rays < 0) return HN_E_SHAPE;
  if (a->n_rays == 0) return HN_OK;
  if (!a->rays || !a->t_vals || !a->u || !a->table || !mlp_ok(a->coarse) || !mlp_ok(a->fine))
    return HN_E_NULL;
  if (cfg->perturb && !a->t_rand) return HN_E_NULL;
  if (!a->rgb || !a->depth || !a->acc || !a->sparsity || !a->rgb0 || !a->depth0 || !a->acc0 ||
      !a->sparsity0 || !a->z_std || !a->z_coarse || !a->z_fine || !a->raw_c || !a->raw_f ||
      !a->fine_src)
    return HN_E_NULL;
  if (!workspace) return HN_E_NULL;
  if (ws_bytes < hn_render_workspace_bytes(cfg, a->n_rays)) return HN_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* Pc = (float*)workspace;
  float* Pf = Pc + G_END;
  if ((st = mlp_pack_launch(&a->coarse, Pc, s))) return st;
  if ((st = mlp_pack_launch(&a->fine, Pf, s))) return st;
  RenderK k;
  k.g = make_grid_args(cfg->grid);
  k.white = cfg->white_bkgd;
  k.lindisp = cfg->lindisp;
  k.perturb = cfg->perturb;
  k.B = a->n_rays;
  k.rays = a->rays; k.tvals = a->t_vals; k.t_rand = a->t_rand; k.u = a->u;
  k.noise_c = a->noise_c; k.noise_f = a->noise_f; k.table = a->table;
  k.Pc = Pc; k.Pf = Pf;
  k.rgb = a->rgb; k.depth = a->depth; k.acc = a->acc; k.sparsity = a->sparsity;
  k.rgb0 = a->rgb0; k.depth0 = a->depth0; k.acc0 = a->acc0; k.sparsity0 = a->sparsity0;
  k.z_std = a->z_std; k.z_coarse = a->z_coarse; k.z_fine = a->z_fine;
  k.raw_c = a->raw_c; k.raw_f = a->raw_f; k.fine_src = a->fine_src;
  const unsigned blocks = (unsigned)((a->n_rays + kFwdWaves - 1) / kFwdWaves);
  hipLaunchKernelGGL(render_fwd_kernel, dim3(blocks), dim3(64 * kFwdWaves), 0, s, k);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_render_bwd(const hn_render_cfg* cfg, const hn_render_bwd_args* a,
                                 void* workspace, size_t ws_bytes, void* stream) {
  int32_t st = check_cfg(cfg);
  if (st) return st;
  if (!a) return HN_E_NULL;
  if (a->n_rays < 0) return HN_E_SHAPE;
  if (a->n_rays == 0) return HN_OK;
  if (!a->rays || !a->table || !mlp_ok(a->coarse) || !mlp_ok(a->fine)) return HN_E_NULL;
  if (!a->z_coarse || !a->z_fine || !a->raw_c || !a->raw_f || !a->fine_src) return HN_E_NULL;
  if (!a->d_table || !grad_ok(a->d_coarse) || !grad_ok(a->d_fine)) return HN_E_NULL;
  if (!workspace) return HN_E_NULL;
  if (ws_bytes < hn_render_workspace_bytes(cfg, a->n_rays)) return HN_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* Pc = (float*)workspace;
  float* Pf = Pc + G_END;
  float* slab = Pf + G_END;
  float* dfeat = slab + (size_t)kBwdBlocks * W_END;
  if ((st = mlp_pack_launch(&a->coarse, Pc, s))) return st;
  if ((st = mlp_pack_launch(&a->fine, Pf, s))) return st;
  RenderBK k;
  k.g = make_grid_args(cfg->grid);
  k.white = cfg->white_bkgd;
  k.B = a->n_rays;
  k.rays = a->rays; k.noise_c = a->noise_c; k.noise_f = a->noise_f; k.table = a->table;
  k.Pc = Pc; k.Pf = Pf;
  k.z_coarse = a->z_coarse; k.z_fine = a->z_fine; k.raw_c = a->raw_c; k.raw_f = a->raw_f;
  k.fine_src = a->fine_src;
  k.dfeat = dfeat;
  k.g_rgb = a->g_rgb; k.g_depth = a->g_depth; k.g_acc = a->g_acc; k.g_sparsity = a->g_sparsity;
  k.g_rgb0 = a->g_rgb0; k.g_depth0 = a->g_depth0; k.g_acc0 = a->g_acc0;
  k.g_sparsity0 = a->g_sparsity0; k.g_raw_f = a->g_raw_f;
  k.d_table = a->d_table;
  k.slab = slab;
  const size_t lds = (size_t)(W_END + kBwdWaves * kBLds + kGsLds) * sizeof(float);
  hipLaunchKernelGGL(render_bwd_kernel, dim3(kBwdBlocks), dim3(64 * kBwdWaves), lds, s, k);
  if ((st = hip_status(hipGetLastError()))) return st;
  hipLaunchKernelGGL(render_scatter_kernel, dim3((unsigned)((a->n_rays + 3) / 4)), dim3(256), 0, s, k);
  if ((st = hip_status(hipGetLastError()))) return st;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((2 * W_END + 255) / 256), dim3(256), 0, s, slab,
                     a->d_coarse, a->d_fine);
  return hip_status(hipGetLastError());
}
