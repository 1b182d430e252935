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
//   composite backward (wave suffix scan) -> per tile: load the features the
//   forward saved, recompute the MLP, MLP backward on MFMA (dW through LDS
//   transposes, accumulated in LDS), store d loss / d feature per point.
// Scatter kernel, one wave per ray over its 192 unique points: trilinear
// backward + float atomics into the hash-table gradient.
#include "hn_mlp.h"
#include "hn_render.h"
#include "hn_loss.h"
#include "hn_tv.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

// The forward's waves raise their issue priority (s_setprio) while they
// encode: a wave that is issuing gathers gets its requests out ahead of the
// SIMD's other waves, whose MLP phases then overlap the gathers' latency.
// Measured (r04x, config 2, two runs each): render_fwd_kernel 0.2743 ->
// 0.2673 ms at priority 1 (0.2671 at 2), step 1.005 / 1.000 -> 0.993 / 0.994
// ms; scheduling only, so every result is unchanged.
#define HN_FWD_PRIO_HI() __builtin_amdgcn_s_setprio(1)
#define HN_FWD_PRIO_LO() __builtin_amdgcn_s_setprio(0)

namespace hn {

// levels per scheduling group of the forward's encode (8 gathers each):
// 1 level 0.2674, 2 levels 0.2666, 4 levels 0.2696 ms (r04z)
constexpr int kEncGroup = 2;
#ifndef HN_FWD_SKIP_STORES
#define HN_FWD_SKIP_STORES 1
#endif

constexpr int kSc = 64, kNi = 128, kSf = 192;
constexpr int kFwdWaves = 4;
constexpr int kBwdBlocks = 256;          // persistent backward: one block per CU
#ifndef HN_DW_BLOCKRED   // the MLP backward's dW summed per block before the slab store (render_bwd_kernel)
#define HN_DW_BLOCKRED 1
#endif

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
  float* feat;    // [B][8 tiles][1024] saved features or NULL
  int feat_nt;    // saved features stored nontemporally (tables past the MALL)
  int skip_dead;  // hn_render_fwd_args.skip_dead_color
};


// Arguments of the backward MLP kernel (kept lean: every field lives in SGPRs).
struct B1K {
  int64_t B;
  int32_t scramble;     // Feistel half-width of the chunk-position -> ray permutation, 0: identity
  int white;
  const float* rays;
  const float *noise_c, *noise_f;
  const float *Pc, *Pf;
  const float *z_coarse, *z_fine, *raw_c, *raw_f;
  const float* feat;
  const float *g_rgb, *g_depth, *g_acc, *g_sparsity, *g_rgb0, *g_depth0, *g_acc0, *g_sparsity0;
  const float* g_raw_f;
  float* slab;
  float* dfeat;         // [B][64][32] coarse-pass feature grads ([f][level] per point)
  float* draw;          // [B][64 + 192][4] d raw of every sample (composite pre-pass)
  // fine kernel: trilinear backward + scatter into the table gradient
  GridArgs g;
  const uint8_t* fine_src;
  float* d_table;
  // binned scatter (bin_geom): record buffer base, records per (block, bin),
  // log2 entries per bin, bins
  float* bins;
  int32_t bin_cap, bin_shift, nbins;
  float* dfeat_f;       // split backward: [B][6 fine tiles][1024] fine-pass feature grads (tile order)
  // ABI 13 training loss formed by the composite pre-pass (hn_render_loss;
  // lout NULL = none): hn_loss_bwd's upstream factors (g = 1), the value's inputs
  const float *ltarget, *lrgb, *lrgb0, *lsp, *lsp0, *ltv;
  int32_t n_tv;
  float lgm, lsparse, lworld, lsparse_w, ltv_w;
  float* lout;
  int32_t skip_zero;    // exact-zero skipping (!hn_render_cfg.dense_bwd)
  uint8_t* uflags;      // [B][kMarkB] marks (composite pre-pass): [0] coarse, [1] fine MLP tiles with a
                        // nonzero d raw -- as bits: 0-3 coarse 16-sample groups, 8-19 fine
                        // groups (the MLP backward's), 20-31 fine groups with a nonzero sample or
                        // coarse twin (the scatter's)
  int32_t* lmeta;       // work lists (render_lists_kernel): [0] coarse tiles, [1] fine tiles, [2] scatter
                        // tiles, [3] gsplit: the MLP waves g < gsplit run coarse tiles (slab_reduce_block)
  int32_t* lists;       // group codes (ray << 4 | group): coarse [4B] | fine [12B] | the scatter's [12B]
};

// Backward schedules (render_bwd_kernel MODE):
//   kModeAtomic  MLP waves 0-2 + a scatter wave issuing float atomics (fused)
//   kModeSplit   MLP backward only (wave 0 coarse units, waves 1-3 fine units), the fine feature
//                grads stored for scatter_bins_kernel
enum : int { kModeAtomic = 0, kModeSplit = 2 };

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

// Saved features: tile t of a ray (t = 0,1 coarse, 2..7 fine) is 1024 floats,
// stored as 4 chunks of [64 lanes][float4] so that both the forward's store
// and the backward's load are fully coalesced dwordx4 accesses.
// After the 8 feature tiles: the tiles' ReLU masks of the two networks (tile
// t: 3 words [h0 | c0 | c1] x 64 lanes, bit 16 ob + r = D register r of
// output block ob of the lane), written by the forward.
constexpr int kTilesPerRay = (kSc + kSf) / 32;
constexpr int kMaskWordsPerTile = 3 * 64;
static_assert(kTilesPerRay * (1024 + kMaskWordsPerTile) == HN_RENDER_FEAT_PER_RAY, "feature cache layout");

// The forward stores its ReLU masks and the backward's forward recompute
// uses them with 2-part products (HN_SPLIT_R 2): the recomputed
// activations then differ from the forward's by ~2^-17 relative (the dW
// operands' own precision), but every ReLU decision is the forward's.

HN_DEV void store_masks(float* __restrict__ base, int64_t ray, int tile, int lane, const uint32_t (&m)[3], bool nt) {
  uint32_t* t = reinterpret_cast<uint32_t*>(base + (size_t)ray * HN_RENDER_FEAT_PER_RAY + kTilesPerRay * 1024) +
                tile * kMaskWordsPerTile;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (nt) __builtin_nontemporal_store(m[j], t + 64 * j + lane);
    else t[64 * j + lane] = m[j];
  }
}
HN_DEV void load_masks(const float* __restrict__ base, int64_t ray, int tile, int lane, uint32_t (&m)[3]) {
  const uint32_t* t = reinterpret_cast<const uint32_t*>(base + (size_t)ray * HN_RENDER_FEAT_PER_RAY +
                                                        kTilesPerRay * 1024) + tile * kMaskWordsPerTile;
#pragma unroll
  for (int j = 0; j < 3; ++j) m[j] = __builtin_nontemporal_load(t + 64 * j + lane);
}
HN_DEV void store_feat(float* __restrict__ base, int64_t ray, int tile, int lane, const f32x16& feat, bool nt) {
  f32x4* t = reinterpret_cast<f32x4*>(base + (size_t)ray * HN_RENDER_FEAT_PER_RAY + (size_t)tile * 1024);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x4 v = {feat[4 * c], feat[4 * c + 1], feat[4 * c + 2], feat[4 * c + 3]};
    if (nt) __builtin_nontemporal_store(v, t + 64 * c + lane);
    else t[64 * c + lane] = v;
  }
}

HN_DEV void load_feat(const float* __restrict__ base, int64_t ray, int tile, int lane, f32x16& feat) {
  const f32x4* t = reinterpret_cast<const f32x4*>(base + (size_t)ray * HN_RENDER_FEAT_PER_RAY + (size_t)tile * 1024);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x4 v = __builtin_nontemporal_load(t + 64 * c + lane);
    feat[4 * c] = v.x; feat[4 * c + 1] = v.y; feat[4 * c + 2] = v.z; feat[4 * c + 3] = v.w;
  }
}

// grid sizes [16][3] staged in LDS (saves 48 SGPRs), then their reciprocals
constexpr int kGsRcp = 48, kGsLds = 96;

// Hash-encode one point into the 32-feature tile layout (lane half h owns
// levels tile_level(m, h), m = 0..7).  hash_encoding.py:84-110.
HN_DEV void encode_tile(const GridArgs& g, const float* gsl, const float* __restrict__ table, const float pt[3], int h,
                        f32x16& feat) {
  // (Software-pipelining the levels -- level m + 1 or m + 2's gathers issued
  // before level m's are consumed -- measured slower: render_fwd_kernel 0.310
  // -> 0.330 / 0.323 ms, r04b; the other three waves of the SIMD already hide
  // the gathers' latency.  Loading a level's x-pairs as 16-B buffer loads
  // where both corners share an aligned pair of rows (4 + 4 loads instead
  // of 8) measured 0.2777 vs 0.2823 ms before the coarse-twin reuse, and
  // 0.2789 vs 0.2731 ms after it (r04h, r04l): not kept.)
  float xc[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) xc[a] = clamp_t(pt[a], g.bmin[a], g.bmax[a]);
  const uint32_t mask = (1u << g.log2T) - 1u;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int l0 = tile_level(m, 0), l1 = tile_level(m, 1);
    const uint32_t l = h ? l1 : l0;
    const float gs[3] = {gsl[3 * l], gsl[3 * l + 1], gsl[3 * l + 2]};
    const float rg[3] = {gsl[kGsRcp + 3 * l], gsl[kGsRcp + 3 * l + 1], gsl[kGsRcp + 3 * l + 2]};
    Voxel v;
    voxel_level_rcp(pt, xc, gs, rg, g.bmin, mask, v);
    float f0, f1;
    encode_level_off(table, l << g.log2T, v, f0, f1);
    feat[2 * m] = f0;
    feat[2 * m + 1] = f1;
    if ((m & (kEncGroup - 1)) == kEncGroup - 1) __builtin_amdgcn_sched_barrier(0);   // <= 8 x kEncGroup gathers in flight
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


HN_DEV void stage_grid_sizes(const GridArgs& g, float* gsl) {
  if (threadIdx.x < 48) {
    const float gs = g.gs[threadIdx.x / 3][threadIdx.x % 3];
    gsl[threadIdx.x] = gs;
    gsl[kGsRcp + threadIdx.x] = 1.f / gs;
  }
}

// LDS per forward wave (floats).
constexpr int kFZc = 0, kFZsrc = 64, kFZs = 256, kFRaw = 448, kFW = 1216, kFBins = 1280,
              kFCdf = 1344, kFC0 = 1408, kFLds = 1472;

#ifndef HN_FWD_WAVES_PER_SIMD
#define HN_FWD_WAVES_PER_SIMD 4
#endif
// 4 waves per SIMD (<= 128 registers; the few spills sit outside the tile
// loops): one ray per wave, so a 4096-ray batch is exactly one round on 256
// CUs (3 waves: 0.427 ms, a 1/3-occupied second round; 4: 0.418 ms)

// Diagnostic phase timers of the forward (HN_PROFILE=1 builds only; never in
// the shipped library): shader-clock cycles per wave in [0] coarse encode,
// [1] coarse MLP + stores, [2] composite + sampling + sort, [3] fine encode,
// [4] fine MLP + stores, [5] final composite, [6] total, [7] waves; printed by
// hn_render_fwd after a synchronising read.  The encode laps wait for the
// features first, so a gather's latency counts in its encode phase.
#ifndef HN_PROFILE
#define HN_PROFILE 0
#endif
#if HN_PROFILE
__device__ unsigned long long g_fwd_prof[8];
#define HN_FT(i) do { const uint64_t n_ = __builtin_amdgcn_s_memtime(); ft[i] += n_ - t_; t_ = n_; } while (0)
#define HN_FT_FEAT(i, f) do { asm volatile("" ::"v"((f)[0]), "v"((f)[15])); HN_FT(i); } while (0)
#else
#define HN_FT(i) ((void)0)
#define HN_FT_FEAT(i, f) ((void)0)
#endif

// (Round 4 measured 16-wave workgroups with each net's forward weight
// fragments staged in LDS instead of streamed from L2 per tile: the MLP phase
// ran ~3x faster but the gathers of 16 waves in step ~2.3x slower,
// render_fwd_kernel 0.294 vs 0.281 ms, and staggering half of the waves made it
// 0.301-0.313 ms; profiles/r04/r04e, r04f.)
constexpr int kFwdBlockWaves = kFwdWaves;


__global__ __launch_bounds__(64 * kFwdBlockWaves)
__attribute__((amdgpu_waves_per_eu(HN_FWD_WAVES_PER_SIMD, HN_FWD_WAVES_PER_SIMD)))
void render_fwd_kernel(RenderK k) {
  __shared__ __attribute__((aligned(16))) float smem[kFwdBlockWaves * kFLds + kGsLds];
  // each wave's split-GEMM fragments one chunk ahead (FragRing, hn_mlp.h):
  // render_fwd_kernel 0.271 -> 0.266 ms, r05 ring (bitwise-identical outputs)
  __shared__ __attribute__((aligned(16))) float fring[kFwdBlockWaves][768];
  // the wave index (and with it the ray, its 11 floats and every per-ray
  // address) on the scalar unit: VGPR spills 45 -> 22, render_fwd_kernel
  // 0.296 -> 0.281 ms (r04e)
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int p = lane & 31, h = lane >> 5;
  float* gsl = smem + kFwdBlockWaves * kFLds;
  stage_grid_sizes(k.g, gsl);
  __syncthreads();
  // XCD-aware: workgroup b runs on XCD b % 8, so consecutive ray groups of a
  // spatially ordered batch go to one XCD and share its L2
  const int64_t nb = gridDim.x;
  // (round 6, r06k: chunks of 4 or 16 ray groups dealt round-robin over the
  // XCDs, or no XCD mapping at all, were no faster: 234.9 / 228.8 / 240.4 us
  // against 229.4 us -- the forward's per-XCD work is balanced already)
  const int64_t grp = nb % 8 == 0 ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
  const int64_t ray = grp * kFwdBlockWaves + wave;
  if (ray >= k.B) return;
#if HN_PROFILE
  uint64_t ft[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t t0_ = __builtin_amdgcn_s_memtime();
  uint64_t t_ = t0_;
#endif
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
  float sh8[8], shx8[8];
  float* c0l = L + kFC0;

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
  ray_sh(r, h, sh8, shx8);
  lds_fence_wave();

  // ---- coarse network (:540) ----
  c0sh_lds_store(opaque_ptr(k.Pc), sh8, c0l, lane);
  lds_fence_wave();
  fwd_ring_start(k.Pc, fring[wave], lane);
  for (int tau = 0; tau < kSc / 32; ++tau) {
    const float* P = opaque_ptr(k.Pc);
    const int q = 32 * tau + p;
    float pt[3];
    ray_point(r, zc[q], pt);
    f32x16 feat;
    HN_FWD_PRIO_HI();
    encode_tile(k.g, gsl, k.table, pt, h, feat);
    HN_FWD_PRIO_LO();
    HN_FT_FEAT(0, feat);
    if (k.feat) store_feat(k.feat, ray, tau, lane, feat, k.feat_nt != 0);
    MlpAct a;
    f32x16 c2;
    mlp_fwd_tile_src<true>(FragRing{P, fring[wave]}, feat, [&](int ob) { return c0sh_lds_load(c0l, ob, lane); },
                           a, c2, lane, k.skip_dead && k.noise_c == nullptr);
    if (k.feat) store_masks(k.feat, ray, tau, lane, a.m, k.feat_nt != 0);
    if (h == 0) {
      const float4 o4 = make_float4(c2[0], c2[1], c2[2], a.s1[0]);
      *reinterpret_cast<float4*>(rawb + 4 * q) = o4;
      *reinterpret_cast<float4*>(k.raw_c + (ray * kSc + q) * 4) = o4;
    }
    HN_FT(1);
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
  // sort(cat(z_vals, z_samples)) (:551): a merge of the sorted coarse run with
  // the bitonic-sorted importance samples (rawb is free until the fine tiles),
  // the all-pairs rank sort if the coarse run is ever out of order
  // (render_fwd_kernel 0.2998 -> 0.2966 ms, r04c)
  uint8_t* org = k.fine_src + ray * kSf;
  if (!merge_sort_z(zsrc, zs, rawb, lane, org)) rank_sort_wave(zsrc, zs, kSf, lane, org, kSc);
  for (int i = lane; i < kSf; i += 64) k.z_fine[ray * kSf + i] = zs[i];

  // ---- fine network (:556) ----
  c0sh_lds_store(opaque_ptr(k.Pf), sh8, c0l, lane);   // the coarse tiles' reads are done (in-order LDS)
  lds_fence_wave();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the coarse ring's last (unused) fill has landed
  fwd_ring_start(k.Pf, fring[wave], lane);
  HN_FT(2);
  for (int tau = 0; tau < kSf / 32; ++tau) {
    const float* P = opaque_ptr(k.Pf);
    const int q = 32 * tau + p;
    float pt[3];
    ray_point(r, zs[q], pt);
    f32x16 feat;
    // a third of the fine samples are the coarse samples again (the merge
    // keeps their z bitwise): with the feature cache present, those lanes load
    // the coarse tile's features (4 dwordx4, written by this wave) instead of
    // gathering 16 levels x 8 corners again -- a quarter of the ray's gathers
    // (render_fwd_kernel 0.282 -> 0.275 ms, r04h).  Encoding only the 128
    // importance samples as 4 full tiles first and loading every fine tile's
    // features back from the cache (a third fewer encode instructions) measured
    // slower: 0.301 ms, the waves then run their MLP tiles in step (r04j).
    const int src = k.feat ? (int)k.fine_src[ray * kSf + q] : 255;
    if (src >= kSc) {
      HN_FWD_PRIO_HI();
      encode_tile(k.g, gsl, k.table, pt, h, feat);
      HN_FWD_PRIO_LO();
    } else {
      const f32x4* t = reinterpret_cast<const f32x4*>(k.feat + (size_t)ray * HN_RENDER_FEAT_PER_RAY +
                                                      (size_t)(src >> 5) * 1024) + (src & 31) + 32 * h;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const f32x4 v = t[64 * c];
        feat[4 * c] = v.x; feat[4 * c + 1] = v.y; feat[4 * c + 2] = v.z; feat[4 * c + 3] = v.w;
      }
    }
    HN_FT_FEAT(3, feat);
    MlpAct a;
    f32x16 c2;
    // skip_dead: a fine tile without density has no nonzero d raw, so the
    // backward (dense_bwd = 0: its work lists) never reads its features or
    // masks -- they are not stored (HN_FWD_SKIP_STORES)
    const bool dead_skip = k.skip_dead && k.noise_f == nullptr;
    bool stored = !HN_FWD_SKIP_STORES || !dead_skip;
    if (k.feat && stored) store_feat(k.feat, ray, kSc / 32 + tau, lane, feat, k.feat_nt != 0);
    mlp_fwd_tile_src<true>(FragRing{P, fring[wave]}, feat, [&](int ob) { return c0sh_lds_load(c0l, ob, lane); },
                           a, c2, lane, dead_skip, [&]() {
                             if (k.feat && !stored) store_feat(k.feat, ray, kSc / 32 + tau, lane, feat, k.feat_nt != 0);
                             stored = true;
                           });
    if (k.feat && stored) store_masks(k.feat, ray, kSc / 32 + tau, lane, a.m, k.feat_nt != 0);
    if (h == 0) {
      const float4 o4 = make_float4(c2[0], c2[1], c2[2], a.s1[0]);
      *reinterpret_cast<float4*>(rawb + 4 * q) = o4;
      *reinterpret_cast<float4*>(k.raw_f + (ray * kSf + q) * 4) = o4;
    }
    HN_FT(4);
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
#if HN_PROFILE
  HN_FT(5);
  ft[6] = __builtin_amdgcn_s_memtime() - t0_;
  ft[7] = 1;
  if (lane == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&g_fwd_prof[i], (unsigned long long)ft[i]);
#endif
}

// ---------------------------------------------------------------------------
// Backward MLP kernel (B1).  One wave per SIMD (4 per CU, 512 registers each):
// the wave keeps ALL twelve 32x32 weight-gradient blocks of its network as
// MFMA accumulators (192 registers, AGPR-resident) for the whole kernel, so a
// tile's dW costs only its MFMAs -- no per-tile LDS accumulation.  The
// operands of the dW products (the point index on the MFMA k axis) come from
// per-wave LDS images of bf16 split parts read back transposed (the weight-
// gradient operand images below).  ReLU masks are kept as bits.
//
// Work units: a coarse unit is one ray's 2 coarse tiles, a fine unit 2 of a
// ray's 6 fine tiles.  Waves 0-2 run units (wave 0 first every coarse unit of
// the block, then fine units with waves 1-2); wave 3 only scatters the fine
// tiles' table gradients, handed over through an LDS ring.  The composite
// backward (d raw per sample) comes from a full-occupancy pre-pass.
// ---------------------------------------------------------------------------
// per-wave LDS: the weight-gradient operand images (9 x 4 KiB) in a slab of
// kRRows x kXS floats (also the fused schedule's slot size unit)
constexpr int kXS = 36;
constexpr int kRRows = 260;
constexpr int kB1Waves = 4;
constexpr int kMW = kB1Waves - 1;                          // MLP waves; wave kMW scatters
constexpr int kB1Img = kMW * kRRows * kXS;                 // floats (112,320 B)
// Fine-tile hand-off ring (MLP waves -> scatter wave): per slot the tile's
// feature grads [32 points][kXS] ([f][level], coarse twin added), the 32
// sample depths and the ray origin / direction.
constexpr int kSlots = 8;
constexpr int kSlotZ = 32 * kXS, kSlotR = kSlotZ + 32, kSlotF = kSlotR + 8;
constexpr int kVoxF = 16 * 16 * 8;                         // scatter wave's voxel buffer
constexpr int kSyncInts = 5 + 2 * kSlots;
constexpr int kB1LdsF = kB1Img + kSlots * kSlotF + kVoxF + kGsLds + kSyncInts;
static_assert(kB1LdsF * 4 <= 160 * 1024, "LDS budget");
// dW slabs in the workspace: [kBwdBlocks][kSlabSlots][W_END], slot 0 the
// block's coarse dW, slots 1-3 its fine MLP waves' dW (slab_reduce_kernel)
constexpr int kSlabSlots = 4;
static_assert(kRRows * kXS % 4 == 0 && kXS % 4 == 0 && kSlotF % 4 == 0, "b128 alignment");

struct DW {
  f32x16 c2[2], c1[4], c0[2], s1[2], s0[2];
};

// ---- weight-gradient operand images --------------------------------------
// A 32 x 32 tile of a layer's activations or output grads (rows = features,
// columns = the tile's points; D layout in registers) is staged as its first
// two split-f32 parts (hn_common.h: p0 = bf16(x), p1 = bf16(x - p0), the NS = 2
// split of the dW products) in a per-wave image [32 points][32 features] of
// bf16 per part (64-B point rows).  The parts come from the split the tile
// already gets as the B operand of the next GEMM of the chain (gemm_w / _w2
// with an image sink), so the dW products need no split of their own.
// dW[o][i] = sum_p G[o][p] X[i][p] contracts the point index (X's column),
// so both operands are read back transposed by ds_read_b64_tr_b16: lane l
// gets feature l & 31 of 4 consecutive points per read.  The 8-byte feature
// quads of point p sit at quad f4 ^ ((p >> 1) & 7): the quad writes of a
// D-layout tile are 2-way (the minimum for 64 lanes x 8 B on 32 banks), the
// transposed reads conflict-free.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kImgBlk = 4096;   // bytes per tile image: 2 parts x 2 KiB
// tile images per wave: features | h0 (2) | [sh16 | sigma | geo15] | c0 (2) |
// c1 (2) | rgb grads; the grads of the backward reuse c1 (dc1, then ds1) and
// c0 (dc0, then dh0) once those are consumed
enum : int { kBF = 0, kBH0 = 1, kBC0in = 3, kBC0 = 4, kBC1 = 6, kBDR = 8, kNImg = 9 };
static_assert(kNImg * kImgBlk <= kRRows * kXS * 4, "images fit the per-wave LDS");

HN_DEV uint32_t img_off(int blk, int part, int p, int f4) {
  return (uint32_t)(blk * kImgBlk + part * 2048 + p * 64 + ((f4 ^ ((p >> 1) & 7)) << 3));
}
HN_DEV void put_quad(char* Xb, int blk, int part, int p, int f4, uint32_t lo, uint32_t hi) {
  *reinterpret_cast<uint2*>(Xb + img_off(blk, part, p, f4)) = uint2{lo, hi};
}
// Parts 0 and 1 of one split B chunk (elements j = D registers 8c' + j of
// lane (p, h): rows 16c' + 4h + j for j < 4, 16c' + 8 + 4h + j - 4 after) to
// quads f4b + h and f4b + 2 + h (f4b = 4c' + the tile's feature offset / 4).
template <int NS>
HN_DEV void put_parts(char* Xb, int blk, int f4b, const SP<NS>& s, int lane) {
  static_assert(NS >= 2, "the images hold two parts");
  const int p = lane & 31, h = lane >> 5;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const u32x4 w = __builtin_bit_cast(u32x4, s.p[q]);
    put_quad(Xb, blk, q, p, f4b + h, w[0], w[1]);
    put_quad(Xb, blk, q, p, f4b + 2 + h, w[2], w[3]);
  }
}
// A D-layout tile not split by any GEMM of the chain (c1): split and stage it.
HN_DEV void put_tile(char* Xb, int blk, const f32x16& v, int lane) {
#pragma unroll
  for (int c = 0; c < 2; ++c) put_parts<2>(Xb, blk, 4 * c, splitn<2>([&](int j) { return v[8 * c + j]; }), lane);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
HN_DEV s16x4 ds_read_tr(const char* a) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(reinterpret_cast<uintptr_t>(a)));
}
// Operand of K = 16 chunk cc (points 16cc .. 16cc + 15) of image tile blk,
// part q: lane l holds feature l & 31 at points 16cc + 8h + j (element j).
HN_DEV bf16x8 img_operand(const char* Xb, int blk, int q, int cc, int lane) {
  const int g = (lane >> 4) & 3, i = lane & 15, h = lane >> 5;
  const int f4 = 4 * (g & 1) + (i & 3), pt = 16 * cc + 8 * h + (i >> 2);
  const s16x4 lo = ds_read_tr(Xb + img_off(blk, q, pt, f4));
  const s16x4 hi = ds_read_tr(Xb + img_off(blk, q, pt + 4, f4));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// acc[NB * a + b] += sum over the tile's 32 points of A(ablk[a]) B(bblk[b])^T
// (two K = 16 chunks, 2-part products in mfma_split's order)
template <int NA, int NB>
HN_DEV void wgrad_n(const char* Xb, const int (&ablk)[NA], const int (&bblk)[NB], f32x16* acc, int lane) {
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    SP<2> a[NA], b[NB];
#pragma unroll
    for (int j = 0; j < NA; ++j)
#pragma unroll
      for (int q = 0; q < 2; ++q) a[j].p[q] = img_operand(Xb, ablk[j], q, cc, lane);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int q = 0; q < 2; ++q) b[j].p[q] = img_operand(Xb, bblk[j], q, cc, lane);
#pragma unroll
    for (int ja = 0; ja < NA; ++ja)
#pragma unroll
      for (int jb = 0; jb < NB; ++jb) acc[NB * ja + jb] = mfma_split<2>(a[ja], b[jb], acc[NB * ja + jb]);
  }
}

template <int I, int N, typename F>
HN_DEV void static_for(F&& f) {
  if constexpr (N > 0) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N - 1>(f);
  }
}

// A weight-gradient block's operands read into registers ahead of its
// products (WgOps), and the products then issued in the gaps of a later
// data-path GEMM (WgX, gemm_w / gemm_w2's `xt`): the image reads leave before
// that GEMM's own image writes (a wave's LDS accesses execute in order), and
// the products -- the same ones, per accumulator in the same order as
// wgrad_n's -- keep the matrix pipe busy while the chain waits on its own
// results and splits.  NoX: no extra products.
template <int NA, int NB>
struct WgOps {
  SP<2> a[2][NA], b[2][NB];   // [K = 16 chunk cc][operand]
};
template <int NA, int NB>
HN_DEV void wg_load(WgOps<NA, NB>& o, const char* Xb, const int (&ablk)[NA], const int (&bblk)[NB], int lane) {
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
#pragma unroll
    for (int j = 0; j < NA; ++j)
#pragma unroll
      for (int q = 0; q < 2; ++q) o.a[cc][j].p[q] = img_operand(Xb, ablk[j], q, cc, lane);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int q = 0; q < 2; ++q) o.b[cc][j].p[q] = img_operand(Xb, bblk[j], q, cc, lane);
  }
}
struct NoX {
  static constexpr int per(int) { return 0; }
  template <int C>
  HN_DEV void run() const {}
};
// the 2 * NA * NB products of a WgOps (cc-major, as wgrad_n) spread over NC chunks
template <int NA, int NB, int NC>
struct WgX {
  const WgOps<NA, NB>& o;
  f32x16* acc;
  static constexpr int P = 2 * NA * NB;
  static constexpr int lo(int c) { return c * P / NC; }
  static constexpr int per(int c) { return 3 * (lo(c + 1) - lo(c)); }   // MFMAs at chunk c
  template <int C>
  HN_DEV void run() const {
    static_for<lo(C), lo(C + 1) - lo(C)>([&](auto pc) {
      constexpr int p = decltype(pc)::value, cc = p / (NA * NB), ja = p % (NA * NB) / NB, jb = p % NB;
      acc[NB * ja + jb] = mfma_split<2>(o.a[cc][ja], o.b[cc][jb], acc[NB * ja + jb]);
    });
  }
};

// ---- weight-fragment stream ----------------------------------------------
// A tile's 15 data-path GEMMs read their packed A-fragment groups (one 1-KiB
// dwordx4 load per wave: 4 f32 k-steps, or one bf16 part of 8 k-steps) in a
// fixed order (92 groups at HN_SPLIT_F = 3, HN_SPLIT_B = 2), padded to a
// multiple of the ring depth so that the ring lines up with the tile period.
// The ring keeps the next 8 groups (~16 bf16 MFMAs with their splits) in
// flight across GEMM, tile and unit boundaries: no GEMM starts on an exposed
// L2 latency at one wave per SIMD.  Depth 4 measured 484 us for the config-2
// MLP backward, 8: 460 us.  The two output blocks of a GEMM are paired
// (kSegs, gemm_w2): one B split per chunk for both, two independent
// accumulator chains (515 -> 484 us together with wgrad_n's shared splits).
struct GemmSeg {
  int r, ob;   // region (hn_mlp.h), output block; ob = -1: both blocks, chunk by chunk
};
constexpr GemmSeg kSegs[] = {{R_F0, -1}, {R_F1, 0}, {R_F2G, -1}, {R_F3, -1}, {R_B4, -1},
                             {R_B3, -1}, {R_B2G, 0}, {R_B1, -1}, {R_B0, 0}};
constexpr int kNSegs = sizeof(kSegs) / sizeof(kSegs[0]);
// HN_SPLIT_R: parts the backward's forward recompute uses of the forward
// regions' HN_SPLIT_F packed parts (the leading parts of a split are the same
// for every part count, so the recompute streams only groups q < HN_SPLIT_R of
// each chunk).  3 = the forward's own products (bit-identical activations).
#ifndef HN_SPLIT_R
#define HN_SPLIT_R 2
#endif
constexpr int seg_ns(const GemmSeg& g) {   // parts this stream uses per chunk (0: f32)
  return g.r < R_B4 && reg_ns(g.r) > HN_SPLIT_R ? HN_SPLIT_R : reg_ns(g.r);
}
constexpr int seg_gpo(const GemmSeg& g) { return seg_ns(g) ? seg_ns(g) * kRegKS[g.r] / 8 : kRegKS[g.r] / 4; }
constexpr int seg_groups(const GemmSeg& g) { return seg_gpo(g) * (g.ob < 0 ? 2 : 1); }
constexpr int seg_start(int i) {   // first group of segment i in the stream
  int n = 0;
  for (int j = 0; j < i; ++j) n += seg_groups(kSegs[j]);
  return n;
}
#ifndef HN_WRING
#define HN_WRING 8
#endif
constexpr int kTileGroups = seg_start(kNSegs), kRing = HN_WRING;
constexpr int kTilePeriod = (kTileGroups + kRing - 1) / kRing * kRing;   // pad groups keep slots static
// A paired segment streams chunk c of block 0 (its NS groups; f32: one
// group), then chunk c of block 1, then chunk c + 1 ...
constexpr int group_off(int idx) {
  idx %= kTilePeriod;
  if (idx >= kTileGroups) idx = 0;              // pad groups re-read group 0
  for (const GemmSeg& g : kSegs) {
    const int n = reg_gpo(g.r), u = seg_gpo(g);   // packed / streamed groups per block
    const int per = seg_ns(g) ? seg_ns(g) : 1, pk = reg_ns(g.r) ? reg_ns(g.r) : 1;   // per chunk
    if (g.ob >= 0) {
      if (idx < u) return reg_off(g.r) + (g.ob * n + pk * (idx / per) + idx % per) * 256;
    } else if (idx < 2 * u) {
      const int c = idx / (2 * per), ob = idx / per % 2, q = idx % per;
      return reg_off(g.r) + (ob * n + pk * c + q) * 256;
    }
    idx -= seg_groups(g);
  }
  return 0;
}
static_assert(group_off(kTileGroups - 1) == G_B0 + (reg_gpo(R_B0) - 1) * 256, "GEMM sequence");
static_assert(HN_SPLIT_F != 3 || HN_SPLIT_FC != 3 || HN_SPLIT_B != 2 || HN_SPLIT_R != 3 ||
              (kTileGroups == 92 && G_END == 30208), "layout");

struct WRing {
  f32x4 b[kRing];
};

// Weight-fragment group load: frag_load (hn_common.h, raw buffer load with a
// scalar offset).
// HN_DIAG_FRAG_L1 (diagnostic builds only, wrong gradients): every group
// load reads the same 1 KiB, so the stream is served from the CU's L1 --
// the bound on what sharing the fragments between waves could save.
#ifndef HN_DIAG_FRAG_L1
#define HN_DIAG_FRAG_L1 0
#endif
HN_DEV f32x4 wload(const float* P, int off, int lane) {
  return frag_load(P, HN_DIAG_FRAG_L1 ? 0 : off, lane);
}

// (offsets are constexpr-evaluated: left to the optimiser, the region
// arithmetic of group_off stays as scalar loops in the kernel)
HN_DEV void wring_prime(WRing& w, const float* P, int lane) {
  static_for<0, kRing>([&](auto jc) {
    constexpr int j = decltype(jc)::value, off = group_off(j);
    w.b[j] = wload(P, off, lane);
  });
}
template <int IDX>
HN_DEV f32x4 wring_take(WRing& w, const float* P, int lane) {
  constexpr int off = group_off(IDX + kRing);
  const f32x4 a = w.b[IDX % kRing];
  w.b[IDX % kRing] = wload(P, off, lane);
  return a;
}

// The next chunk's B split (VALU) is issued in the gaps of this
// chunk's MFMAs (sched_group_barrier: one MFMA, then V VALU) instead of after
// them; the same splits and the same MFMA order, so results are unchanged.
// Measured (r03g, config 2, two runs each on one box): backward launch
// 0.812 -> 0.789 ms, step 1.159 -> 1.134 ms; the kernel's 24 VGPR spills go to 0.
// The same pipelining in the forward's gemm (round 3, removed) changed
// nothing there (render_fwd 0.304 ms either way).
// (VALU per MFMA slot, 2-part splits: 7 in gemm_w, 4 in gemm_w2.  Measured
// round 4, r04sw: 5 / 3 took render_bwd_kernel from 0.2343 to 0.2426 ms,
// 10 / 6 to 0.2364 ms.)
template <int NMFMA, int NVALU>
HN_DEV void swp_pattern() {
  static_for<0, NMFMA>([&](auto) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);       // one MFMA
    __builtin_amdgcn_sched_group_barrier(0x002, NVALU, 0);   // then VALU
  });
}

// acc += A(segment SEG of the stream) . B, bval(s) = B operand of f32 k-step s.
// IMG >= 0: chunk c's first two B parts also go to image tile IMG + c / 2 at
// quad offset F4B + 4 (c % 2) (put_parts; Xb = the wave's images).
// XT: extra independent MFMAs issued after chunk c's own (WgX; NoX: none),
// their VALU slots sharing the next chunk's split (kSplitV VALU per split).
template <int NS, bool PAIR>
constexpr int kSplitV = NS == 3 ? 36 : (PAIR ? 24 : 21);
constexpr int ceil_div(int a, int b) { return (a + b - 1) / b; }
template <int SEG, int IMG = -1, int F4B = 0, typename BF, typename XT = NoX>
HN_DEV f32x16 gemm_w(WRing& w, const float* P, f32x16 acc, int lane, BF bval, char* Xb = nullptr,
                     const XT& xt = XT{}) {
  constexpr int R = kSegs[SEG].r, KS = kRegKS[R], NS = seg_ns(kSegs[SEG]), START = seg_start(SEG);
  static_assert(IMG < 0 || NS >= 2, "image sinks take split B operands");
  if constexpr (NS > 0 && KS > 8) {   // split-f32, next chunk's split in the MFMA gaps
    constexpr int NC = KS / 8;
    SP<NS> b = splitn<NS>([&](int j) { return bval(j); });
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, NC>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      SP<NS> a;
      static_for<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        a.p[q] = as_bf16x8(wring_take<START + NS * c + q>(w, P, lane));
      });
      if constexpr (IMG >= 0) put_parts<NS>(Xb, IMG + c / 2, F4B + 4 * (c % 2), b, lane);
      acc = mfma_split<NS>(a, b, acc);
      xt.template run<c>();
      if constexpr (c + 1 < NC) {
        b = splitn<NS>([&](int j) { return bval(8 * (c + 1) + j); });
        constexpr int M = NS + XT::per(c);
        swp_pattern<M, XT::per(c) ? ceil_div(kSplitV<NS, false>, M) : (NS == 3 ? 6 : 7)>();
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  } else if constexpr (NS > 0) {                // split-f32: NS groups per K = 16 chunk
    static_for<0, KS / 8>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      SP<NS> a;
      static_for<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        a.p[q] = as_bf16x8(wring_take<START + NS * c + q>(w, P, lane));
      });
      const SP<NS> b = splitn<NS>([&](int j) { return bval(8 * c + j); });
      if constexpr (IMG >= 0) put_parts<NS>(Xb, IMG + c / 2, F4B + 4 * (c % 2), b, lane);
      acc = mfma_split<NS>(a, b, acc);
      xt.template run<c>();
      __builtin_amdgcn_sched_barrier(0);
    });
  } else {
    static_for<0, KS / 4>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      const f32x4 a = wring_take<START + g>(w, P, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma(a[j], bval(4 * g + j), acc);
      xt.template run<g>();
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  return acc;
}

// acc0 / acc1 += blocks 0 / 1 of the paired segment SEG . B: one B split per
// chunk for both blocks, and two independent accumulator chains
template <int SEG, int IMG = -1, int F4B = 0, typename BF, typename XT = NoX>
HN_DEV void gemm_w2(WRing& w, const float* P, f32x16& acc0, f32x16& acc1, int lane, BF bval, char* Xb = nullptr,
                    const XT& xt = XT{}) {
  constexpr int R = kSegs[SEG].r, KS = kRegKS[R], NS = seg_ns(kSegs[SEG]), START = seg_start(SEG);
  static_assert(kSegs[SEG].ob < 0, "paired segment");
  static_assert(IMG < 0 || NS >= 2, "image sinks take split B operands");
  if constexpr (NS > 0 && KS > 8) {
    constexpr int NC = KS / 8;
    SP<NS> b = splitn<NS>([&](int j) { return bval(j); });
    __builtin_amdgcn_sched_barrier(0);
    static_for<0, NC>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      SP<NS> a0, a1;
      static_for<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        a0.p[q] = as_bf16x8(wring_take<START + 2 * NS * c + q>(w, P, lane));
      });
      static_for<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        a1.p[q] = as_bf16x8(wring_take<START + 2 * NS * c + NS + q>(w, P, lane));
      });
      if constexpr (IMG >= 0) put_parts<NS>(Xb, IMG + c / 2, F4B + 4 * (c % 2), b, lane);
      mfma_split2<NS>(a0, a1, b, acc0, acc1);
      xt.template run<c>();
      if constexpr (c + 1 < NC) {
        b = splitn<NS>([&](int j) { return bval(8 * (c + 1) + j); });
        constexpr int M = 2 * NS + XT::per(c);
        swp_pattern<M, XT::per(c) ? ceil_div(kSplitV<NS, true>, M) : (NS == 3 ? 3 : 4)>();
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  } else if constexpr (NS > 0) {
    constexpr int NC = KS / 8;
    static_for<0, NC>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      SP<NS> a0, a1;
      static_for<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        a0.p[q] = as_bf16x8(wring_take<START + 2 * NS * c + q>(w, P, lane));
      });
      static_for<0, NS>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        a1.p[q] = as_bf16x8(wring_take<START + 2 * NS * c + NS + q>(w, P, lane));
      });
      const SP<NS> b = splitn<NS>([&](int j) { return bval(8 * c + j); });
      if constexpr (IMG >= 0) put_parts<NS>(Xb, IMG + c / 2, F4B + 4 * (c % 2), b, lane);
      mfma_split2<NS>(a0, a1, b, acc0, acc1);
      xt.template run<c>();
      __builtin_amdgcn_sched_barrier(0);
    });
  } else {
    static_for<0, KS / 4>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      const f32x4 a0 = wring_take<START + 2 * g>(w, P, lane);
      const f32x4 a1 = wring_take<START + 2 * g + 1>(w, P, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc0 = mfma(a0[j], bval(4 * g + j), acc0);
        acc1 = mfma(a1[j], bval(4 * g + j), acc1);
      }
      xt.template run<g>();
      __builtin_amdgcn_sched_barrier(0);
    });
  }
}

constexpr int seg_of(int r) {   // first stream segment of region r
  for (int i = 0; i < kNSegs; ++i)
    if (kSegs[i].r == r) return i;
  return -1;
}
// acc[0..1] += both output blocks of region R . B (image sink: gemm_w)
template <int R, int IMG = -1, int F4B = 0, typename BF, typename XT = NoX>
HN_DEV void gemm2(WRing& w, const float* P, f32x16 acc[2], int lane, BF bval, char* Xb = nullptr,
                  const XT& xt = XT{}) {
  constexpr int S = seg_of(R);
  if constexpr (kSegs[S].ob < 0) {
    gemm_w2<S, IMG, F4B>(w, P, acc[0], acc[1], lane, bval, Xb, xt);
  } else {
    static_assert(std::is_same<XT, NoX>::value, "extra products go to paired segments");
    acc[0] = gemm_w<S, IMG, F4B>(w, P, acc[0], lane, bval, Xb);
    acc[1] = gemm_w<S + 1>(w, P, acc[1], lane, bval);
  }
}

// ReLU with its mask bits, in integer forms that keep no lane masks
// live (the compare forms held 16+ SGPR-pair masks across the GEMMs and
// spilled them to VGPR lanes): relu = the bits with the sign-extended sign
// cleared (v > 0 ? v : 0 for every non-NaN v, -0 -> +0), bit = relu > 0 from
// the relu's bits, and the gradient masked by AND with the sign-extended bit.
// (No inline asm here: an asm operand that is an MFMA result gets none of the
// MFMA-to-VALU wait states the compiler inserts for its own instructions.)
HN_DEV void relu_bits(f32x16& v, uint32_t& m, int ob) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint32_t b = __float_as_uint(v[r]);
    const uint32_t u = b & ~(uint32_t)((int32_t)b >> 31);
    m |= min(u, 1u) << (16 * ob + r);
    v[r] = __uint_as_float(u);
  }
}
HN_DEV void mask_bits(f32x16& g, uint32_t m, int ob) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe((int)m, 16 * ob + r, 1);   // 0 or ~0
    g[r] = __uint_as_float(__float_as_uint(g[r]) & keep);
  }
}

// Ordering of a wave's own LDS image writes and transposed reads inside a
// tile.  The LDS unit executes one wave's ds instructions in order, so a read
// issued after a write sees it (also another lane's) and a write after a read
// does not overwrite what the read returns: only the compiler must keep the
// program order: a compiler barrier (the reads' own lgkmcnt waits stay)
// instead of s_waitcnt lgkmcnt(0) at each hand-over (lds_fence_wave), which
// also waits for every write still in flight (measured equal, round 3).
HN_DEV void tile_lds_order() {
  asm volatile("" ::: "memory");
}

// color_net.0 applied to the ray's sh features (the same for every point of
// the ray): its 64 rows are kept in the wave's LDS slab after the
// images (read back as the c0 accumulators' seed, 8 broadcast ds_read_b128
// per tile) instead of 32 VGPRs live across the unit's tiles.
constexpr int kC0shF = kNImg * kImgBlk / 4;   // float offset in the wave's slab
static_assert(kC0shF + 128 <= kRRows * kXS, "c0sh (two groups' rays) fits the per-wave slab");
struct C0Sh {
  const float* lds;
};
HN_DEV void c0sh_seed(const C0Sh& c, f32x16 (&c0)[2], int h) {
#pragma unroll
  for (int ob = 0; ob < 2; ++ob)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(c.lds + 32 * ob + row_of(4 * g, h));
#pragma unroll
      for (int j = 0; j < 4; ++j) c0[ob][4 * g + j] = v[j];
    }
}

// One 32-point tile: recompute the forward (features from the cache), then
// the MLP backward; dW into the wave's accumulators, d feature to dst.
HN_DEV f32x16 b1_tile(const float* __restrict__ P, WRing& wr, float* X, const f32x16& feat,
                      const C0Sh& c0sh, float4 dr, DW& dw, const uint32_t (&sm)[3]) {
  const int lane = lane_id();   // opaque: lane-derived LDS addresses are not hoisted out of the loop
  const int h = lane >> 5;
  char* Xb = reinterpret_cast<char*>(X);
  uint32_t mh0 = sm[0], mc0 = sm[1], mc1 = sm[2], mdead = 0;
#define HN_RELU(v, m, ob) relu_bits(v, mdead, ob)
  // ---- forward recompute (models.py:151-174); each GEMM stages its B
  // operand's parts as a dW operand image ----
  f32x16 h0[2] = {zero16(), zero16()};
  gemm2<R_F0, kBF>(wr, P, h0, lane, [&](int s) { return feat[s]; }, Xb);
  HN_RELU(h0[0], mh0, 0);
  HN_RELU(h0[1], mh0, 1);
  const f32x16 s1 = gemm_w<seg_of(R_F1), kBH0>(wr, P, zero16(), lane, [&](int s) { return h0[s >> 4][s & 15]; }, Xb);
  f32x16 c0[2];
  c0sh_seed(c0sh, c0, h);
  // s1 rows 0..15 = [sigma | geo15] -> features 16..31 of [sh16 | sigma | geo15]
  gemm2<R_F2G, kBC0in, 4>(wr, P, c0, lane, [&](int s) { return s1[s]; }, Xb);
  HN_RELU(c0[0], mc0, 0);
  HN_RELU(c0[1], mc0, 1);
  {
    f32x16 c1[2] = {zero16(), zero16()};
    gemm2<R_F3, kBC0>(wr, P, c1, lane, [&](int s) { return c0[s >> 4][s & 15]; }, Xb);
    HN_RELU(c1[0], mc1, 0);
    HN_RELU(c1[1], mc1, 1);
    put_tile(Xb, kBC1, c1[0], lane);
    put_tile(Xb, kBC1 + 1, c1[1], lane);
  }
  if (h == 0) {   // rgb grads: features 0..2 of the kBDR tile (features >= 3 are never stored)
    const SP<2> d = splitn<2>([&](int j) { return j == 0 ? dr.x : j == 1 ? dr.y : j == 2 ? dr.z : 0.f; });
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const u32x4 w = __builtin_bit_cast(u32x4, d.p[q]);
      put_quad(Xb, kBDR, q, lane & 31, 0, w[0], w[1]);
    }
  }
  tile_lds_order();
  // Each layer's weight-gradient products run inside the NEXT data-path GEMM
  // (WgX): its operands are read here, before that GEMM's image writes, and
  // its MFMAs fill the chain's gaps -- per accumulator the same products in
  // the same order as the separate wgrad_n form of round 4 (bitwise-equal dW;
  // step 0.988 -> 0.980 ms, r05i).
  // ---- color_net.2 (dW rows >= 3 are discarded) inside color_net.2^T ----
  WgOps<1, 2> w_c2;
  {
    const int ab[1] = {kBDR}, bb[2] = {kBC1, kBC1 + 1};
    wg_load(w_c2, Xb, ab, bb, lane);
  }
  const float dy2[2] = {h ? dr.y : dr.x, h ? 0.f : dr.z};
  f32x16 dc1[2] = {zero16(), zero16()};
  gemm2<R_B4>(wr, P, dc1, lane, [&](int s) { return s < 2 ? dy2[s] : 0.f; }, nullptr, WgX<1, 2, 1>{w_c2, dw.c2});
  mask_bits(dc1[0], mc1, 0);
  mask_bits(dc1[1], mc1, 1);
  // ---- color_net.1 (dc1 image over c1) ----
  f32x16 dc0[2] = {zero16(), zero16()};
  gemm2<R_B3, kBC1>(wr, P, dc0, lane, [&](int s) { return dc1[s >> 4][s & 15]; }, Xb);
  mask_bits(dc0[0], mc0, 0);
  mask_bits(dc0[1], mc0, 1);
  tile_lds_order();
  // ---- color_net.0 (dc0 image over c0; B = [sh16 | sigma | geo15]), color_net.1's dW inside ----
  WgOps<2, 2> w_c1;
  {
    const int ab[2] = {kBC1, kBC1 + 1}, bb[2] = {kBC0, kBC0 + 1};
    wg_load(w_c1, Xb, ab, bb, lane);            // dw.c1[2 * nb + kb]
  }
  f32x16 ds1 = gemm_w<seg_of(R_B2G), kBC0>(wr, P, zero16(), lane, [&](int s) { return dc0[s >> 4][s & 15]; }, Xb,
                                           WgX<2, 2, 4>{w_c1, dw.c1});
  if (h == 0) ds1[0] = dr.w;                    // row 0 = sigma (A row 0 is zero)
  tile_lds_order();
  // ---- sigma_net.1 (ds1 image over dc1's first tile; rows 16..31 discarded), color_net.0's dW inside ----
  WgOps<2, 1> w_c0;
  {
    const int ab[2] = {kBC0, kBC0 + 1}, bb[1] = {kBC0in};
    wg_load(w_c0, Xb, ab, bb, lane);
  }
  f32x16 dh0[2] = {zero16(), zero16()};
  gemm2<R_B1, kBC1>(wr, P, dh0, lane, [&](int s) { return ds1[s]; }, Xb, WgX<2, 1, 1>{w_c0, dw.c0});
  mask_bits(dh0[0], mh0, 0);
  mask_bits(dh0[1], mh0, 1);
  tile_lds_order();
  // ---- sigma_net.0 (dh0 image over dc0), sigma_net.1's dW inside ----
  WgOps<1, 2> w_s1;
  {
    const int ab[1] = {kBC1}, bb[2] = {kBH0, kBH0 + 1};
    wg_load(w_s1, Xb, ab, bb, lane);
  }
  const f32x16 dfeat = gemm_w<seg_of(R_B0), kBC0>(wr, P, zero16(), lane, [&](int s) { return dh0[s >> 4][s & 15]; },
                                                  Xb, WgX<1, 2, 4>{w_s1, dw.s1});
  tile_lds_order();
  {
    const int ab[2] = {kBC0, kBC0 + 1}, bb[1] = {kBF};
    wgrad_n<2, 1>(Xb, ab, bb, dw.s0, lane);
  }
  static_for<kTileGroups, kTilePeriod - kTileGroups>([&](auto gc) {   // pad groups: keep the ring
    (void)wring_take<decltype(gc)::value>(wr, P, lane);                 // aligned with the tile
  });
  tile_lds_order();                             // image reads done before any later writes
  (void)mdead;
#undef HN_RELU
  return dfeat;
}

// Scatter of one fine tile's table gradient (embedding_dense_backward of
// hash_encoding.py:106 + trilinear backward).  A fine sample that is one of
// the 64 coarse samples (fine_src < 64) is the same point in both passes: its
// coarse-pass feature grads (written by the coarse kernel) are added first,
// so every unique point is scattered once (25 % fewer atomics).
//
// Lane layout: lane = 16 * (2 * xi + f) + point, 16 points per pass.  One
// atomic wave-instruction covers corners (0,j,k) and (1,j,k) of both features
// of 16 points: h(x+1) differs from h(x) only in low bits (prime 1 on x), so
// 7/8 of the x-pairs fall in one 64-byte segment and the four dwords of a
// point go out as ~1 memory request instead of 2 (the float-atomic path is
// request-rate bound for random rows).  Points are consecutive samples along
// the ray and sit along a 16-lane DPP row, so a run of samples inside one
// voxel is summed by a segmented suffix sum of row shifts (no LDS round
// trips, no branches) and only the run head issues atomics.
// DPP row shifts; lanes whose source is outside the row read 0 (bound_ctrl),
// which lets the compiler fold the shift into the consuming VALU op.
template <int CTRL>
HN_DEV uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, true);
}
template <int CTRL>
HN_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, true));
}
constexpr int kRowShr1 = 0x111;              // lane i <- lane i-1 within its row
template <int D> constexpr int kRowShl = 0x100 + D;   // lane i <- lane i+D within its row

// Voxel of one (point, level) for the scatter: cell corner index and
// trilinear weights in the op order of hash_encoding.py:62-72 / :130-140.
HN_DEV void voxel_cw(const GridArgs& g, const float* gsl, const float pt[3], const float xc[3], int l,
                     int32_t cell[3], float w[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float gs = gsl[3 * l + a];
    const float q = (xc[a] - g.bmin[a]) / gs;   // exact IEEE divisions
    const int32_t i = (int32_t)floorf(q);
    const float vmin = (float)i * gs + g.bmin[a];
    const float vmax = vmin + gs;
    w[a] = (pt[a] - vmin) / (vmax - vmin);
    cell[a] = i;
  }
}

// Atomic wave-instructions the scatter wave may have in flight before it
// issues a level's 4 (-1: no cap).  Uncapped, its atomics crowd the CU's
// vector-memory pipeline and the MLP waves' weight loads stall behind them
// (backward 1.59 ms at config 2); capped too tightly, the scatter wave waits
// on atomic latency.  Measured with the f32-MFMA MLP (scripts/variants.sh):
// 1: 1.59 ms, 2: 1.56, 4: 1.496, 6: 1.508.  With the split-f32 MLP and
// Morton-ordered batches (scripts/variants_env.sh, two runs each): 4: 1.282 /
// 1.278 ms, 8: 1.258 / 1.252, 12: 1.275 / 1.274.
#ifndef HN_SW_VMCNT
#define HN_SW_VMCNT 8
#endif
// The cap when the table does not fit the 256 MiB MALL (T >= 21): config 3
// (T=22, B=8192) measured 2.93 / 2.94 ms at cap 8 and 2.82 / 2.82 ms at 4.
#ifndef HN_SW_VMCNT_BIG
#define HN_SW_VMCNT_BIG 4
#endif
// One level of the scatter for the 16 points of a pass; v = this lane's
// point's voxel {cell x, cell y * PY, cell z * PZ, w x, y, z} from the compact
// pass (the prime products are precomputed there: (c + 1) * P = c * P + P,
// and c -> c * P is a bijection, so run heads compare the products).
template <int CAP>   // in-flight atomic cap: HN_SW_VMCNT, or HN_SW_VMCNT_BIG for a table beyond the MALL
HN_DEV void scatter_level_x(const GridArgs& g, float* __restrict__ dtable, const f32x4 v0, const float2 v1,
                            uint32_t l, float gl, int lane) {
  const int pp = lane & 15, xi = lane >> 5;
  const int f = (lane >> 4) & 1;
  const uint32_t cx = (uint32_t)__float_as_int(v0.x), y0 = (uint32_t)__float_as_int(v0.y),
                 z0 = (uint32_t)__float_as_int(v0.z);
  const float w[3] = {v0.w, v1.x, v1.y};
  const uint32_t mask = (1u << g.log2T) - 1u;
  const uint32_t hx = cx + (uint32_t)xi;
  const uint32_t y1 = y0 + kPrimeY, z1 = z0 + kPrimeZ;
  // d feat / d e_c = ((g * fz) * fy) * fx  (trilerp_bwd order), c = 4*xi + jk
  const float fx = xi ? w[0] : 1.f - w[0];
  const float gz0 = gl * (1.f - w[2]), gz1 = gl * w[2];
  float cv[4];
  cv[0] = (gz0 * (1.f - w[1])) * fx;   // j=0 k=0
  cv[1] = (gz1 * (1.f - w[1])) * fx;   // j=0 k=1
  cv[2] = (gz0 * w[1]) * fx;           // j=1 k=0
  cv[3] = (gz1 * w[1]) * fx;           // j=1 k=1
  const uint32_t q0 = dpp_u<kRowShr1>(cx), q1 = dpp_u<kRowShr1>(y0), q2 = dpp_u<kRowShr1>(z0);
  const bool head = pp == 0 || q0 != cx || q1 != y0 || q2 != z0;
  const uint32_t pm = (uint32_t)__ballot(head) & 0xffffu;   // every row sees the same points
  // Segmented suffix sum over runs of samples in one voxel: lane p absorbs
  // lane p+d iff no run starts in (p, p+d].  Step d is only needed when some
  // run is longer than d (k consecutive non-heads = a run of > k samples);
  // the tests are on the wave-uniform head mask, so skipped steps cost nothing.
  const uint32_t nz1 = ~pm & 0xfffeu, nz2 = nz1 & (nz1 >> 1), nz4 = nz2 & (nz2 >> 2);
  auto seg_sum = [&](float (&v)[4]) {
    if (!nz1) return;
    auto absorb = [&](auto dc, int d) {
      const bool same = pp + d < 16 && ((pm >> (pp + 1)) & ((1u << d) - 1u)) == 0u;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float o = dpp_f<decltype(dc)::value>(v[c]);
        v[c] = same ? v[c] + o : v[c];
      }
    };
    absorb(std::integral_constant<int, kRowShl<1>>{}, 1);
    if (nz2) {
      absorb(std::integral_constant<int, kRowShl<2>>{}, 2);
      if (nz4) {
        absorb(std::integral_constant<int, kRowShl<4>>{}, 4);
        if (nz4 & (nz4 >> 4)) absorb(std::integral_constant<int, kRowShl<8>>{}, 8);
      }
    }
  };
  seg_sum(cv);
  if (head) {
    const uint32_t row0 = l << g.log2T;
    const uint32_t hh[4] = {(hx ^ y0 ^ z0) & mask, (hx ^ y0 ^ z1) & mask, (hx ^ y1 ^ z0) & mask,
                            (hx ^ y1 ^ z1) & mask};
    // cap the atomics in flight (they share the CU's vector-memory pipeline
    // with the MLP waves' weight loads); waiting only here, after this
    // level's VALU, overlaps the wait with it
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CAP) : "memory");
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float* dst = reinterpret_cast<float*>(reinterpret_cast<char*>(dtable) +
                                            (row0 + hh[c]) * 8u + 4u * f);
      atomic_add_f32(dst, cv[c]);
    }
  }
}



// ---- fine-tile hand-off ring ----------------------------------------------
// The MLP waves never issue an atomic and the scatter wave never issues a
// global load: a load behind outstanding atomics waits for all of them
// (in-order vmcnt), so mixing the two in one wave exposes the atomic latency.
// Protocol (LDS ints, single consumer): a producer takes ticket t, waits until
// slot t % kSlots has been consumed t / kSlots times, fills it and publishes
// ready[slot] = t + 1; the consumer takes tickets in order.  The producer
// holding the oldest unconsumed ticket never waits, so the ring cannot
// deadlock.  Flags are relaxed LDS atomics ordered by lgkmcnt(0) fences (an
// acquire / release would also wait vmcnt(0), draining the atomics).
struct Ring {
  float* slots;
  int* tick;    // next ticket
  int* ready;   // [kSlots] ticket + 1 of the slot's contents
  int* freed;   // [kSlots] times consumed
  const float* gsl;
};

// Sticky device fault word (hn_device_faults): a bounded wait that runs out
// sets its bit, so a protocol bug ends in an error the host sees, never in a
// hung GPU or in silently partial gradients.
__device__ int g_hn_fault;
enum : int { kFaultSlot = 1, kFaultDrain = 2, kFaultCoarse = 4, kFaultDwBuf = 8 };
constexpr int kSpinCap = 1 << 22;   // iterations of >= 128 cycles: ~0.25 s
HN_DEV void raise_fault(int bit) {
  if (lane_id() == 0) __hip_atomic_fetch_or(&g_hn_fault, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bounded spin on a workgroup-local flag.
HN_DEV void spin_until(int* flag, int need, int fault_bit, int prof_slot = -1) {
  bool ok = false;
  for (int it = 0; it < kSpinCap; ++it) {
    const int v = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (v >= need) {
      ok = true;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  if (!ok) raise_fault(fault_bit);
  asm volatile("" ::: "memory");
}

HN_DEV int lds_load(int* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}

HN_DEV void ring_publish(int* flag, int v) {
  lds_fence_wave();                               // the slot's LDS accesses are done
  if (lane_id() == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A slot: the tile's feature grads [32 points][kXS] ([f][level]), the coarse
// twin's grads added (tw, lane (point, feature h)), depths and the ray.
HN_DEV void fill_slot(float* S, const Ray& r, float z, const f32x16& dfeat, const f32x4 tw[4]) {
  const int lane = lane_id();
  const int p = lane & 31, h = lane >> 5;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int l = h ? tile_level(m, 1) : tile_level(m, 0);
    S[p * kXS + l] = dfeat[2 * m];
    S[p * kXS + 16 + l] = dfeat[2 * m + 1];
  }
  lds_fence_wave();
  // fine grad + twin grad: the order of the former two-kernel scatter
  f32x4* g4 = reinterpret_cast<f32x4*>(S + p * kXS + 16 * h);
#pragma unroll
  for (int c = 0; c < 4; ++c) g4[c] = g4[c] + tw[c];
  if (h == 0) S[kSlotZ + p] = z;
  if (lane == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      S[kSlotR + a] = r.o[a];
      S[kSlotR + 3 + a] = r.d[a];
    }
  }
  lds_fence_wave();
}

constexpr int kMarkB = 4;   // unit-mark bytes per ray (B1K::uflags)
// Samples with d raw = 0 (relu(sigma) = 0) have no gradient at all: the MLP
// backward skips their units and the scatter their feature grads and zero
// records (b1_unit_split, scatter_bins_kernel), unless hn_render_cfg.dense_bwd
// asks for every sample to be computed (B1K / ScK skip_zero = 0).
HN_DEV bool draw_nonzero(const float4& d) {
  return ((__float_as_uint(d.x) | __float_as_uint(d.y) | __float_as_uint(d.z) | __float_as_uint(d.w)) << 1) != 0u;
}

// ---- binned table-gradient scatter (HN_SCATTER=split) ----------------------
// The memory-side float-atomic rate (~20 G requests/s, one per 64-B segment
// of a wave-instruction) bounds the atomic scatter.  The binned scatter sends
// no float atomic to memory: each run head's x-pair of a corner row becomes
// one 20-B record {4 sums: (x0 f0, x0 f1, x1 f0, x1 f1), entry word}, written
// into the region of its bin (2^bin_shift consecutive table entries,
// level-major); bin_reduce_kernel then owns each bin and writes its slice of
// the gradient once.  Entry word = (l << T) + h(x0) | nbits << 28: the x1
// corner's row is h(x0) ^ ((2^nbits - 1) & mask), since the x prime is 1 and
// x1 = x0 + 1 differs from x0 in its trailing ones and the bit above (nbits
// <= 11 for cells <= 1024, so both rows fall in one 2^13-entry bin).
// Layout (floats from bins): vals f32x4 [nbins][kBwdBlocks][cap] (a bin's
// regions are contiguous for its owner) then the overflow lists
// [kBwdBlocks][ovf_per_block]; idx u32 over the same record index; counts u32
// [nbins][kBwdBlocks]; largest |value| per level f32 [16][kBwdBlocks] (the
// owner's fixed-point scale); then the overflow book (OvfBook).  The producer
// counts its records per bin in LDS (ds_add_rtn); a record past its region's
// capacity goes to the block's own overflow list (one more LDS counter), so
// spilling costs no global atomic.  A block's list holds every record the
// block can make (64 samples x 16 levels x 4 corner rows per unit): clumped
// input (a scene box inside the sample range, where every out-of-box sample
// clamps onto the box surface; the coarse levels of a T = 22 table) spills
// but never runs out.  ovf_place_kernel buckets the spilled records by bin so
// that each owner reads only its own.
// kFaultNonFinite: a record input (feature grad or sample point) was NaN / Inf.
// The fixed-point owner pass cannot carry such a value (the reference's
// autograd would propagate it into embeddings[l].grad, hash_encoding.py:106),
// so the gradient of that launch is flagged invalid instead of silently
// dropping the contribution.
enum : int { kFaultBins = 16, kFaultNonFinite = 32, kFaultDeadRow = 64 };

// Record r in memory: the values [nrec] f32x4 then the words [nrec] u32.
// Measured and removed (round 2): groups of 4 records = 4 value quads
// then their 4 entry words (80 B), a record's value and word in one line and
// one write stream per region -- measured slower on config 2 (scatter +5 us,
// owner +6.5 us, two A/B pairs on one box): the owner's value loads then span
// 80-B strides instead of dense 1-KiB runs.  Either way the records take
// 5 * nrec floats from `bins` and the book words follow at bins + 5 * nrec
// (ovf_book's idx base = bins + 4 * nrec).
HN_DEV size_t rec_vofs(size_t r) { return 4 * r; }
HN_DEV size_t rec_wofs(size_t r, size_t nrec) { return 4 * nrec + r; }
// A record store.  The staged pool's runs of records (whole lines, read
// once by the owner pass) are written nontemporally; the direct stores (partial
// lines, scattered over the regions) go through L2 as usual, where their
// lines fill up.  Measured (config 2): direct stores nontemporal too, scatter
// 0.197 -> 0.321 ms; staged runs only, scatter and owner both faster (the L2s
// hold fewer dirty record lines to write back).
template <bool kStaged = false>
HN_DEV void rec_put(float* bins, size_t r, size_t nrec, f32x4 v, uint32_t w) {
  f32x4* pv = reinterpret_cast<f32x4*>(bins + rec_vofs(r));
  uint32_t* pw = reinterpret_cast<uint32_t*>(bins) + rec_wofs(r, nrec);
  if (kStaged) {
    __builtin_nontemporal_store(v, pv);
    __builtin_nontemporal_store(w, pw);
  } else {
    *pv = v;
    *pw = w;
  }
}
struct BinW {
  float* bins;
  size_t nrec;
  unsigned long long* lcnt;   // LDS [nbins]: records of the bin (low 32 bits: the slot
                              // counter), records of it in the current staging phase (high 32)
  uint32_t* lovf;      // LDS: this block's overflow records
  size_t base;         // first record of this block's region of bin 0
  size_t stride;       // records between a block's regions of consecutive bins
  size_t ovf_base;     // first record of this block's overflow list
  uint32_t n_ovf;      // its length
  uint32_t cap, shift;
};

__host__ __device__ inline int64_t sc_units_per_block(int64_t n_rays) {   // scatter_bins_kernel: 3 units per ray
  return (3 * (n_rays > 0 ? n_rays : 1) + kBwdBlocks - 1) / kBwdBlocks;
}
// TV records (the scatter blocks' share of the x-pairs, cubes <= kTvRecMaxCube):
// at most L x ((c + 2) / 2) x (c + 1)^2 pairs over the 256 blocks
constexpr int kTvRecMaxCube = 50;
constexpr size_t kTvRecPerBlock = (16 * ((kTvRecMaxCube + 2) / 2) * (kTvRecMaxCube + 1) * (kTvRecMaxCube + 1) +
                                   kBwdBlocks - 1) / kBwdBlocks;
// a producer's overflow list holds everything it can write: its units' render
// records (64 samples x 16 levels x 4 corner rows each) plus its TV share
__host__ __device__ inline size_t ovf_per_block(int64_t n_rays) {
  return (size_t)sc_units_per_block(n_rays) * 64 * 64 + kTvRecPerBlock;
}
__host__ __device__ inline size_t bin_records(int nbins, int cap, int64_t n_rays) {
  return (size_t)kBwdBlocks * nbins * cap + (size_t)kBwdBlocks * ovf_per_block(n_rays);
}
// Overflow book, u32 words after the counts and level maxima (idx + nrec +
// kBwdBlocks * (nbins + 16)): total spilled, spilled per bin, placement
// cursors, first slot per bin, the scatter blocks' slab-block counter,
// spilled per producer block, record ids (relative to the first overflow
// record) bucketed by bin.  All of it lives in the call's workspace, so
// concurrent hn_render_bwd calls with their own workspaces share nothing.
struct OvfBook {
  uint32_t *cnt, *per_bin, *cur, *first, *slab_next, *blk, *ids;
};
__host__ __device__ inline size_t ovf_book_words(int nbins, int64_t n_rays) {
  return 2 + 3 * (size_t)nbins + kBwdBlocks + (size_t)kBwdBlocks * ovf_per_block(n_rays);
}
__host__ __device__ inline OvfBook ovf_book(uint32_t* idx, size_t nrec, int nbins) {
  OvfBook o;
  o.cnt = idx + nrec + (size_t)kBwdBlocks * (nbins + 16);
  o.per_bin = o.cnt + 1;
  o.cur = o.per_bin + nbins;
  o.first = o.cur + nbins;
  o.slab_next = o.first + nbins;
  o.blk = o.slab_next + 1;
  o.ids = o.blk + kBwdBlocks;
  return o;
}

// max(|a|, |b|, m) for m >= 0 as one v_max3_f32 with abs modifiers: the
// compiler's fmaxf in IEEE mode first quiets each input (v_max_f32 x, x), two
// extra instructions per value.  Plain VALU operands (no MFMA or DPP result
// read here), so the asm needs no hazard padding; the values are finite (a
// non-finite one has already set the fault bit).
HN_DEV float max3_abs(float a, float b, float m) {
  float r;
  asm("v_max3_f32 %0, |%1|, |%2|, %3" : "=v"(r) : "v"(a), "v"(b), "v"(m));
  return r;
}

// Segmented suffix sum over runs of samples in one voxel along a 16-lane
// DPP row (the sum of scatter_level_x): lane pp absorbs lane pp + d iff no
// run head lies in (pp, pp + d]; pm = the row's head mask.  s1..s8:
// wave-uniform "some run is longer than 1 / 2 / 4 / 8" (steps skipped when
// no row needs them; a lane whose row does not, absorbs nothing).
// v + (same ? o : 0) is computed as fma(o, same, v): fma(o, 1, v) rounds
// like v + o, and fma(o, 0, v) = v (up to the sign of a zero v, which no
// record value carries into the owner's integer sums).
// All 4 corner rows of a level at once (the runs, and so `same`, are the
// rows' common ones), each step 16 v_fmac_f32_dpp: left to the compiler, the
// fma is packed into v_pk_fma_f32, which cannot take a DPP source, with a
// v_mov_b32_dpp per value (r05: scatter 0.213 -> 0.202 ms).
#define HN_SEG_FMAC(C, E, D) \
  "v_fmac_f32_dpp %[v" #C #E "], %[v" #C #E "], %[sf] row_shl:" #D " row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
// The steps as one asm block with wave-uniform branches inside (n = steps
// to run): the 16 values enter and leave once, without the copies the
// compiler puts at the joins of separately branched blocks.  Step d's `same`
// is computed in the block (v_cmp writes vcc, s_nop 1 before the v_cndmask
// reads it, as the compiler does); its 4 instructions also give the first
// DPP read its 2 wait states.
#define HN_SEG_SAME(M)                                                                                       \
  "v_lshrrev_b32 %[t], %[sh], %[pm]\n"                                                                       \
  "v_and_b32 %[t], " #M ", %[t]\n"                                                                           \
  "v_cmp_eq_u32 vcc, 0, %[t]\n"                                                                              \
  "s_nop 1\n"                                                                                                \
  "v_cndmask_b32_e64 %[sf], 0, 1.0, vcc\n"
#define HN_SEG_BODY(D)                                                                                       \
  HN_SEG_FMAC(0, 0, D) HN_SEG_FMAC(0, 1, D) HN_SEG_FMAC(0, 2, D) HN_SEG_FMAC(0, 3, D) HN_SEG_FMAC(1, 0, D)    \
  HN_SEG_FMAC(1, 1, D) HN_SEG_FMAC(1, 2, D) HN_SEG_FMAC(1, 3, D) HN_SEG_FMAC(2, 0, D) HN_SEG_FMAC(2, 1, D)    \
  HN_SEG_FMAC(2, 2, D) HN_SEG_FMAC(2, 3, D) HN_SEG_FMAC(3, 0, D) HN_SEG_FMAC(3, 1, D) HN_SEG_FMAC(3, 2, D)    \
  HN_SEG_FMAC(3, 3, D)
HN_DEV void seg_sum16(float (&v)[4][4], uint32_t pm, int pp, bool s1, bool s2, bool s4, bool s8) {
  // wave-uniform (from ballots); readfirstlane keeps it in an SGPR
  const int n = __builtin_amdgcn_readfirstlane(s1 ? (s2 ? (s4 ? (s8 ? 4 : 3) : 2) : 1) : 0);
  float t, sf;
  asm("s_cmp_eq_u32 %[n], 0\n s_cbranch_scc1 Lseg_end%=\n"
      HN_SEG_SAME(1) HN_SEG_BODY(1)
      "s_cmp_eq_u32 %[n], 1\n s_cbranch_scc1 Lseg_end%=\n"
      HN_SEG_SAME(3) HN_SEG_BODY(2)
      "s_cmp_eq_u32 %[n], 2\n s_cbranch_scc1 Lseg_end%=\n"
      HN_SEG_SAME(15) HN_SEG_BODY(4)
      "s_cmp_eq_u32 %[n], 3\n s_cbranch_scc1 Lseg_end%=\n"
      HN_SEG_SAME(0xff) HN_SEG_BODY(8)
      "Lseg_end%=:\n"
      : [v00] "+v"(v[0][0]), [v01] "+v"(v[0][1]), [v02] "+v"(v[0][2]), [v03] "+v"(v[0][3]),
        [v10] "+v"(v[1][0]), [v11] "+v"(v[1][1]), [v12] "+v"(v[1][2]), [v13] "+v"(v[1][3]),
        [v20] "+v"(v[2][0]), [v21] "+v"(v[2][1]), [v22] "+v"(v[2][2]), [v23] "+v"(v[2][3]),
        [v30] "+v"(v[3][0]), [v31] "+v"(v[3][1]), [v32] "+v"(v[3][2]), [v33] "+v"(v[3][3]),
        [t] "=&v"(t), [sf] "=&v"(sf)
      : [n] "s"(n), [sh] "v"((uint32_t)pp + 1u), [pm] "v"(pm)
      : "vcc", "scc");
}
#undef HN_SEG_SAME
#undef HN_SEG_BODY
#undef HN_SEG_FMAC

// round(v * 2^S) as int64 without f64 arithmetic: x = v * 2^S is exact in fp32
// (|x| < 2^47, a power-of-2 scale), a = trunc(x / 2^16) is an exact integer
// (|a| < 2^31),
// b = x - a * 2^16 exact with |b| < 2^16, and round(x) = a * 2^16 + rint(b)
// (ties to even agree: a * 2^16 is even).
HN_DEV long long fx_of(float v, float scale) {
  const float x = v * scale;
  const float a = truncf(x * 0x1p-16f);
  const float b = __builtin_fmaf(-a, 0x1p16f, x);
  return ((long long)(int32_t)a << 16) + (long long)(int32_t)rintf(b);
}

// A run head's record: the x-pair (x0 = cx, x1 = cx + 1) of corner row (yy, zz)
// (the y / z coordinates times their primes) at level l.  rec_slot takes the
// record's slot in its bin (LDS counter); rec_store writes it -- split so a
// caller can have several counter round trips in flight.
struct RecSlot {
  uint32_t word, bin, slot, pj;   // pj: the record's index among the bin's records of the staging phase
};
// staged = count the record in the bin's staging-phase half too (one 64-bit
// LDS add returns both counts: the staging index needs no separate read of
// the phase's first slot)
constexpr unsigned long long kCntRec = 1ull, kCntStaged = (1ull << 32) | 1ull;
HN_DEV RecSlot rec_slot(const BinW& bw, uint32_t l, uint32_t log2T, uint32_t cx, uint32_t yy, uint32_t zz,
                        unsigned long long inc = kCntRec) {
  const uint32_t mask = (1u << log2T) - 1u;
  const uint32_t flat = (l << log2T) + ((cx ^ yy ^ zz) & mask);
  const uint32_t nbits = (uint32_t)__builtin_ctz(~cx) + 1u;
  RecSlot r;
  r.word = flat | (nbits << 28);
  r.bin = flat >> bw.shift;
  const unsigned long long old =
      __hip_atomic_fetch_add(bw.lcnt + r.bin, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  r.slot = (uint32_t)old;
  r.pj = (uint32_t)(old >> 32);
  return r;
}
HN_DEV void rec_store(const BinW& bw, const RecSlot& rs, const float (&v)[4]) {
  size_t r = bw.base + (size_t)rs.bin * bw.stride + rs.slot;
  bool ok = true;
  if (rs.slot >= bw.cap) {
    const uint32_t o = __hip_atomic_fetch_add(bw.lovf, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    ok = o < bw.n_ovf;   // always, by the list's size
    r = bw.ovf_base + o;
    if (!ok) __hip_atomic_fetch_or(&g_hn_fault, kFaultBins, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (ok) {
    rec_put(bw.bins, r, bw.nrec, f32x4{v[0], v[1], v[2], v[3]}, rs.word);
  }
}

// Voxel of one (point, level) for the split scatter: the cell from cell_floor
// (the forward's), the weights by the reference's IEEE divisions.
HN_DEV void voxel_cw_sc(const GridArgs& g, const float* gsl, const float pt[3], const float xc[3], int l,
                        int32_t cell[3], float w[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float gs = gsl[3 * l + a];
    const int32_t i = cell_floor(xc[a] - g.bmin[a], gs, gsl[kGsRcp + 3 * l + a]);
    const float vmin = (float)i * gs + g.bmin[a];
    const float vmax = vmin + gs;
    w[a] = div_rn(pt[a] - vmin, vmax - vmin);
    cell[a] = i;
  }
}

// ---- split backward: the table-gradient scatter as its own kernel ---------
// kModeSplit's render_bwd_kernel stores each fine tile's feature grads; this
// kernel then runs the scatter at full occupancy (16 waves per CU) instead of
// in one wave per SIMD next to the MLP waves.  One wave per (ray, third of
// its 192 fine samples), lane = sample: its point o + d z, its grads (fine +
// coarse twin, the order of the fused ring), its voxel computed once per
// level; per corner row the x-pair sums over runs of samples in one voxel
// (16-lane rows, as in the fused scatter) and one record per run head.  Block
// b is producer b of the record layout (kBwdBlocks blocks).
// Coarse-pass feature grads, per ray: 64 samples x 32 features (workspace-internal)
constexpr size_t kDcRay = (size_t)kSc * 32;
// dW(coarse) (+)= sum_b slab[b][0], dW(fine) (+)= sum_b (slab[b][1] +
// slab[b][2] + slab[b][3]).  64 consecutive elements per block, kSlabGroups
// slab-groups per element (8 loads in flight per thread, ~18 waves per CU: the
// read is latency bound otherwise), LDS combine in a fixed order, so the sums
// are deterministic given the slabs.
constexpr int kSlabGroups = 16;
constexpr int kSlabIlp = 8;   // slab loads in flight per thread (a power of 2)
// One slab-reduce block's 64 elements (vblock): the arithmetic of every
// element is fixed (the group partials, then the pairwise combines), so the
// sums are the same whichever kernel runs it (slab_reduce_kernel, or the
// binned scatter's tail).  1024 threads; part[16][64] in LDS.
// ms (binned scatter, optional): the ten NeRFSmall tensors' RAdam steps
// ([network_fn's 5 | network_fine's 5], hn_mlp order), applied to each element
// with its final gradient (radam_kernel's update) where that is formed.
HN_DEV void slab_reduce_block(const float* __restrict__ slab, int n_blocks, const hn_mlp_grad& dc,
                              const hn_mlp_grad& df, int overwrite, int vblock, float (*part)[64],
                              const hn_radam_tensor* ms = nullptr, const int32_t* gsplit = nullptr) {
  const int lane = threadIdx.x & 63;
  const int e = vblock * 64 + lane;
  const int grp = threadIdx.x >> 6;
  const bool fine = e >= W_END;
  const int i = fine ? e - W_END : e;
  // the slabs summed for this element.  gsplit (the split schedule's balanced
  // unit lists): one slab per MLP wave g = wave * n_blocks + block, waves
  // g < *gsplit coarse, the others fine; otherwise (block, slot) pairs, slot
  // 0 (coarse) or 1..3 (fine), flattened
  const int gs = gsplit ? *gsplit : 0;
  const int per = fine ? kSlabSlots - 1 : 1;
  // HN_DW_BLOCKRED: only each block's run leaders hold a slab -- coarse: the
  // waves 4j < gs; fine: gs, then the waves 4j > gs
  const int n_lead = fine ? (kSlabSlots * n_blocks) / 4 - gs / 4 : (gs + 3) / 4;
  const int n_slabs = gsplit ? (HN_DW_BLOCKRED ? n_lead : (fine ? kSlabSlots * n_blocks - gs : gs)) : n_blocks * per;
  auto slab_at = [&](int q) {
    if (gsplit && HN_DW_BLOCKRED) {
      const int g = !fine ? 4 * q : (gs % 4 == 0 ? gs + 4 * q : (q == 0 ? gs : 4 * (gs / 4 + q)));
      return slab[(size_t)g * W_END + i];
    }
    if (gsplit) return slab[(size_t)(fine ? gs + q : q) * W_END + i];
    const int b = q / per, slot = fine ? 1 + q % per : 0;
    return slab[((size_t)b * kSlabSlots + slot) * W_END + i];
  };
  float s = 0.f;
  if (e < 2 * W_END) {
    float acc[kSlabIlp];
#pragma unroll
    for (int u = 0; u < kSlabIlp; ++u) acc[u] = 0.f;
    int q = grp;
    for (; q + (kSlabIlp - 1) * kSlabGroups < n_slabs; q += kSlabIlp * kSlabGroups)
#pragma unroll
      for (int u = 0; u < kSlabIlp; ++u) acc[u] += slab_at(q + kSlabGroups * u);
    for (; q < n_slabs; q += kSlabGroups) acc[0] += slab_at(q);
#pragma unroll
    for (int w = kSlabIlp / 2; w >= 1; w /= 2)   // pairwise, fixed order
#pragma unroll
      for (int u = 0; u < w; ++u) acc[u] = acc[u] + acc[u + w];
    s = acc[0];
  }
  part[grp][lane] = s;
  __syncthreads();
  if (grp == 0 && e < 2 * W_END) {
    float t[kSlabGroups];
#pragma unroll
    for (int g = 0; g < kSlabGroups; ++g) t[g] = part[g][lane];
#pragma unroll
    for (int w = kSlabGroups / 2; w >= 1; w /= 2)
#pragma unroll
      for (int g = 0; g < w; ++g) t[g] = t[g] + t[g + w];
    s = t[0];
    const hn_mlp_grad& d = fine ? df : dc;
    const int ly = i < W_S1 ? 0 : i < W_C0 ? 1 : i < W_C1 ? 2 : i < W_C2 ? 3 : 4;   // the torch tensor
    const int j = i - (ly == 0 ? 0 : ly == 1 ? W_S1 : ly == 2 ? W_C0 : ly == 3 ? W_C1 : W_C2);
    float* dst = (ly == 0 ? d.sigma0 : ly == 1 ? d.sigma1 : ly == 2 ? d.color0 : ly == 3 ? d.color1 : d.color2) + j;
    const float gv = overwrite ? s : *dst + s;
    *dst = gv;
    if (ms) {
      const hn_radam_tensor& r = ms[(fine ? 5 : 0) + ly];
      float p = r.p[j], m = r.m[j], v = r.v[j];
      radam_elem(r, p, gv, m, v);
      r.m[j] = m;
      r.v[j] = v;
      if (r.mode != 0) r.p[j] = p;
    }
  }
}
constexpr int kSlabVBlocks = (2 * W_END + 63) / 64;
struct ScK {
  GridArgs g;
  int64_t B;
  const float* rays;
  const float* z_fine;
  const uint8_t* fine_src;
  const float* dfeat_f;   // [B][6][1024] tile order (split render_bwd_kernel)
  const float* dfeat_c;   // [B][2][1024] tile order (coarse units of the split render_bwd_kernel)
  const float* draw;      // [B][64 + 192][4] d raw (composite pre-pass): zero = no feature grads to read
  int32_t scramble;       // the MLP backward's ray permutation (B1K::scramble; 0: identity)
  int32_t skip_zero;      // exact-zero skipping (!hn_render_cfg.dense_bwd)
  const int32_t* lmeta;   // render_lists_kernel's counts ([2] scatter groups, [3] the MLP waves' split)
  const int32_t* slist;   // its scatter group codes (ray << 4 | 16-sample group), or null: every unit
  float* bins;
  int32_t bin_cap, bin_shift, nbins;
  // TV term (loss.py:11-43) as records of the same bins: tv_off[l] = first
  // x-pair of level l (tv_off[L] pairs in all; 0 = no TV term), split evenly
  // over the blocks after their units
  int32_t tv_off[17];
  const float* g_tv;
  TvK tv;
  // The blocks then reduce the MLP backward's dW slabs (the
  // slab_reduce_kernel launch folded into this one; same per-element sums)
  const float* slab;       // NULL: no slab reduction here
  hn_mlp_grad dc, df;
  int32_t overwrite_mlp;
  int32_t has_mstep;       // the NeRFSmall tensors' RAdam steps run in the slab reduction (mstep)
  hn_radam_tensor mstep[10];
};
constexpr int kScWaves = 16;
constexpr int kScMaxBinsLog2 = 13;
constexpr int kScMaxBins = 1 << kScMaxBinsLog2;   // LDS counters (32 KiB): T <= 22 at 2^13 entries per bin
#ifndef HN_BIN_SHIFT_DEFAULT
#define HN_BIN_SHIFT_DEFAULT 13
#endif
constexpr int kBinShift = HN_BIN_SHIFT_DEFAULT;   // preferred log2 entries per bin (bin_geom)

// Record staging: level-major phases across the block's waves (all 16 waves
// take level l of their units, then the block syncs), each head lane's record
// put into an LDS pool at (bin of the level, slot - the bin's first slot of the
// phase) and the pool flushed by the block in slot order: a bin's records of
// the phase leave as contiguous runs (one 16-B value and one word per lane,
// consecutive lanes on consecutive slots) instead of 64 scattered 16-B and 4-B
// stores per instruction.  Records past the pool's share of their bin (2^kStLog2
// records over the level's bins) or past the region's capacity are stored
// directly.  The slot of every record is the same as without staging, so the
// record buffer, and the owner's sums, are identical.  Measured (r03g, config
// 2): WRITE_SIZE 548 -> 395 MB per launch for 352 MB of records (1.56x ->
// 1.12x), backward launch time unchanged (0.813 / 0.814 vs 0.813 / 0.812 ms):
// the scatter waits on its own dependency chains (SQ_WAIT_INST_ANY 44% of its
// wave cycles), not on the write traffic.
constexpr int kStLog2 = 12, kStPool = 1 << kStLog2;   // 64 KiB of values + 16 KiB of words
constexpr int kStMinLog2C = 3;                          // fewer than 8 records per bin: no staging
constexpr size_t kLdsMax = 160 * 1024;
__global__ void scatter_bins_kernel(ScK k);
// the kernel's static LDS, read once from the code object (a
// constant here would silently go stale if the static arrays grow)
static size_t sc_static_lds() {
  static size_t v = 0;
  if (!v) {
    hipFuncAttributes at{};
    v = hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&scatter_bins_kernel)) == hipSuccess
            ? at.sharedSizeBytes : (size_t)16 * 1024;
  }
  return v;
}
// dynamic LDS of scatter_bins_kernel: the bins' counters, then the staging pool
static size_t sc_lds_bytes(int nbins) {
  return (size_t)((nbins + 3) & ~3) * 8 + (size_t)kStPool * 20;
}
struct StPhase {
  int b0, log2c;   // first bin of the phase's levels, log2 pool records per bin (< kStMinLog2C: direct)
  int nbl;         // bins of the phase's levels
};
// a staging phase: levels l .. l + 2^lg2n - 1 (their bins are consecutive;
// several levels per phase only where every level owns whole bins)
HN_DEV StPhase st_phase(int l, int log2T, int shift, int lg2n = 0) {
  StPhase ph;
  ph.b0 = (int)(((uint32_t)l << log2T) >> shift);
  const int lg = log2T > shift ? log2T - shift : 0;
  ph.nbl = 1 << (lg + lg2n);
  ph.log2c = kStLog2 - lg - lg2n;
  return ph;
}
// log2 levels per staging phase where the pool still holds 8 records per bin
// (one block barrier pair per phase; r05h: 1 level 0.984-0.987 ms per step,
// 2: 0.988-1.005, 4: 1.012-1.014, 8: 1.037-1.039)
constexpr int kScLpp = 1;

__global__ __launch_bounds__(64 * kScWaves) void scatter_bins_kernel(ScK k) {
  // dynamic LDS: the bins' record counters, then the staging pool
  // (sc_lds_bytes)
  extern __shared__ __attribute__((aligned(16))) uint32_t sc_dyn[];
  unsigned long long* const bcnt = reinterpret_cast<unsigned long long*>(sc_dyn);   // BinW::lcnt
  __shared__ float gsl[kGsLds], lvmx[16];
  __shared__ uint32_t lovf;
  __shared__ uint32_t lvmxl[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += blockDim.x) lvmxl[i] = 0u;
  // wave-uniform work-unit arithmetic (u, ray = u / 3, u % 3, act) on the scalar unit
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = lane_id();
  for (int i = threadIdx.x; i < k.nbins; i += blockDim.x) bcnt[i] = 0ull;
  if (threadIdx.x < 16) lvmx[threadIdx.x] = 0.f;
  if (threadIdx.x == 0) lovf = 0u;
  stage_grid_sizes(k.g, gsl);
  __syncthreads();
  BinW bw;
  const size_t nrec = bin_records(k.nbins, k.bin_cap, k.B);
  bw.bins = k.bins;
  bw.nrec = nrec;
  uint32_t* const book = reinterpret_cast<uint32_t*>(k.bins + 4 * nrec);
  const OvfBook ob = ovf_book(book, nrec, k.nbins);
  bw.lovf = &lovf;
  bw.n_ovf = (uint32_t)ovf_per_block(k.B);
  bw.lcnt = bcnt;
  bw.base = (size_t)blockIdx.x * k.bin_cap;
  bw.stride = (size_t)kBwdBlocks * k.bin_cap;
  bw.ovf_base = (size_t)kBwdBlocks * k.nbins * k.bin_cap + (size_t)blockIdx.x * bw.n_ovf;

  bw.cap = (uint32_t)k.bin_cap;
  bw.shift = (uint32_t)k.bin_shift;
  // The block's units.  With exact-zero skipping: its slice of the list of
  // fine 16-sample groups that have feature grads to scatter
  // (render_lists_kernel, from the composite pre-pass's marks), the list in
  // ray order and cut into equal slices over the blocks -- every block the
  // same share of the work, whatever the scene leaves nonzero; a wave's unit
  // is four consecutive groups of the slice, one per 16-lane run row (often of
  // different rays; runs never cross rows, so the records are the dense
  // form's).  Otherwise (dense_bwd) every unit is a third of one ray's fine
  // samples, the rays permuted as the MLP backward's (unit_ray).
  const bool use_list = k.slist != nullptr;
  int64_t u0 = 0, u1 = 0;
  int64_t s0 = 0, s1 = 0;   // this block's slice of the group list
  if (use_list) {
    const int64_t Ns = __builtin_amdgcn_readfirstlane(k.lmeta[2]);
    s0 = (int64_t)blockIdx.x * Ns / gridDim.x;
    s1 = (int64_t)(blockIdx.x + 1) * Ns / gridDim.x;
    u1 = (s1 - s0 + 3) / 4;   // a unit = four consecutive groups of the slice, one per 16-lane row
  } else {
    const int64_t units = 3 * k.B;
    const int64_t per = (units + gridDim.x - 1) / gridDim.x;
    u0 = (int64_t)blockIdx.x * per;
    u1 = u0 + per < units ? u0 + per : units;
  }
  const int pp = lane & 15;
  // the staging pool: 80 KiB
  uint32_t* const st_raw = sc_dyn + 2 * ((k.nbins + 3) & ~3);   // 16-B aligned after the counters
  f32x4* const stv = reinterpret_cast<f32x4*>(st_raw);
  uint32_t* const stw = st_raw + 4 * kStPool;
  __shared__ uint32_t stfl[2][kStPool >> kStMinLog2C];   // per phase parity: first staged slot per bin
  const int log2T = (int)k.g.log2T, sh = k.bin_shift;
  // first staged slot of each bin of level l (the bins' counts so far, capped)
  // (stfl alternates between phases: par = the phase's parity)
  int par = 0;
  auto st_init = [&](const StPhase& ph, int pr) {
    if (ph.log2c < kStMinLog2C) return;
    for (int i = threadIdx.x; i < ph.nbl; i += blockDim.x) {
      const unsigned long long c = bcnt[ph.b0 + i];
      stfl[pr][i] = min((uint32_t)c, bw.cap);
      bcnt[ph.b0 + i] = c & 0xffffffffull;   // the phase's count from 0 (no atomics in flight on it now)
    }
  };
  // the pool's records of level l to their regions, in slot order
  auto st_flush = [&](const StPhase& ph) {
    if (ph.log2c < kStMinLog2C) return;
    const uint32_t c = 1u << ph.log2c;
    for (int p = threadIdx.x; p < kStPool; p += blockDim.x) {
      const int bl = p >> ph.log2c, b = ph.b0 + bl;
      const uint32_t j = (uint32_t)p & (c - 1u), f = stfl[par][bl];
      const uint32_t end = min(min((uint32_t)bcnt[b], bw.cap), f + c);
      if (f + j < end) {
        const size_t r = bw.base + (size_t)b * bw.stride + f + j;
        rec_put<true>(bw.bins, r, bw.nrec, stv[p], stw[p]);
      }
    }
  };
  const int64_t n_it = (u1 - u0 + kScWaves - 1) / kScWaves;   // the same for every wave of the block
  // one unit's inputs: its ray, point and (fine + coarse twin) grads of one level
  struct Unit {
    bool act;
    Ray r;
    float pt[3], xc[3];
    const float* tb;   // the sample's fine grads (tile order), or null: exactly zero
    const float* tw;   // its coarse twin's grads, or null (none, or exactly zero)
    float g0, g1;      // the current level's two feature grads (fine + coarse twin)
  };
  bool bad = false;   // a non-finite grad or point seen by this lane
  // the MLP backward's ray order (render_bwd_kernel's block_ray): block b's
  // units are the rays MLP block b processed, spread over the batch, so the
  // units without any gradient (below) spread evenly over the blocks
#ifndef HN_SC_CHUNK
#define HN_SC_CHUNK 1
#endif
  auto unit_ray = [&](int64_t j) -> int64_t {
    if (HN_SC_CHUNK == 0) return j;
    if (HN_SC_CHUNK > 1 && k.B % HN_SC_CHUNK == 0 && k.B >= 4 * HN_SC_CHUNK) {
      // chunks of HN_SC_CHUNK consecutive (Morton-neighbour) rays, the chunks
      // permuted over the batch
      int bits = 2;
      while ((1ll << bits) < k.B / HN_SC_CHUNK) bits += 2;
      uint32_t c = (uint32_t)(j / HN_SC_CHUNK);
      do {
        c = feistel(c, bits / 2, 0x5bd1e995u);
      } while ((int64_t)c >= k.B / HN_SC_CHUNK);
      return (int64_t)c * HN_SC_CHUNK + j % HN_SC_CHUNK;
    }
    uint32_t x = (uint32_t)j;
    if (k.scramble) {
      do {
        x = feistel(x, k.scramble, 0x5bd1e995u);
      } while ((int64_t)x >= k.B);
    }
    return (int64_t)x;
  };
  // unit u0 + wave + it * kScWaves: its ray, the lane's sample point and grad rows
  auto unit_base = [&](int64_t it) {
    Unit q;
    const int64_t u = u0 + wave + it * kScWaves;
    q.act = u < u1;
    q.g0 = q.g1 = 0.f;
    q.tb = q.tw = nullptr;
    if (q.act) {
      int64_t ray;
      int i;   // the lane's fine sample
      bool none = false;   // a second tile that does not exist: no grads
      if (use_list) {
        // row r of the unit: group s0 + 4 u + r, a group of 16 consecutive
        // samples of one ray -- the run rows are the dense form's, so the
        // records are too (minus the all-zero ones)
        const int64_t gj = s0 + 4 * u + (lane >> 4);
        const int c0 = k.slist[s0 + 4 * u];
        const int code = gj < s1 ? k.slist[gj] : c0;
        none = gj >= s1;
        ray = code >> 4;
        i = 16 * (code & 15) + (lane & 15);
      } else {
        ray = unit_ray(u / 3);
        i = 64 * (int)(u % 3) + lane;
      }
      {
        const float* rb = k.rays + 11 * ray;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          q.r.o[a] = rb[a];
          q.r.d[a] = rb[3 + a];
        }
      }
      ray_point(q.r, k.z_fine[ray * kSf + i], q.pt);
#pragma unroll
      for (int a = 0; a < 3; ++a) q.xc[a] = clamp_t(q.pt[a], k.g.bmin[a], k.g.bmax[a]);
      bad |= !(fabsf((q.pt[0] + q.pt[1]) + q.pt[2]) <= 3.402823466e38f);
      // a sample whose d raw is exactly zero has exactly zero feature grads (the
      // MLP backward did not store them: b1_unit_split's skip); the same for
      // its coarse twin
      const float* dr = k.draw + (size_t)ray * (kSc + kSf) * 4;
      if (!none && (!k.skip_zero || draw_nonzero(*reinterpret_cast<const float4*>(dr + 4 * (kSc + i)))))
        q.tb = k.dfeat_f + ((size_t)ray * (kSf / 32) + (i >> 5)) * 1024 + 4 * (i & 31);
      const int src = k.fine_src[ray * kSf + i];
      if (!none && src < kSc && (!k.skip_zero || draw_nonzero(*reinterpret_cast<const float4*>(dr + 4 * src))))
        q.tw = k.dfeat_c + (size_t)ray * kDcRay + (size_t)(src >> 5) * 1024 + 4 * (src & 31);
      // no lane with a gradient: the unit writes no record (wave-uniform)
      q.act = __ballot(q.tb != nullptr || q.tw != nullptr) != 0ull;
    }
    return q;
  };
  // level l's grads = elements 2 (l & 1) .. of level pair l / 2 (tile_level:
  // chunk lp / 2 of lane half lp % 2); a coarse twin adds its coarse grads
  // (the fused ring's order); no twin: the fine grads as they are.  (Loading
  // level l + 1's while level l runs measured no faster, r05g.)
  auto unit_grads = [&](Unit& q, int l) {
    if (!q.act) return;
    const int lp = l >> 1, o = 4 * (64 * (lp >> 1) + 32 * (lp & 1)) + 2 * (l & 1);
    float2 gq = q.tb ? *reinterpret_cast<const float2*>(q.tb + o) : make_float2(0.f, 0.f);
    if (q.tw) {
      const float2 t = *reinterpret_cast<const float2*>(q.tw + o);
      gq = make_float2(gq.x + t.x, gq.y + t.y);
    }
    q.g0 = gq.x;
    q.g1 = gq.y;
    bad |= !(fabsf(gq.x + gq.y) <= 3.402823466e38f);
  };
  // The records of one level of a unit: voxel, run heads, per corner row the
  // x-pair sums over runs of samples in one voxel (16-lane rows), then each
  // head lane's record into the staging pool, or stored directly (slots from
  // the LDS counters)
  auto level = [&](const Unit& q, const int l, const StPhase& ph) {
    if (!q.act) return;
    const bool staged = ph.log2c >= kStMinLog2C;
    int32_t cell[3];
    float w[3];
    voxel_cw_sc(k.g, gsl, q.pt, q.xc, l, cell, w);
    const uint32_t cx = (uint32_t)cell[0], y0 = (uint32_t)cell[1] * kPrimeY, z0 = (uint32_t)cell[2] * kPrimeZ;
    const uint32_t q0 = dpp_u<kRowShr1>(cx), q1 = dpp_u<kRowShr1>(y0), q2 = dpp_u<kRowShr1>(z0);
    bool head = pp == 0 || q0 != cx || q1 != y0 || q2 != z0;
    const uint64_t hb = __ballot(head);
    const uint32_t pm = ((uint32_t)(hb >> (lane & 48)) & 0xffffu) | 0x10000u;   // + virtual head 16 (seg_same)
    // lane 0 of every row is a head, so these never carry across rows
    const uint64_t nz1 = ~hb & 0xfffefffefffefffeull, nz2 = nz1 & (nz1 >> 1), nz4 = nz2 & (nz2 >> 2);
    const bool s1 = nz1 != 0ull, s2 = nz2 != 0ull, s4 = nz4 != 0ull, s8 = (nz4 & (nz4 >> 4)) != 0ull;
    const float az = 1.f - w[2], ay = 1.f - w[1], ax = 1.f - w[0];
    // d feat / d e_c = ((g * wz) * wy) * wx (trilerp_bwd's order)
    // the two features as one packed pair (v_pk_mul_f32: the same fp32
    // products, half the instructions; the asm below would otherwise leave
    // them unpacked)
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 g2 = {q.g0, q.g1};
    const f2 gz[2] = {g2 * az, g2 * w[2]};   // [k] (features f0, f1)
    float vmax = 0.f;   // largest |record value| of the level: the owner's fixed-point scale
    float v[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j = c >> 1, kk = c & 1;
      const float wy = j ? w[1] : ay;
      const f2 a = gz[kk] * wy;
      const f2 x0 = a * ax, x1 = a * w[0];
      v[c][0] = x0.x; v[c][1] = x0.y; v[c][2] = x1.x; v[c][3] = x1.y;
    }
    seg_sum16(v, pm, pp, s1, s2, s4, s8);
#pragma unroll
    for (int c = 0; c < 4; ++c) vmax = max3_abs(v[c][2], v[c][3], max3_abs(v[c][0], v[c][1], vmax));
    RecSlot rs[4];
    // a run whose four sums are exactly zero (samples without gradient, or a
    // zero trilinear weight) adds nothing to the owner's integer sums: no
    // record (the same table gradient bitwise; not with dense_bwd)
    bool put[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
      put[c] = head && (!k.skip_zero || ((__float_as_uint(v[c][0]) | __float_as_uint(v[c][1]) |
                                           __float_as_uint(v[c][2]) | __float_as_uint(v[c][3])) << 1) != 0u);
    if (head) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {   // 4 counter round trips in flight
        const int j = c >> 1, kk = c & 1;
        if (put[c])
          rs[c] = rec_slot(bw, (uint32_t)l, (uint32_t)log2T, cx, j ? y0 + kPrimeY : y0, kk ? z0 + kPrimeZ : z0,
                           staged ? kCntStaged : kCntRec);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (!put[c]) continue;
        // staged index = the record's place among the bin's records of this
        // phase (its slot minus the phase's first slot whenever slot < cap)
        const uint32_t bl = rs[c].bin - (uint32_t)ph.b0, j = rs[c].pj;
        if (staged && rs[c].slot < bw.cap && j < (1u << ph.log2c)) {
          const int qq = (int)((bl << ph.log2c) + j);
          stv[qq] = f32x4{v[c][0], v[c][1], v[c][2], v[c][3]};
          stw[qq] = rs[c].word;
          continue;
        }
        rec_store(bw, rs[c], v[c]);
      }
    }
    __hip_atomic_fetch_max(&lvmxl[l * 64 + lane], __float_as_uint(vmax), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  // staging phases of 2^lpp levels where each level owns whole bins and the
  // pool still holds >= 2^kStMinLog2C records per bin (T=19: 2 levels per
  // phase, 32 records per bin; T=22: 1 level, 8 per bin)
  const int lg_bins = log2T - sh;   // log2 bins per level
  const int lpp = lg_bins < 0 ? 0 : max(0, min(kScLpp, kStLog2 - kStMinLog2C - lg_bins));
  auto phase_of = [&](int l) { return st_phase(l, log2T, sh, l + (1 << lpp) <= 16 ? lpp : 0); };
  st_init(phase_of(0), par);
  __syncthreads();
  // the levels unit by unit (each unit's ray and rows loaded once), their
  // records through the staging pool, one phase per (unit round, level group)
  for (int64_t it = 0; it < n_it; ++it) {
    Unit q = unit_base(it);
    for (int l = 0; l < 16;) {
      const StPhase ph = phase_of(l);
      const int np = l + (1 << lpp) <= 16 ? 1 << lpp : 1;
      for (int j = 0; j < np; ++j, ++l) {
        unit_grads(q, l);
        level(q, l, ph);
      }
      __syncthreads();   // the phase's records are in the pool, its counts final
      st_flush(ph);
      // the next phase's bins (other parity), counts unchanged by the flush
      const int ln = l < 16 ? l : (it + 1 < n_it ? 0 : 16);
      if (ln < 16) st_init(phase_of(ln), par ^ 1);
      __syncthreads();   // the pool is free again
      par ^= 1;
    }
  }
  // non-finite inputs (NaN / Inf in a grad or the point): one test per lane
  if (__ballot(bad) != 0ull && lane == 0)
    __hip_atomic_fetch_or(&g_hn_fault, kFaultNonFinite, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (k.tv_off[16] > 0) {
    // The TV term's table gradient: one record per x-pair (x0, x0 + 1) of cube
    // vertices of one (y, z) row, d TV_l / d e (tv_grad) scaled by g_tv[l] /
    // cube, through the same region / overflow path as the render records
    // (so the owner pass sums render + TV exactly and the table step stays fused)
    const int total = k.tv_off[16], per = (total + (int)gridDim.x - 1) / (int)gridDim.x;
    const int q0 = (int)blockIdx.x * per, q1 = q0 + per < total ? q0 + per : total;
    const uint32_t T = (uint32_t)k.g.log2T;
    for (int q = q0 + (int)threadIdx.x; q < q1; q += (int)blockDim.x) {
      int l = 0;
      while (l + 1 < k.tv.L && q >= k.tv_off[l + 1]) ++l;
      const int c = k.tv.cube[l], n1 = c + 1, np = (n1 + 1) / 2, loc = q - k.tv_off[l];
      const int ip = loc % np, j = (loc / np) % n1, kk = loc / (np * n1);
      const uint32_t x0 = (uint32_t)(k.tv.mv[3 * l] + 2 * ip), y = (uint32_t)(k.tv.mv[3 * l + 1] + j),
                     z = (uint32_t)(k.tv.mv[3 * l + 2] + kk);
      const float scale = k.g_tv[l] / (float)c;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int f = 0; f < 2; ++f) v[f] = scale * tv_grad(k.tv, l, c, 2 * ip, j, kk, x0, y, z, f);
      if (2 * ip + 1 <= c)
#pragma unroll
        for (int f = 0; f < 2; ++f) v[2 + f] = scale * tv_grad(k.tv, l, c, 2 * ip + 1, j, kk, x0 + 1u, y, z, f);
      const float chk = (v[0] + v[1]) + (v[2] + v[3]);
      if (!(fabsf(chk) <= 3.402823466e38f))
        __hip_atomic_fetch_or(&g_hn_fault, kFaultNonFinite, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const float vmax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
      __hip_atomic_fetch_max(reinterpret_cast<uint32_t*>(&lvmx[l]), __float_as_uint(vmax), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      const RecSlot rs = rec_slot(bw, (uint32_t)l, T, x0, y * kPrimeY, z * kPrimeZ);
      rec_store(bw, rs, v);
    }
  }
  __syncthreads();
  if (wave == 0) {   // lane = level: the max of its 64 lane slots
    const int l = lane & 15, q = lane >> 4;
    uint32_t m = 0u;
    for (int j = 0; j < 16; ++j) m = max(m, lvmxl[l * 64 + 16 * q + j]);
    __hip_atomic_fetch_max(reinterpret_cast<uint32_t*>(&lvmx[l]), m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  uint32_t* cnt = book + nrec + blockIdx.x;
  for (int i = threadIdx.x; i < k.nbins; i += blockDim.x) {
    const uint32_t c = (uint32_t)bcnt[i];
    cnt[(size_t)i * kBwdBlocks] = c;
    if (c > bw.cap)   // spilled records of bin i (ovf_place_kernel's bucket sizes)
      __hip_atomic_fetch_add(ob.per_bin + i, c - bw.cap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  float* mxo = reinterpret_cast<float*>(book + nrec + (size_t)kBwdBlocks * k.nbins) + blockIdx.x;
  if (threadIdx.x < 16) mxo[threadIdx.x * kBwdBlocks] = lvmx[threadIdx.x];
  if (threadIdx.x == 0) {
    const uint32_t n = lovf < bw.n_ovf ? lovf : bw.n_ovf;
    ob.blk[blockIdx.x] = n;
    if (n) __hip_atomic_fetch_add(ob.cnt, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (k.slab) {   // the dW slabs are complete (the MLP-backward kernel ran before this one)
    float(*part)[64] = reinterpret_cast<float(*)[64]>(stv);   // the staging pool is free now
    static_assert(kStPool * 20 >= sizeof(float) * kSlabGroups * 64 && 64 * kScWaves == 64 * kSlabGroups,
                  "slab-reduce blocks inside the scatter blocks");
    // the 292 slab blocks go to the scatter blocks as they finish (a counter
    // reset by render_comp_bwd_kernel): the sums do not depend on who runs them
    __shared__ int vb_sh;
    for (;;) {
      __syncthreads();   // part and vb_sh are free (the pool's last readers, or the previous combine)
      if (threadIdx.x == 0)
        vb_sh = (int)__hip_atomic_fetch_add(ob.slab_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int vb = vb_sh;
      if (vb >= kSlabVBlocks) break;
      slab_reduce_block(k.slab, kBwdBlocks, k.dc, k.df, k.overwrite_mlp, vb, part, k.has_mstep ? k.mstep : nullptr,
                        k.lmeta + 3);
    }
  }
}

// The table-gradient scatter of one slot (embedding_dense_backward of
// hash_encoding.py:106 + trilinear backward); V = 2048-float voxel buffer.
template <int CAP>
HN_DEV void scatter_slot(const B1K& k, const float* S, float* V, const float* gsl) {
  const int lane = lane_id();
  const int pp = lane & 15, f = (lane >> 4) & 1, lq = lane >> 4;
  Ray r;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    r.o[a] = S[kSlotR + a];
    r.d[a] = S[kSlotR + 3 + a];
  }
#pragma unroll
  for (int grp = 0; grp < 2; ++grp) {
    float pt[3], xc[3];
    ray_point(r, S[kSlotZ + 16 * grp + pp], pt);
#pragma unroll
    for (int a = 0; a < 3; ++a) xc[a] = clamp_t(pt[a], k.g.bmin[a], k.g.bmax[a]);
    // compact pass: lane (row lq, point pp) computes levels lq, lq+4, lq+8,
    // lq+12 once, instead of every (x offset, feature) row repeating the divisions
    if (grp) lds_fence_wave();                  // previous pass's voxel reads done
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int l = 4 * b + lq;
      int32_t cell[3];
      float w[3];
      voxel_cw(k.g, gsl, pt, xc, l, cell, w);
      float* dst = V + (l * 16 + pp) * 8;
      *reinterpret_cast<f32x4*>(dst) = f32x4{__int_as_float(cell[0]), __uint_as_float((uint32_t)cell[1] * kPrimeY),
                                              __uint_as_float((uint32_t)cell[2] * kPrimeZ), w[0]};
      *reinterpret_cast<float2*>(dst + 4) = make_float2(w[1], w[2]);
    }
    lds_fence_wave();
    float gl[16];
    const f32x4* src4 = reinterpret_cast<const f32x4*>(S + (16 * grp + pp) * kXS + 16 * f);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x4 v = src4[c];
      gl[4 * c] = v.x; gl[4 * c + 1] = v.y; gl[4 * c + 2] = v.z; gl[4 * c + 3] = v.w;
    }
    // voxel records are read one level ahead (one wave per SIMD: nothing
    // else hides the LDS latency)
    const float* vs = V + pp * 8;
    f32x4 v0 = *reinterpret_cast<const f32x4*>(vs);
    float2 v1 = *reinterpret_cast<const float2*>(vs + 4);
#pragma unroll
    for (int l = 0; l < 16; ++l) {
      const f32x4 c0 = v0;
      const float2 c1 = v1;
      if (l < 15) {
        v0 = *reinterpret_cast<const f32x4*>(vs + (l + 1) * 128);
        v1 = *reinterpret_cast<const float2*>(vs + (l + 1) * 128 + 4);
      }
      scatter_level_x<CAP>(k.g, k.d_table, c0, c1, l, gl[l], lane);
      if ((l & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  lds_fence_wave();                             // slot and voxel reads done
}

// Producer: one fine tile.  A fine sample that is one of the 64 coarse
// samples (fine_src < 64) is the same point in both passes: its coarse-pass
// grads are added, so every unique point is scattered once.  z / src: this
// lane's point's depth and fine_src (prefetched per unit).
HN_DEV void ring_put(const B1K& k, const Ring& q, float* X, const Ray& r, int64_t ray, float z, int src,
                     const f32x16& dfeat) {
  const int lane = lane_id();
  const int h = lane >> 5;
  const bool twin = src < kSc;
  const f32x4* dc =
      reinterpret_cast<const f32x4*>(k.dfeat + (size_t)ray * kDcRay + (size_t)(twin ? src : 0) * 32 + 16 * h);
  f32x4 tw[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) tw[c] = twin ? dc[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  int t = 0;
  if (lane == 0) t = atomicAdd(q.tick, 1);
  t = __builtin_amdgcn_readfirstlane(t);
  const int s = t % kSlots;
  spin_until(&q.freed[s], t / kSlots, kFaultSlot, 2);
  float* S = q.slots + s * kSlotF;
  fill_slot(S, r, z, dfeat, tw);
  ring_publish(&q.ready[s], t + 1);
}

// Consumer: takes tickets in order until every one of the n_tiles fine tiles
// has a ticket.  tick only grows and a tile takes its ticket before it is
// handed over, so tick == n_tiles with t >= tick means no ticket t will ever
// come.
template <int CAP>
HN_DEV void ring_drain(const B1K& k, const Ring& q, float* V, int n_tiles) {
  for (int t = 0;; ++t) {
    const int s = t % kSlots;
    bool have = false, done = false;
    for (int it = 0; it < kSpinCap; ++it) {
      if (lds_load(&q.ready[s]) >= t + 1) {
        have = true;
        break;
      }
      const int tk = lds_load(q.tick);
      if (tk >= n_tiles && t >= tk) {
        done = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!have && !done) raise_fault(kFaultDrain);   // tiles left unscattered
    asm volatile("" ::: "memory");
    if (!have) break;
    const float* S = q.slots + s * kSlotF;
    scatter_slot<CAP>(k, S, V, q.gsl);
    ring_publish(&q.freed[s], t / kSlots + 1);
  }
}

HN_DEV void wait_flag(int* flag, int need) {
  for (int it = 0; it < kSpinCap; ++it) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= need) return;
    __builtin_amdgcn_s_sleep(8);
  }
  raise_fault(kFaultCoarse);
}

// One work unit: composite backward of the ray (:541/:558 chain), then 2 tiles.
// Fine units hand each tile to the scatter wave; before the first hand-off
// they wait until wave 0 has published this ray's coarse feature grads
// (*done >= need)
template <int S, int MODE>
HN_DEV void b1_unit(const B1K& k, int64_t ray, int part, float* X, DW& dw, WRing& wr, const Ring* ring,
                    int* done = nullptr, int need = 0) {
  const int lane = lane_id();
  constexpr bool fine = S == kSf;
  const int p = lane & 31, h = lane >> 5;
  Ray r;
  load_ray(k.rays, ray, r);
  const int tile0 = 2 * part;                   // tile within this pass
  const float* drs = k.draw + ((size_t)ray * (kSc + kSf) + (fine ? kSc : 0) + 32 * tile0 + p) * 4;
  float4 dr[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) dr[t] = *reinterpret_cast<const float4*>(drs + 128 * t);
  float sh8[8], shx8[8];
  ray_sh(r, h, sh8, shx8);
  {   // sh part of color_net.0's input: features 8h .. 8h + 7 of the [sh16 | sigma | geo15] image
    const SP<2> sp = splitn<2>([&](int j) { return shx8[j]; });
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const u32x4 w = __builtin_bit_cast(u32x4, sp.p[q]);
      put_quad(reinterpret_cast<char*>(X), kBC0in, q, p, 2 * h, w[0], w[1]);
      put_quad(reinterpret_cast<char*>(X), kBC0in, q, p, 2 * h + 1, w[2], w[3]);
    }
  }
  const float* P = opaque_ptr(fine ? k.Pf : k.Pc);
  // color_net.0 applied to the sh part: the same for every point of the ray
  // (and bit-identical to starting each point's chain with it)
  C0Sh c0sh;
  {
    float* cl = X + kC0shF;
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) {
      const f32x16 v = gemm<R_F2S>(P, ob, zero16(), lane, [&](int s) { return sh8[s]; });
      if (p == 0)   // every point's column holds the same rows: lanes 0 and 32 store them
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(cl + 32 * ob + row_of(4 * g, h)) =
              f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
    }
    lds_fence_wave();
    c0sh.lds = cl;
  }
  const int ctile = (fine ? kSc / 32 : 0) + tile0;
  float zq[2] = {0.f, 0.f};
  int srcq[2] = {0, 0};
  if constexpr (fine) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      zq[t] = k.z_fine[ray * kSf + 32 * (tile0 + t) + p];
      srcq[t] = k.fine_src[ray * kSf + 32 * (tile0 + t) + p];
    }
  }
  f32x16 feat, featn;
  load_feat(k.feat, ray, ctile, lane, feat);
  load_feat(k.feat, ray, ctile + 1, lane, featn);
  static_for<0, 2>([&](auto tc) {   // unrolled: the ring's slots and the per-tile arrays stay static
    constexpr int t = decltype(tc)::value;
    uint32_t sm[3] = {0u, 0u, 0u};
    load_masks(k.feat, ray, ctile + t, lane, sm);
    const f32x16 dfeat = b1_tile(P, wr, X, t ? featn : feat, c0sh, dr[t], dw, sm);
    const int qbase = 32 * (tile0 + t);
    if constexpr (fine && MODE == kModeSplit) {
      // split backward: the tile's feature grads in the saved-feature tile
      // order (4 coalesced dwordx4 stores); scatter_bins_kernel adds the
      // coarse twins and scatters
      f32x4* dst = reinterpret_cast<f32x4*>(k.dfeat_f + ((size_t)ray * (kSf / 32) + tile0 + t) * 1024);
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[64 * c + lane] = f32x4{dfeat[4 * c], dfeat[4 * c + 1], dfeat[4 * c + 2], dfeat[4 * c + 3]};
    } else if constexpr (fine) {
      if (t == 0) wait_flag(done, need);       // the coarse twin grads are written
      ring_put(k, *ring, X, r, ray, zq[t], srcq[t], dfeat);
    } else if constexpr (MODE == kModeSplit) {
      // coarse, split backward: the tile's feature grads in the saved-feature
      // tile order like the fine tiles (4 coalesced dwordx4 stores; the
      // per-point layout below took 16 scattered 4-B stores per lane and tile)
      f32x4* dst = reinterpret_cast<f32x4*>(k.dfeat + (size_t)ray * kDcRay + (size_t)(tile0 + t) * 1024);
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[64 * c + lane] = f32x4{dfeat[4 * c], dfeat[4 * c + 1], dfeat[4 * c + 2], dfeat[4 * c + 3]};
    } else {
      // coarse, fused backward: per-point feature grads [point][feature f][level]
      // for the fine units' ring hand-off (lane half h holds levels tile_level(m, h))
      float* dst = k.dfeat + (size_t)ray * kDcRay + (size_t)(qbase + p) * 32;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int l = h ? tile_level(m, 1) : tile_level(m, 0);
        dst[l] = dfeat[2 * m];
        dst[16 + l] = dfeat[2 * m + 1];
      }
    }
  });
}

// Split backward: the coarse and fine units share one code
// path (the pass is a runtime flag: weights, draw offset, tile index and
// destination are selects) and the unit's two tiles run as a loop, so the
// kernel holds ONE copy of b1_tile instead of four (two unrolled tiles x two
// unit templates): 87 KB of code -> ~25 KB, under the 64 KB instruction cache
// two CUs share (wave 0 ran the coarse copies, waves 1-3 the fine ones, at
// the same time).
// A tile whose 32 samples all have d raw = 0 (raw2outputs' backward gives
// exactly that to every sample with relu(sigma) = 0: alpha = 0, weight 0,
// run_nerf_helpers.py:577-628) has an exactly zero MLP backward: zero
// feature grads, and it adds 0 to every dW accumulator.  Such tiles are
// skipped -- the same results (an accumulator plus exact zeros is unchanged)
// for ~2/3 of the tiles of a trained scene (config 2: 57 % of the coarse and
// 70 % of the fine tiles, scripts/zero_grad_frac.py).
// Nothing is stored for them: the scatter kernel reads a sample's feature
// grads only where its own d raw (or its coarse twin's) is nonzero.  The
// weight ring is aligned to the tile period, so a skipped unit leaves it
// ready for the next one.  The composite pre-pass marks the tiles with a
// nonzero d raw (B1K::uflags), and the waves run lists of the marked tiles
// (render_bwd_kernel): the same loop shape as over every tile (a per-tile
// test inside the loop made the register allocator spill).
// new_ray: the previous tile of this wave was another ray's (or none), so
// the ray's SH operand image and color_net.0's SH rows (c0sh) are set up;
// otherwise they are still in the wave's LDS from that tile.
// One MLP tile of two listed 16-sample groups (round 6): points 0-15 group
// code ca, 16-31 group cb (codes ray << 4 | group; cb < 0: none, those lanes
// run with d raw 0 and store nothing).  Each lane's ray gives its own SH
// columns, and color_net.0's SH half is formed for both groups' rays at once
// (column p of that product is point p's ray), kept in LDS per group.  The
// two groups are often of different rays; every per-point input (features,
// masks, d raw) is read at the point's own place in the ray's tiles and its
// feature grads are written there, so the dW products and grads are those of
// the dense form's tiles, grouped differently.
HN_DEV void b1_groups(const B1K& k, int ca, int cb, bool fine, float* X, DW& dw, WRing& wr) {
  const int lane = lane_id();
  const int p = lane & 31, h = lane >> 5;
  const bool none = p >= 16 && cb < 0;
  const int code = p < 16 || cb < 0 ? ca : cb;
  const int64_t ray = code >> 4;
  const int i = 16 * (code & 15) + (p & 15);          // the point within its pass
  float4 dr = *reinterpret_cast<const float4*>(k.draw + ((size_t)ray * (kSc + kSf) + (fine ? kSc : 0) + i) * 4);
  if (none) dr = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* P = opaque_ptr(fine ? k.Pf : k.Pc);
  C0Sh c0sh;
  {
    Ray r;
    load_ray(k.rays, ray, r);
    float sh8[8], shx8[8];
    ray_sh(r, h, sh8, shx8);
    const SP<2> sp = splitn<2>([&](int j) { return shx8[j]; });
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const u32x4 w = __builtin_bit_cast(u32x4, sp.p[q]);
      put_quad(reinterpret_cast<char*>(X), kBC0in, q, p, 2 * h, w[0], w[1]);
      put_quad(reinterpret_cast<char*>(X), kBC0in, q, p, 2 * h + 1, w[2], w[3]);
    }
    float* cl = X + kC0shF;
#pragma unroll
    for (int ob = 0; ob < 2; ++ob) {
      const f32x16 v = gemm<R_F2S>(P, ob, zero16(), lane, [&](int s) { return sh8[s]; });
      if ((p & 15) == 0)   // columns 0 and 16: the two groups' rays
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(cl + 64 * (p >> 4) + 32 * ob + row_of(4 * g, h)) =
              f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
    }
    lds_fence_wave();
    c0sh.lds = cl + 64 * (p >> 4);
  }
  // the point's place in the saved tiles: tile (pass offset + i / 32), lane (i % 32) + 32 h
  const int ctile = (fine ? kSc / 32 : 0) + (i >> 5), pl = (i & 31) + 32 * h;
  const float* fb = k.feat + (size_t)ray * HN_RENDER_FEAT_PER_RAY;
  f32x16 feat;
  {
    const f32x4* t = reinterpret_cast<const f32x4*>(fb + (size_t)ctile * 1024);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x4 v = __builtin_nontemporal_load(t + 64 * c + pl);
      feat[4 * c] = v.x; feat[4 * c + 1] = v.y; feat[4 * c + 2] = v.z; feat[4 * c + 3] = v.w;
    }
  }
  uint32_t sm[3];
  {
    const uint32_t* t = reinterpret_cast<const uint32_t*>(fb + kTilesPerRay * 1024) + ctile * kMaskWordsPerTile;
#pragma unroll
    for (int j = 0; j < 3; ++j) sm[j] = __builtin_nontemporal_load(t + 64 * j + pl);
  }
  const f32x16 dfeat = b1_tile(P, wr, X, feat, c0sh, dr, dw, sm);
  // this point's feature grads (the saved-feature tile order of both passes)
  if (!none) {
    f32x4* dst = fine ? reinterpret_cast<f32x4*>(k.dfeat_f + ((size_t)ray * (kSf / 32) + (i >> 5)) * 1024)
                      : reinterpret_cast<f32x4*>(k.dfeat + (size_t)ray * kDcRay + (size_t)(i >> 5) * 1024);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const f32x4 v = f32x4{dfeat[4 * c], dfeat[4 * c + 1], dfeat[4 * c + 2], dfeat[4 * c + 3]};
      __builtin_nontemporal_store(v, dst + 64 * c + pl);   // read once, by the scatter
    }
  }
}

// The binned scatter's overflow book starts empty (count, per bin, cursors,
// the scatter blocks' slab-block counter): reset by workgroup 0 of the first
// kernel of the backward.
HN_DEV void zero_ovf_book(const B1K& k) {
  const size_t nrec = bin_records(k.nbins, k.bin_cap, k.B);
  uint32_t* o = ovf_book(reinterpret_cast<uint32_t*>(k.bins + 4 * nrec), nrec, k.nbins).cnt;
  for (int i = threadIdx.x; i < 1 + 2 * k.nbins; i += blockDim.x) o[i] = 0u;
  if (threadIdx.x == 0) o[1 + 3 * k.nbins] = 0u;   // the scatter kernel's slab-block counter (ob.slab_next)
}

// Composite backward pre-pass (raw2outputs backward, run_nerf_helpers.py:577-628
// via the :541 / :558 chain): one wave per (ray, pass) at full occupancy
// writes d raw of every sample, so the MLP units only load one float4 per
// point instead of each redoing the ray's scans.
__global__ __launch_bounds__(256) void render_comp_bwd_kernel(B1K k) {
  __shared__ float lds[kFwdWaves][kSf * 5];
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k.bins && blockIdx.x == 0) zero_ovf_book(k);   // binned scatter: no overflow records yet
  // the loss value (hn_loss_fwd's reduction): an extra workgroup 0 of its own,
  // dispatched first, so its serial sums run beside the rays' workgroups
  if (k.lout && blockIdx.x == 0) {
    loss_fwd_block<64 * kFwdWaves>(k.lrgb, k.lrgb0, k.ltarget, k.lsp, k.lsp0, k.B, k.ltv, k.n_tv, k.lworld,
                                   k.lsparse_w, k.ltv_w, k.lout);
    return;
  }
  const int64_t w = (int64_t)(blockIdx.x - (k.lout ? 1 : 0)) * kFwdWaves + wave;
  // the two waves of a ray (coarse 2r, fine 2r + 1) share the workgroup: the
  // coarse wave's nonzero-sample mask reaches the fine wave through LDS
  __shared__ unsigned long long cmask[kFwdWaves / 2];
  const bool active = w < 2 * k.B;
  uint32_t nzf = 0u;   // the fine wave's MLP groups
  const int64_t ray = w >> 1;
  const bool fine = (w & 1) != 0;
  float* rawb = lds[wave] + kSf;
  if (active) {
    const int S = fine ? kSf : kSc;
    float* zb = lds[wave];
    const float* zsrc = (fine ? k.z_fine : k.z_coarse) + ray * S;
    const float* rsrc = (fine ? k.raw_f : k.raw_c) + ray * S * 4;
    for (int j = lane; j < S; j += 64) {
      zb[j] = zsrc[j];
      *reinterpret_cast<float4*>(rawb + 4 * j) = *reinterpret_cast<const float4*>(rsrc + 4 * j);
    }
    lds_fence_wave();
    Ray r;
    load_ray(k.rays, ray, r);
    CompGrad g;
    const float* grgb = fine ? k.g_rgb : k.g_rgb0;
    const float* gacc = fine ? k.g_acc : k.g_acc0;
    const float* gdep = fine ? k.g_depth : k.g_depth0;
    const float* gent = fine ? k.g_sparsity : k.g_sparsity0;
    if (k.lout) {   // the training loss's gradients (hn_loss_bwd_elem's op forms, g_loss = 1)
      const float* x = fine ? k.lrgb : k.lrgb0;
      g.has_rgb = g.has_entropy = true;
      g.has_acc = g.has_depth = false;
#pragma unroll
      for (int c = 0; c < 3; ++c) g.rgb[c] = k.lgm * (2.f * (x[3 * ray + c] - k.ltarget[3 * ray + c]));
      g.acc = g.depth = 0.f;
      g.entropy = k.lsparse;
    } else {
      g.has_rgb = grgb != nullptr;
      g.has_acc = gacc != nullptr;
      g.has_depth = gdep != nullptr;
      g.has_entropy = gent != nullptr;
#pragma unroll
      for (int c = 0; c < 3; ++c) g.rgb[c] = g.has_rgb ? grgb[3 * ray + c] : 0.f;
      g.acc = g.has_acc ? gacc[ray] : 0.f;
      g.depth = g.has_depth ? gdep[ray] : 0.f;
      g.entropy = g.has_entropy ? gent[ray] : 0.f;
    }
    const float* noise = fine ? (k.noise_f ? k.noise_f + ray * S : nullptr)
                              : (k.noise_c ? k.noise_c + ray * S : nullptr);
    const float* graw = (fine && k.g_raw_f) ? k.g_raw_f + ray * S * 4 : nullptr;
    float* dst = k.draw + ((size_t)ray * (kSc + kSf) + (fine ? kSc : 0)) * 4;
    if (fine)
      composite_bwd<kSf / 64>(rawb, zb, noise, S, r.dnorm, k.white != 0, g, nullptr, graw, rawb, lane);
    else
      composite_bwd<kSc / 64>(rawb, zb, noise, S, r.dnorm, k.white != 0, g, nullptr, graw, rawb, lane);
    lds_fence_wave();
    uint32_t nzu = 0u;   // bit t: a sample of 16-sample group t has a nonzero d raw (the MLP's)
    for (int j = lane; j < S; j += 64) {
      const float4 d = *reinterpret_cast<const float4*>(rawb + 4 * j);
      *reinterpret_cast<float4*>(dst + 4 * j) = d;
      const uint64_t b = __ballot(draw_nonzero(d));
#pragma unroll
      for (int q = 0; q < 4; ++q) nzu |= (((b >> (16 * q)) & 0xffffull) != 0ull ? 1u : 0u) << (4 * (j >> 6) + q);
    }
    if (lane == 0 && !fine) k.uflags[kMarkB * ray] = (uint8_t)nzu;   // byte 0: the coarse groups
    nzf = nzu;
    if (!fine) cmask[wave >> 1] = __ballot(draw_nonzero(*reinterpret_cast<const float4*>(rawb + 4 * lane)));
  }
  __syncthreads();
  if (active && fine) {
    // the scatter's marks: bit t = a sample of fine tile t, or its coarse twin
    // (the same point, fine_src < 64), has a nonzero d raw -- the tile has
    // feature grads to scatter (scatter_bins_kernel's lists)
    const unsigned long long cm = cmask[wave >> 1];
    uint32_t su = 0u;   // bit t: fine 16-sample group t has feature grads to scatter
    for (int j = lane; j < kSf; j += 64) {
      const int src = k.fine_src[ray * kSf + j];
      const bool nz = draw_nonzero(*reinterpret_cast<const float4*>(rawb + 4 * j)) ||
                      (src < kSc && ((cm >> src) & 1ull) != 0ull);
      const uint64_t b = __ballot(nz);
#pragma unroll
      for (int q = 0; q < 4; ++q) su |= (((b >> (16 * q)) & 0xffffull) != 0ull ? 1u : 0u) << (4 * (j >> 6) + q);
    }
    if (lane == 0) {   // bits 8-19: the fine MLP groups, 20-31: the scatter's groups
      const uint32_t v = nzf | (su << 12);
      k.uflags[kMarkB * ray + 1] = (uint8_t)v;
      k.uflags[kMarkB * ray + 2] = (uint8_t)(v >> 8);
      k.uflags[kMarkB * ray + 3] = (uint8_t)(v >> 16);
    }
  }
}

// acc[base + n*ld + k] += D[n - n0][k - k0] for n < nmax, k < kmax (LDS),
// or = (plain stores) when STORE: every dW element belongs to exactly one
// (block, lane, register) of the twelve blocks.
template <bool STORE>
HN_DEV void dw_block(float* acc, int base, int ld, int n0, int nmax, int k0, int kmax, const f32x16& d,
                     int lane) {
  if constexpr (STORE) {
    const int i = lane & 31, h = lane >> 5;
    const int kk = k0 + i;
    if (kk >= kmax) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = n0 + row_of(r, h);
      if (n < nmax) acc[base + n * ld + kk] = d[r];
    }
  } else {
    accum_block(acc, base, ld, n0, nmax, k0, kmax, d, lane);
  }
}

// color_net.0's dW block: its columns are the image features [sh16 | sigma |
// geo15] (b1_tile): feature 16 (sigma, no weight) is dropped, 17..31 are
// weight columns 16..30.
template <bool STORE>
HN_DEV void dw_block_c0(float* acc, int nb, const f32x16& d, int lane) {
  const int i = lane & 31, h = lane >> 5;
  if (i == 16) return;
  const int col = i < 16 ? i : i - 1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float* dst = acc + W_C0 + (32 * nb + row_of(r, h)) * 31 + col;
    if constexpr (STORE)
      *dst = d[r];
    else
      atomicAdd(dst, d[r]);
  }
}

template <bool STORE>
HN_DEV void dw_flush(const DW& dw, float* acc, int lane) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) dw_block<STORE>(acc, W_C2, 64, 0, 3, 32 * kb, 64, dw.c2[kb], lane);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      dw_block<STORE>(acc, W_C1, 64, 32 * nb, 64, 32 * kb, 64, dw.c1[2 * nb + kb], lane);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) dw_block_c0<STORE>(acc, nb, dw.c0[nb], lane);
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) dw_block<STORE>(acc, W_S1, 64, 0, 16, 32 * kb, 64, dw.s1[kb], lane);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) dw_block<STORE>(acc, W_S0, 32, 32 * nb, 64, 0, 32, dw.s0[nb], lane);
}

HN_DEV void dw_zero(DW& dw) {
#pragma unroll
  for (int j = 0; j < 2; ++j) dw.c2[j] = dw.c0[j] = dw.s1[j] = dw.s0[j] = zero16();
#pragma unroll
  for (int j = 0; j < 4; ++j) dw.c1[j] = zero16();
}

// The block's MLP waves sum their dW before the slab store (HN_DW_BLOCKRED):
// a wave's 12 accumulator blocks through LDS as [block][quad][lane] f32x4
// (48 KiB; conflict-free b128 accesses), added by the first wave of the block
// that runs the same net, in wave order.
template <typename F>
HN_DEV void dw_each(DW& dw, F&& f) {
#pragma unroll
  for (int j = 0; j < 2; ++j) f(dw.c2[j], j);
#pragma unroll
  for (int j = 0; j < 4; ++j) f(dw.c1[j], 2 + j);
#pragma unroll
  for (int j = 0; j < 2; ++j) f(dw.c0[j], 6 + j);
#pragma unroll
  for (int j = 0; j < 2; ++j) f(dw.s1[j], 8 + j);
#pragma unroll
  for (int j = 0; j < 2; ++j) f(dw.s0[j], 10 + j);
}
HN_DEV void dw_to_lds(DW& dw, f32x4* L, int lane) {
  dw_each(dw, [&](f32x16& v, int b) {
#pragma unroll
    for (int q = 0; q < 4; ++q) L[(b * 4 + q) * 64 + lane] = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
  });
}
HN_DEV void dw_add_lds(DW& dw, const f32x4* L, int lane) {
  dw_each(dw, [&](f32x16& v, int b) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 t = L[(b * 4 + q) * 64 + lane];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * q + j] = v[4 * q + j] + t[j];
    }
  });
}

// The backward's work lists (round 6), from the composite pre-pass's marks
// (B1K::uflags; every group with dense_bwd): the coarse and the fine 16-sample
// groups with a nonzero d raw (the MLP backward's) and the fine groups with
// feature grads (the scatter's), each in ray order, as
// codes (ray << 4 | 16-sample group); their lengths and the MLP waves' coarse / fine
// split.  Workgroup w writes the codes of rays [w R, (w + 1) R): it counts
// the marks of every earlier ray itself (a few loads per thread; no
// workgroup waits for another), then takes 256 rays at a time, one per
// thread, with a block-wide prefix of their counts.  (One 1,024-thread
// workgroup for the whole batch took 14 us; computed redundantly by every
// block of the kernels that use the lists it cost the MLP backward ~28 us.)
constexpr int kListThreads = 256;
constexpr int kListMaxBlocks = 64;
HN_DEV int list_block_scan(int v, int* sh) {   // inclusive scan over the workgroup; sh: 4 ints of LDS
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  __syncthreads();   // sh free (its previous use is complete)
  if (lane == 63) sh[wave] = v;
  __syncthreads();
  for (int q = 0; q < wave; ++q) v += sh[q];
  return v;
}
HN_DEV int list_block_sum(int v, int* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  return sh[0] + sh[1] + sh[2] + sh[3];
}
__global__ __launch_bounds__(kListThreads) void render_lists_kernel(B1K k) {
  static_assert(kListThreads == 256, "list_block_scan: 4 waves");
  __shared__ int sh[3][4];
  const int t = threadIdx.x;
  // bits [coarse groups (4), -, fine groups (12), the scatter's groups (12)]
  auto mword = [&](int64_t r) -> uint32_t {
    return k.skip_zero ? *reinterpret_cast<const uint32_t*>(k.uflags + kMarkB * r) : 0xffffff0fu;
  };
  const int64_t R = (k.B + gridDim.x - 1) / gridDim.x;
  const int64_t ra = (int64_t)blockIdx.x * R, rb = ra + R < k.B ? ra + R : k.B;
  // the counts of the rays before this workgroup's range, and of all rays
  int bc = 0, bf = 0, bs = 0, tc = 0, tf = 0, ts = 0;
  for (int64_t r = t; r < k.B; r += kListThreads) {
    const uint32_t w = mword(r);
    const int c = __builtin_popcount(w & 15u), f = __builtin_popcount((w >> 8) & 0xfffu),
              g = __builtin_popcount(w >> 20);
    tc += c; tf += f; ts += g;
    if (r < ra) { bc += c; bf += f; bs += g; }
  }
  int64_t xc = list_block_sum(bc, sh[0]), xf = list_block_sum(bf, sh[1]), xs = list_block_sum(bs, sh[2]);
  const int64_t Nc = list_block_sum(tc, sh[0]), Nf = list_block_sum(tf, sh[1]), Ns = list_block_sum(ts, sh[2]);
  int32_t* lc = k.lists;
  int32_t* lf = lc + 4 * k.B;
  int32_t* ls = lf + 12 * k.B;
  for (int64_t r0 = ra; r0 < rb; r0 += kListThreads) {
    const int64_t r = r0 + t;
    const uint32_t w = r < rb ? mword(r) : 0u;
    const int c = __builtin_popcount(w & 15u), f = __builtin_popcount((w >> 8) & 0xfffu),
              g = __builtin_popcount(w >> 20);
    const int ic = list_block_scan(c, sh[0]), jf = list_block_scan(f, sh[1]), ks = list_block_scan(g, sh[2]);
    int64_t oc = xc + ic - c, of = xf + jf - f, os = xs + ks - g;
    for (int i = 0; i < 4; ++i)
      if ((w >> i) & 1u) lc[oc++] = (int32_t)(r << 4) | i;
    for (int i = 0; i < 12; ++i)
      if ((w >> (8 + i)) & 1u) lf[of++] = (int32_t)(r << 4) | i;
    for (int i = 0; i < 12; ++i)
      if ((w >> (20 + i)) & 1u) ls[os++] = (int32_t)(r << 4) | i;
    xc += list_block_sum(c, sh[0]);
    xf += list_block_sum(f, sh[1]);
    xs += list_block_sum(g, sh[2]);
  }
  if (blockIdx.x == 0 && t == 0) {
    const int G = kB1Waves * kBwdBlocks;
    int gc = Nc > 0 ? G : 0;   // MLP waves on the coarse list, in proportion to the lists
    if (Nc > 0 && Nf > 0) {
      gc = (int)((2 * (int64_t)G * Nc + Nc + Nf) / (2 * (Nc + Nf)));
      gc = gc < 1 ? 1 : (gc > G - 1 ? G - 1 : gc);
    }
    k.lmeta[0] = (int32_t)Nc;
    k.lmeta[1] = (int32_t)Nf;
    k.lmeta[2] = (int32_t)Ns;
    k.lmeta[3] = gc;
  }
}

// One persistent block per CU owns rays blockIdx.x + i * gridDim.x.  Wave 0
// first runs the block's coarse units (MLP backward of network_fn only) and
// publishes each ray's coarse feature grads through an LDS counter; then it
// stores its coarse dW to the block's slab and joins the fine units.  Waves
// 1-2 (and wave 0 once free) take fine units from an LDS work counter (MLP
// backward of network_fine) and hand every fine tile's feature grads to
// wave 3 through the LDS ring; wave 3 only scatters (the table gradient is
// bound by the memory-side float-atomic rate, so the MLP work runs under it).
// Every wave that waits, waits on a wave of its own workgroup: co-resident.
template <int CAP, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void render_bwd_kernel(B1K k) {
  constexpr bool SPLIT = MODE == kModeSplit;
  extern __shared__ f32x4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  float* X = smem + wave * kRRows * kXS;
  float* slots = smem + kB1Img;
  float* V = slots + kSlots * kSlotF;
  float* gsl = V + kVoxF;                        // [voxel buffer | grid sizes | sync]
  // [0] coarse rays done, [1] fine units taken, [2] ring tickets, [3] dW buffer zeroed,
  // [4] unused, [5..) ready, freed
  int* sync = reinterpret_cast<int*>(gsl + kGsLds);
  stage_grid_sizes(k.g, gsl);
  if (threadIdx.x < kSyncInts) sync[threadIdx.x] = 0;
  __syncthreads();
  const Ring ring{slots, &sync[2], &sync[5], &sync[5 + kSlots], gsl};
  const int64_t nb = gridDim.x;
  const int n_rays = k.B > (int64_t)blockIdx.x ? (int)((k.B - 1 - blockIdx.x) / nb + 1) : 0;
  // ray of the block's i-th unit: a contiguous chunk per block when the
  // batch divides evenly, so the rays in flight at one time across the chip
  // are far apart in a spatially ordered batch (concurrent atomics on the
  // same rows serialize at the memory side); strided otherwise
  const bool chunked = k.B % nb == 0;
  auto block_ray = [&](int64_t i) -> int64_t {
    if (!chunked) return (int64_t)blockIdx.x + i * nb;
    // a fixed pseudo-random permutation of the batch scatters both the rays in
    // flight across the chip (one per block) and a block's consecutive rays
    uint32_t x = (uint32_t)((int64_t)blockIdx.x * (k.B / nb) + i);
    if (k.scramble) {
      do {
        x = feistel(x, k.scramble, 0x5bd1e995u);
      } while ((int64_t)x >= k.B);
    }
    return (int64_t)x;
  };
  DW dw;
  dw_zero(dw);
  WRing wr;
  if (wave == kMW && !SPLIT) {
    ring_drain<CAP>(k, ring, V, 2 * kSf / 64 * n_rays);
  } else if (SPLIT) {
    // Balanced tile lists (round 6).  The tiles with a nonzero d raw (the
    // composite pre-pass's marks; all of them with dense_bwd) form two lists in
    // ray order -- coarse tiles, then fine tiles (ray, tile), render_lists_kernel
    // -- and the kB1Waves x nb MLP waves g = wave * nb + block split them: the
    // first gsplit waves the coarse list, the others the fine list, in
    // contiguous slices of equal length (gsplit in proportion to the two
    // lists).  Every wave then runs ~1/1024 of the work, whatever the scene
    // leaves nonzero; each wave keeps one net's dW and stores it to slab g,
    // which the scatter kernel's slab reduction sums in g order:
    // deterministic (the split is a function of the marks alone).  Tiles, not
    // the two-tile units of the static split: a live unit often holds a dead
    // tile.  A wave reads its codes 64 at a time (one vector load; the tile
    // loop takes them by readlane).
    const int wv = __builtin_amdgcn_readfirstlane(wave);    // wave-uniform (SGPR)
    const int64_t Nc = __builtin_amdgcn_readfirstlane(k.lmeta[0]), Nf = __builtin_amdgcn_readfirstlane(k.lmeta[1]);
    const int gc = __builtin_amdgcn_readfirstlane(k.lmeta[3]);
    static_assert(kB1Waves == 4 && kSlabSlots == kB1Waves, "slab_reduce_block's run leaders: 4 waves per block");
    const int G = kB1Waves * (int)nb,
              g_me = HN_DW_BLOCKRED ? (int)blockIdx.x * kB1Waves + wv : wv * (int)nb + (int)blockIdx.x;
    const bool fine = g_me >= gc;                            // wave-uniform
    const int64_t N = fine ? Nf : Nc;
    const int gi = fine ? g_me - gc : g_me, GG = fine ? G - gc : gc;
    // slices of whole group pairs (a tile = two consecutive listed groups)
    const int64_t NP = (N + 1) / 2;
    const int64_t lo = GG ? 2 * ((int64_t)gi * NP / GG) : 0, hi2 = GG ? 2 * ((int64_t)(gi + 1) * NP / GG) : 0;
    const int64_t hi = hi2 < N ? hi2 : N;
    const int32_t* L = k.lists + (fine ? 4 * k.B : 0);
    wring_prime(wr, fine ? k.Pf : k.Pc, lane);
#ifndef HN_DIAG_NOTILES
#define HN_DIAG_NOTILES 0   // diagnostic builds: 1 = no tiles
#endif
    for (int64_t c0 = lo; c0 < (HN_DIAG_NOTILES ? lo : hi); c0 += 64) {   // lo even: pairs never straddle
      const int cnt = (int)(hi - c0 < 64 ? hi - c0 : 64);
      const int codes = lane < cnt ? L[c0 + lane] : -1;
      for (int j = 0; j < cnt; j += 2) {
        const int ca = __builtin_amdgcn_readlane(codes, j);
        const int cb = j + 1 < cnt ? __builtin_amdgcn_readlane(codes, j + 1) : -1;
        b1_groups(k, ca, cb, fine, X, dw, wr);
      }
    }
    if (HN_DW_BLOCKRED) {
      // the block's waves g0 .. g0 + 3 run the coarse net below gc, the fine
      // one from gc: each run of same-net waves is summed into its first wave
      // (wave order), which alone stores a slab (slab_reduce_block's leaders)
      const int g0 = (int)blockIdx.x * kB1Waves;
      f32x4* red = smem4;
      for (int w = 1; w < kB1Waves; ++w) {
        const bool w_leads = g0 + w == gc;                  // first fine wave of the block
        int ldr = 0;                                        // the leader of wave w
        if (g0 + w >= gc && g0 < gc) ldr = gc - g0;         // a fine wave behind the block's coarse ones
        __syncthreads();
        if (!w_leads && wv == w) dw_to_lds(dw, red, lane);
        __syncthreads();
        if (!w_leads && wv == ldr) dw_add_lds(dw, red, lane);
      }
      const bool leader = wv == 0 || g_me == gc;
      if (leader) dw_flush<true>(dw, k.slab + (size_t)g_me * W_END, lane);
    } else {
      dw_flush<true>(dw, k.slab + (size_t)g_me * W_END, lane);
    }
  } else {
    if (wave == 0) {
      wring_prime(wr, k.Pc, lane);
      for (int i = 0; i < n_rays; ++i) {
        b1_unit<kSc, MODE>(k, block_ray(i), 0, X, dw, wr, nullptr);
        if constexpr (!SPLIT) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this ray's feature grads are in L2
          if (lane == 0) __hip_atomic_store(&sync[0], i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      dw_flush<true>(dw, k.slab + (size_t)blockIdx.x * kSlabSlots * W_END, lane);   // slot 0: coarse
      dw_zero(dw);
    }
    // split: wave 0 has the block's 2 * n_rays coarse tiles, waves 1-3 share
    // its 6 * n_rays fine tiles (balanced); fused: wave 0 joins waves 1-2
    if (SPLIT && wave != 0) {
      // split: wave w owns part w - 1 (tiles 2(w-1), 2(w-1)+1) of every ray of
      // the block, in ray order -- a static split (the units are equal), so each
      // dW slab, and with the fixed-order slab reduce the MLP gradients, are
      // bitwise reproducible
      wring_prime(wr, k.Pf, lane);
      for (int i = 0; i < n_rays; ++i) b1_unit<kSf, MODE>(k, block_ray(i), wave - 1, X, dw, wr, &ring, &sync[0], i + 1);
    } else if (!SPLIT) {
      wring_prime(wr, k.Pf, lane);
      for (;;) {
        int u = 0;
        if (lane == 0) u = atomicAdd(&sync[1], 1);
        u = __builtin_amdgcn_readfirstlane(u);
        if (u >= 3 * n_rays) break;
        b1_unit<kSf, MODE>(k, block_ray(u / 3), u % 3, X, dw, wr, &ring, &sync[0], u / 3 + 1);
      }
    }
    // every fine MLP wave stores its fine dW to its own slab slot (split:
    // waves 1-3 -> slots 1-3; fused: waves 0-2 -> slots 1-3), inside this
    // branch: the accumulators must not be live in the scatter wave's code (a
    // spill there would wait vmcnt(0), i.e. drain its atomics).  Formerly the
    // waves summed into one LDS image with LDS atomics after waiting for wave
    // 0: ~0.1 M cycles of the kernel's tail.
    if (!SPLIT || wave != 0)
      dw_flush<true>(dw, k.slab + ((size_t)blockIdx.x * kSlabSlots + (SPLIT ? wave : wave + 1)) * W_END, lane);
  }
}

__global__ __launch_bounds__(64 * kSlabGroups) void slab_reduce_kernel(const float* __restrict__ slab, int n_blocks,
                                                                       hn_mlp_grad dc, hn_mlp_grad df, int overwrite) {
  __shared__ float part[kSlabGroups][64];
  slab_reduce_block(slab, n_blocks, dc, df, overwrite, blockIdx.x, part);
}

// Owner pass of the binned scatter: workgroup b sums every record of bin b
// (the regions of all kBwdBlocks producers, then the overflow records that
// belong to it) and writes its slice of 2^shift entries of the table
// gradient once: = (overwrite) or +=.  Every entry is written by exactly one
// workgroup.
//
// The sums are exact integer sums.  On gfx950 ds_add_f32 runs ~20x slower than
// integer LDS atomics (config 2: ~600 us for the bins' 71 M float adds, against
// ~145 us with ds_add_u32 on the same addresses, ~125 us for the record loads
// alone), and a bin's records are heavily duplicated (surfaces: e.g. 37.5 K
// records on 2.9 K distinct entries at level 8), which defeats claiming
// entries for plain read-modify-writes.  So each value is converted to a
// 64-bit fixed-point integer in units of 2^(E - 40), E the exponent of the
// bin's largest |value| (every value < 2^41 units, 2^20 of them < 2^61), and
// added with ds_add_u64; the slice is converted back (one rounding to fp32).
// Integer adds are associative, so the gradient is bitwise reproducible, and
// every entry keeps full fp32 precision down to 2^-16 of the bin's largest
// contribution (2^-40 absolute resolution below that).  Measured on recorded
// config 2 bins (scripts/bin_stats.py): median relative error 1e-8 (fp32
// sequential sums 6e-9 .. 2e-8); the worst entries, at |g| ~ 1e-17 with a bin
// maximum ~ 5e-7, within 8e-3 -- where fp32 atomics cannot resolve them
// either once a larger contribution has been added.
struct BinR {
  const float* bins;
  int64_t n_rays;
  int32_t nbins, cap, shift, log2T;
  float* d_table;          // or NULL (fused step only)
  int32_t overwrite;
  int32_t fused;           // 1: apply `step` to the table (p, m, v) with the bin's gradient
  hn_radam_tensor step;
  const uint32_t* live;    // fused step: live row pairs of levels < live_levels (hn_render_bwd_args.table_live)
  int32_t live_levels;
  int32_t bin0;            // first bin of the launch (hn_render_bwd_owner ranges)
};
constexpr int kBinThreads = 1024;
constexpr int kSliceF4 = 4;   // float4s of a 2^13-entry slice per thread (2 x 2^13 floats / 4 / 1024)
// The fused step's optimizer-state loads: 0 in the epilogue; 1 at kernel
// start.  Measured on one box (config 2): 207.5 vs 214.8 / 204.5 us; loaded
// after the setup 238 us, after the thread's last record fetch 217 us (64
// VGPR spills): vmcnt waits are in order, so an earlier issue only moves the
// wait to the first records.
static_assert(kSliceF4 * kBinThreads * 4 >= (2 << 13), "bins are at most 2^13 entries (bin_geom)");
constexpr int kBrDepth = 4;   // records per thread and fetch group (two groups in flight)
constexpr int kBrChunks = 8192;   // table entries (16 KiB of LDS): bins of up to 512 K records


// acc: [feature][entry] (entry e's accumulators 8 B apart per feature: a
// wave's random entries spread over twice the LDS banks of [entry][feature])
HN_DEV void bin_add(unsigned long long* acc, uint32_t se, const f32x4 v, uint32_t w, uint32_t sel,
                    uint32_t tmask, float scale) {
  const uint32_t e0 = w & 0x0fffffffu & sel;
  const uint32_t e1 = e0 ^ (((1u << (w >> 28)) - 1u) & tmask);
  const long long q[4] = {fx_of(v.x, scale), fx_of(v.y, scale), fx_of(v.z, scale), fx_of(v.w, scale)};
  __hip_atomic_fetch_add(acc + e0, (unsigned long long)q[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_add(acc + se + e0, (unsigned long long)q[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_add(acc + e1, (unsigned long long)q[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __hip_atomic_fetch_add(acc + se + e1, (unsigned long long)q[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Buckets the spilled records by bin.  Block j handles producer block j's
// overflow list: it scans the per-bin spill counts (block 0 publishes the
// first slot of each bin), counts its own records per bin in LDS, reserves one
// range per touched bin with a single global atomic, and places the record
// ids through LDS cursors (spilled records clump into few bins: per-record
// global cursors serialise on them).  Returns at once when nothing spilled
// (the usual case).
constexpr int kPlaceThreads = 1024;   // 256 measured the same (r05: the launch, not its work)
// The stepped NeRFSmall weights' MFMA copies (hn_render_bwd_args.repack):
// extra workgroups of the placement launch, which runs after the scatter
// kernel's slab reduction has stepped every weight (mlp_pack2_kernel's values)
struct PackK {
  hn_mlp c, f;
  float* P;   // [2][G_END]: the workspace's packed copies (hn_render_fwd's Pc, Pf)
};
__global__ __launch_bounds__(kPlaceThreads) void ovf_place_kernel(BinR k, PackK pk) {
  if (blockIdx.x >= kBwdBlocks) {
    const int idx = (int)(blockIdx.x - kBwdBlocks) * kPlaceThreads + (int)threadIdx.x;
    if (idx < 2 * G_END) pk.P[idx] = idx < G_END ? pack_value(pk.c, idx) : pack_value(pk.f, idx - G_END);
    return;
  }
  __shared__ uint32_t cur[kScMaxBins], lc[kScMaxBins];
  __shared__ uint32_t part[kPlaceThreads];
  const size_t nrec = bin_records(k.nbins, k.cap, k.n_rays);
  uint32_t* idx = const_cast<uint32_t*>(reinterpret_cast<const uint32_t*>(k.bins + 4 * nrec));
  const OvfBook ob = ovf_book(idx, nrec, k.nbins);
  if (*ob.cnt == 0u) return;
  const uint32_t mine = ob.blk[blockIdx.x];
  if (mine == 0u && blockIdx.x != 0) return;   // block 0 publishes `first`
  const int per = (k.nbins + kPlaceThreads - 1) / kPlaceThreads, t = threadIdx.x;
  uint32_t sum = 0;
  for (int j = 0; j < per; ++j) {
    const int bb = t * per + j;
    if (bb < k.nbins) {
      sum += ob.per_bin[bb];
      lc[bb] = 0u;
    }
  }
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < kPlaceThreads; d <<= 1) {   // inclusive scan of the thread sums
    const uint32_t v = t >= d ? part[t - d] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (int j = 0; j < per; ++j) {
    const int bb = t * per + j;
    if (bb < k.nbins) {
      cur[bb] = run;
      if (blockIdx.x == 0) ob.first[bb] = run;
      run += ob.per_bin[bb];
    }
  }
  const size_t o0 = (size_t)blockIdx.x * ovf_per_block(k.n_rays);   // this list, relative to the overflow
  const size_t l0 = (size_t)kBwdBlocks * k.nbins * k.cap + o0;   // first record of this list
  const uint32_t* words = reinterpret_cast<const uint32_t*>(k.bins);
  auto bin_of = [&](uint32_t s) { return (words[rec_wofs(l0 + s, nrec)] & 0x0fffffffu) >> k.shift; };
  for (uint32_t s = t; s < mine; s += kPlaceThreads)
    __hip_atomic_fetch_add(lc + bin_of(s), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  for (int j = 0; j < per; ++j) {
    const int bb = t * per + j;
    if (bb < k.nbins && lc[bb])
      cur[bb] += __hip_atomic_fetch_add(ob.cur + bb, lc[bb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (uint32_t s = t; s < mine; s += kPlaceThreads) {
    const uint32_t pos = __hip_atomic_fetch_add(cur + bin_of(s), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    ob.ids[pos] = (uint32_t)(o0 + s);
  }
}

// Records of the bin, flattened over the producers' regions: thread i takes
// records i, i + 1024, ... (4 at a time, independent loads in flight) and
// finds each one's region by binary search over the LDS prefix of the
// regions' counts.
__global__ __launch_bounds__(kBinThreads) void bin_reduce_kernel(BinR k) {
  extern __shared__ f32x4 acc4[];
  __shared__ uint32_t pre[kBwdBlocks + 1];
  __shared__ uint32_t wsum[kBwdBlocks / 64], wmax[kBwdBlocks / 64];
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(acc4);
  const int n4 = (2 << k.shift) / 2;   // f32x4 = 2 accumulators
  const uint32_t b = (uint32_t)k.bin0 + blockIdx.x;
  const size_t e0 = (size_t)b << (k.shift + 1);   // first float of the slice
  const int nd4 = (2 << k.shift) / 4;             // float4s of the slice (<= 4 per thread)
  // fused step on a coarse level: the row pairs no gradient can reach (their
  // moments are zero, so the dense update leaves p, m, v bitwise unchanged)
  // are neither loaded nor stored (table_live; T=19: levels 0-6)
  const uint32_t* lw = nullptr;
  if (k.fused && k.live && k.shift <= k.log2T && (int)(((uint32_t)b << k.shift) >> k.log2T) < k.live_levels)
    lw = k.live + (((size_t)b << k.shift) >> 6);
  auto live_at = [&](int i) { return lw == nullptr || ((lw[i >> 5] >> (i & 31)) & 1u) != 0u; };
  for (int i = threadIdx.x; i < n4; i += kBinThreads) acc4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const size_t nrec = bin_records(k.nbins, k.cap, k.n_rays);
  const uint32_t* words = reinterpret_cast<const uint32_t*>(k.bins);
  const uint32_t* idx = reinterpret_cast<const uint32_t*>(k.bins + 4 * nrec);   // book base
  const uint32_t* cnt = idx + nrec;
  const float* mxs = reinterpret_cast<const float*>(cnt + (size_t)kBwdBlocks * k.nbins);   // [16][blocks]
  const OvfBook obk = ovf_book(const_cast<uint32_t*>(idx), nrec, k.nbins);
  const uint32_t n_ovf = *obk.cnt;
  static_assert(kBwdBlocks == 256 && kBinThreads >= 256, "one count per thread of waves 0-3");
  // levels of this bin: one, or all 16 when the whole table is one bin
  const int lev0 = (int)(((uint32_t)b << k.shift) >> k.log2T);
  const int nlev = k.shift > k.log2T ? 1 << (k.shift - k.log2T) : 1;
  uint32_t n = 0;
  float mx = 0.f;
  if (threadIdx.x < kBwdBlocks) {
    const uint32_t c = cnt[(size_t)b * kBwdBlocks + threadIdx.x];
    n = c < (uint32_t)k.cap ? c : (uint32_t)k.cap;
    for (int l = lev0; l < lev0 + nlev; ++l) mx = fmaxf(mx, mxs[l * kBwdBlocks + threadIdx.x]);
  }
  const uint32_t inc = (uint32_t)wave_incl_sum((double)n);   // exact: counts < 2^53
  const float wmx = wave_max_f32(mx);
  if (threadIdx.x < kBwdBlocks && (threadIdx.x & 63) == 63) {
    wsum[threadIdx.x >> 6] = inc;
    wmax[threadIdx.x >> 6] = wmx;
  }
  __syncthreads();
  if (threadIdx.x < kBwdBlocks) {
    uint32_t add = 0;
    for (int q = 0; q < (int)(threadIdx.x >> 6); ++q) add += wsum[q];
    pre[threadIdx.x + 1] = inc + add;
  }
  if (threadIdx.x == 0) pre[0] = 0;
  // bin scale: every record value (overflow records included: the producers
  // take every record) is below 2^(E+1) -> below 2^41 units
  const float bmx = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  const int E = ilogbf(bmx > 0.f ? bmx : 1.f);
  // 2^(40 - E) as fp32 (E >= -126 + ... : the scale stays a normal float for
  // every E in [-87, 127]; smaller maxima use 2^127, still < 2^41 units)
  const int S = 40 - (E < -126 ? -126 : E);
  const float scale = ldexpf(1.f, S > 127 ? 127 : S);
  __syncthreads();
  const uint32_t total = pre[kBwdBlocks];
  const uint32_t sel = (1u << k.shift) - 1u, tmask = (1u << k.log2T) - 1u, se = 1u << k.shift;
  // region of the first record of every 64-record chunk: a record's region is
  // then a short forward walk from its chunk's (regions hold ~24-114 records)
  // instead of an 8-step binary search
  __shared__ uint16_t first_reg[kBrChunks];
  const bool tab = ((total + 63) >> 6) <= (uint32_t)kBrChunks;   // uniform
  if (tab) {
    for (uint32_t c = threadIdx.x; c < ((total + 63) >> 6); c += kBinThreads) {
      const uint32_t r = c << 6;
      int lo = 0;
#pragma unroll
      for (int st = kBwdBlocks / 2; st >= 1; st >>= 1)
        if (pre[lo + st] <= r) lo += st;
      first_reg[c] = (uint16_t)lo;
    }
    __syncthreads();
  }
  const size_t bbase = (size_t)b * kBwdBlocks * k.cap;
  // records r0 + q * 1024 (lane-consecutive: coalesced loads), each found in
  // the regions' prefix from its 64-record chunk's first region (a binary
  // search per record measured slower; both faster than one search per 4
  // lane-consecutive records with their 64-B-strided loads); the next group
  // of records is loaded before the current one is added
  auto fetch = [&](uint32_t r0, f32x4 (&v)[kBrDepth], uint32_t (&w)[kBrDepth]) {
#pragma unroll
    for (int q = 0; q < kBrDepth; ++q) {
      const uint32_t r = r0 + q * kBinThreads;
      if (r < total) {
        int lo = 0;   // largest p with pre[p] <= r
        if (tab) {
          lo = first_reg[r >> 6];
          while (pre[lo + 1] <= r) ++lo;   // r < total = pre[kBwdBlocks]: stops by lo = 255
        } else
        {
#pragma unroll
          for (int st = kBwdBlocks / 2; st >= 1; st >>= 1)
            if (pre[lo + st] <= r) lo += st;
        }
        const size_t rec = bbase + (size_t)lo * k.cap + (r - pre[lo]);
        v[q] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(k.bins + rec_vofs(rec)));   // read once
        w[q] = __builtin_nontemporal_load(words + rec_wofs(rec, nrec));
      }
    }
  };
  auto add = [&](uint32_t r0, const f32x4 (&v)[kBrDepth], const uint32_t (&w)[kBrDepth]) {
#pragma unroll
    for (int q = 0; q < kBrDepth; ++q)
      if (r0 + q * kBinThreads < total) {
        bin_add(acc, se, v[q], w[q], sel, tmask, scale);
      }
  };
  f32x4 va[kBrDepth], vb[kBrDepth];
  uint32_t wa[kBrDepth], wb[kBrDepth];
  uint32_t r0 = threadIdx.x;
  if (r0 < total) fetch(r0, va, wa);
  for (; r0 < total; r0 += 2 * kBrDepth * kBinThreads) {
    const uint32_t r1 = r0 + kBrDepth * kBinThreads;
    if (r1 < total) fetch(r1, vb, wb);
    add(r0, va, wa);
    if (r1 >= total) break;
    if (r1 + kBrDepth * kBinThreads < total) fetch(r1 + kBrDepth * kBinThreads, va, wa);
    add(r1, vb, wb);
  }
  if (n_ovf) {   // this bin's spilled records (bucketed by ovf_place_kernel)
    const size_t ob = (size_t)kBwdBlocks * k.nbins * k.cap;
    const uint32_t lo = obk.first[b], hi = lo + obk.per_bin[b];
    for (uint32_t s = lo + threadIdx.x; s < hi; s += kBinThreads) {
      const uint32_t o = obk.ids[s];
      bin_add(acc, se, *reinterpret_cast<const f32x4*>(k.bins + rec_vofs(ob + o)), words[rec_wofs(ob + o, nrec)],
              sel, tmask, scale);
    }
  }
  __syncthreads();
  const double inv = 1.0 / (double)scale;
  float4* dst = k.d_table ? reinterpret_cast<float4*>(k.d_table + e0) : nullptr;
  if (k.fused && dst == nullptr) {
    // fused step: the thread's live flags, then all of its p, m, v loads in
    // flight at once (one HBM round trip instead of one per float4: the
    // pass 90.5 -> 88.6 us on config 2)
    bool lv[kSliceF4];
#pragma unroll
    for (int j = 0; j < kSliceF4; ++j) {
      const int i = threadIdx.x + j * kBinThreads;
      lv[j] = i < nd4 && live_at(i);
    }
    f32x4 p4[kSliceF4], m4[kSliceF4], v4[kSliceF4];
#pragma unroll
    for (int j = 0; j < kSliceF4; ++j) {
      const int i = threadIdx.x + j * kBinThreads;
      if (lv[j]) {
        p4[j] = reinterpret_cast<const f32x4*>(k.step.p + e0)[i];
        m4[j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(k.step.m + e0) + i);
        v4[j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(k.step.v + e0) + i);
      }
    }
#pragma unroll
    for (int j = 0; j < kSliceF4; ++j) {
      const int i = threadIdx.x + j * kBinThreads;
      if (i >= nd4) break;
      float4 a;
      a.x = (float)((double)(long long)acc[2 * i] * inv);
      a.y = (float)((double)(long long)acc[se + 2 * i] * inv);
      a.z = (float)((double)(long long)acc[2 * i + 1] * inv);
      a.w = (float)((double)(long long)acc[se + 2 * i + 1] * inv);
      if (!lv[j]) {
        if (a.x != 0.f || a.y != 0.f || a.z != 0.f || a.w != 0.f)
          __hip_atomic_fetch_or(&g_hn_fault, kFaultDeadRow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      float4 p{p4[j][0], p4[j][1], p4[j][2], p4[j][3]}, m{m4[j][0], m4[j][1], m4[j][2], m4[j][3]},
          v{v4[j][0], v4[j][1], v4[j][2], v4[j][3]};
      radam_elem(k.step, p.x, a.x, m.x, v.x);
      radam_elem(k.step, p.y, a.y, m.y, v.y);
      radam_elem(k.step, p.z, a.z, m.z, v.z);
      radam_elem(k.step, p.w, a.w, m.w, v.w);
      __builtin_nontemporal_store(f32x4{m.x, m.y, m.z, m.w}, reinterpret_cast<f32x4*>(k.step.m + e0) + i);
      __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(k.step.v + e0) + i);
      if (k.step.mode != 0) reinterpret_cast<f32x4*>(k.step.p + e0)[i] = f32x4{p.x, p.y, p.z, p.w};
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < kSliceF4; ++j) {   // entries 2i, 2i + 1
    const int i = threadIdx.x + j * kBinThreads;
    if (i >= nd4) break;
    float4 a;
    a.x = (float)((double)(long long)acc[2 * i] * inv);
    a.y = (float)((double)(long long)acc[se + 2 * i] * inv);
    a.z = (float)((double)(long long)acc[2 * i + 1] * inv);
    a.w = (float)((double)(long long)acc[se + 2 * i + 1] * inv);
    if (dst) {
      if (!k.overwrite) {
        const float4 d = dst[i];
        a.x = a.x + d.x; a.y = a.y + d.y; a.z = a.z + d.z; a.w = a.w + d.w;
      }
      dst[i] = a;
    }
    if (k.fused && !live_at(i)) {   // a dead pair: its gradient is a structural zero
      if (a.x != 0.f || a.y != 0.f || a.z != 0.f || a.w != 0.f)
        __hip_atomic_fetch_or(&g_hn_fault, kFaultDeadRow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (k.fused) {   // RAdam on these 4 table elements (radam_kernel's update, same op forms)
      f32x4* pp = reinterpret_cast<f32x4*>(k.step.p + e0) + i;
      f32x4* pm = reinterpret_cast<f32x4*>(k.step.m + e0) + i;
      f32x4* pv = reinterpret_cast<f32x4*>(k.step.v + e0) + i;
      // m and v are nontemporal (next read by the next step's owner pass);
      // p stays cached: the next forward gathers it (p nontemporal too
      // measured the forward +10 us)
      const f32x4 p4 = *pp, m4 = __builtin_nontemporal_load(pm), v4 = __builtin_nontemporal_load(pv);
      float4 p{p4[0], p4[1], p4[2], p4[3]}, m{m4[0], m4[1], m4[2], m4[3]}, v{v4[0], v4[1], v4[2], v4[3]};
      radam_elem(k.step, p.x, a.x, m.x, v.x);
      radam_elem(k.step, p.y, a.y, m.y, v.y);
      radam_elem(k.step, p.z, a.z, m.z, v.z);
      radam_elem(k.step, p.w, a.w, m.w, v.w);
      __builtin_nontemporal_store(f32x4{m.x, m.y, m.z, m.w}, pm);
      __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, pv);
      if (k.step.mode != 0) *pp = f32x4{p.x, p.y, p.z, p.w};
    }
  }
}

static int32_t check_cfg(const hn_render_cfg* c) {
  if (!c) return HN_E_NULL;
  const hn_grid& g = c->grid;
  if (g.n_levels != 16 || g.n_features != 2) return HN_E_SHAPE;
  if (g.log2_hashmap_size < 1 || g.log2_hashmap_size > 24) return HN_E_SHAPE;
  if (c->n_samples != kSc || c->n_importance != kNi) return HN_E_SHAPE;
  if (c->scatter < 0 || c->scatter > 2) return HN_E_SHAPE;
  if (c->bin_cap < 0 || (c->bin_cap & 63)) return HN_E_SHAPE;
  if (c->dense_bwd < 0 || c->dense_bwd > 1) return HN_E_SHAPE;
  return HN_OK;
}

static bool mlp_ok(const hn_mlp& w) { return w.sigma0 && w.sigma1 && w.color0 && w.color1 && w.color2; }
static bool grad_ok(const hn_mlp_grad& w) {
  return w.sigma0 && w.sigma1 && w.color0 && w.color1 && w.color2;
}

// Binned scatter geometry.  A bin is 2^13 consecutive table entries (its
// 2 x 2^13 64-bit accumulators are the owner's 128 KiB of LDS), or the whole
// table when that is smaller.  Region capacity per (block, bin): the records
// a block's rays can write into one bin without any run merging on average
// (192 unique points x 4 corner rows per level and ray, spread over the
// level's 2^T / 2^shift bins) + 128; sized so, a region overflows only on
// strongly clumped input (into the shared overflow records).
struct BinGeom {
  int shift, nbins, cap;
  size_t floats;
};
static BinGeom bin_geom(int T, int64_t n_rays, int cap_override) {
  BinGeom g;
  // 2^12-entry bins (64 KiB of accumulators: two owner workgroups per CU;
  // compile-time HN_BIN_SHIFT_DEFAULT=12) unless that needs more bins than the
  // scatter's LDS counters hold
  const int want = T + 4 - kBinShift <= kScMaxBinsLog2 ? kBinShift : 13;
  g.shift = T + 4 < want ? T + 4 : want;
  g.nbins = 1 << (T + 4 - g.shift);
  const double rpb = (double)((n_rays + kBwdBlocks - 1) / kBwdBlocks);
  const double avg = rpb * (kSf * 4) * ldexp(1.0, g.shift - T);
  g.cap = cap_override > 0 ? cap_override : (int)(((int64_t)avg + 128 + 63) & ~(int64_t)63);
  // an odd multiple of 64 records: the regions' stride (16 B x cap) then has
  // as few factors of two as the 64-record granule allows.  Measured on
  // config 2 (scatter / owner): 320 224 / 225 us, 448 227 / 226, 384 233 /
  // 224, 256 247 / 237, 512 254 / 235 -- the 256 regions of a bin at a
  // power-of-two stride share memory channels
  if (cap_override <= 0 && ((g.cap >> 6) & 1) == 0) g.cap += 64;
  const size_t nrec = bin_records(g.nbins, g.cap, n_rays);
  g.floats = nrec * 5 + (size_t)kBwdBlocks * (g.nbins + 16) + ovf_book_words(g.nbins, n_rays) + 4;
  return g;
}
// Backward schedule: cfg->scatter 1 = float atomics (fused), 2 or 0 = binned
// (split).  The binned scatter keeps per-bin counters in LDS: nbins <=
// kScMaxBins (T <= 22); past that, and where a record's two x corners could
// leave one bin, the float-atomic schedule runs.  (The release library reads
// no environment: every schedule choice is in hn_render_cfg.)
static int bwd_mode(const hn_render_cfg* c, int64_t n_rays) {
  if (!c) return kModeAtomic;
  const int want = c->scatter == 1 ? kModeAtomic : kModeSplit;
  const int T = c->grid.log2_hashmap_size;
  if (want != kModeSplit || (16ll << T) > (long long)kScMaxBins << 13) return kModeAtomic;
  // A record keeps its x1 corner's row as h(x0) ^ (2^nbits - 1), nbits =
  // ctz(~x0) + 1 <= bit_length(x0) + 1 (4 bits of the entry word), and assumes
  // both rows lie in one bin.  The cell index of a clamped point is at most
  // (bmax - bmin) / grid_size, so that must fit the bin (or the level, when a
  // bin holds whole levels: the xor is taken modulo 2^T).
  const int shift = bin_geom(T, n_rays, c->bin_cap).shift;
  if (shift < T) {
    double cells = 0.0;
    for (int l = 0; l < c->grid.n_levels; ++l)
      for (int a = 0; a < 3; ++a) {
        const double gs = c->grid.grid_size[l][a];
        const double n = gs > 0.0 ? ((double)c->grid.box_max[a] - c->grid.box_min[a]) / gs : 1e30;
        cells = n > cells ? n : cells;
      }
    int bits = 0;
    while (bits < 40 && ldexp(1.0, bits) <= cells + 1.0) ++bits;   // bit_length of the largest cell index
    if (bits + 1 > shift || bits + 1 > 15) return kModeAtomic;
  }
  return kModeSplit;
}
// Workspace (floats): packed coarse + fine weights | dW slabs [256][2][9344] |
// coarse-pass feature grads [n][64][32] | d raw [n][256][4] | unit marks [n][4] u8 + wave split | split: fine
// feature grads [n][6][1024] and the records (bin_geom).
struct WsLayout {
  size_t dfeat_f, bins, total;
};
static WsLayout ws_layout(const hn_render_cfg* cfg, int64_t n_rays, int mode) {
  const size_t n = n_rays > 0 ? (size_t)n_rays : 0;
  WsLayout w;
  w.dfeat_f = (size_t)2 * G_END + (size_t)kBwdBlocks * kSlabSlots * W_END + n * kDcRay + n * (kSc + kSf) * 4 +
              ((29 * n + 8 + 3) & ~(size_t)3);   // + the marks [n][4] u8, the lists' counts [8], the lists
                                                 // [(4 + 12 + 12) n]
  w.bins = w.dfeat_f + (mode == kModeSplit ? n * kSf * 32 : 0);
  w.total = w.bins + (mode == kModeSplit ? bin_geom(cfg->grid.log2_hashmap_size, n_rays, cfg->bin_cap).floats : 0);
  return w;
}

}  // namespace hn

using namespace hn;

// Workspace: packed coarse + fine weights | dW slabs [256][2][9344] |
// coarse-pass feature grads [n_rays][64][32] | d raw [n_rays][256][4] |
// binned-scatter records (bin_geom) when the binned scatter is used.
extern "C" size_t hn_render_workspace_bytes(const hn_render_cfg* cfg, int64_t n_rays) {
  return ws_layout(cfg, n_rays, bwd_mode(cfg, n_rays)).total * sizeof(float);
}

extern "C" int32_t hn_render_scatter_mode(const hn_render_cfg* cfg, int64_t n_rays) {
  return bwd_mode(cfg, n_rays) == kModeSplit ? 2 : 1;
}

extern "C" int32_t hn_device_faults(int32_t* faults, int32_t clear) {
  if (!faults) return HN_E_NULL;
  int32_t st = hip_status(hipMemcpyFromSymbol(faults, HIP_SYMBOL(g_hn_fault), sizeof(int32_t)));
  if (st || !clear || *faults == 0) return st;
  const int32_t zero = 0;
  return hip_status(hipMemcpyToSymbol(HIP_SYMBOL(g_hn_fault), &zero, sizeof(int32_t)));
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
  if (!a->weights_packed && (st = mlp_pack2_launch(&a->coarse, Pc, &a->fine, Pf, s))) return st;
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
  k.raw_c = a->raw_c; k.raw_f = a->raw_f; k.fine_src = a->fine_src; k.feat = a->feat;
  // the saved features (32 KB + 6 KB per ray) go through L2 while the table
  // (16 x 2^T x 8 B) leaves room for them in the 256 MiB MALL, where the
  // backward finds them (config 2, T=19: forward 260.7 -> 253.6 us, step
  // -8 us); past it they are streamed (config 3, T=22, cached: forward
  // 633 -> 682 us)
  k.feat_nt = cfg->grid.log2_hashmap_size > 20;
  k.skip_dead = a->skip_dead_color != 0;
  const unsigned blocks = (unsigned)((a->n_rays + kFwdBlockWaves - 1) / kFwdBlockWaves);
  hipLaunchKernelGGL(render_fwd_kernel, dim3(blocks), dim3(64 * kFwdBlockWaves), 0, s, k);
#if HN_PROFILE
  {
    unsigned long long f[8];
    (void)hipStreamSynchronize(s);
    (void)hipMemcpyFromSymbol(f, HIP_SYMBOL(g_fwd_prof), sizeof(f));
    const double w = f[7] ? (double)f[7] : 1.;
    fprintf(stderr, "hn_fwd_profile cycles/wave: coarse encode %.0f mlp %.0f | sample %.0f | fine encode %.0f "
            "mlp %.0f | composite %.0f | total %.0f\n", f[0] / w, f[1] / w, f[2] / w, f[3] / w, f[4] / w,
            f[5] / w, f[6] / w);
    memset(f, 0, sizeof(f));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fwd_prof), f, sizeof(f));
  }
#endif
  return hip_status(hipGetLastError());
}

// The owner pass's arguments (bins [bin0, ...) of one launch)
static BinR owner_args(const hn_render_cfg* cfg, const hn_render_bwd_args* a, float* bins, const BinGeom& bg,
                       int bin0) {
  BinR r;
  r.bins = bins;
  r.n_rays = a->n_rays;
  r.nbins = bg.nbins;
  r.cap = bg.cap;
  r.shift = bg.shift;
  r.log2T = cfg->grid.log2_hashmap_size;
  r.d_table = a->d_table;
  r.overwrite = (a->d_table_mode & 1) != 0;
  r.fused = a->table_step != nullptr;
  if (r.fused) r.step = *a->table_step;
  r.live = r.fused ? a->table_live : nullptr;
  r.live_levels = r.live ? a->table_live_levels : 0;
  r.bin0 = bin0;
  return r;
}

extern "C" int32_t hn_render_bins(const hn_render_cfg* cfg, int64_t n_rays, int32_t* shift) {
  if (!cfg || !shift) return 0;
  if (check_cfg(cfg) || bwd_mode(cfg, n_rays) != kModeSplit) {
    *shift = 0;
    return 0;
  }
  const BinGeom bg = bin_geom(cfg->grid.log2_hashmap_size, n_rays, cfg->bin_cap);
  *shift = bg.shift;
  return bg.nbins;
}

extern "C" int32_t hn_render_bwd_owner(const hn_render_cfg* cfg, const hn_render_bwd_args* a, void* workspace,
                                       size_t ws_bytes, int32_t bin_lo, int32_t bin_hi, void* stream) {
  int32_t st = check_cfg(cfg);
  if (st) return st;
  if (!a || !workspace) return HN_E_NULL;
  if (!a->owner_defer || a->n_rays <= 0 || bwd_mode(cfg, a->n_rays) != kModeSplit) return HN_E_SHAPE;
  if (!a->d_table && !a->table_step) return HN_E_NULL;
  if (ws_bytes < hn_render_workspace_bytes(cfg, a->n_rays)) return HN_E_WORKSPACE;
  const BinGeom bg = bin_geom(cfg->grid.log2_hashmap_size, a->n_rays, cfg->bin_cap);
  if (bin_lo < 0 || bin_hi > bg.nbins || bin_lo > bin_hi) return HN_E_SHAPE;
  if (bin_lo == bin_hi) return HN_OK;
  const WsLayout wl = ws_layout(cfg, a->n_rays, kModeSplit);
  const BinR r = owner_args(cfg, a, (float*)workspace + wl.bins, bg, bin_lo);
  hipLaunchKernelGGL(bin_reduce_kernel, dim3((unsigned)(bin_hi - bin_lo)), dim3(kBinThreads),
                     (size_t)(2 << bg.shift) * sizeof(unsigned long long), (hipStream_t)stream, r);
  return hip_status(hipGetLastError());
}

// hn_render_bwd with no rays and a TV term (ABI 14): a data-parallel rank that
// drew no rays still carries the TV term (train.dp_loss puts it on rank 0,
// run_nerf.py:551-555 / :626-635).  Its gradient goes through the same TV
// records, overflow placement and exact fixed-point owner pass as a rendering
// rank's (scatter_bins_kernel with no units and no slab reduction), so it is
// bitwise reproducible where hn_tv_bwd's float atomics are not.
static int32_t tv_only_bwd(const hn_render_cfg* cfg, const hn_render_bwd_args* a, void* workspace,
                           size_t ws_bytes, hipStream_t s) {
  const int T = cfg->grid.log2_hashmap_size;
  if (!a->g_tv || (!a->d_table && !a->table_step) || !workspace) return HN_E_NULL;
  if (a->d_table_mode < 0 || a->d_table_mode > 3 || a->owner_defer || a->mlp_step || a->repack || a->loss)
    return HN_E_SHAPE;
  if (bwd_mode(cfg, 0) != kModeSplit) return HN_E_SHAPE;
  if (a->table_step) {
    const hn_radam_tensor& ts = *a->table_step;
    if (ts.n != ((int64_t)16 << T) * 2) return HN_E_SHAPE;
    if (!ts.p || !ts.m || !ts.v) return HN_E_NULL;
    if (a->table_live && (a->table_live_levels < 0 || a->table_live_levels > cfg->grid.n_levels || T < 6))
      return HN_E_SHAPE;
  }
  TvK tvk;
  int nbf, nbb;
  int32_t st = make_tv(a->tv, tvk, nbf, nbb);
  if (st) return st;
  if (a->tv->n_levels != cfg->grid.n_levels || a->tv->log2_hashmap_size != T) return HN_E_SHAPE;
  for (int l = 0; l < a->tv->n_levels; ++l)
    if (a->tv->cube[l] > kTvRecMaxCube) return HN_E_SHAPE;
  if (ws_bytes < hn_render_workspace_bytes(cfg, 0)) return HN_E_WORKSPACE;
  const BinGeom bg = bin_geom(T, 0, cfg->bin_cap);
  const size_t sc_lds = sc_lds_bytes(bg.nbins);
  if (sc_lds + sc_static_lds() > kLdsMax) return HN_E_SHAPE;
  float* bins = (float*)workspace + ws_layout(cfg, 0, kModeSplit).bins;
  // the overflow book starts empty (render_comp_bwd_kernel's zero_ovf_book
  // on a rendering rank): total, per-bin spills, placement cursors
  const size_t nrec = bin_records(bg.nbins, bg.cap, 0);
  const OvfBook ob = ovf_book(reinterpret_cast<uint32_t*>(bins + 4 * nrec), nrec, bg.nbins);
  if ((st = hip_status(hipMemsetAsync(ob.cnt, 0, (1 + 2 * (size_t)bg.nbins) * sizeof(uint32_t), s)))) return st;
  ScK sk{};
  sk.g = make_grid_args(cfg->grid);
  sk.B = 0;
  sk.bins = bins;
  sk.bin_cap = bg.cap;
  sk.bin_shift = bg.shift;
  sk.nbins = bg.nbins;
  sk.g_tv = a->g_tv;
  sk.tv = tvk;
  int off = 0;
  for (int l = 0; l < a->tv->n_levels; ++l) {
    sk.tv_off[l] = off;
    const int n1 = a->tv->cube[l] + 1;
    off += (n1 + 1) / 2 * n1 * n1;
  }
  for (int l = a->tv->n_levels; l <= 16; ++l) sk.tv_off[l] = off;
  sk.slab = nullptr;   // no MLP gradients: the caller's stay untouched
  hipLaunchKernelGGL(scatter_bins_kernel, dim3(kBwdBlocks), dim3(64 * kScWaves), sc_lds, s, sk);
  if ((st = hip_status(hipGetLastError()))) return st;
  hn_render_bwd_args b = *a;
  b.n_rays = 0;
  const BinR r = owner_args(cfg, &b, bins, bg, 0);
  hipLaunchKernelGGL(ovf_place_kernel, dim3(kBwdBlocks), dim3(kPlaceThreads), 0, s, r, PackK{});
  if ((st = hip_status(hipGetLastError()))) return st;
  hipLaunchKernelGGL(bin_reduce_kernel, dim3((unsigned)bg.nbins), dim3(kBinThreads),
                     (size_t)(2 << bg.shift) * sizeof(unsigned long long), s, r);
  return hip_status(hipGetLastError());
}

extern "C" int32_t hn_render_bwd(const hn_render_cfg* cfg, const hn_render_bwd_args* a,
                                 void* workspace, size_t ws_bytes, void* stream) {
  int32_t st = check_cfg(cfg);
  if (st) return st;
  if (!a) return HN_E_NULL;
  if (a->n_rays < 0) return HN_E_SHAPE;
  if (a->n_rays == 0) return a->tv ? tv_only_bwd(cfg, a, workspace, ws_bytes, (hipStream_t)stream) : HN_OK;
  if (!a->rays || !a->table || !mlp_ok(a->coarse) || !mlp_ok(a->fine)) return HN_E_NULL;
  if (!a->z_coarse || !a->z_fine || !a->raw_c || !a->raw_f || !a->fine_src || !a->feat)
    return HN_E_NULL;
  if ((!a->d_table && !a->table_step) || !grad_ok(a->d_coarse) || !grad_ok(a->d_fine)) return HN_E_NULL;
  if (a->d_table_mode < 0 || a->d_table_mode > 3) return HN_E_SHAPE;
  if (!workspace) return HN_E_NULL;
  if (ws_bytes < hn_render_workspace_bytes(cfg, a->n_rays)) return HN_E_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* Pc = (float*)workspace;
  float* Pf = Pc + G_END;
  float* slab = Pf + G_END;
  float* dfeat = slab + (size_t)kBwdBlocks * kSlabSlots * W_END;
  float* draw = dfeat + (size_t)a->n_rays * kDcRay;
  uint8_t* uflags = reinterpret_cast<uint8_t*>(draw + (size_t)a->n_rays * (kSc + kSf) * 4);
  if (!a->weights_packed && (st = mlp_pack2_launch(&a->coarse, Pc, &a->fine, Pf, s))) return st;
  B1K k;
  k.B = a->n_rays;
  k.scramble = 0;
  if (a->n_rays > 1) {
    int bits = 2;
    while ((1ll << bits) < a->n_rays) bits += 2;
    k.scramble = bits / 2;
  }
  k.white = cfg->white_bkgd;
  k.rays = a->rays; k.noise_c = a->noise_c; k.noise_f = a->noise_f;
  k.Pc = Pc; k.Pf = Pf;
  k.z_coarse = a->z_coarse; k.z_fine = a->z_fine; k.raw_c = a->raw_c; k.raw_f = a->raw_f;
  k.feat = a->feat;
  k.g_rgb = a->g_rgb; k.g_depth = a->g_depth; k.g_acc = a->g_acc; k.g_sparsity = a->g_sparsity;
  k.g_rgb0 = a->g_rgb0; k.g_depth0 = a->g_depth0; k.g_acc0 = a->g_acc0;
  k.g_sparsity0 = a->g_sparsity0; k.g_raw_f = a->g_raw_f;
  k.slab = slab;
  k.dfeat = dfeat;
  k.draw = draw;
  k.uflags = uflags;
  // the work lists' counts and the lists, after the marks
  k.lmeta = reinterpret_cast<int32_t*>(uflags + kMarkB * (size_t)a->n_rays);
  k.lists = k.lmeta + 8;
  k.ltarget = k.lrgb = k.lrgb0 = k.lsp = k.lsp0 = k.ltv = nullptr;
  k.n_tv = 0;
  k.lgm = k.lsparse = k.lworld = k.lsparse_w = k.ltv_w = 0.f;
  k.lout = nullptr;
  k.skip_zero = cfg->dense_bwd ? 0 : 1;
  if (a->loss) {   // ABI 13: the training loss formed by the pre-pass (hn_render_loss)
    const hn_render_loss& L = *a->loss;
    if (!L.target || !L.rgb || !L.rgb0 || !L.sparsity || !L.sparsity0 || !L.out || (L.n_tv && !L.tv))
      return HN_E_NULL;
    if (L.n_tv < 0 || !(L.world > 0.f)) return HN_E_SHAPE;
    const float g = 1.f;   // hn_loss_bwd's factors with g_loss = 1
    k.lgm = (g / L.world) / (float)(3 * a->n_rays);
    k.lsparse = g * L.sparse_w;
    k.ltarget = L.target; k.lrgb = L.rgb; k.lrgb0 = L.rgb0; k.lsp = L.sparsity; k.lsp0 = L.sparsity0;
    k.ltv = L.n_tv ? L.tv : nullptr;
    k.n_tv = L.n_tv;
    k.lworld = L.world; k.lsparse_w = L.sparse_w; k.ltv_w = L.tv_w;
    k.lout = L.out;
  }
  k.g = make_grid_args(cfg->grid);
  k.fine_src = a->fine_src;
  k.d_table = a->d_table;
  const int T = cfg->grid.log2_hashmap_size;
  const int mode = bwd_mode(cfg, a->n_rays);
  if (a->table_step) {   // the fused step lives in the binned scatter's owner pass
    const hn_radam_tensor& ts = *a->table_step;
    if (mode != kModeSplit || ts.n != ((int64_t)16 << cfg->grid.log2_hashmap_size) * 2) return HN_E_SHAPE;
    if (!ts.p || !ts.m || !ts.v) return HN_E_NULL;
    if (a->table_live && (a->table_live_levels < 0 || a->table_live_levels > cfg->grid.n_levels || T < 6))
      return HN_E_SHAPE;
  }
  // TV term: records of the binned scatter, or hn_tv_bwd into d_table (atomic schedule)
  TvK tvk;
  bool tv_rec = false, tv_atomic = false;
  if (a->tv) {
    if (!a->g_tv) return HN_E_NULL;
    int nbf, nbb;
    if ((st = make_tv(a->tv, tvk, nbf, nbb))) return st;
    if (a->tv->n_levels != cfg->grid.n_levels || a->tv->log2_hashmap_size != T) return HN_E_SHAPE;
    bool small = a->tv->n_levels <= 16;
    for (int l = 0; l < a->tv->n_levels && small; ++l) small = a->tv->cube[l] <= kTvRecMaxCube;
    if (mode == kModeSplit && small) {   // the overflow lists hold these records (ovf_per_block)
      tv_rec = true;
    } else {
      if (a->table_step || !a->d_table) return HN_E_SHAPE;
      tv_atomic = true;
    }
  }
  if (a->owner_defer && mode != kModeSplit) return HN_E_SHAPE;
  if (a->repack && !a->mlp_step) return HN_E_SHAPE;
  if (a->mlp_step) {   // the MLP steps live in the binned scatter's slab reduction
    if (mode != kModeSplit) return HN_E_SHAPE;
    static constexpr int64_t numel[5] = {W_S1, W_C0 - W_S1, W_C1 - W_C0, W_C2 - W_C1, W_END - W_C2};
    for (int t = 0; t < 10; ++t) {
      const hn_radam_tensor& r = a->mlp_step[t];
      if (!r.p || !r.m || !r.v) return HN_E_NULL;
      if (r.n != numel[t % 5]) return HN_E_SHAPE;
    }
  }
  const WsLayout wl = ws_layout(cfg, a->n_rays, mode);
  // the scatter's LDS (bins' counters + staging pool), checked before anything is queued
  size_t sc_lds = 0;
  if (mode == kModeSplit) {
    sc_lds = sc_lds_bytes(bin_geom(T, a->n_rays, cfg->bin_cap).nbins);
    if (sc_lds + sc_static_lds() > kLdsMax) return HN_E_SHAPE;   // bins beyond the LDS counters' room
  }
  BinGeom bg{};
  k.bins = nullptr;
  k.bin_cap = k.bin_shift = k.nbins = 0;
  k.dfeat_f = mode == kModeSplit ? (float*)workspace + wl.dfeat_f : nullptr;
  if (mode != kModeAtomic) {
    bg = bin_geom(T, a->n_rays, cfg->bin_cap);
    k.bins = (float*)workspace + wl.bins;
    k.bin_cap = bg.cap;
    k.bin_shift = bg.shift;
    k.nbins = bg.nbins;
  } else if (a->d_table_mode & 1) {
    const size_t tb = ((size_t)16 << T) * 2 * sizeof(float);
    if ((st = hip_status(hipMemsetAsync(a->d_table, 0, tb, s)))) return st;
  }
  hipLaunchKernelGGL(render_comp_bwd_kernel,
                     dim3((unsigned)((2 * a->n_rays + kFwdWaves - 1) / kFwdWaves + (k.lout ? 1 : 0))),
                     dim3(64 * kFwdWaves), 0, s, k);
  const size_t lds = (size_t)kB1LdsF * sizeof(float);
  if (mode == kModeSplit) {   // the backward's work lists (from the pre-pass's marks)
    const int64_t nlb = (a->n_rays + kListThreads - 1) / kListThreads;
    hipLaunchKernelGGL(render_lists_kernel, dim3((unsigned)(nlb < kListMaxBlocks ? nlb : kListMaxBlocks)),
                       dim3(kListThreads), 0, s, k);
    if ((st = hip_status(hipGetLastError()))) return st;
  }
  // 16 levels x 2^T x 8 B >= 256 MiB from T = 21: the table no longer fits the MALL
  if (mode == kModeSplit)
    hipLaunchKernelGGL((render_bwd_kernel<HN_SW_VMCNT, kModeSplit>), dim3(kBwdBlocks), dim3(64 * kB1Waves), lds, s,
                       k);
  else if (T >= 21)
    hipLaunchKernelGGL((render_bwd_kernel<HN_SW_VMCNT_BIG, kModeAtomic>), dim3(kBwdBlocks), dim3(64 * kB1Waves),
                       lds, s, k);
  else
    hipLaunchKernelGGL((render_bwd_kernel<HN_SW_VMCNT, kModeAtomic>), dim3(kBwdBlocks), dim3(64 * kB1Waves), lds,
                       s, k);
  if ((st = hip_status(hipGetLastError()))) return st;
  if (mode == kModeSplit) {
    ScK sk;
    sk.g = k.g;
    sk.B = a->n_rays;
    sk.rays = a->rays;
    sk.draw = draw;
    sk.scramble = k.scramble;
    sk.skip_zero = k.skip_zero;
    sk.lmeta = k.lmeta;
    // the scatter's group list
    sk.slist = k.skip_zero ? k.lists + 16 * a->n_rays : nullptr;
    sk.z_fine = a->z_fine;
    sk.fine_src = a->fine_src;
    sk.dfeat_f = k.dfeat_f;
    sk.dfeat_c = k.dfeat;
    sk.bins = k.bins;
    sk.bin_cap = k.bin_cap;
    sk.bin_shift = k.bin_shift;
    sk.nbins = k.nbins;
    for (int l = 0; l <= 16; ++l) sk.tv_off[l] = 0;
    sk.g_tv = a->g_tv;
    if (tv_rec) {
      sk.tv = tvk;
      int off = 0;
      for (int l = 0; l < a->tv->n_levels; ++l) {
        sk.tv_off[l] = off;
        const int n1 = a->tv->cube[l] + 1;
        off += (n1 + 1) / 2 * n1 * n1;
      }
      for (int l = a->tv->n_levels; l <= 16; ++l) sk.tv_off[l] = off;
    }
    sk.slab = slab;
    sk.dc = a->d_coarse;
    sk.df = a->d_fine;
    sk.overwrite_mlp = (a->d_table_mode & 2) ? 1 : 0;
    sk.has_mstep = a->mlp_step != nullptr;
    for (int t = 0; t < 10; ++t) sk.mstep[t] = sk.has_mstep ? a->mlp_step[t] : hn_radam_tensor{};
    hipLaunchKernelGGL(scatter_bins_kernel, dim3(kBwdBlocks), dim3(64 * kScWaves), sc_lds, s, sk);
    if ((st = hip_status(hipGetLastError()))) return st;
  }
  if (mode != kModeAtomic) {
    const BinR r = owner_args(cfg, a, k.bins, bg, 0);
    PackK pk{};
    unsigned pblocks = 0;
    if (a->repack) {   // checked above: mlp_step given, binned scatter
      pk.c = a->coarse;
      pk.f = a->fine;
      pk.P = (float*)workspace;
      pblocks = (unsigned)((2 * G_END + kPlaceThreads - 1) / kPlaceThreads);
    }
    hipLaunchKernelGGL(ovf_place_kernel, dim3(kBwdBlocks + pblocks), dim3(kPlaceThreads), 0, s, r, pk);
    if ((st = hip_status(hipGetLastError()))) return st;
    if (!a->owner_defer) {
      hipLaunchKernelGGL(bin_reduce_kernel, dim3((unsigned)bg.nbins), dim3(kBinThreads),
                         (size_t)(2 << bg.shift) * sizeof(unsigned long long), s, r);
      if ((st = hip_status(hipGetLastError()))) return st;
    }
  }
  if (mode != kModeSplit) {
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(kSlabVBlocks), dim3(64 * kSlabGroups), 0, s, slab, kBwdBlocks,
                       a->d_coarse, a->d_fine, (a->d_table_mode & 2) ? 1 : 0);
    if ((st = hip_status(hipGetLastError()))) return st;
  }
  if (tv_atomic) return hn_tv_bwd(a->tv, a->g_tv, a->d_table, stream);
  return HN_OK;
}
