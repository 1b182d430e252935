// hn_common.h -- device building blocks shared by every HashNeRF kernel (gfx950).
//
// Compiled with -ffp-contract=off: every fp32 expression below rounds after
// each operation exactly like the reference's sequence of eager torch ops, so
// the hash-grid encoding and SH features are bit-identical to the reference.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hashnerf_amd.h"

#define HN_DEV __device__ __forceinline__

namespace hn {

constexpr uint32_t kPrimeY = 2654435761u;   // hash_encoding.py:7
constexpr uint32_t kPrimeZ = 805459861u;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Kernel-argument copy of hn_grid (passed by value).
struct GridArgs {
  int32_t n_levels;
  int32_t log2T;
  float bmin[3];
  float bmax[3];
  float gs[HN_MAX_LEVELS][3];
};

inline GridArgs make_grid_args(const hn_grid& g) {
  GridArgs a;
  a.n_levels = g.n_levels;
  a.log2T = g.log2_hashmap_size;
  for (int i = 0; i < 3; ++i) { a.bmin[i] = g.box_min[i]; a.bmax[i] = g.box_max[i]; }
  for (int l = 0; l < HN_MAX_LEVELS; ++l)
    for (int i = 0; i < 3; ++i) a.gs[l][i] = g.grid_size[l][i];
  return a;
}

// torch.clamp(x, min=lo, max=hi) with NaN propagation (hash_encoding.py:69).
HN_DEV float clamp_t(float x, float lo, float hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}

// One hash level of one point (hash_encoding.py:59-82 + :112-128 + :143).
//   xc: clamped point (corners), x: unclamped point (trilinear weights).
// Outputs the 8 hashed row indices (corner c = 4i+2j+k) and the weights.
struct Voxel {
  uint32_t h[8];
  float w[3];
};

HN_DEV void voxel_level(const float x[3], const float xc[3], const float gs[3],
                        const float bmin[3], uint32_t mask, Voxel& v) {
  uint32_t c[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float q = (xc[a] - bmin[a]) / gs[a];
    const int32_t i = (int32_t)floorf(q);                 // floor(...).int()
    const float vmin = (float)i * gs[a] + bmin[a];        // idx * grid + min
    const float vmax = vmin + gs[a];                      // + 1.0 * grid
    v.w[a] = (x[a] - vmin) / (vmax - vmin);
    c[a] = (uint32_t)i;
  }
  const uint32_t x0 = c[0], x1 = c[0] + 1u;               // prime 1
  const uint32_t y0 = c[1] * kPrimeY, y1 = (c[1] + 1u) * kPrimeY;
  const uint32_t z0 = c[2] * kPrimeZ, z1 = (c[2] + 1u) * kPrimeZ;
  v.h[0] = (x0 ^ y0 ^ z0) & mask;
  v.h[1] = (x0 ^ y0 ^ z1) & mask;
  v.h[2] = (x0 ^ y1 ^ z0) & mask;
  v.h[3] = (x0 ^ y1 ^ z1) & mask;
  v.h[4] = (x1 ^ y0 ^ z0) & mask;
  v.h[5] = (x1 ^ y0 ^ z1) & mask;
  v.h[6] = (x1 ^ y1 ^ z0) & mask;
  v.h[7] = (x1 ^ y1 ^ z1) & mask;
}

// The cell's quotient q = (xc - min) / g from the correctly rounded reciprocal
// rg = RN(1/g): q0 = num * rg, r = fma(-g, q0, num) (exact), q = fma(r, rg, q0)
// is the correctly rounded quotient for num >= 2^-100 (one correction step with
// RN(1/g); checked against IEEE division on 575 M quotients over the grid
// sizes of six boxes x three finest resolutions, scripts/div_check.c), and
// below that both floors are 0.  Only the floor is used: 3 instructions for
// the division's ~11.
HN_DEV int32_t cell_floor(float num, float g, float rg) {
  const float q0 = num * rg;
  const float r = __builtin_fmaf(-g, q0, num);
  return (int32_t)floorf(__builtin_fmaf(r, rg, q0));
}
// n / d, correctly rounded, for operands the division's scaling never
// touches (|n|, |d| well inside [2^-96, 2^96], d != 0, finite): the FMA
// sequence hipcc emits for an IEEE f32 division (rcp, two refinements, the
// final residual correction) without its v_div_scale pair and v_div_fixup,
// which leave such operands unchanged -- the same bits in 8 instructions
// instead of 11.  The trilinear weights (x - vmin) / (vmax - vmin): grid
// sizes and sample coordinates of a NeRF scene are far inside that range.
HN_DEV float div_rn(float n, float d) {
  float y = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, y, 1.f);
  y = __builtin_fmaf(e, y, y);
  float q = n * y;
  const float r = __builtin_fmaf(-d, q, n);
  q = __builtin_fmaf(r, y, q);
  const float r2 = __builtin_fmaf(-d, q, n);
  return __builtin_fmaf(r2, y, q);
}
// voxel_level with the cells from cell_floor (rg[a] = RN(1/gs[a])); the
// weights keep the reference's IEEE divisions (div_rn: the same bits).
HN_DEV void voxel_level_rcp(const float x[3], const float xc[3], const float gs[3], const float rg[3],
                            const float bmin[3], uint32_t mask, Voxel& v) {
  uint32_t c[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const int32_t i = cell_floor(xc[a] - bmin[a], gs[a], rg[a]);   // floor((x - min) / g).int()
    const float vmin = (float)i * gs[a] + bmin[a];
    const float vmax = vmin + gs[a];
    v.w[a] = div_rn(x[a] - vmin, vmax - vmin);
    c[a] = (uint32_t)i;
  }
  const uint32_t x0 = c[0], x1 = c[0] + 1u;
  const uint32_t y0 = c[1] * kPrimeY, y1 = (c[1] + 1u) * kPrimeY;
  const uint32_t z0 = c[2] * kPrimeZ, z1 = (c[2] + 1u) * kPrimeZ;
  v.h[0] = (x0 ^ y0 ^ z0) & mask;
  v.h[1] = (x0 ^ y0 ^ z1) & mask;
  v.h[2] = (x0 ^ y1 ^ z0) & mask;
  v.h[3] = (x0 ^ y1 ^ z1) & mask;
  v.h[4] = (x1 ^ y0 ^ z0) & mask;
  v.h[5] = (x1 ^ y0 ^ z1) & mask;
  v.h[6] = (x1 ^ y1 ^ z0) & mask;
  v.h[7] = (x1 ^ y1 ^ z1) & mask;
}

// voxel_level that also returns the integer cell (run detection along rays).
HN_DEV void voxel_level_cell(const float x[3], const float xc[3], const float gs[3],
                             const float bmin[3], uint32_t mask, Voxel& v, uint32_t cell[3]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float q = (xc[a] - bmin[a]) / gs[a];
    const int32_t i = (int32_t)floorf(q);
    const float vmin = (float)i * gs[a] + bmin[a];
    const float vmax = vmin + gs[a];
    v.w[a] = (x[a] - vmin) / (vmax - vmin);
    cell[a] = (uint32_t)i;
  }
  const uint32_t x0 = cell[0], x1 = cell[0] + 1u;
  const uint32_t y0 = cell[1] * kPrimeY, y1 = (cell[1] + 1u) * kPrimeY;
  const uint32_t z0 = cell[2] * kPrimeZ, z1 = (cell[2] + 1u) * kPrimeZ;
  v.h[0] = (x0 ^ y0 ^ z0) & mask;
  v.h[1] = (x0 ^ y0 ^ z1) & mask;
  v.h[2] = (x0 ^ y1 ^ z0) & mask;
  v.h[3] = (x0 ^ y1 ^ z1) & mask;
  v.h[4] = (x1 ^ y0 ^ z0) & mask;
  v.h[5] = (x1 ^ y0 ^ z1) & mask;
  v.h[6] = (x1 ^ y1 ^ z0) & mask;
  v.h[7] = (x1 ^ y1 ^ z1) & mask;
}

// trilinear_interp (hash_encoding.py:130-163): x first, then y, then z.
HN_DEV float trilerp(const float e[8], const float w[3]) {
  const float ax = 1.f - w[0], ay = 1.f - w[1], az = 1.f - w[2];
  const float c00 = e[0] * ax + e[4] * w[0];
  const float c01 = e[1] * ax + e[5] * w[0];
  const float c10 = e[2] * ax + e[6] * w[0];
  const float c11 = e[3] * ax + e[7] * w[0];
  const float c0 = c00 * ay + c10 * w[1];
  const float c1 = c01 * ay + c11 * w[1];
  return c0 * az + c1 * w[2];
}

// d feat / d e_c = ((g * az) * ay) * ax: autograd's multiplication order.
HN_DEV void trilerp_bwd(float g, const float w[3], float out[8]) {
  const float ax = 1.f - w[0], ay = 1.f - w[1], az = 1.f - w[2];
  const float gz0 = g * az, gz1 = g * w[2];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float gzy = ((c & 1) ? gz1 : gz0) * ((c & 2) ? w[1] : ay);
    out[c] = gzy * ((c & 4) ? w[0] : ax);
  }
}

// RAdam per element (radam.py:58-92) in the op forms of torch's CPU kernels
// (verified bit-exact on the reference's RAdam trace, tests/golden/radam.npz):
// add_(x, alpha) = fma(alpha, x, self); addcmul_ = fma(value * t1, t2, self);
// addcdiv_ = self + (value * t1) / t2.
HN_DEV void radam_elem(const hn_radam_tensor& d, float& p, float g, float& m, float& v) {
  v = __builtin_fmaf(d.one_minus_beta2 * g, g, v * d.beta2);   // exp_avg_sq.mul_(b2).addcmul_
  m = __builtin_fmaf(d.one_minus_beta1, g, m * d.beta1);       // exp_avg.mul_(b1).add_
  if (d.mode != 0) {
    if (d.has_wd) p = __builtin_fmaf(d.neg_wd_lr, p, p);      // p.add_(-wd*lr, p)
    if (d.mode == 2) p = p + (d.neg_step_lr * m) / (sqrtf(v) + d.eps);   // addcdiv_
    else p = __builtin_fmaf(d.neg_step_lr, m, p);              // add_(-step_size*lr, exp_avg)
  }
}

HN_DEV void atomic_add_f32(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Gather one level's two features for a point: table_l is [2^T][2].
HN_DEV void encode_level(const float* __restrict__ table_l, const Voxel& v, float& f0, float& f1) {
  float e0[8], e1[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float2 t = *reinterpret_cast<const float2*>(table_l + 2 * (size_t)v.h[c]);
    e0[c] = t.x;
    e1[c] = t.y;
  }
  f0 = trilerp(e0, v.w);
  f1 = trilerp(e1, v.w);
}

// Same, addressed as uniform table base + 32-bit byte offset (row r of level
// l sits at byte (((l << T) + r) * 8)); lets hipcc use the SGPR-base +
// 32-bit-VGPR-offset addressing mode instead of 64-bit per-lane addresses.
HN_DEV float2 ld_row(const float* __restrict__ table, uint32_t byte_off) {
  return *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(table) + byte_off);
}
HN_DEV void encode_level_off(const float* __restrict__ table, uint32_t lvl_row0, const Voxel& v,
                             float& f0, float& f1) {
  float e0[8], e1[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float2 t = ld_row(table, (lvl_row0 + v.h[c]) * 8u);
    e0[c] = t.x;
    e1[c] = t.y;
  }
  f0 = trilerp(e0, v.w);
  f1 = trilerp(e1, v.w);
}
HN_DEV void atomic_add_row(float* table, uint32_t byte_off, float g0, float g1) {
  float* p = reinterpret_cast<float*>(reinterpret_cast<char*>(table) + byte_off);
  atomic_add_f32(p, g0);
  atomic_add_f32(p + 1, g1);
}

// SHEncoder.forward degree 4 (spherical_harmonic.py:65-103); constants are
// rounded to fp32 first, exactly as torch does for python-scalar * tensor.
HN_DEV void sh16(float x, float y, float z, float o[16]) {
  const float C0 = 0.28209479177387814f, C1 = 0.4886025119029199f;
  const float C2_0 = 1.0925484305920792f, C2_1 = -1.0925484305920792f,
              C2_2 = 0.31539156525252005f, C2_3 = -1.0925484305920792f,
              C2_4 = 0.5462742152960396f;
  const float C3_0 = -0.5900435899266435f, C3_1 = 2.890611442640554f,
              C3_2 = -0.4570457994644658f, C3_3 = 0.3731763325901154f,
              C3_4 = -0.4570457994644658f, C3_5 = 1.445305721320277f,
              C3_6 = -0.5900435899266435f;
  const float xx = x * x, yy = y * y, zz = z * z;
  const float xy = x * y, yz = y * z, xz = x * z;
  o[0] = C0;
  o[1] = -C1 * y;
  o[2] = C1 * z;
  o[3] = -C1 * x;
  o[4] = C2_0 * xy;
  o[5] = C2_1 * yz;
  o[6] = C2_2 * (2.0f * zz - xx - yy);
  o[7] = C2_3 * xz;
  o[8] = C2_4 * (xx - yy);
  o[9] = C3_0 * y * (3.f * xx - yy);
  o[10] = C3_1 * xy * z;
  o[11] = C3_2 * y * (4.f * zz - xx - yy);
  o[12] = C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
  o[13] = C3_4 * x * (4.f * zz - xx - yy);
  o[14] = C3_5 * z * (xx - yy);
  o[15] = C3_6 * x * (xx - 3.f * yy);
}

// ---------------------------------------------------------------------------
// Wave (64-lane) primitives
// ---------------------------------------------------------------------------
// The lane index behind an empty asm: the optimiser cannot treat it as loop-
// invariant, so persistent kernels do not hoist every shuffle's address and
// lane-compare mask out of their work loop (hundreds of registers).
HN_DEV int lane_id() {
  int l = (int)__lane_id();
  asm volatile("" : "+v"(l));
  return l;
}

// v from lane src (ds_bpermute; exact move).
HN_DEV float shfl_from(float v, int src) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
HN_DEV double shfl_from(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

HN_DEV uint32_t shfl_from(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

HN_DEV float wave_max_f32(float v) {
  const int l = lane_id();
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = fmaxf(v, __int_as_float(__builtin_amdgcn_ds_bpermute((l ^ d) << 2, __float_as_int(v))));
  return v;
}

template <typename T>
HN_DEV T wave_sum(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += shfl_from(v, l ^ o);
  return v;
}

// Inclusive scans across the 64 lanes (Hillis-Steele).
HN_DEV double wave_incl_sum(double v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = shfl_from(v, l >= o ? l - o : l);
    if (l >= o) v += t;
  }
  return v;
}
HN_DEV double wave_incl_prod(double v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = shfl_from(v, l >= o ? l - o : l);
    if (l >= o) v *= t;
  }
  return v;
}

// ---------------------------------------------------------------------------
// MFMA 32x32x2 f32 (exact f32 FMA chain).  Lane l: i = l & 31, h = l >> 5.
//   A operand: A[i][k=h]   B operand: B[k=h][j=i]
//   C/D: col = l & 31, row(r) = (r & 3) + 8 * (r >> 2) + 4 * h
// ---------------------------------------------------------------------------
HN_DEV f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
HN_DEV constexpr int row_of(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---------------------------------------------------------------------------
// Split-f32 products on the bf16 MFMA.  An f32 x is carried as NS bf16 parts
// x = p0 + p1 (+ p2) + r, p_q = bf16(x - p0 - .. - p_{q-1}) (RNE, each residual
// exact in f32), |r| <= 2^-18 |x| for NS = 2 and 2^-27 |x| for NS = 3.  The
// products p_q(a) p_q'(b) are exact in the f32 accumulator; keeping those with
// q + q' < NS gives a . b to ~2^-17 (NS = 2) or ~2^-25 (NS = 3) relative per
// product -- NS = 3 is as accurate as one f32 rounding.
// v_mfma_f32_32x32x16_bf16 contracts K = 16 in 32 cycles per SIMD: NS = 3 is
// six of them (192 cycles) against eight v_mfma_f32_32x32x2_f32 (512 cycles)
// for the same K, NS = 2 three (96 cycles).
//   Operand map (32x32x16 bf16): lane l holds A[row l&31][k = 8(l>>5) + j] and
//   B[k = 8(l>>5) + j][col l&31] in element j = 0..7; C/D as the f32 form.
// A K = 16 chunk c of a chained GEMM takes element j of lane half h from the
// f32 k-step s = 8c + j of the same lane half: the k <-> input-row map is the
// f32 form's, so packed A fragments and D -> B chaining keep their layout.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
template <int NS>
struct SP {   // one K = 16 operand chunk as NS bf16 parts, p[0] the largest
  bf16x8 p[NS];
};
template <int NS, typename F>
HN_DEV SP<NS> splitn(F x) {
  SP<NS> s;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = x(j);
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      const __bf16 b = (__bf16)v;
      s.p[q][j] = b;
      if (q + 1 < NS) v = v - (float)b;
    }
  }
  return s;
}
template <int NS>
HN_DEV SP<NS> splitn(const f32x4 a, const f32x4 b) {
  return splitn<NS>([&](int j) { return j < 4 ? a[j] : b[j - 4]; });
}
HN_DEV bf16x8 as_bf16x8(const f32x4 v) { return __builtin_bit_cast(bf16x8, v); }
HN_DEV f32x16 mfma_bf(const bf16x8 a, const bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// acc += A . B, both as NS parts; the smallest products first
template <int NS>
HN_DEV f32x16 mfma_split(const SP<NS>& a, const SP<NS>& b, f32x16 c) {
  static_assert(NS == 2 || NS == 3, "parts");
  if constexpr (NS == 3) {
    c = mfma_bf(a.p[2], b.p[0], c);
    c = mfma_bf(a.p[0], b.p[2], c);
    c = mfma_bf(a.p[1], b.p[1], c);
  }
  c = mfma_bf(a.p[1], b.p[0], c);
  c = mfma_bf(a.p[0], b.p[1], c);
  return mfma_bf(a.p[0], b.p[0], c);
}
// c0 += A0 . B, c1 += A1 . B (one split of B, the two chains interleaved;
// each accumulator sees the products in mfma_split's order)
template <int NS>
HN_DEV void mfma_split2(const SP<NS>& a0, const SP<NS>& a1, const SP<NS>& b, f32x16& c0, f32x16& c1) {
  static_assert(NS == 2 || NS == 3, "parts");
  if constexpr (NS == 3) {
    c0 = mfma_bf(a0.p[2], b.p[0], c0);
    c1 = mfma_bf(a1.p[2], b.p[0], c1);
    c0 = mfma_bf(a0.p[0], b.p[2], c0);
    c1 = mfma_bf(a1.p[0], b.p[2], c1);
    c0 = mfma_bf(a0.p[1], b.p[1], c0);
    c1 = mfma_bf(a1.p[1], b.p[1], c1);
  }
  c0 = mfma_bf(a0.p[1], b.p[0], c0);
  c1 = mfma_bf(a1.p[1], b.p[0], c1);
  c0 = mfma_bf(a0.p[0], b.p[1], c0);
  c1 = mfma_bf(a1.p[0], b.p[1], c1);
  c0 = mfma_bf(a0.p[0], b.p[0], c0);
  c1 = mfma_bf(a1.p[0], b.p[0], c1);
}
// Level handled by register pair (2m, 2m+1) of lane half h in the 32-feature
// tile layout: feature ROW(2m,h) = 2 * lev(m,h).
HN_DEV constexpr int tile_level(int m, int h) { return (m & 1) + 4 * (m >> 1) + 2 * h; }

// Order this wave's LDS writes before its later LDS reads of other lanes' data
// (LDS executes one wave's instructions in order; this pins the compiler).
// Deliberately NOT a memory fence: a wavefront-scope fence also waits for
// vmcnt(0), i.e. for every outstanding global atomic of the wave -- in the
// fused scatter kernel that drained the atomic queue at every LDS hand-off.
HN_DEV void lds_fence_wave() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Hide a uniform pointer's value from the optimiser.  Used at the top of tile
// loops so hipcc cannot hoist hundreds of loop-invariant weight-fragment loads
// out of the loop (which blows the register file and spills).
// The result stays a GLOBAL (address space 1) pointer: a laundered generic
// pointer turns every load through it into a FLAT load, and a pending FLAT op
// makes the waitcnt pass wait vmcnt(0) lgkmcnt(0) -- no prefetch distance
// survives and every outstanding atomic of the wave is drained.
template <typename T>
HN_DEV T* opaque_ptr(T* p) {
  uint64_t v = reinterpret_cast<uint64_t>(p);
  asm volatile("" : "+s"(v));
  return (T*)((__attribute__((address_space(1))) T*)v);
}

// One 1-KiB packed weight-fragment group (lane's 16 bytes at float offset off
// of P): a raw buffer load, voffset = the lane's 16 bytes, soffset = the
// group's byte offset laundered on the scalar unit (not hoisted: ~100
// loop-invariant offsets would spill SGPRs), so a load costs no vector
// address arithmetic (a global load of base + group + lane took a 64-bit
// VALU add per load).
HN_DEV f32x4 frag_load(const float* P, int off, int lane) {
  int so = off * 4;
  asm volatile("" : "+s"(so));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(opaque_ptr(P)), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, so, 0));
}

// ---------------------------------------------------------------------------
// Keyed 4-round Feistel permutation of [0, 2^(2 half)) (pixel sampling without
// replacement, hn_train.hip; ray scrambling in the render backward) and its
// inverse.
// ---------------------------------------------------------------------------
HN_DEV uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

HN_DEV uint32_t feistel(uint32_t x, int half, uint64_t seed) {
  const uint32_t mask = (1u << half) - 1u;
  uint32_t L = x >> half, R = x & mask;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t key = (uint32_t)(seed >> (16 * r)) ^ (0x9e3779b9u * (uint32_t)(r + 1));
    const uint32_t F = mix32(R ^ key) & mask;
    const uint32_t t = R;
    R = L ^ F;
    L = t;
  }
  return (L << half) | R;
}

HN_DEV uint32_t feistel_inv(uint32_t x, int half, uint64_t seed) {
  const uint32_t mask = (1u << half) - 1u;
  uint32_t L = x >> half, R = x & mask;
#pragma unroll
  for (int r = 3; r >= 0; --r) {
    const uint32_t key = (uint32_t)(seed >> (16 * r)) ^ (0x9e3779b9u * (uint32_t)(r + 1));
    const uint32_t t = L;
    L = R ^ (mix32(t ^ key) & mask);
    R = t;
  }
  return (L << half) | R;
}

inline int32_t hip_status(hipError_t e) { return e == hipSuccess ? HN_OK : HN_E_HIP + (int32_t)e; }

HN_DEV f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

}  // namespace hn
