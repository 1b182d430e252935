// hn_mlp.h -- NeRFSmall (models.py:96-174) on the gfx950 MFMA, one wave per
// 32-point tile.
//
// Orientation: every layer computes Y[out][pt] = W[out][in] . X[in][pt] with
// 32x32 MFMA tiles (v_mfma_f32_32x32x16_bf16 on split-f32 operands, see
// hn_common.h; v_mfma_f32_32x32x2_f32 in the f32 build), so points sit on the
// MFMA columns (lane & 31) and neurons on the accumulator rows.  A layer's D
// tile is then directly the B operand of the next layer (and of the W^T
// data-gradient products): lane half h at f32 k-step s supplies its own
// register s, i.e. input row row_of(s & 15, h) of tile s >> 4 -- no lane
// movement between layers.  The weights are pre-packed ("fragment order") so
// the A operands of a group are one coalesced 1-KiB dwordx4 load (regions and
// groups below).
//
// Layouts per lane (p = lane & 31 = point, h = lane >> 5):
//   feat  f32x16: reg r = feature row_of(r,h) = (level tile_level(r>>1,h), r&1)
//   h0[2], c0[2], c1[2]: hidden 64 = two 32-row tiles
//   s1    f32x16: rows 0..15 valid (row 0 = sigma, rows 1..15 = geo_feat)
//   c2    f32x16: rows 0..2 valid (rgb)
//   sh8   float[8]: sh[2s + h], s = 0..7 (pair order)
#pragma once
#include "hn_common.h"

namespace hn {

// Packed A-operand GEMMs ("regions"), per net, in this order.  KS = f32 k-steps
// (K = 2 each), OB = 32-row output blocks.  A region is OB x groups x 256
// floats; a group is one 1-KiB dwordx4 load per wave.
//   f32 region  (NS = 0): group g = the f32 fragments of k-steps 4g .. 4g+3;
//   split region (NS parts, hn_common.h): chunk c (k-steps 8c .. 8c+7) is NS
//   groups, group NS*c + q = part q of those 8 values as bf16 (dword d of a
//   lane = elements 2d, 2d+1).
// HN_SPLIT_F: parts in the forward GEMMs (the forward pass and the backward's
// recompute, which therefore reproduce each other's activations bit for bit);
// 3 makes them as accurate as f32.  HN_SPLIT_B: parts in the data-gradient and
// weight-gradient GEMMs.  0 = f32 MFMA (an exact FMA chain).  color_net.2^T
// (4 k-steps, 2 used) is always f32 (a 2-part split of its 3 rgb grads as one
// K = 16 chunk measured no faster: 1.154-1.155 ms vs 1.159 ms per step, r03g).
#ifndef HN_SPLIT_F
#define HN_SPLIT_F 3
#endif
#ifndef HN_SPLIT_B
#define HN_SPLIT_B 2
#endif
enum : int { R_F0, R_F1, R_F2G, R_F2S, R_F3, R_F4, R_B4, R_B3, R_B2G, R_B2S, R_B1, R_B0, R_N };
//  F0 sigma_net.0  F1 sigma_net.1  F2G/F2S color_net.0 geo/sh  F3 color_net.1  F4 color_net.2
//  B4 color_net.2^T  B3 color_net.1^T  B2G/B2S color_net.0^T geo/sh  B1 sigma_net.1^T  B0 sigma_net.0^T
constexpr int kRegKS[R_N] = {16, 32, 8, 8, 32, 32, 4, 32, 32, 32, 8, 32};
constexpr int kRegOB[R_N] = {2, 1, 2, 2, 2, 1, 2, 2, 1, 1, 2, 1};
#ifndef HN_SPLIT_FC   // parts in the forward colour-net GEMMs (color_net.0-2)
#define HN_SPLIT_FC HN_SPLIT_F
#endif
constexpr int reg_ns(int r) {
  return kRegKS[r] % 8 ? 0 : (r < R_F2G ? HN_SPLIT_F : (r < R_B4 ? HN_SPLIT_FC : HN_SPLIT_B));
}
constexpr int reg_gpo(int r) { return reg_ns(r) ? reg_ns(r) * kRegKS[r] / 8 : kRegKS[r] / 4; }   // groups per OB
constexpr int reg_off(int r) {
  int o = 0;
  for (int i = 0; i < r; ++i) o += kRegOB[i] * reg_gpo(i) * 256;
  return o;
}
enum : int {
  G_F0 = reg_off(R_F0), G_F1 = reg_off(R_F1), G_F2G = reg_off(R_F2G), G_F2S = reg_off(R_F2S),
  G_F3 = reg_off(R_F3), G_F4 = reg_off(R_F4), G_B4 = reg_off(R_B4), G_B3 = reg_off(R_B3),
  G_B2G = reg_off(R_B2G), G_B2S = reg_off(R_B2S), G_B1 = reg_off(R_B1), G_B0 = reg_off(R_B0),
  G_END = reg_off(R_N)
};
static_assert(G_END <= HN_MLP_PACKED_FLOATS, "packed size");

// Weight-gradient accumulator layout (torch [out][in] row-major, concatenated).
enum : int { W_S0 = 0, W_S1 = 2048, W_C0 = 3072, W_C1 = 5056, W_C2 = 9152, W_END = 9344 };
static_assert(W_END == HN_MLP_PARAMS, "param count");

// acc += A(region R, block ob) . B where bval(s) is the B operand of f32 k-step s.
// Split-f32: each chunk's A fragments are loaded at use (round 3: loading the
// next chunk's into registers during the current one's MFMAs measured 0.324
// against 0.314 ms for render_fwd_kernel, identical results), or, with a
// FragRing source (the render forward, round 5), read from the wave's LDS slot
// that a DMA filled during the previous chunk (0.271 -> 0.266 ms, no registers
// held).  f32: one group ahead.  The scheduling barrier stops hipcc from
// hoisting all loads (register blowup).
// Where a GEMM's packed A fragments come from (the packed buffer in global
// memory: frag_load).
struct FragGlobal {
  static constexpr bool kRing = false;
  const float* P;
  HN_DEV f32x4 operator()(int off, int lane) const { return frag_load(P, off, lane); }
};
// The forward tile's split-GEMM chunks (3 fragment groups each, contiguous)
// in the order mlp_fwd_tile_src runs them; a tile's last chunk is followed by
// the next tile's first.
struct FwdChunk {
  int r, ob, c;
};
constexpr FwdChunk kFwdSeq[] = {
    {R_F0, 0, 0}, {R_F0, 0, 1}, {R_F0, 1, 0}, {R_F0, 1, 1}, {R_F1, 0, 0}, {R_F1, 0, 1}, {R_F1, 0, 2},
    {R_F1, 0, 3}, {R_F2G, 0, 0}, {R_F2G, 1, 0}, {R_F3, 0, 0}, {R_F3, 0, 1}, {R_F3, 0, 2}, {R_F3, 0, 3},
    {R_F3, 1, 0}, {R_F3, 1, 1}, {R_F3, 1, 2}, {R_F3, 1, 3}, {R_F4, 0, 0}, {R_F4, 0, 1}, {R_F4, 0, 2},
    {R_F4, 0, 3}};
constexpr int kFwdSeqN = sizeof(kFwdSeq) / sizeof(kFwdSeq[0]);
constexpr int fwd_chunk_off(const FwdChunk& q) { return reg_off(q.r) + (q.ob * reg_gpo(q.r) + reg_ns(q.r) * q.c) * 256; }
// float offset of the chunk after (r, ob, c) in the sequence
constexpr int fwd_next_off(int r, int ob, int c) {
  for (int i = 0; i < kFwdSeqN; ++i)
    if (kFwdSeq[i].r == r && kFwdSeq[i].ob == ob && kFwdSeq[i].c == c) return fwd_chunk_off(kFwdSeq[(i + 1) % kFwdSeqN]);
  return -1;
}
// Split-GEMM fragments prefetched one chunk ahead into this wave's LDS slot
// (3 x 1 KiB; buffer_load ... lds, no registers held): a chunk's groups are
// read from the slot, the slot is refilled with the next chunk of kFwdSeq,
// and that DMA runs under the chunk's split and MFMAs.  fwd_ring_start puts a
// net's first chunk in the slot before its tiles.
struct FragRing {
  static constexpr bool kRing = true;
  const float* P;
  float* slot;   // LDS, this wave's 768 floats
  HN_DEV f32x4 operator()(int off, int lane) const { return frag_load(P, off, lane); }
};
HN_DEV void ring_fill(const float* P, float* slot, int off, int lane) {
  int so = off * 4;
  asm volatile("" : "+s"(so));
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(opaque_ptr(P)), (short)0, 0x7fffffff, 0x00020000);
#ifndef HN_DIAG_RING2
#define HN_DIAG_RING2 0
#endif
#pragma unroll
  for (int q = 0; q < (HN_DIAG_RING2 ? 2 : 3); ++q)   // HN_DIAG_RING2: timing diagnostic only (stale third part)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(slot + 256 * q), 16,
                                             lane * 16, so + 1024 * q, 0, 0);
}
HN_DEV void fwd_ring_start(const float* P, float* slot, int lane) {
  if (HN_DIAG_RING2) *reinterpret_cast<f32x4*>(slot + 512 + 4 * lane) = f32x4{0.f, 0.f, 0.f, 0.f};
  ring_fill(P, slot, fwd_chunk_off(kFwdSeq[0]), lane);
}
template <int R, typename BF, typename Src>
HN_DEV f32x16 gemm_src(const Src& src, int ob, f32x16 acc, int lane, BF bval);
template <int R, typename BF>
HN_DEV f32x16 gemm(const float* __restrict__ P, int ob, f32x16 acc, int lane, BF bval) {
  return gemm_src<R>(FragGlobal{P}, ob, acc, lane, bval);
}
template <int R, typename BF, typename Src>
HN_DEV f32x16 gemm_src(const Src& src, int ob, f32x16 acc, int lane, BF bval) {
  constexpr int KS = kRegKS[R], NS = reg_ns(R), GPO = reg_gpo(R), OFF = reg_off(R);
  // fragment group g of this block (frag_load: scalar offsets, hn_common.h)
  auto ld = [&](int g) { return src(OFF + (ob * GPO + g) * 256, lane); };
  if constexpr (NS > 0) {        // split-f32, fragments loaded at use
#pragma unroll
    for (int c = 0; c < KS / 8; ++c) {
      SP<NS> a;
      if constexpr (Src::kRing && NS == 3) {
        // this chunk from the slot, then the slot refilled with the next one
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < NS; ++q) a.p[q] = as_bf16x8(*reinterpret_cast<const f32x4*>(src.slot + 256 * q + 4 * lane));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ring_fill(src.P, src.slot, fwd_next_off(R, ob, c), lane);
      } else {
#pragma unroll
        for (int q = 0; q < NS; ++q) a.p[q] = as_bf16x8(ld(NS * c + q));
      }
      const SP<NS> b = splitn<NS>([&](int j) { return bval(8 * c + j); });
      acc = mfma_split<NS>(a, b, acc);
      __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
  } else {
    f32x4 an = ld(0);
#pragma unroll
    for (int g = 0; g < KS / 4; ++g) {
      const f32x4 a = an;
      if (g + 1 < KS / 4) an = ld(g + 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma(a[j], bval(4 * g + j), acc);
      __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
  }
}

struct MlpAct {
  f32x16 h0[2];
  f32x16 s1;
  f32x16 c0[2];
  f32x16 c1[2];
  uint32_t m[3];   // ReLU masks of h0, c0, c1 (bit 16 ob + r: value > 0), formed as each is ReLU'd
};
// mask bits of one ReLU'd D-layout block: its values are +0 or positive, so a
// bit is (bits + 0x7fffffff) >> 31 (integer ops only: the compare forms, which
// min(bits, 1) also becomes, hold lane masks in SGPR pairs and spilled the forward)
// Two ops per value: t = 0 - bits has bit 31 set iff bits >= 1 (a ReLU'd value
// is +0 or positive, so bits < 2^31), and (m << 1) | (t >> 31) is one
// v_alignbit_b32 that shifts the word's bits up and inserts the new one at
// bit 0 -- so r runs from 15 down and bit r ends at position r.
HN_DEV void relu_mask_or(const f32x16& v, uint32_t& m, int ob) {
  uint32_t w = 0u;
#pragma unroll
  for (int r = 15; r >= 0; --r) w = __builtin_amdgcn_alignbit(w, 0u - __float_as_uint(v[r]), 31u);
  m |= w << (16 * ob);
}

// ReLU as one integer max on the bits (a negative float or -0 is a negative
// int32): equal to v > 0 ? v : +0 for every non-NaN v, and one v_max_i32
// where the float form is a v_max_f32 plus the IEEE-mode canonicalisation of
// its input.  A NaN with the sign bit clear passes through (as torch.relu
// propagates NaN); one with the sign bit set is a negative int32 and becomes
// +0 here.
HN_DEV void relu16(f32x16& v) {
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = __int_as_float(max(__float_as_int(v[r]), 0));
}
HN_DEV void mask16(f32x16& g, const f32x16& act) {   // relu backward (result > 0)
#pragma unroll
  for (int r = 0; r < 16; ++r) g[r] = act[r] > 0.f ? g[r] : 0.f;
}

// Forward of one tile.  Returns activations (post-ReLU) and c2 (raw rgb).
// MASKS: also form a.m (pinned right after each ReLU by an empty asm, so the
// compiler cannot sink the bit ops to the masks' late use and keep every
// activation live until then -- that spilled the render forward 39 -> 158).
// C0Init(ob): color_net.0's SH half for output block ob (constant along a ray:
// the fused forward computes it once per ray and seeds every tile with it).
struct NoLive {
  HN_DEV void operator()() const {}
};
template <bool MASKS = false, typename C0Init, typename Src, typename OnLive = NoLive>
HN_DEV void mlp_fwd_tile_src(const Src& P, const f32x16& feat, C0Init&& c0init, MlpAct& a, f32x16& c2,
                             int lane, bool skip_dead = false, OnLive&& on_live = OnLive{});
template <bool MASKS = false, typename C0Init>
HN_DEV void mlp_fwd_tile_c0(const float* __restrict__ P, const f32x16& feat, C0Init&& c0init,
                            MlpAct& a, f32x16& c2, int lane) {
  mlp_fwd_tile_src<MASKS>(FragGlobal{P}, feat, c0init, a, c2, lane);
}
template <bool MASKS, typename C0Init, typename Src, typename OnLive>
HN_DEV void mlp_fwd_tile_src(const Src& P, const f32x16& feat, C0Init&& c0init, MlpAct& a, f32x16& c2,
                             int lane, bool skip_dead, OnLive&& on_live) {
  a.m[0] = a.m[1] = a.m[2] = 0u;
  // sigma_net.0: 32 -> 64, ReLU
  // (Both output blocks of a GEMM sharing one B split per chunk, as the
  // backward's gemm_w2 does, measured slower here: render_fwd_kernel 0.300 ->
  // 0.307 ms, more spills at 4 waves per SIMD; r04c.)
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    a.h0[ob] = gemm_src<R_F0>(P, ob, zero16(), lane, [&](int s) { return feat[s]; });
    relu16(a.h0[ob]);
    if constexpr (MASKS) relu_mask_or(a.h0[ob], a.m[0], ob);
  }
  if constexpr (MASKS) asm volatile("" : "+v"(a.m[0]));
  // sigma_net.1: 64 -> 16 (sigma, geo15), no activation
  a.s1 = gemm_src<R_F1>(P, 0, zero16(), lane, [&](int s) { return a.h0[s >> 4][s & 15]; });
  // skip_dead (the trainer's forward, no raw noise): a tile whose 32 raw
  // sigmas (row 0, lanes 0-31) are all <= 0 has alpha = 0 and weight 0 at
  // every sample (raw2outputs, run_nerf_helpers.py:577-628), so its colours
  // enter no output and no gradient: the colour net is not evaluated (raw rgb
  // written as 0, its ReLU masks 0) and the weight stream restarts at the next
  // tile's first chunk
  if (skip_dead && __ballot(lane < 32 && a.s1[0] > 0.f) == 0ull) {
    c2 = zero16();
    if constexpr (Src::kRing) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the slot's pending fill has landed
      ring_fill(P.P, P.slot, fwd_chunk_off(kFwdSeq[0]), lane);
    }
    return;
  }
  on_live();   // the tile has density (or nothing is skipped): e.g. its features are stored
  // color_net.0: [sh16 | geo15] -> 64, ReLU
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    f32x16 acc = c0init(ob);
    acc = gemm_src<R_F2G>(P, ob, acc, lane, [&](int s) { return a.s1[s]; });
    relu16(acc);
    if constexpr (MASKS) relu_mask_or(acc, a.m[1], ob);
    a.c0[ob] = acc;
  }
  if constexpr (MASKS) asm volatile("" : "+v"(a.m[1]));
  // color_net.1: 64 -> 64, ReLU
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    a.c1[ob] = gemm_src<R_F3>(P, ob, zero16(), lane, [&](int s) { return a.c0[s >> 4][s & 15]; });
    relu16(a.c1[ob]);
    if constexpr (MASKS) relu_mask_or(a.c1[ob], a.m[2], ob);
  }
  if constexpr (MASKS) asm volatile("" : "+v"(a.m[2]));
  // color_net.2: 64 -> 3, no activation
  c2 = gemm_src<R_F4>(P, 0, zero16(), lane, [&](int s) { return a.c1[s >> 4][s & 15]; });
}
template <bool MASKS = false>
HN_DEV void mlp_fwd_tile(const float* __restrict__ P, const f32x16& feat, const float sh8[8],
                         MlpAct& a, f32x16& c2, int lane) {
  mlp_fwd_tile_c0<MASKS>(P, feat, [&](int ob) { return gemm<R_F2S>(P, ob, zero16(), lane, [&](int s) { return sh8[s]; }); },
                         a, c2, lane);
}
// The SH half of color_net.0 for one ray (every point's column holds the same
// rows), kept in 64 floats of LDS: lanes 0 and 32 store their rows; a tile
// then seeds its accumulators with c0sh_lds_load (bitwise the per-tile GEMM).
HN_DEV void c0sh_lds_store(const float* __restrict__ P, const float sh8[8], float* lds, int lane) {
  const int p = lane & 31, h = lane >> 5;
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    const f32x16 v = gemm<R_F2S>(P, ob, zero16(), lane, [&](int s) { return sh8[s]; });
    if (p == 0)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(lds + 32 * ob + row_of(4 * g, h)) = f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
  }
}
HN_DEV f32x16 c0sh_lds_load(const float* lds, int ob, int lane) {
  const int h = lane >> 5;
  f32x16 c;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(lds + 32 * ob + row_of(4 * g, h));
#pragma unroll
    for (int j = 0; j < 4; ++j) c[4 * g + j] = v[j];
  }
  return c;
}

// ---------------------------------------------------------------------------
// Weight gradients: dW[n][k] += sum_p dY[n][p] X[k][p] needs the point index
// on the MFMA k axis for both operands, so the two 32x32 blocks go through a
// per-wave LDS transpose T[pt][row] (stride 33: conflict-free writes and reads).
// ---------------------------------------------------------------------------
constexpr int kTS = 33;                 // transpose row stride (floats)
constexpr int kTBuf = 32 * kTS;         // one [32][33] buffer

// Stage a D-layout tile: T[p][row_of(r,h)] = v[r].
HN_DEV void stage_tile(float* T, const f32x16& v, int lane) {
  const int p = lane & 31, h = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) T[p * kTS + row_of(r, h)] = v[r];
}

// 32x32 block: returns D with row n = row_of(r,h) of dY, col k = lane & 31 of X.
HN_DEV f32x16 wgrad_block(const float* Tdy, const float* Tx, int lane) {
  const int i = lane & 31, h = lane >> 5;
  f32x16 acc = zero16();
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int pt = 2 * s + h;
    acc = mfma(Tdy[pt * kTS + i], Tx[pt * kTS + i], acc);
  }
  return acc;
}

// acc_lds[base + n*ld + k] += D[n - n0][k - k0] for n < nmax, k < kmax.
HN_DEV void accum_block(float* acc_lds, int base, int ld, int n0, int nmax, int k0, int kmax,
                        const f32x16& d, int lane) {
  const int i = lane & 31, h = lane >> 5;
  const int k = k0 + i;
  if (k >= kmax) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = n0 + row_of(r, h);
    if (n < nmax) atomicAdd(acc_lds + base + n * ld + k, d[r]);
  }
}

// One staged weight-gradient block: Tdy/Tx already hold the operands.
HN_DEV void wgrad_accum(const float* Tdy, const float* Tx, float* Wacc, int base, int ld, int n0,
                        int nmax, int k0, int kmax, int lane) {
  lds_fence_wave();
  const f32x16 d = wgrad_block(Tdy, Tx, lane);
  lds_fence_wave();
  accum_block(Wacc, base, ld, n0, nmax, k0, kmax, d, lane);
  __builtin_amdgcn_sched_barrier(0);
}

// Backward of one tile given the recomputed activations.
//   dy2[2]: B operand of the rgb gradient (lane half 0: ch 0, 2; half 1: ch 1, 0)
//   dsig  : d sigma (valid on lane half 0)
//   rgbg  : the point's 3 rgb grads (for the dW_c2 staging; lane half 0)
//   shx8  : sh[8h .. 8h+7] of the point (dW_c0 staging)
//   T     : this wave's 2 transpose buffers; Wacc: the workgroup's dW accumulator
//   dsh   : if non-null, also return d sh (standalone NeRFSmall backward)
HN_DEV void mlp_bwd_tile(const float* __restrict__ P, const f32x16& feat, const float shx8[8],
                         MlpAct& a, const float dy2[2], float dsig, const float rgbg[3], float* T,
                         float* Wacc, f32x16& dfeat, f32x16* dsh, int lane) {
  const int p = lane & 31, h = lane >> 5;
  float* Tdy = T;
  float* Tx = T + kTBuf;
  // ---- color_net.2 ----
  if (h == 0) {
    Tdy[p * kTS + 0] = rgbg[0];
    Tdy[p * kTS + 1] = rgbg[1];
    Tdy[p * kTS + 2] = rgbg[2];
  }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    stage_tile(Tx, a.c1[kb], lane);
    wgrad_accum(Tdy, Tx, Wacc, W_C2, 64, 0, 3, kb * 32, 64, lane);
  }
  f32x16 dc1[2];
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    dc1[ob] = gemm<R_B4>(P, ob, zero16(), lane, [&](int s) { return s < 2 ? dy2[s] : 0.f; });
    mask16(dc1[ob], a.c1[ob]);
  }
  // ---- color_net.1 ----
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    stage_tile(Tdy, dc1[nb], lane);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int kb = nb ? 1 - kk : kk;   // reuse the staged X block across nb
      if (!(nb == 1 && kk == 0)) stage_tile(Tx, a.c0[kb], lane);
      wgrad_accum(Tdy, Tx, Wacc, W_C1, 64, nb * 32, 64, kb * 32, 64, lane);
    }
  }
  f32x16 dc0[2];
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    dc0[ob] = gemm<R_B3>(P, ob, zero16(), lane, [&](int s) { return dc1[s >> 4][s & 15]; });
    mask16(dc0[ob], a.c0[ob]);
  }
  // ---- color_net.0: X = [sh16 | geo15] ----
#pragma unroll
  for (int j = 0; j < 8; ++j) Tx[p * kTS + 8 * h + j] = shx8[j];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int row = row_of(r, h);               // s1 rows 0..15
    if (row >= 1) Tx[p * kTS + 15 + row] = a.s1[r];
  }
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    stage_tile(Tdy, dc0[nb], lane);
    wgrad_accum(Tdy, Tx, Wacc, W_C0, 31, nb * 32, 64, 0, 31, lane);
  }
  f32x16 ds1 = gemm<R_B2G>(P, 0, zero16(), lane, [&](int s) { return dc0[s >> 4][s & 15]; });
  if (h == 0) ds1[0] = dsig;                    // row 0 = sigma (A row 0 is zero)
  if (dsh != nullptr)
    *dsh = gemm<R_B2S>(P, 0, zero16(), lane, [&](int s) { return dc0[s >> 4][s & 15]; });
  // ---- sigma_net.1 ----
  stage_tile(Tdy, ds1, lane);
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    stage_tile(Tx, a.h0[kb], lane);
    wgrad_accum(Tdy, Tx, Wacc, W_S1, 64, 0, 16, kb * 32, 64, lane);
  }
  f32x16 dh0[2];
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    dh0[ob] = gemm<R_B1>(P, ob, zero16(), lane, [&](int s) { return ds1[s]; });
    mask16(dh0[ob], a.h0[ob]);
  }
  // ---- sigma_net.0 ----
  stage_tile(Tx, feat, lane);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    stage_tile(Tdy, dh0[nb], lane);
    wgrad_accum(Tdy, Tx, Wacc, W_S0, 32, nb * 32, 64, 0, 32, lane);
  }
  dfeat = gemm<R_B0>(P, 0, zero16(), lane, [&](int s) { return dh0[s >> 4][s & 15]; });
}

// Packing: natural torch weights -> fragment-ordered A operands (per net).
// f32 value of region r's A fragment: out block ob, k-step s, lane; W(t, i) =
// element i of torch tensor t (0 sigma_net.0 .. 4 color_net.2).
template <class W>
HN_DEV float pack_f32(const W& w, int r, int ob, int s, int lane) {
  const int i = lane & 31, h = lane >> 5;
  const int o = ob * 32 + i;
  const int kc = 32 * (s >> 4) + row_of(s & 15, h);   // chain order (D-layout input)
  const int kp = 2 * s + h;                            // pair order
  switch (r) {
    case R_F0: return w(0, o * 32 + kc);
    case R_F1: return i < 16 ? w(1, i * 64 + kc) : 0.f;
    case R_F2G: return (kc >= 1 && kc <= 15) ? w(2, o * 31 + 15 + kc) : 0.f;
    case R_F2S: return w(2, o * 31 + kp);
    case R_F3: return w(3, o * 64 + kc);
    case R_F4: return i < 3 ? w(4, i * 64 + kc) : 0.f;
    case R_B4: return kp < 3 ? w(4, kp * 64 + o) : 0.f;
    case R_B3: return w(3, kc * 64 + o);
    case R_B2G: return (i >= 1 && i <= 15) ? w(2, kc * 31 + 15 + i) : 0.f;
    case R_B2S: return i < 16 ? w(2, kc * 31 + i) : 0.f;
    case R_B1: return w(1, kc * 64 + o);
    default: return w(0, kc * 32 + i);   // R_B0
  }
}

// Float idx of the packed buffer (layout above), inside region r.
template <class W>
HN_DEV float pack_value_r(const W& w, int r, int idx) {
  const int rel = idx - reg_off(r), d = rel & 3, lane = (rel >> 2) & 63, t = rel >> 8;
  const int gpo = reg_gpo(r), ns = reg_ns(r), g = t % gpo, ob = t / gpo;
  if (ns == 0) return pack_f32(w, r, ob, 4 * g + d, lane);
  const int c = g / ns, part = g % ns;
  uint32_t out = 0;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    float v = pack_f32(w, r, ob, 8 * c + 2 * d + e, lane);
    __bf16 b = (__bf16)v;
    for (int q = 0; q < part; ++q) {
      v = v - (float)b;
      b = (__bf16)v;
    }
    out |= (uint32_t)__builtin_bit_cast(uint16_t, b) << (16 * e);
  }
  return __uint_as_float(out);
}
// the natural weights of one net (hn_mlp's tensors)
struct MlpW {
  const hn_mlp& m;
  HN_DEV float operator()(int t, int i) const {
    const float* p = t == 0 ? m.sigma0 : t == 1 ? m.sigma1 : t == 2 ? m.color0 : t == 3 ? m.color1 : m.color2;
    return p[i];
  }
};
HN_DEV float pack_value(const hn_mlp& w, int idx) {
  int r = 0;
  while (r + 1 < R_N && idx >= reg_off(r + 1)) ++r;
  return pack_value_r(MlpW{w}, r, idx);
}

// Launch the packing kernel (hn_mlp.hip).
int32_t mlp_pack_launch(const hn_mlp* w, float* packed, hipStream_t s);
int32_t mlp_pack2_launch(const hn_mlp* w0, float* p0, const hn_mlp* w1, float* p1, hipStream_t s);

}  // namespace hn
