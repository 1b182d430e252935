// hn_mlp.h -- NeRFSmall (models.py:96-174) on gfx950 f32 MFMA, one wave per
// 32-point tile.
//
// Orientation: every layer computes Y[out][pt] = W[out][in] . X[in][pt] with
// v_mfma_f32_32x32x2_f32, so points sit on the MFMA columns (lane & 31) and
// neurons on the accumulator rows.  A layer's D tile is then directly the B
// operand of the next layer (and of the W^T data-gradient products): lane
// half h at k-step s supplies its own register s, i.e. input row
// row_of(s & 15, h) of tile s >> 4 -- no lane movement between layers.  The
// weights are pre-packed ("fragment order") so the A operands of four k-steps
// are one coalesced 1-KiB dwordx4 load: packed[gemm][ob][s/4][lane][s%4].
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

// Packed A-operand GEMMs (offsets in floats; size = OB * KS * 64, KS % 4 == 0).
enum : int {
  G_F0 = 0,        // sigma_net.0        OB 2  KS 16
  G_F1 = 2048,     // sigma_net.1        OB 1  KS 32
  G_F2G = 4096,    // color_net.0 geo    OB 2  KS 8
  G_F2S = 5120,    // color_net.0 sh     OB 2  KS 8
  G_F3 = 6144,     // color_net.1        OB 2  KS 32
  G_F4 = 10240,    // color_net.2        OB 1  KS 32
  G_B4 = 12288,    // color_net.2^T      OB 2  KS 4 (2 used)
  G_B3 = 12800,    // color_net.1^T      OB 2  KS 32
  G_B2G = 16896,   // color_net.0^T geo  OB 1  KS 32
  G_B2S = 18944,   // color_net.0^T sh   OB 1  KS 32
  G_B1 = 20992,    // sigma_net.1^T      OB 2  KS 8
  G_B0 = 22016,    // sigma_net.0^T      OB 1  KS 32
  G_END = 24064
};
static_assert(G_END == HN_MLP_PACKED_FLOATS, "packed size");

// Weight-gradient accumulator layout (torch [out][in] row-major, concatenated).
enum : int { W_S0 = 0, W_S1 = 2048, W_C0 = 3072, W_C1 = 5056, W_C2 = 9152, W_END = 9344 };
static_assert(W_END == HN_MLP_PARAMS, "param count");

// acc += A(gemm at off, block ob) . B where bval(s) is the B operand of k-step s.
// The next group's A fragment is loaded while the current group's 4 MFMAs run;
// the scheduling barrier stops hipcc from hoisting all loads (register blowup).
template <int KS, typename BF>
HN_DEV f32x16 gemm(const float* __restrict__ P, int off, int ob, f32x16 acc, int lane, BF bval) {
  // opaque BEFORE the offset: keeps hipcc from precomputing ~50 uniform GEMM
  // base addresses at the top of the tile loop (SGPR pairs that then spill)
  const float* base = opaque_ptr(P) + off + ob * (KS / 4) * 256 + lane * 4;
  f32x4 an = *reinterpret_cast<const f32x4*>(base);
#pragma unroll
  for (int g = 0; g < KS / 4; ++g) {
    const f32x4 a = an;
    if (g + 1 < KS / 4) an = *reinterpret_cast<const f32x4*>(base + (g + 1) * 256);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = mfma(a[j], bval(4 * g + j), acc);
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

struct MlpAct {
  f32x16 h0[2];
  f32x16 s1;
  f32x16 c0[2];
  f32x16 c1[2];
};

HN_DEV void relu16(f32x16& v) {
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
}
HN_DEV void mask16(f32x16& g, const f32x16& act) {   // relu backward (result > 0)
#pragma unroll
  for (int r = 0; r < 16; ++r) g[r] = act[r] > 0.f ? g[r] : 0.f;
}

// Forward of one tile.  Returns activations (post-ReLU) and c2 (raw rgb).
HN_DEV void mlp_fwd_tile(const float* __restrict__ P, const f32x16& feat, const float sh8[8],
                         MlpAct& a, f32x16& c2, int lane) {
  // sigma_net.0: 32 -> 64, ReLU
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    a.h0[ob] = gemm<16>(P, G_F0, ob, zero16(), lane, [&](int s) { return feat[s]; });
    relu16(a.h0[ob]);
  }
  // sigma_net.1: 64 -> 16 (sigma, geo15), no activation
  a.s1 = gemm<32>(P, G_F1, 0, zero16(), lane, [&](int s) { return a.h0[s >> 4][s & 15]; });
  // color_net.0: [sh16 | geo15] -> 64, ReLU
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    f32x16 acc = gemm<8>(P, G_F2S, ob, zero16(), lane, [&](int s) { return sh8[s]; });
    acc = gemm<8>(P, G_F2G, ob, acc, lane, [&](int s) { return a.s1[s]; });
    relu16(acc);
    a.c0[ob] = acc;
  }
  // color_net.1: 64 -> 64, ReLU
#pragma unroll
  for (int ob = 0; ob < 2; ++ob) {
    a.c1[ob] = gemm<32>(P, G_F3, ob, zero16(), lane, [&](int s) { return a.c0[s >> 4][s & 15]; });
    relu16(a.c1[ob]);
  }
  // color_net.2: 64 -> 3, no activation
  c2 = gemm<32>(P, G_F4, 0, zero16(), lane, [&](int s) { return a.c1[s >> 4][s & 15]; });
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
#if HN_ABLATE == 3
  return;
#endif
  lds_fence_wave();
  const f32x16 d = wgrad_block(Tdy, Tx, lane);
  lds_fence_wave();
#if HN_ABLATE == 4
  if (d[0] == 1234.5f && d[1] == -1234.5f) Wacc[lane] = d[2];
#else
  accum_block(Wacc, base, ld, n0, nmax, k0, kmax, d, lane);
#endif
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
    dc1[ob] = gemm<4>(P, G_B4, ob, zero16(), lane, [&](int s) { return s < 2 ? dy2[s] : 0.f; });
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
    dc0[ob] = gemm<32>(P, G_B3, ob, zero16(), lane, [&](int s) { return dc1[s >> 4][s & 15]; });
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
  f32x16 ds1 = gemm<32>(P, G_B2G, 0, zero16(), lane, [&](int s) { return dc0[s >> 4][s & 15]; });
  if (h == 0) ds1[0] = dsig;                    // row 0 = sigma (A row 0 is zero)
  if (dsh != nullptr)
    *dsh = gemm<32>(P, G_B2S, 0, zero16(), lane, [&](int s) { return dc0[s >> 4][s & 15]; });
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
    dh0[ob] = gemm<8>(P, G_B1, ob, zero16(), lane, [&](int s) { return ds1[s]; });
    mask16(dh0[ob], a.h0[ob]);
  }
  // ---- sigma_net.0 ----
  stage_tile(Tx, feat, lane);
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    stage_tile(Tdy, dh0[nb], lane);
    wgrad_accum(Tdy, Tx, Wacc, W_S0, 32, nb * 32, 64, 0, 32, lane);
  }
  dfeat = gemm<32>(P, G_B0, 0, zero16(), lane, [&](int s) { return dh0[s >> 4][s & 15]; });
}

// Packing: natural torch weights -> fragment-ordered A operands (per net).
HN_DEV float pack_value(const hn_mlp& w, int idx) {
  int off, KS;
  if (idx < G_F1) { off = G_F0; KS = 16; }
  else if (idx < G_F2G) { off = G_F1; KS = 32; }
  else if (idx < G_F2S) { off = G_F2G; KS = 8; }
  else if (idx < G_F3) { off = G_F2S; KS = 8; }
  else if (idx < G_F4) { off = G_F3; KS = 32; }
  else if (idx < G_B4) { off = G_F4; KS = 32; }
  else if (idx < G_B3) { off = G_B4; KS = 4; }
  else if (idx < G_B2G) { off = G_B3; KS = 32; }
  else if (idx < G_B2S) { off = G_B2G; KS = 32; }
  else if (idx < G_B1) { off = G_B2S; KS = 32; }
  else if (idx < G_B0) { off = G_B1; KS = 8; }
  else { off = G_B0; KS = 32; }
  const int rel = idx - off;
  const int j = rel & 3;
  const int lane = (rel >> 2) & 63;
  const int t = rel >> 8;
  const int g = t % (KS / 4), ob = t / (KS / 4);
  const int s = 4 * g + j;
  const int i = lane & 31, h = lane >> 5;
  const int o = ob * 32 + i;
  const int kc = 32 * (s >> 4) + row_of(s & 15, h);   // chain order (D-layout input)
  const int kp = 2 * s + h;                            // pair order
  switch (off) {
    case G_F0: return w.sigma0[o * 32 + kc];
    case G_F1: return i < 16 ? w.sigma1[i * 64 + kc] : 0.f;
    case G_F2G: return (kc >= 1 && kc <= 15) ? w.color0[o * 31 + 15 + kc] : 0.f;
    case G_F2S: return w.color0[o * 31 + kp];
    case G_F3: return w.color1[o * 64 + kc];
    case G_F4: return i < 3 ? w.color2[i * 64 + kc] : 0.f;
    case G_B4: return kp < 3 ? w.color2[kp * 64 + o] : 0.f;
    case G_B3: return w.color1[kc * 64 + o];
    case G_B2G: return (i >= 1 && i <= 15) ? w.color0[kc * 31 + 15 + i] : 0.f;
    case G_B2S: return i < 16 ? w.color0[kc * 31 + i] : 0.f;
    case G_B1: return w.sigma1[kc * 64 + o];
    default: return w.sigma0[kc * 32 + i];   // G_B0
  }
}

// Launch the packing kernel (hn_mlp.hip).
int32_t mlp_pack_launch(const hn_mlp* w, float* packed, hipStream_t s);
int32_t mlp_pack2_launch(const hn_mlp* w0, float* p0, const hn_mlp* w1, float* p1, hipStream_t s);

}  // namespace hn
