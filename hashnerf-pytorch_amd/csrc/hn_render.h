// hn_render.h -- per-ray (one wave64 per ray) volume rendering building blocks:
//   composite_fwd / composite_bwd  raw2outputs (run_nerf_helpers.py:577-628)
//   sample_pdf_wave                sample_pdf  (run_nerf_helpers.py:264-307)
//   rank_sort_wave                 torch.sort of the merged z  (:551)
//
// Samples of a ray are "blocked" over lanes: lane l owns samples l*N .. l*N+N-1
// (N = ceil(S/64), template parameter).  Per-ray arrays live in LDS (or global)
// and are addressed by sample index.  The exclusive transmittance product and
// the cdf cumsum run as wave scans in fp64 and are rounded to fp32 per
// element -- torch's CPU cumprod/cumsum accumulate in double too.
#pragma once
#include "hn_common.h"

namespace hn {

constexpr float kEps32 = 1.1920928955078125e-07f;   // torch.finfo(float32).eps

HN_DEV float sigmoidf_t(float x) { return 1.f / (1.f + expf(-x)); }

// Exclusive product over samples given each lane's N factors (fp64).
template <int N>
HN_DEV void excl_prod(const double (&x)[N], double (&T)[N], int lane) {
  double loc = 1.0;
#pragma unroll
  for (int k = 0; k < N; ++k) loc *= x[k];
  const double inc = wave_incl_prod(loc);
  double ex = shfl_from(inc, lane > 0 ? lane - 1 : 0);
  if (lane == 0) ex = 1.0;
#pragma unroll
  for (int k = 0; k < N; ++k) { T[k] = ex; ex *= x[k]; }
}

// Exclusive suffix sum (sum over later samples) of each lane's N values.
template <int N>
HN_DEV void excl_suffix_sum(const double (&v)[N], double (&S)[N], int lane) {
  double loc = 0.0;
#pragma unroll
  for (int k = 0; k < N; ++k) loc += v[k];
  const double inc = wave_incl_sum(loc);          // prefix incl. this lane
  const double tot = shfl_from(inc, 63);
  double after = tot - inc;                       // sum of later lanes
#pragma unroll
  for (int k = N - 1; k >= 0; --k) { S[k] = after; after += v[k]; }
}

struct CompOut {
  float rgb[3];
  float depth, disp, acc, entropy;
};

// Per-sample forward quantities of raw2outputs (:590-611).
template <int N>
struct CompSamples {
  float c[N][3];     // sigmoid(rgb)
  float z[N];
  float sig[N];      // relu(sigma + noise)
  float delta[N];    // dists * |d|
  float e[N];        // exp(-sig * delta)
  float alpha[N];
  float x[N];        // (1 - alpha) + 1e-10
  float T[N];
  float w[N];
  bool valid[N];
};

template <int N>
HN_DEV void composite_samples(const float* raw, const float* z, const float* noise, int S,
                              float dnorm, CompSamples<N>& cs, int lane) {
  double xd[N], Td[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int j = lane * N + k;
    const bool v = j < S;
    cs.valid[k] = v;
    const float4 r = v ? *reinterpret_cast<const float4*>(raw + 4 * j) : make_float4(0, 0, 0, 0);
    const float zj = v ? z[j] : 0.f;
    const float zn = (j + 1 < S) ? z[j + 1] : 0.f;
    const float dist = (j + 1 < S) ? (zn - zj) : 1e10f;
    const float delta = dist * dnorm;
    const float sn = (noise != nullptr && v) ? r.w + noise[j] : r.w;
    const float sg = sn > 0.f ? sn : 0.f;
    const float e = expf(-sg * delta);
    const float a = v ? 1.f - e : 0.f;
    const float xx = v ? (1.f - a) + 1e-10f : 1.f;
    cs.c[k][0] = sigmoidf_t(r.x);
    cs.c[k][1] = sigmoidf_t(r.y);
    cs.c[k][2] = sigmoidf_t(r.z);
    cs.z[k] = zj;
    cs.sig[k] = sg;
    cs.delta[k] = delta;
    cs.e[k] = e;
    cs.alpha[k] = a;
    cs.x[k] = xx;
    xd[k] = (double)xx;
  }
  excl_prod<N>(xd, Td, lane);
#pragma unroll
  for (int k = 0; k < N; ++k) {
    cs.T[k] = (float)Td[k];
    cs.w[k] = cs.alpha[k] * cs.T[k];
  }
}

struct CompTotals {
  float acc, num, rgb[3];
  float qS, Q;
};

template <int N>
HN_DEV void composite_totals(const CompSamples<N>& cs, CompTotals& t) {
  double sw = 0, swz = 0, sr = 0, sg = 0, sb = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (!cs.valid[k]) continue;
    const float w = cs.w[k];
    sw += w;
    swz += (double)(w * cs.z[k]);
    sr += (double)(w * cs.c[k][0]);
    sg += (double)(w * cs.c[k][1]);
    sb += (double)(w * cs.c[k][2]);
  }
  sw = wave_sum(sw); swz = wave_sum(swz);
  sr = wave_sum(sr); sg = wave_sum(sg); sb = wave_sum(sb);
  t.acc = (float)sw;
  t.num = (float)swz;
  t.rgb[0] = (float)sr; t.rgb[1] = (float)sg; t.rgb[2] = (float)sb;
  t.qS = (1.f - t.acc) + 1e-6f;                  // 1.0 - w.sum() + 1e-6 (:623)
  t.Q = (float)(sw + (double)t.qS);             // Categorical normalisation
}

HN_DEV float ent_logit(float p) { return logf(p < kEps32 ? kEps32 : (p > 1.f - kEps32 ? 1.f - kEps32 : p)); }
HN_DEV bool ent_inside(float p) { return p >= kEps32 && p <= 1.f - kEps32; }

// Forward.  Writes per-sample weights to wout (may be null).
template <int N>
HN_DEV void composite_fwd(const float* raw, const float* z, const float* noise, int S, float dnorm,
                          bool white, float* wout, CompOut& o, int lane) {
  CompSamples<N> cs;
  composite_samples<N>(raw, z, noise, S, dnorm, cs, lane);
  CompTotals t;
  composite_totals<N>(cs, t);
  double ent = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    if (!cs.valid[k]) continue;
    if (wout) wout[lane * N + k] = cs.w[k];
    const float p = cs.w[k] / t.Q;
    ent += (double)(ent_logit(p) * p);
  }
  ent = wave_sum(ent);
  const float pS = t.qS / t.Q;
  const float entS = ent_logit(pS) * pS;
  o.acc = t.acc;
  o.depth = t.num / t.acc;
  o.disp = (o.depth != o.depth) ? o.depth : 1.f / (o.depth > 1e-10f ? o.depth : 1e-10f);
#pragma unroll
  for (int c = 0; c < 3; ++c) o.rgb[c] = white ? t.rgb[c] + (1.f - t.acc) : t.rgb[c];
  o.entropy = -(float)(ent + (double)entS);
}

// Upstream gradients of one ray.  has_* false => that output has no grad.
struct CompGrad {
  float rgb[3];
  float acc, depth, entropy;
  bool has_rgb, has_acc, has_depth, has_entropy;
};

// Backward w.r.t. raw: writes draw[j] (float4, may alias raw: each lane reads
// its own samples before writing them).  gw: per-sample grad of weights or
// null; graw: external grad of raw (added) or null.
template <int N>
HN_DEV void composite_bwd(const float* raw, const float* z, const float* noise, int S, float dnorm,
                          bool white, const CompGrad& g, const float* gw, const float* graw,
                          float* draw, int lane) {
  CompSamples<N> cs;
  composite_samples<N>(raw, z, noise, S, dnorm, cs, lane);
  CompTotals t;
  composite_totals<N>(cs, t);
  // entropy: dH/dw_j = (g_j - g_S) / Q with g_k = -(log(clamp p_k) + inside_k)
  const float pS = t.qS / t.Q;
  const float gS = -(ent_logit(pS) + (ent_inside(pS) ? 1.f : 0.f));
  const float white_term = (g.has_rgb && white) ? -(g.rgb[0] + g.rgb[1] + g.rgb[2]) : 0.f;
  const float gd_over_a = g.has_depth ? g.depth / t.acc : 0.f;
  const float gd_num = g.has_depth ? -(g.depth * t.num) / (t.acc * t.acc) : 0.f;
  float G[N];
  double Gw[N], Sfx[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    float gk = 0.f;
    if (cs.valid[k]) {
      if (g.has_rgb) gk = g.rgb[0] * cs.c[k][0] + g.rgb[1] * cs.c[k][1] + g.rgb[2] * cs.c[k][2] + white_term;
      if (g.has_acc) gk += g.acc;
      if (g.has_depth) gk += cs.z[k] * gd_over_a + gd_num;
      if (g.has_entropy) {
        const float p = cs.w[k] / t.Q;
        const float gp = -(ent_logit(p) + (ent_inside(p) ? 1.f : 0.f));
        gk += g.entropy * ((gp - gS) / t.Q);
      }
      if (gw != nullptr) gk += gw[lane * N + k];
    }
    G[k] = gk;
    Gw[k] = (double)(gk * cs.w[k]);
  }
  excl_suffix_sum<N>(Gw, Sfx, lane);
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const int j = lane * N + k;
    if (!cs.valid[k]) continue;
    const float dalpha = G[k] * cs.T[k] - (float)Sfx[k] / cs.x[k];
    const float dsig_t = dalpha * cs.e[k] * cs.delta[k];
    float4 d;
    d.w = cs.sig[k] > 0.f ? dsig_t : 0.f;
    if (g.has_rgb) {
      d.x = (g.rgb[0] * cs.w[k]) * (1.f - cs.c[k][0]) * cs.c[k][0];
      d.y = (g.rgb[1] * cs.w[k]) * (1.f - cs.c[k][1]) * cs.c[k][1];
      d.z = (g.rgb[2] * cs.w[k]) * (1.f - cs.c[k][2]) * cs.c[k][2];
    } else {
      d.x = d.y = d.z = 0.f;
    }
    if (graw != nullptr) {
      const float4 e = *reinterpret_cast<const float4*>(graw + 4 * j);
      d.x += e.x; d.y += e.y; d.z += e.z; d.w += e.w;
    }
    *reinterpret_cast<float4*>(draw + 4 * j) = d;
  }
}

// torch.sum over a contiguous fp32 row on the CPU (ATen SumKernel.cpp
// vectorized_inner_sum: 8-float vectors, row_sum with 4-way ILP, scalar tail,
// then the 8 vector lanes) restated for n < 512, so that
// `weights / torch.sum(weights)` (run_nerf_helpers.py:267) is bit-identical.
// Every lane evaluates it redundantly from LDS (broadcast reads).
HN_DEV float torch_row_sum(const float* x, int n) {
  const int nv = n >> 3;
  float acc[8];
  if (nv >= 4) {
    const int size_ilp = nv >> 2;
    float p[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < 8; ++l) p[k][l] = 0.f;
    for (int i = 0; i < size_ilp; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < 8; ++l) p[k][l] += x[(i * 4 + k) * 8 + l];
    for (int i = size_ilp * 4; i < nv; ++i)
#pragma unroll
      for (int l = 0; l < 8; ++l) p[0][l] += x[i * 8 + l];
#pragma unroll
    for (int k = 1; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < 8; ++l) p[0][l] += p[k][l];
#pragma unroll
    for (int l = 0; l < 8; ++l) acc[l] = p[0][l];
  } else {
#pragma unroll
    for (int l = 0; l < 8; ++l) acc[l] = 0.f;
    for (int i = 0; i < nv; ++i)
#pragma unroll
      for (int l = 0; l < 8; ++l) acc[l] += x[i * 8 + l];
  }
  float fin = 0.f;
  for (int k = nv * 8; k < n; ++k) fin += x[k];
#pragma unroll
  for (int l = 0; l < 8; ++l) fin += acc[l];
  return fin;
}

// sample_pdf for one ray.  bins[nw+1], w[nw] (any memory), cdf: LDS scratch
// [nw+1], u[ns] (global), out[ns].  nw + 1 <= 256.
HN_DEV void sample_pdf_wave(const float* bins, const float* w, int nw, float* cdf_lds,
                            const float* u, int ns, float* out, int lane) {
  constexpr int NPL = 4;                       // weights per lane (nw <= 255)
  float wp[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int j = lane * NPL + k;
    wp[k] = j < nw ? w[j] + 1e-5f : 0.f;      // weights + 1e-5 (:266)
    if (j < nw) cdf_lds[j + 1] = wp[k];       // staged for the row sum
  }
  lds_fence_wave();
  const float sum = torch_row_sum(cdf_lds + 1, nw);
  lds_fence_wave();
  double pd[NPL], loc = 0;
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int j = lane * NPL + k;
    pd[k] = j < nw ? (double)(wp[k] / sum) : 0.0;
    loc += pd[k];
  }
  double run = wave_incl_sum(loc) - loc;       // exclusive lane prefix
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int j = lane * NPL + k;
    run += pd[k];
    if (j < nw) cdf_lds[j + 1] = (float)run;
  }
  if (lane == 0) cdf_lds[0] = 0.f;
  lds_fence_wave();
  const int nb = nw + 1;
  for (int i = lane; i < ns; i += 64) {
    const float ui = u[i];
    // searchsorted(cdf, u, right=True): first index with cdf > u
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf_lds[mid] > ui) hi = mid; else lo = mid + 1;
    }
    const int below = lo - 1 > 0 ? lo - 1 : 0;
    const int above = lo < nb - 1 ? lo : nb - 1;
    const float c0 = cdf_lds[below], c1 = cdf_lds[above];
    const float b0 = bins[below], b1 = bins[above];
    float denom = c1 - c0;
    denom = denom < 1e-5f ? 1.f : denom;
    const float tt = (ui - c0) / denom;
    out[i] = b0 + tt * (b1 - b0);
  }
}

// Sort S (<= 256) floats of src (LDS) into dst (LDS) by rank; ties keep
// source order.  Values are what torch.sort returns.  If origin != null,
// origin[rank] = e for source elements e < n_tag, else 255 (where each sorted
// element came from: lets the backward merge a coarse sample's two passes).
HN_DEV void rank_sort_wave(const float* src, float* dst, int S, int lane, uint8_t* origin = nullptr,
                           int n_tag = 0) {
  for (int e = lane; e < S; e += 64) {
    const float v = src[e];
    int rank = 0;
    for (int j = 0; j < S; ++j) {
      const float o = src[j];
      rank += (o < v || (o == v && j < e)) ? 1 : 0;
    }
    dst[rank] = v;
    if (origin != nullptr) origin[rank] = e < n_tag ? (uint8_t)e : (uint8_t)255;
  }
  lds_fence_wave();
}

// float <-> uint32 key with the same order (negative floats reversed); -0
// maps to +0's key, so equal floats have equal keys.
HN_DEV uint32_t sort_key(float v) {
  uint32_t b = __float_as_uint(v);
  if (b == 0x80000000u) b = 0u;
  return b ^ ((b >> 31) ? 0xffffffffu : 0x80000000u);
}
HN_DEV float key_value(uint32_t k) { return __uint_as_float(k ^ ((k >> 31) ? 0x80000000u : 0xffffffffu)); }

// The same result as rank_sort_wave(src, dst, 192, lane, origin, 64) -- the
// values torch.sort returns, and origin[rank] = the coarse index or 255 --
// for src = [64 coarse z, non-decreasing | 128 importance z]: the importance
// samples are sorted by a bitonic network over the wave (2 per lane, cross-
// lane exchanges by ds_bpermute), then each element's rank is its position in
// its own run plus a binary search in the other run (coarse before importance
// on ties, as the rank sort's index tie-break puts them; ties among importance
// samples are equal values tagged 255, so their order is not observable).
// ~0.5 k instructions per wave where the rank sort's 192 x 192 compares take
// ~3 k.  Returns false (dst untouched) when the coarse run is not sorted.
HN_DEV bool merge_sort_z(const float* src, float* dst, float* tmp, int lane, uint8_t* origin) {
  const float zc = src[lane];
  const float zn = lane < 63 ? src[lane + 1] : zc;
  if (__ballot(sort_key(zn) < sort_key(zc)) != 0ull) return false;
  uint32_t k[2] = {sort_key(src[64 + lane]), sort_key(src[128 + lane])};
#pragma unroll
  for (int kk = 2; kk <= 128; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
      if (j == 64) {   // partner in the other register of this lane (kk = 128: ascending)
        const uint32_t lo = min(k[0], k[1]), hi = max(k[0], k[1]);
        k[0] = lo;
        k[1] = hi;
      } else {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int i = lane + 64 * r;
          const uint32_t kp = shfl_from(k[r], lane ^ j);
          const bool asc = (i & kk) == 0, lower = (i & j) == 0;
          k[r] = (lower == asc) ? min(k[r], kp) : max(k[r], kp);
        }
      }
    }
  }
  tmp[lane] = key_value(k[0]);
  tmp[64 + lane] = key_value(k[1]);
  lds_fence_wave();
  // coarse e: e + #{importance < v} (lower bound in the sorted importance run)
  {
    const uint32_t kc = sort_key(zc);
    int lo = 0, hi = 128;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sort_key(tmp[mid]) < kc) lo = mid + 1; else hi = mid;
    }
    dst[lane + lo] = zc;
    if (origin) origin[lane + lo] = (uint8_t)lane;
  }
  // importance at sorted position p: p + #{coarse <= v} (upper bound in the coarse run)
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = lane + 64 * r;
    int lo = 0, hi = 64;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sort_key(src[mid]) <= k[r]) lo = mid + 1; else hi = mid;
    }
    dst[p + lo] = key_value(k[r]);
    if (origin) origin[p + lo] = (uint8_t)255;
  }
  lds_fence_wave();
  return true;
}

}  // namespace hn
