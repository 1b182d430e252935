// hn_tv.h -- hash-table total variation (loss.py:11-43) shared by the TV
// kernels (hn_optim.hip) and the binned backward's TV records (hn_render.hip).
#pragma once
#include "hn_common.h"

namespace hn {

struct TvK {
  int32_t L, log2T;
  int32_t cube[HN_MAX_LEVELS];
  // packed 1-D grids: level l owns blocks [boff[l], boff[l+1]) of the
  // forward (kTvFwdV vertices per thread) and [bofb[l], bofb[l+1]) of the
  // backward (one thread per (vertex, feature)), instead of a (max blocks) x L
  // grid that is mostly idle blocks
  int32_t boff[HN_MAX_LEVELS + 1], bofb[HN_MAX_LEVELS + 1];
  const int32_t* mv;
  const float* table;
};

// Entry of grid vertex (x, y, z) of level l (hash_encoding.py:112-128).
HN_DEV float2 tv_row(const TvK& k, int l, uint32_t x, uint32_t y, uint32_t z) {
  const uint32_t mask = (1u << k.log2T) - 1u;
  const uint32_t h = (x ^ (y * kPrimeY) ^ (z * kPrimeZ)) & mask;
  return ld_row(k.table, (((uint32_t)l << k.log2T) + h) * 8u);
}

// level of packed block b (wave-uniform; at most 16 scalar compares)
HN_DEV int tv_level(const TvK& k, const int32_t* off, int b) {
  int l = 0;
  while (l + 1 < k.L && b >= off[l + 1]) ++l;
  return l;
}

// vertices per forward thread: fewer blocks, so fewer same-address atomics
// on the 16 level sums
constexpr int kTvFwdV = 4;

HN_DEV float tv_val(const TvK& k, int l, uint32_t x, uint32_t y, uint32_t z, int f) {
  const uint32_t mask = (1u << k.log2T) - 1u;
  const uint32_t h = (x ^ (y * kPrimeY) ^ (z * kPrimeZ)) & mask;
  return k.table[((((size_t)l << k.log2T) + h) << 1) + f];
}

// d TV_l / d e of cube vertex (i, j, kk) = grid vertex (x, y, z), feature f,
// times cube (the caller scales by g_tv[l] / cube): the sum over the vertex's
// incident edges of d(d^2)/de = -+2d (loss.py:23-43's three squared-difference
// sums, autograd's sub / pow backward)
HN_DEV float tv_grad(const TvK& k, int l, int c, int i, int j, int kk, uint32_t x, uint32_t y, uint32_t z,
                     int f) {
  const float e = tv_val(k, l, x, y, z, f);
  float g = 0.f;
  const int idx[3] = {i, j, kk};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (idx[a] < c) g -= 2.f * (tv_val(k, l, x + (a == 0), y + (a == 1), z + (a == 2), f) - e);
    if (idx[a] > 0) g += 2.f * (e - tv_val(k, l, x - (a == 0), y - (a == 1), z - (a == 2), f));
  }
  return g;
}


inline int32_t make_tv(const hn_tv_args* a, TvK& k, int& fwd_blocks, int& bwd_blocks) {
  if (!a || !a->min_vertex || !a->table) return HN_E_NULL;
  if (a->n_levels < 1 || a->n_levels > HN_MAX_LEVELS) return HN_E_SHAPE;
  if (a->log2_hashmap_size < 1 || a->log2_hashmap_size > 24) return HN_E_SHAPE;
  k.L = a->n_levels;
  k.log2T = a->log2_hashmap_size;
  k.mv = a->min_vertex;
  k.table = a->table;
  for (int l = 0; l < HN_MAX_LEVELS; ++l) k.cube[l] = l < a->n_levels ? a->cube[l] : 1;
  k.boff[0] = k.bofb[0] = 0;
  for (int l = 0; l < HN_MAX_LEVELS; ++l) {
    int nv = 0;
    if (l < a->n_levels) {
      const int c = a->cube[l];
      if (c < 1 || c > 1000) return HN_E_SHAPE;
      nv = (c + 1) * (c + 1) * (c + 1);
    }
    k.boff[l + 1] = k.boff[l] + (nv + 256 * kTvFwdV - 1) / (256 * kTvFwdV);
    k.bofb[l + 1] = k.bofb[l] + (2 * nv + 255) / 256;
  }
  fwd_blocks = k.boff[a->n_levels];
  bwd_blocks = k.bofb[a->n_levels];
  return HN_OK;
}

}  // namespace hn
