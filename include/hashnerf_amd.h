/*
 * hashnerf_amd.h -- C ABI of the MI355X (gfx950) HashNeRF hot path.
 *
 * Plain pointers + sizes, no torch types.  Every pointer is a DEVICE pointer
 * (HBM, fp32, contiguous, row-major) unless documented otherwise; config
 * structs are HOST pointers read at call time.  `stream` is a hipStream_t
 * passed as void*.  The library never allocates or frees, and synchronises
 * only in hn_device_faults: scratch comes in through `workspace`; outputs are
 * caller-allocated.
 * Gradient outputs named d* are ACCUMULATED (+=) so the caller zeroes them,
 * mirroring autograd's .grad accumulation.  Return value: 0 on success,
 * a positive HN_E_* code for argument errors, or a hipError_t + 1000.
 *
 * Each entry point cites the reference interface it replaces
 * (mache102/HashNeRF-pytorch, file:line).
 */
#ifndef HASHNERF_AMD_H
#define HASHNERF_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HN_ABI_VERSION 14
#define HN_MAX_LEVELS 32

enum {
  HN_OK = 0,
  HN_E_NULL = 1,        /* required pointer is NULL */
  HN_E_SHAPE = 2,       /* unsupported size (e.g. n_levels, n_samples) */
  HN_E_WORKSPACE = 3,   /* workspace too small */
  HN_E_HIP = 1000       /* + hipError_t */
};

/* Hash-grid description (embedding/hash_encoding.py:14-57).  grid_size is
 * (box_max - box_min) / resolution_l evaluated on the host in fp32 exactly as
 * hash_encoding.py:72/:101 do, so the device sees bit-identical cell sizes.
 * Table layout in HBM: [n_levels][2^log2_hashmap_size][n_features] fp32
 * (the stacked `embeddings.{l}.weight` tensors). */
typedef struct hn_grid {
  int32_t n_levels;            /* L <= HN_MAX_LEVELS (16) */
  int32_t n_features;          /* F, must be 2 */
  int32_t log2_hashmap_size;   /* T, 1..24 */
  int32_t reserved;
  float box_min[3];
  float box_max[3];
  float grid_size[HN_MAX_LEVELS][3];
} hn_grid;

/* NeRFSmall weights (models.py:96-149; num_layers=2, hidden 64, geo 15,
 * num_layers_color=3): torch nn.Linear layout [out][in], no biases. */
typedef struct hn_mlp {
  const float* sigma0;   /* sigma_net.0.weight [64][32] */
  const float* sigma1;   /* sigma_net.1.weight [16][64] */
  const float* color0;   /* color_net.0.weight [64][31]  (in = [sh16 | geo15]) */
  const float* color1;   /* color_net.1.weight [64][64] */
  const float* color2;   /* color_net.2.weight [3][64] */
} hn_mlp;

typedef struct hn_mlp_grad {
  float* sigma0; float* sigma1; float* color0; float* color1; float* color2;  /* += */
} hn_mlp_grad;

#define HN_MLP_PARAMS 9344          /* 2048 + 1024 + 1984 + 4096 + 192 */
#define HN_MLP_PACKED_FLOATS 30208  /* MFMA fragment-ordered copy (split-f32 bf16 parts), per net */

int32_t hn_abi_version(void);
const char* hn_status_string(int32_t status);
/* Sticky device fault word.  The persistent render backward synchronises its
 * waves through bounded LDS waits; a wait that runs out (a protocol failure,
 * never expected) sets a bit here instead of hanging the GPU: 1 ring slot,
 * 2 ring drain (tiles left unscattered), 4 coarse-grad flag, 8 dW buffer,
 * 16 binned-scatter overflow records exhausted (gradient records lost),
 * 32 a NaN / Inf feature gradient or sample point reached the binned scatter
 * (its exact fixed-point sums cannot carry it; the reference's autograd would
 * propagate it into the table gradient), 64 a gradient on a row pair table_live
 * marks dead (hn_render_bwd_args).
 * Nonzero means the gradients of the launches since the last clear are
 * invalid.  This is the one entry point that synchronises (a blocking copy
 * from the device); call it at points where the host syncs anyway.
 * *faults = the word; clear != 0 resets it. */
int32_t hn_device_faults(int32_t* faults, int32_t clear);

/* ---- L1 encodings --------------------------------------------------------
 * HashEmbedder.forward (hash_encoding.py:84-110): x[n][3] -> feat[n][L*F],
 * keep_mask[n] (uint8, may be NULL).  Corners from the clamped point, trilinear
 * weights from the unclamped point, every level hashed (SURVEY 8a traps 1-3). */
int32_t hn_encode_fwd(const hn_grid* g, const float* x, int64_t n, const float* table,
                      float* feat, uint8_t* keep_mask, void* stream);
/* Autograd of the above (embedding_dense_backward x L): dtable += scatter. */
int32_t hn_encode_bwd(const hn_grid* g, const float* x, int64_t n, const float* dfeat,
                      float* dtable, void* stream);
/* SHEncoder.forward, degree 4 (embedding/spherical_harmonic.py:65-103):
 * dirs[n][3] -> out[n][16]. */
int32_t hn_sh_fwd(const float* dirs, int64_t n, float* out, void* stream);

/* ---- L2 NeRFSmall (MFMA) ------------------------------------------------
 * NeRFSmall.forward (models.py:151-174): x[n][48] = [feat32 | sh16] ->
 * out[n][4] = [rgb3 | sigma].  workspace >= hn_mlp_workspace_bytes(). */
size_t hn_mlp_workspace_bytes(void);
int32_t hn_mlp_fwd(const hn_mlp* w, const float* x, int64_t n, float* out,
                   void* workspace, size_t ws_bytes, void* stream);
/* Backward: dx[n][48] (overwritten; may be NULL), dw (+=). */
int32_t hn_mlp_bwd(const hn_mlp* w, const float* x, const float* dout, int64_t n,
                   float* dx, const hn_mlp_grad* dw, void* workspace, size_t ws_bytes,
                   void* stream);

/* ---- L3 volume rendering --------------------------------------------------
 * raw2outputs (run_nerf_helpers.py:577-628), n_samples <= 256 per ray:
 * raw[n_rays][S][4], z[n_rays][S], rays_d[n_rays][3], noise[n_rays][S] or NULL
 * -> rgb[n_rays][3], disp, acc, depth, entropy [n_rays], weights[n_rays][S]. */
int32_t hn_composite_fwd(const float* raw, const float* z, const float* rays_d,
                         const float* noise, int64_t n_rays, int32_t n_samples,
                         int32_t white_bkgd, float* rgb, float* disp, float* acc,
                         float* weights, float* depth, float* entropy, void* stream);
/* Backward w.r.t. raw (overwritten): upstream grads of rgb[n][3], acc[n],
 * depth[n], entropy[n], weights[n][S] (any may be NULL = 0). */
int32_t hn_composite_bwd(const float* raw, const float* z, const float* rays_d,
                         const float* noise, int64_t n_rays, int32_t n_samples,
                         int32_t white_bkgd, const float* g_rgb, const float* g_acc,
                         const float* g_depth, const float* g_entropy,
                         const float* g_weights, float* d_raw, void* stream);
/* sample_pdf (run_nerf_helpers.py:264-307) with u given:
 * bins[n_rays][nb], weights[n_rays][nb-1], u[n_rays][ns] -> out[n_rays][ns];
 * nb <= 256. */
int32_t hn_sample_pdf(const float* bins, const float* weights, const float* u,
                      int64_t n_rays, int32_t n_bins, int32_t n_samples, float* out,
                      void* stream);

/* ---- fused render_rays (run_nerf_helpers.py:464-574) ---------------------
 * One kernel for the whole forward of a ray batch (coarse 64 -> composite ->
 * sample_pdf 128 -> sort -> fine 192 -> composite) and one for its backward.
 * Hash grid must have L=16, F=2; N_samples=64, N_importance=128. */
typedef struct hn_render_cfg {
  hn_grid grid;
  int32_t n_samples;      /* 64 */
  int32_t n_importance;   /* 128 */
  int32_t white_bkgd;
  int32_t lindisp;
  int32_t perturb;        /* 1: stratified jitter from t_rand */
  int32_t scatter;        /* backward table-gradient scatter: 0 auto (= binned where the
                             table allows it), 1 float atomics, 2 binned (records +
                             exact per-bin owner pass; T <= 22).  The library reads no
                             environment variables (ABI 14). */
  int32_t bin_cap;        /* binned scatter: records per (producer block, bin) region, a
                             multiple of 64; 0 = sized from the batch.  Small values
                             exercise the shared overflow records (tests). */
  int32_t dense_bwd;      /* ABI 14 (in ABI 12-13's merge_levels slot, whose merged coarse-level
                             records were removed): 0 = the backward skips the samples whose
                             d raw is exactly zero (relu(sigma) = 0: alpha = 0, weight 0), whose
                             feature and weight gradients are exactly zero -- the same results
                             up to the sign of zero; 1 = every sample computed (A/B, tests) */
} hn_render_cfg;

#define HN_RENDER_FEAT_PER_RAY 9728   /* (64 + 192) points x 16 levels x 2 features, then the
                                         MLPs' ReLU masks of those points (ABI 10) */

/* ABI 13: the training loss fused into hn_render_bwd (the trainer's step;
 * replaces its hn_loss_fwd_bwd launch).  The loss is run_nerf.py:612-636
 * under train.dp_loss's data-parallel rule:
 *   loss = (mse(rgb) + mse(rgb0)) / world + sparse_w * sum(entropy + entropy0)
 *          + tv_w * sum(tv)
 * With hn_render_bwd_args.loss set, the backward's composite pre-pass forms
 * the upstream gradients itself from the forward's outputs (hn_loss_bwd's op
 * forms with g_loss = 1; the g_* arguments are not read) and one of its
 * workgroups reduces the loss value into out[4] = loss, mse, mse0, sum of
 * entropies (hn_loss_fwd's fp64 sums, another thread count).  The TV term's
 * gradient still comes in as tv / g_tv (= tv_w per level). */
typedef struct hn_render_loss {
  const float* target;      /* [B][3] */
  const float* rgb; const float* rgb0;            /* the forward's [B][3] outputs */
  const float* sparsity; const float* sparsity0;  /* the forward's [B] entropies */
  const float* tv;          /* [n_tv] per-level TV values (hn_tv_fwd), or NULL */
  int32_t n_tv;
  float world, sparse_w, tv_w;
  float* out;               /* [4] */
} hn_render_loss;

typedef struct hn_render_fwd_args {
  int64_t n_rays;
  const float* rays;        /* [B][11] = [o3 d3 near far viewdir3] (run_nerf_helpers.py:509-512) */
  const float* t_vals;      /* [64]   torch.linspace(0,1,64) (:514) */
  const float* t_rand;      /* [B][64] jitter (:528) or NULL if !perturb */
  const float* u;           /* [B][128] importance uniforms (:276) */
  const float* noise_c;     /* [B][64] or NULL (raw_noise_std = 0) */
  const float* noise_f;     /* [B][192] or NULL */
  const float* table;       /* [16][2^T][2] */
  hn_mlp coarse;            /* network_fn */
  hn_mlp fine;              /* network_fine */
  /* outputs (render_rays ret, :560-568) */
  float* rgb; float* depth; float* acc; float* sparsity;        /* fine: [B][3],[B],[B],[B] */
  float* rgb0; float* depth0; float* acc0; float* sparsity0;    /* coarse */
  float* z_std;             /* [B] */
  /* saved for backward (also returned: raw = raw_f) */
  float* z_coarse;          /* [B][64] */
  float* z_fine;            /* [B][192] */
  float* raw_c;             /* [B][64][4] */
  float* raw_f;             /* [B][192][4] */
  uint8_t* fine_src;        /* [B][192]: coarse index of each fine sample, 255 = importance */
  float* feat;              /* [B][HN_RENDER_FEAT_PER_RAY] hash features of the 64 + 192
                               evaluated points and their ReLU masks (MFMA-tile order,
                               opaque); NULL = not kept (inference); required by hn_render_bwd */
  int32_t weights_packed;   /* ABI 13: nonzero = `workspace` already holds both nets' packed MFMA
                               copies of these weights (an hn_render_bwd with repack wrote them and the
                               weights are unchanged since): no packing launch */
  int32_t skip_dead_color;  /* ABI 14: nonzero (and no noise for that pass) = a tile of 32 samples
                               whose raw sigmas are all <= 0 -- alpha 0 and weight 0 at every sample,
                               so its colours enter no output and no gradient -- skips the colour
                               net: raw_c / raw_f rgb of those samples are written as 0 (rgb, depth,
                               acc, the entropies and every gradient unchanged), and such fine
                               tiles' features and ReLU masks are not stored in `feat` (no d raw of
                               theirs is nonzero, so a dense_bwd = 0 backward never reads them; a
                               dense_bwd = 1 backward of this state is invalid).  0 = every sample's
                               raw rgb computed (the reference's `raw` output), every tile stored */
} hn_render_fwd_args;

typedef struct hn_render_bwd_args {
  int64_t n_rays;
  const float* rays;
  const float* noise_c; const float* noise_f;
  const float* table;
  hn_mlp coarse; hn_mlp fine;
  const float* z_coarse; const float* z_fine; const float* raw_c; const float* raw_f;
  const uint8_t* fine_src;  /* from the forward */
  const float* feat;        /* from the forward (saved hash features) */
  int32_t weights_packed;   /* nonzero: `workspace` is the one hn_render_fwd used and the weights
                               are unchanged since, so its packed MFMA copies are reused */
  int32_t d_table_mode;     /* bit 0 clear: d_table += gradient (as every d* output); set: d_table =
                               gradient (every entry written, the caller need not zero it).
                               bit 1 set: d_coarse / d_fine = their gradients likewise (ABI 8) */
  /* upstream grads (NULL = 0) */
  const float* g_rgb; const float* g_depth; const float* g_acc; const float* g_sparsity;
  const float* g_rgb0; const float* g_depth0; const float* g_acc0; const float* g_sparsity0;
  const float* g_raw_f;     /* [B][192][4] or NULL */
  /* gradient outputs (+=) */
  float* d_table;           /* [16][2^T][2]; may be NULL when table_step is given */
  hn_mlp_grad d_coarse; hn_mlp_grad d_fine;
  /* Optional fused optimizer step (binned scatter only, else HN_E_SHAPE): the
   * owner pass applies this RAdam step (hn_radam_step's per-element update,
   * g = the table gradient of this backward) to the table right where it forms
   * the gradient; p / m / v are the table and its moments, g is ignored.
   * NULL = no step (the gradient goes to d_table). */
  const struct hn_radam_tensor* table_step;
  /* Optional total-variation term (loss.py:11-43; run_nerf.py:626-635) in the same
   * backward (ABI 9): tv = the TV args of the hn_tv_fwd call (host), g_tv = device
   * [L] upstream gradients of its per-level values.  With the binned scatter and
   * cubes <= 50 its gradient goes into the bins as records (so table_step stays
   * fused); otherwise it is added to d_table (hn_tv_bwd; table_step not allowed).
   * NULL = no TV term.
   * ABI 14: n_rays == 0 with a TV term (a data-parallel rank that drew no rays,
   * run_nerf.py:551-555, still carries the TV term) runs the TV term alone through
   * the same records and exact owner pass -- bitwise reproducible, unlike
   * hn_tv_bwd's float atomics; only cfg, tv, g_tv, d_table (or table_step),
   * d_table_mode and the workspace (hn_render_workspace_bytes(cfg, 0)) are read,
   * the MLP gradients are not touched, owner_defer must be 0.  The binned scatter
   * is required (else HN_E_SHAPE: use hn_tv_bwd).  n_rays == 0 without a TV term
   * does nothing. */
  const struct hn_tv_args* tv;
  const float* g_tv;
  /* Optional with table_step (ABI 11): the live row pairs of the table's leading
   * table_live_levels levels, a device bitmap over the flat [level][row] index:
   * bit (R >> 1) & 31 of word R >> 6 covers rows R and R + 1.  A clear bit
   * promises that neither row can ever receive a gradient (render or TV: level l's
   * corners lie in [0, res_l + 1]^3 once the point is clamped to the box,
   * hash_encoding.py:66-76, so the other rows of a level with (res_l + 2)^3 < 2^T
   * are structural zeros) and that their moments are zero; the fused step then
   * neither loads nor stores p / m / v there -- the dense update would leave them
   * bitwise unchanged.  A nonzero gradient on a clear pair sets fault bit 64.
   * NULL = every row stepped. */
  const uint32_t* table_live;
  int32_t table_live_levels;
  /* ABI 12, binned scatter only: nonzero = stop before the owner pass; the
   * caller then runs it per range of bins with hn_render_bwd_owner (e.g. to
   * start each range's gradient exchange while the next range is reduced).
   * The workspace must not be touched in between. */
  int32_t owner_defer;
  const hn_render_loss* loss;   /* ABI 13: NULL, or the training loss formed here (above) */
  const struct hn_radam_tensor* mlp_step;   /* ABI 13 (binned scatter only, else HN_E_SHAPE): NULL, or [10] the
                               NeRFSmall tensors' RAdam steps (network_fn's sigma_net.0, sigma_net.1,
                               color_net.0, color_net.1, color_net.2, then network_fine's; g unused),
                               applied where each weight's final gradient is formed (hn_radam_step's
                               per-element update; the gradient is still written to d_coarse / d_fine) */
  int32_t repack;           /* ABI 13, with mlp_step: then write the stepped weights' packed MFMA copies
                               into `workspace` (in the overflow-placement launch), so the next
                               hn_render_fwd on this workspace may set weights_packed */
} hn_render_bwd_args;

/* The binned scatter's bins for this cfg and batch: returns their number (0:
 * the float-atomic schedule, no bins) and sets *shift: bin b holds the table
 * entries (flat level-major rows) [b << shift, (b + 1) << shift). */
int32_t hn_render_bins(const hn_render_cfg* cfg, int64_t n_rays, int32_t* shift);
/* The owner pass of hn_render_bwd (owner_defer set) over bins [bin_lo,
 * bin_hi): writes (or steps, with table_step) exactly those bins' slices of
 * the table gradient.  Same cfg / args / workspace as the deferred call. */
int32_t hn_render_bwd_owner(const hn_render_cfg* cfg, const hn_render_bwd_args* a, void* workspace,
                            size_t ws_bytes, int32_t bin_lo, int32_t bin_hi, void* stream);

/* ---- L4 hash-table total variation (loss.py:11-43), all levels at once ---
 * Level l samples the cube of (cube[l]+1)^3 grid vertices starting at
 * min_vertex[l] (device int32 [L][3], the reference's torch.randint draw),
 * hashes them like hash_encoding.py:112-128 and sums squared differences of
 * the entries along x, y and z, divided by cube[l]. */
typedef struct hn_tv_args {
  int32_t n_levels;
  int32_t log2_hashmap_size;
  int32_t cube[HN_MAX_LEVELS];
  const int32_t* min_vertex;   /* device [L][3] */
  const float* table;          /* device [L][2^T][2] */
} hn_tv_args;
/* tv[L] (device) is overwritten with the per-level TV values. */
int32_t hn_tv_fwd(const hn_tv_args* a, float* tv, void* stream);
/* dtable += sum_l g_tv[l] * d tv_l / d table  (g_tv: device [L]). */
int32_t hn_tv_bwd(const hn_tv_args* a, const float* g_tv, float* dtable, void* stream);

/* ---- L4 RAdam step (radam.py:28-94) over many tensors in one launch -----
 * Per element, in the op forms of torch's CPU kernels (bit-exact on the
 * reference's trace):
 *   v = fma((1-beta2)*g, g, v*beta2) ; m = fma(1-beta1, g, m*beta1)
 *   mode 2 (N_sma >= 5): p = fma(neg_wd_lr, p, p) (if wd); p += (neg_step_lr*m)/(sqrt(v)+eps)
 *   mode 1 (step_size > 0, N_sma < 5): p = fma(neg_wd_lr, p, p) (if wd); p = fma(neg_step_lr, m, p)
 *   mode 0: moments only (the reference's first steps at beta2=0.99).
 * Scalars are the fp32 values torch would use (host computes N_sma/step_size). */
#define HN_RADAM_MAX_TENSORS 16
typedef struct hn_radam_tensor {
  float* p; const float* g; float* m; float* v; int64_t n;
  float beta1, beta2, one_minus_beta1, one_minus_beta2, eps, neg_wd_lr, neg_step_lr;
  int32_t mode;
  int32_t has_wd;
  int32_t reserved;
} hn_radam_tensor;
int32_t hn_radam_step(const hn_radam_tensor* ts, int32_t n_tensors, void* stream);

/* ---- L5 training-step driver (run_nerf.py:576-636) -----------------------
 * Device ray sampler: n_rays DISTINCT pixels of one training image drawn
 * without replacement (np.random.choice(..., replace=False) at
 * run_nerf.py:595; here a seeded Feistel permutation of the crop window with
 * cycle walking), the rays of ray_util.py:62-80 for them, and their target
 * colours.  rays[n][11] = [o3 d3 near far viewdir3] (the ray batch render()
 * builds, run_nerf_helpers.py:355-368); target[n][3]. */
typedef struct hn_ray_sampler {
  int32_t H, W;                        /* image size */
  int32_t crop_y0, crop_x0, crop_h, crop_w;   /* sampling window (precrop, :584-593) */
  float fx, fy, cx, cy;                /* intrinsics K */
  float near, far;
  uint64_t seed;                       /* per step and rank */
} hn_ray_sampler;
int32_t hn_sample_rays(const hn_ray_sampler* s, const float* image, const float* c2w, int64_t n_rays,
                       float* rays, float* target, void* stream);
/* The same draw (same set for the same seed) listed in Morton order of its
 * pixels (window-relative row, column), so consecutive rays are spatial
 * neighbours: hn_render_fwd gives consecutive ray groups to one XCD and they
 * share its L2.  Pixel x is drawn iff perm^-1(x) < n_rays, so the Morton walk
 * of the window compacts the draw in order, without a sort.  Window sides up
 * to HN_SAMPLER_MORTON_MAX; workspace = hn_sample_rays_morton_workspace_bytes. */
#define HN_SAMPLER_MORTON_MAX 4096
size_t hn_sample_rays_morton_workspace_bytes(const hn_ray_sampler* s);
int32_t hn_sample_rays_morton(const hn_ray_sampler* s, const float* image, const float* c2w, int64_t n_rays,
                              float* rays, float* target, void* workspace, size_t ws_bytes, void* stream);

/* ABI 13: torch.rand on the device's default generator, restated bit for bit
 * (render_rays' draws, run_nerf_helpers.py:528 t_rand and :276 via :548 u):
 * ATen's uniform_ kernel runs `threads` = blockDim x gridDim threads of
 * hiprand Philox4x32-10 (key = seed, subsequence = thread, counter = offset / 4
 * + call), four values per call, element li from thread li % threads, call
 * li / (4 threads), component (li / threads) % 4; value 2^-32 + v 2^-32, with
 * 1 mapped to 0.  The caller supplies the generator's seed and each draw's
 * offset and threads as torch would use them (and advances the generator). */
typedef struct hn_uniform_draw {
  float* out;               /* [numel] */
  int64_t numel;
  int64_t threads;          /* torch's launch for this numel: 256 x min(ceil(numel / 256), CUs x 2048 / 256) */
  uint64_t offset;          /* the generator's philox offset at this draw (a multiple of 4) */
} hn_uniform_draw;
#define HN_UNIFORM_MAX_DRAWS 4
int32_t hn_uniform_philox(uint64_t seed, const hn_uniform_draw* draws, int32_t n_draws, void* stream);
/* hn_sample_rays_morton with the step's uniform draws made in its first
 * launch (one launch less than the sampler + torch.rand's own launches). */
int32_t hn_sample_batch_morton(const hn_ray_sampler* s, const float* image, const float* c2w, int64_t n_rays,
                               float* rays, float* target, void* workspace, size_t ws_bytes, uint64_t seed,
                               const hn_uniform_draw* draws, int32_t n_draws, void* stream);

/* use_batching ray pool (run_nerf.py:505-521 builds rays_rgb from every training
 * pixel and shuffles it; :544-555 takes consecutive N_rand slices and reshuffles
 * after each epoch).  The pool is never materialised: position q of an epoch
 * maps to pool pixel perm(q) (a keyed, cycle-walked Feistel bijection of
 * [0, n_images * H * W), the epoch's shuffle; pool order is (image, row,
 * column) as rays_rgb's reshape), whose ray is get_rays_np's (ray_util.py:82-93:
 * float64 arithmetic, rounded to float32 as rays_rgb.astype(np.float32)) and
 * whose target is the image pixel.  Batch k of an epoch = positions
 * [k N_rand, min((k + 1) N_rand, pool size)): the caller passes start = k N_rand
 * and the batch length (the last batch of an epoch is short, as the
 * reference's slice).  rays[n][11] and target[n][3] as hn_sample_rays. */
typedef struct hn_ray_pool {
  int32_t n_images;       /* training images in the pool (image_ids[n_images]) */
  int32_t H, W;
  int32_t pose_stride;    /* floats between consecutive c2w matrices in `poses` (12 or 16) */
  double fx, fy, cx, cy;  /* intrinsics K, float64 as get_rays_np uses them */
  float near, far;
  uint64_t seed;          /* the epoch's shuffle key */
} hn_ray_pool;
/* images: device [n_all][H][W][3]; poses: device [n_all][.][4] (row-major
 * c2w, pose_stride floats apart); image_ids: device int32 [n_images] (i_train). */
int32_t hn_sample_pool(const hn_ray_pool* p, const float* images, const float* poses, const int32_t* image_ids,
                       int64_t start, int64_t n_rays, float* rays, float* target, void* stream);

/* Blender image preparation (load/load_blender.py:63, :78-86; run_nerf.py:259-262):
 * rgba: device uint8 [n][H][W][4] (the PNGs) -> out, float32:
 *   x = float32(u8 / 255.0)  (float64 division, as np.array(imgs) / 255.);
 *   half_res: 2 x 2 box mean (cv2.resize INTER_AREA to H/2 x W/2; H, W even);
 *   mode 0: RGBA [n][H'][W'][4] (what load_blender_data returns);
 *   mode 1: white background, rgb * a + (1 - a) -> [n][H'][W'][3] (float32
 *           arithmetic at full resolution, float64 after half_res as the
 *           reference's float64 half-res array, rounded to float32);
 *   mode 2: rgb only -> [n][H'][W'][3] (white_bkgd False). */
int32_t hn_blender_images(const uint8_t* rgba, int64_t n_images, int32_t H, int32_t W, int32_t half_res,
                          int32_t mode, float* out, void* stream);

/* Training loss (run_nerf.py:612-636 with the data-parallel rule of
 * SURVEY 8e): loss = (mse(rgb) + mse(rgb0)) / world + sparse_w * (sum sp + sum sp0)
 * + tv_w * sum tv.  rgb0/sp0/tv may be NULL.  out[4] (device) = loss, mse, mse0,
 * sum of entropies.  The backward writes the upstream gradients of the five
 * inputs in torch autograd's op order (mean/pow/div/mul backward), g_loss is
 * the device scalar d L_total / d loss. */
int32_t hn_loss_fwd(const float* rgb, const float* rgb0, const float* target, const float* sp,
                    const float* sp0, int64_t n_rays, const float* tv, int32_t n_tv, float world,
                    float sparse_w, float tv_w, float* out, void* stream);
int32_t hn_loss_bwd(const float* rgb, const float* rgb0, const float* target, int64_t n_rays,
                    int32_t n_tv, float world, float sparse_w, float tv_w, const float* g_loss,
                    float* g_rgb, float* g_rgb0, float* g_sp, float* g_sp0, float* g_tv, void* stream);
/* hn_loss_fwd and hn_loss_bwd in one launch (the trainer's step: the backward
 * does not depend on the loss value); out and the gradients bitwise those of
 * the two calls. */
int32_t hn_loss_fwd_bwd(const float* rgb, const float* rgb0, const float* target, const float* sp,
                        const float* sp0, int64_t n_rays, const float* tv, int32_t n_tv, float world,
                        float sparse_w, float tv_w, float* out, const float* g_loss, float* g_rgb,
                        float* g_rgb0, float* g_sp, float* g_sp0, float* g_tv, void* stream);

size_t hn_render_workspace_bytes(const hn_render_cfg* cfg, int64_t n_rays);
/* The table-gradient scatter hn_render_bwd runs for this configuration and
 * batch (1 float atomics, 2 binned), after cfg->scatter, the table size and
 * the box's cell counts. */
int32_t hn_render_scatter_mode(const hn_render_cfg* cfg, int64_t n_rays);
int32_t hn_render_fwd(const hn_render_cfg* cfg, const hn_render_fwd_args* a,
                      void* workspace, size_t ws_bytes, void* stream);
int32_t hn_render_bwd(const hn_render_cfg* cfg, const hn_render_bwd_args* a,
                      void* workspace, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HASHNERF_AMD_H */
