"""Training-step driver: the loop of run_nerf.py:541-651 with on-device ray
sampling, plus data-parallel gradient exchange.

One step = draw one training image per rank, N_rand pixels without
replacement (centre crop for the first ``precrop_iters``) -- or, with
use_batching (no_batching False, run_nerf.py:505-521, 544-555), the next
N_rand positions of the shuffled pool of every training ray -- render with the
fused kernels, loss (MSE fine + coarse + sparse_loss_weight * entropy sums
+ tv_loss_weight * TV), backward, gradient all-reduce (DP), RAdam step and
the exponential lr decay of run_nerf.py:647-651 (applied after step() with
the pre-increment global_step).

DP semantics: every rank renders its own rays; per-rank MSE
terms are divided by world_size and the entropy sums are not, so a SUM
all-reduce yields exactly the gradient of the global-batch reference loss;
the TV term (one random cube per level) is added on rank 0 only.
"""
from __future__ import annotations

import math
import types
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import functional as HF
from .create import create_nerf
from .loss import draw_tv_cubes, tv_loss_levels
from .rays import bbox_for_blender, blender_cameras, blender_intrinsics, get_rays, pose_spherical
from .render import img2mse, mse2psnr, render, render_ray_batch


def dp_loss(mse_fine, mse_coarse, entropy_sum, world, sparse_loss_weight, tv=None,
            tv_loss_weight=0.0):
    """Per-rank loss whose SUM-all-reduced gradient equals the gradient of the
    reference loss (run_nerf.py:612-636) over the global batch: the MSE terms
    are means (divide by world), the entropy term is a sum over rays (do not),
    and the TV term is counted once (pass tv on one rank only)."""
    loss = (mse_fine + (mse_coarse if mse_coarse is not None else 0.0)) / world
    loss = loss + sparse_loss_weight * entropy_sum
    if tv is not None:
        loss = loss + tv_loss_weight * tv
    return loss


def live_rows(resolutions, log2_hashmap_size):
    """Rows of the coarse levels that a gradient can ever touch.

    A point is clamped to the bbox before its cell is taken
    (hash_encoding.py:66-76), so level l's corners lie in [0, res_l + 1]^3 and
    its gradient (render scatter and TV alike) only lands on the hashed rows of
    those (res_l + 2)^3 vertices.  For the leading levels where that is fewer
    than 2^T rows, every other row's gradient is a structural zero on every
    rank.  Returns (n_sparse_levels, int64 row index into the first
    n_sparse_levels levels, flattened) -- e.g. T=19, finest 512: levels 0-6,
    ~0.5 M of 3.7 M rows; None when no level qualifies."""
    T = log2_hashmap_size
    idx, n_lv = [], 0
    for l, res in enumerate(int(r) for r in resolutions):
        n = res + 2
        if n ** 3 >= 2 ** T:
            break
        g = np.arange(n, dtype=np.uint64)
        x, y, z = np.meshgrid(g, g, g, indexing="ij")
        h = (x * np.uint64(1)) ^ (y * np.uint64(2654435761)) ^ (z * np.uint64(805459861))   # hash_encoding.py:112-128
        rows = np.unique((h & np.uint64(2 ** T - 1)).astype(np.int64).ravel())
        idx.append(rows + (l << T))
        n_lv = l + 1
    if not n_lv:
        return None
    return n_lv, torch.from_numpy(np.concatenate(idx))


def live_pair_mask(resolutions, log2_hashmap_size):
    """live_rows as the bitmap of hn_render_bwd_args.table_live: bit
    (R >> 1) & 31 of word R >> 6 is set when row R or R + 1 of the flat
    [level][row] index is live.  Returns (n_levels, int32 tensor) or None."""
    lv = live_rows(resolutions, log2_hashmap_size)
    if lv is None or log2_hashmap_size < 6:
        return None
    n_lv, rows = lv
    pairs = rows.numpy().astype(np.uint64) >> np.uint64(1)
    words = np.zeros(n_lv << (log2_hashmap_size - 6), dtype=np.uint32)
    np.bitwise_or.at(words, (pairs >> np.uint64(5)).astype(np.int64),
                     (np.uint32(1) << (pairs & np.uint64(31)).astype(np.uint32)))
    return n_lv, torch.from_numpy(words.view(np.int32))


def allreduce_grads(table, mlp_params, group=None, live=None):
    """SUM all-reduce of the hash-table gradient and of the flattened
    NeRFSmall gradients, issued asynchronously back to back so RCCL can run
    them concurrently.

    ``live`` = live_rows(...) of the table: the coarse levels' structurally
    zero rows are left out of the exchange -- their live rows are gathered
    into one compact bucket and scattered back, the dense levels are reduced
    in place (T=19, finest 512: 40 MB on the wire instead of 64 MiB).  The
    result is identical to reducing the whole table."""
    mlp = [p for p in mlp_params if p.grad is not None]
    flat = torch.cat([p.grad.reshape(-1) for p in mlp]) if mlp else None
    works, compact = [], None
    g = table.grad
    if g is not None:
        if live is None:
            works.append(dist.all_reduce(g, group=group, async_op=True))
        else:
            n_lv, rows = live
            rows = rows.to(g.device)
            head = g[:n_lv].reshape(-1, g.shape[-1])
            compact = head.index_select(0, rows)
            works.append(dist.all_reduce(compact, group=group, async_op=True))
            if n_lv < g.shape[0]:
                works.append(dist.all_reduce(g[n_lv:], group=group, async_op=True))
    if flat is not None:
        works.append(dist.all_reduce(flat, group=group, async_op=True))
    for w in works:
        w.wait()
    if compact is not None:
        head.index_copy_(0, rows, compact)
    off = 0
    for p in mlp:
        n = p.numel()
        p.grad.copy_(flat[off:off + n].view_as(p))
        off += n


class Collectives:
    """The two collectives of the sharded table step: ``reduce_scatter(out,
    inp)`` = ``reduce_scatter_tensor`` (SUM; ``out`` is this rank's 1/world
    slice of ``inp``'s sum) and ``all_gather(out, inp)`` =
    ``all_gather_into_tensor`` (``inp`` may be ``out``'s own slice: in
    place).  These production calls run on RCCL and on gloo with host
    tensors (torch 2.10's gloo implements both, async reduce-scatter and the
    in-place all-gather included), so the CPU gloo tests execute exactly the
    calls an RCCL run makes.

    ``emulate=True`` replaces each call by an emulation INTO THE SAME out
    tensor (all-reduce + copy of the rank's slice; a list all-gather over
    ``out``'s views).  It is the default only for gloo on device tensors
    (the GPU DP tests run two ranks of one GPU over gloo); the gloo tests hold
    the two forms bitwise equal on host tensors (tests/test_dp_gloo.py) and
    on device tensors (tests/test_gpu_dp.py)."""

    def __init__(self, rank, world, group=None, emulate=None, device=None):
        self.rank, self.world, self.group = rank, world, group
        dev = torch.device(device) if device is not None else torch.device("cpu")
        gloo_dev = dist.get_backend(group) == "gloo" and dev.type != "cpu"
        self.emulate = gloo_dev if emulate is None else emulate

    def reduce_scatter(self, out, inp, async_op=False):
        """Returns the RCCL work handle with async_op (None under gloo, whose
        emulation completes in the call)."""
        n = out.numel()
        if inp.numel() != n * self.world:
            raise ValueError(f"reduce_scatter: input {inp.numel()} != {self.world} x output {n}")
        if self.emulate:
            dist.all_reduce(inp, group=self.group)
            out.copy_(inp[self.rank * n:(self.rank + 1) * n])
            return None
        return dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=async_op)

    def all_gather(self, out, inp):
        n = inp.numel()
        if out.numel() != n * self.world:
            raise ValueError(f"all_gather: output {out.numel()} != {self.world} x input {n}")
        if self.emulate:
            dist.all_gather(list(out.chunk(self.world)), inp.clone(), group=self.group)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.group)


class ShardedTableStep:
    """Data-parallel exchange + RAdam step of the hash table as reduce-scatter
    -> RAdam on this rank's shard -> all-gather (SURVEY 8e's alternative to
    one all-reduce): the same bytes on the wire as the
    all-reduce, 1/world of the dense optimizer work per rank (radam.py:28-94
    over 16.7 M / 134 M parameters).

    The exchanged vector is the table packed as [levels n_lv.. (dense) |
    the live rows of the coarse levels 0..n_lv-1 (train.live_rows: the rest
    of those levels is a structural zero on every rank) | zero pad], so the
    wire carries 40 MB instead of 64 MiB at T=19 / finest 512.  Gradient and
    parameters each live in one buffer laid out [coarse dense | dense tail |
    packed coarse | pad]: the render backward writes the table gradient into
    its first part as usual, and the packed vector is the buffer from the
    tail on -- contiguous, no copy of the 60 MB tail.  The table parameter is
    re-pointed into the parameter buffer, so the all-gather updates the tail
    in place and the coarse live rows are scattered back (4 MB).

    Segments (overlap with the backward).  With ``bins`` =
    (nbins, shift) of the binned scatter, the vector is cut into up to
    ``n_chunks`` segments at bin boundaries (each a multiple of world floats):
    tail pieces, then [rest of the tail | packed coarse | pad].  Each segment
    is reduce-scattered on its own, right after ``produce(k)`` has formed its
    bins' gradient (the render backward's deferred owner pass over
    ``seg_bins[k]``; segment 0's range also holds the coarse levels), so on
    RCCL segment k's exchange runs while the owner pass reduces segment k+1.
    A rank's shard is the concatenation of its slices of the segments (its
    p / g / m / v shards all in that order); one segment is the plain
    layout.  The stepped shards come back in ONE all-gather (rank-major, then
    one strided copy per segment), so the segmentation adds reduce-scatter
    calls only.

    The table's RAdam moments live for this rank's shard only.  They start
    from ``state`` (the optimizer's exp_avg / exp_avg_sq of the table, e.g.
    loaded from a checkpoint, run_nerf.py:158-168), packed like the gradient;
    gather_state() rebuilds the full ones (dead rows: zero, as the dense
    reference keeps them).  ``stale`` is set by every step and cleared by
    gather_state(): RAdam.state_dict() refuses to write a checkpoint while the
    optimizer's full-size copy is stale (Trainer.sync_optimizer_state)."""

    def __init__(self, table, live, rank, world, group=None, state=None, stepper=None, bins=None, n_chunks=4,
                 emulate=None):
        L_, R, F_ = table.shape
        self.table, self.rank, self.world, self.group = table, rank, world, group
        self.coll = Collectives(rank, world, group, emulate=emulate, device=table.device)
        self.stepper = HF.radam_step if stepper is None else stepper
        self.full = L_ * R * F_
        n_lv, rows = live if live is not None else (0, None)
        self.rows = rows
        self.head = n_lv * R * F_
        self.nc = 0 if rows is None else rows.numel() * F_
        n = self.full - self.head + self.nc
        self.P = (n + world - 1) // world * world
        self.s = self.P // world
        self.segs, self.seg_bins = self._segments(bins, n_chunks)
        offs = [0]
        for lo, hi in self.segs:
            offs.append(offs[-1] + (hi - lo) // world)
        self.shard_offs = offs
        dev = table.device
        self.gbuf = torch.zeros(self.head + self.P, dtype=torch.float32, device=dev)
        self.pbuf = torch.zeros(self.head + self.P, dtype=torch.float32, device=dev)
        self.g_shard = torch.empty(self.s, dtype=torch.float32, device=dev)
        self.p_shard = torch.empty(self.s, dtype=torch.float32, device=dev)
        with torch.no_grad():
            self.pbuf[:self.full].copy_(table.data.reshape(-1))
        table.data = self.pbuf[:self.full].view(L_, R, F_)
        self.m = torch.zeros(self.s, dtype=torch.float32, device=dev)
        self.v = torch.zeros(self.s, dtype=torch.float32, device=dev)
        self._gath = None   # rank-major all-gather buffer (segmented exchange)
        self.load_state(state)

    @torch.no_grad()
    def load_state(self, state):
        """(Re)seed this rank's moment shards from the table's full-size
        optimizer state (exp_avg / exp_avg_sq); zeros without one.  Called at
        construction and by RAdam.load_state_dict (a checkpoint loaded after
        the sharded step began)."""
        if state is not None and "exp_avg" in state:
            self.m.copy_(self._shard_of(state["exp_avg"]))
            self.v.copy_(self._shard_of(state["exp_avg_sq"]))
        else:
            self.m.zero_()
            self.v.zero_()
        self.stale = False

    def _segments(self, bins, n_chunks):
        """[(lo, hi)] over the packed vector (offsets from ``head``) and each
        segment's bins [(b_lo, b_hi)] (None without ``bins``)."""
        if not bins or n_chunks <= 1:
            return [(0, self.P)], None
        nbins, shift = bins
        bf = 2 << shift                              # floats per bin
        tail = self.full - self.head
        unit = self.world * bf
        if self.head % bf or self.full % bf or tail < unit:
            return [(0, self.P)], None
        nu = tail // unit                            # whole units in the tail
        k = min(n_chunks - 1, nu)
        cuts = [0] + [unit * ((nu * (j + 1)) // k) for j in range(k)]
        segs = [(cuts[j], cuts[j + 1]) for j in range(k)]
        if cuts[-1] < self.P:
            segs.append((cuts[-1], self.P))
        b0 = self.head // bf
        sb = [(0 if j == 0 else b0 + lo // bf, min(nbins, b0 + hi // bf) if hi <= tail else nbins)
              for j, (lo, hi) in enumerate(segs)]
        sb[-1] = (sb[-1][0], nbins)
        return segs, sb

    def _packed_vector(self, full):
        """A full-size table tensor packed like the exchanged vector ([dense
        tail | coarse live rows | zero pad], P floats)."""
        F_ = self.table.shape[2]
        flat = full.detach().reshape(-1).to(device=self.pbuf.device, dtype=torch.float32)
        parts = [flat[self.head:]]
        if self.nc:
            parts.append(flat[:self.head].view(-1, F_).index_select(0, self.rows).reshape(-1))
        packed = torch.cat(parts)
        return torch.cat([packed, packed.new_zeros(self.P - packed.numel())])

    def _shard_slices(self, vec):
        """This rank's slices of the segments of a packed vector (views)."""
        out = []
        for lo, hi in self.segs:
            n = (hi - lo) // self.world
            out.append(vec[lo + self.rank * n:lo + (self.rank + 1) * n])
        return out

    def _shard_of(self, full):
        """This rank's shard of a full-size table tensor (segment order)."""
        return torch.cat(self._shard_slices(self._packed_vector(full)))

    def grad_view(self):
        """Where the render backward writes the table gradient (overwrite)."""
        return self.gbuf[:self.full].view(self.table.shape)

    def _packed_coarse(self, buf):
        F_ = self.table.shape[2]
        return buf[self.full:self.full + self.nc].view(-1, F_)

    def exchange_bytes(self):
        """Bytes each collective of one step moves per rank buffer: the
        reduce-scatter's input and the all-gather's output (P floats each: the
        dense tail + the coarse levels' live rows + pad)."""
        return 4 * self.P

    @torch.no_grad()
    def step(self, coeffs, produce=None, extra=(), pre_step=None):
        """After the backward: exchange the gradient, RAdam step on the shard
        (hn_radam_step, the reference's per-element op forms), all-gather.
        ``produce(k)``: forms segment k's gradient first (the deferred owner
        pass over seg_bins[k]); None = the gradient is complete.  ``extra``:
        more (p, g, m, v, coeffs) to step in the same hn_radam_step launch
        (the trainer's NeRFSmall tensors), after ``pre_step()`` (their
        gradients' all-reduce wait).  bench.py times the reduce-scatter
        (issue to wait), the step launch and the all-gather on the compute
        stream (HF.TIMER names xchg_*)."""
        F_ = self.table.shape[2]
        vec_g, vec_p = self.gbuf[self.head:], self.pbuf[self.head:]
        works = []
        last = len(self.segs) - 1
        # (bench.py: the deferred owner pass's launches, bracketed on the compute stream)
        t_own = HF.TIMER.begin("render_bwd_owner") if produce is not None else None
        t_rs = None
        for k, (lo, hi) in enumerate(self.segs):
            if produce is not None:
                produce(k)
            if k == last and self.nc:   # the coarse levels' bins are in segment 0's range
                torch.index_select(self.gbuf[:self.head].view(-1, F_), 0, self.rows, out=self._packed_coarse(self.gbuf))
            o0, o1 = self.shard_offs[k], self.shard_offs[k + 1]
            if t_rs is None:
                t_rs = HF.TIMER.begin("xchg_reduce_scatter")
            works.append(self.coll.reduce_scatter(self.g_shard[o0:o1], vec_g[lo:hi], async_op=True))
        HF.TIMER.end("render_bwd_owner", t_own)
        # the shard's parameters (the table may have been loaded since the last step)
        if self.nc:
            torch.index_select(self.pbuf[:self.head].view(-1, F_), 0, self.rows, out=self._packed_coarse(self.pbuf))
        torch.cat(self._shard_slices(vec_p), out=self.p_shard)
        for w in works:
            if w is not None:
                w.wait()
        HF.TIMER.end("xchg_reduce_scatter", t_rs)
        if pre_step is not None:
            pre_step()
        t_st = HF.TIMER.begin("xchg_step")
        self.stepper([(self.p_shard, self.g_shard, self.m, self.v, coeffs)] + list(extra))
        HF.TIMER.end("xchg_step", t_st)
        t_ag = HF.TIMER.begin("xchg_all_gather")
        if len(self.segs) == 1:   # the shard is one slice of the vector: gathered in place
            self.coll.all_gather(vec_p, self.p_shard)
        else:
            # one all-gather (one collective call, not one per segment) into a
            # rank-major buffer, then each segment's [world, n_k] block copied
            # into place
            if self._gath is None:
                self._gath = torch.empty(self.P, dtype=torch.float32, device=self.pbuf.device)
            self.coll.all_gather(self._gath, self.p_shard)
            g2 = self._gath.view(self.world, self.s)
            for k, (lo, hi) in enumerate(self.segs):
                o0, o1 = self.shard_offs[k], self.shard_offs[k + 1]
                vec_p[lo:hi].view(self.world, o1 - o0).copy_(g2[:, o0:o1])
        if self.nc:
            self.pbuf[:self.head].view(-1, F_).index_copy_(0, self.rows, self._packed_coarse(self.pbuf))
        HF.TIMER.end("xchg_all_gather", t_ag)
        self.stale = True

    @torch.no_grad()
    def gather_state(self):
        """Full-size (exp_avg, exp_avg_sq) of the table from every rank's shard."""
        out = []
        F_ = self.table.shape[2]
        for sh in (self.m, self.v):
            packed = torch.empty(self.P, dtype=torch.float32, device=sh.device)
            for k, (lo, hi) in enumerate(self.segs):
                self.coll.all_gather(packed[lo:hi], sh[self.shard_offs[k]:self.shard_offs[k + 1]])
            full = torch.zeros(self.full, dtype=torch.float32, device=sh.device)
            full[self.head:] = packed[:self.full - self.head]
            if self.nc:
                full[:self.head].view(-1, F_).index_copy_(0, self.rows,
                                                          packed[self.full - self.head:][:self.nc].view(-1, F_))
            out.append(full.view(self.table.shape))
        self.stale = False
        return out


def default_args(**over):
    """chair.txt + run_nerf.py defaults (configs/chair.txt:1-19, README.md:20)."""
    a = dict(N_rand=1024, N_samples=64, N_importance=128, use_viewdirs=True, white_bkgd=True,
             perturb=1.0, raw_noise_std=0.0, lrate=0.01, lrate_decay=10, precrop_iters=500,
             precrop_frac=0.5, finest_res=512, log2_hashmap_size=19, sparse_loss_weight=1e-10,
             tv_loss_weight=1e-6, netchunk=1024 * 64, chunk=1024 * 32, dataset_type="blender",
             i_embed=1, i_embed_views=2, no_reload=True, ft_path=None, basedir=None, expname=None,
             H=400, W=400, n_train=100, lindisp=False, no_ndc=False, tv_until=1001, no_batching=True)
    a.update(over)
    return types.SimpleNamespace(**a)


def _box_sdf(p, c, h):
    q = (p - p.new_tensor(c)).abs() - p.new_tensor(h)
    return q.clamp(min=0).norm(dim=-1) + q.max(-1).values.clamp(max=0)


# (centre, half extent, albedo) of the procedural chair: seat, back, 4 legs
_CHAIR_BOXES = (((0., 0., 0.), (.55, .55, .07), (.80, .45, .20)),
                ((0., -.50, .55), (.55, .06, .48), (.70, .35, .15)),
                ((.45, .45, -.52), (.06, .06, .45), (.25, .25, .30)),
                ((-.45, .45, -.52), (.06, .06, .45), (.25, .25, .30)),
                ((.45, -.45, -.52), (.06, .06, .45), (.25, .25, .30)),
                ((-.45, -.45, -.52), (.06, .06, .45), (.25, .25, .30)))
_CHAIR_BALL = ((.15, .10, .30), .22, (.20, .45, .85))


def procedural_field(pts):
    """Analytic chair-like radiance field (density from a sharpened box/sphere
    SDF union, albedo with a sinusoidal texture): pts [..., 3] -> sigma [...],
    rgb [..., 3].  The stand-in for nerf-synthetic's chair, which is not in
    the image: a scene the hash grid can learn, so PSNR curves mean something."""
    sdfs = [_box_sdf(pts, c, h) for c, h, _ in _CHAIR_BOXES]
    sdfs.append((pts - pts.new_tensor(_CHAIR_BALL[0])).norm(dim=-1) - _CHAIR_BALL[1])
    sdf = torch.stack(sdfs, -1)
    d, k = sdf.min(-1)
    albedo = pts.new_tensor([a for _, _, a in _CHAIR_BOXES] + [_CHAIR_BALL[2]])[k]
    s = lambda k: torch.sin(k * pts[..., 0]) * torch.sin(k * pts[..., 1]) * torch.sin(k * pts[..., 2])
    # a coarse pattern plus grain finer than a finest-level voxel and than a
    # pixel at 200x200 (period 0.0086 vs 0.016 / 0.014)
    tex = 0.65 + 0.15 * s(14.) + 0.2 * s(733.)
    sigma = 60. * torch.sigmoid(-60. * d)
    return sigma, (albedo * tex[..., None]).clamp(0., 1.)


@torch.no_grad()
def render_procedural(H, W, K, c2w, near=2., far=6., n_samples=384, chunk=8192, white_bkgd=True):
    """Ground-truth image [H, W, 3] of procedural_field by dense midpoint
    quadrature of the volume-rendering integral (alpha compositing as
    raw2outputs, white background as blender)."""
    ro, rd = get_rays(H, W, K, c2w[:3, :4])
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    t = near + (far - near) * (torch.arange(n_samples, device=ro.device) + .5) / n_samples
    delta = (far - near) / n_samples
    out = []
    for i in range(0, ro.shape[0], chunk):
        o, d = ro[i:i + chunk], rd[i:i + chunk]
        pts = o[:, None] + d[:, None] * t[None, :, None]
        sigma, rgb = procedural_field(pts)
        alpha = 1. - torch.exp(-sigma * delta * d.norm(dim=-1, keepdim=True))
        trans = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1. - alpha + 1e-10], -1), -1)[:, :-1]
        w = alpha * trans
        c = (w[..., None] * rgb).sum(1)
        if white_bkgd:
            c = c + (1. - w.sum(-1, keepdim=True))
        out.append(c)
    return torch.cat(out, 0).reshape(H, W, 3)


class SyntheticBlender:
    """Synthetic nerf-synthetic-shaped dataset held in HBM: n training
    cameras on the hemisphere (camera_angle_x of chair), bbox from bbox.py's
    rule.  scene="uniform": targets uniform in [0,1]^3 (speed runs);
    scene="procedural": images of procedural_field rendered on the device
    (PSNR runs), plus n_test held-out views (test_poses, test_images)."""

    def __init__(self, H, W, n, device, seed=0, scene="uniform", n_test=0):
        self.H, self.W = H, W
        self.focal, self.K = blender_intrinsics(H, W)
        poses = blender_cameras(n)
        self.poses = torch.stack(poses, 0).to(device)
        self.bounding_box = bbox_for_blender(poses, H, W, self.focal)
        if scene == "uniform":
            g = torch.Generator(device="cpu").manual_seed(seed)
            self.images = torch.rand((n, H, W, 3), generator=g).to(device)
        elif scene == "procedural":
            self.images = torch.stack([render_procedural(H, W, self.K, c) for c in self.poses], 0)
        else:
            raise ValueError(f"SyntheticBlender scene {scene!r}")
        self.i_train = torch.arange(n)
        # held-out views between the training azimuths, elevation -45
        th = np.linspace(-180, 180, n_test + 1)[:-1] + 180. / max(n, 1)
        self.test_poses = torch.stack([pose_spherical(float(t), -45., 4.0) for t in th], 0).to(device) \
            if n_test else None
        self.test_images = torch.stack([render_procedural(H, W, self.K, c) for c in self.test_poses], 0) \
            if (n_test and scene == "procedural") else None


def _step_seed(seed, rank, step):
    """64-bit splitmix of (seed, rank, step): the device sampler's key."""
    x = (seed * 0x9E3779B97F4A7C15 + rank * 0xBF58476D1CE4E5B9 + step * 0x94D049BB133111EB) & (2 ** 64 - 1)
    x ^= x >> 30
    x = (x * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)
    x ^= x >> 27
    x = (x * 0x94D049BB133111EB) & (2 ** 64 - 1)
    return x ^ (x >> 31)


class Trainer:
    """One training iteration of run_nerf.py:541-651.

    mode="explicit" (default): the step as an explicit launch sequence -- device
    ray sampler, fused render forward, TV forward, fused loss forward and
    backward, render backward and TV backward accumulating into ONE persistent
    table-gradient buffer, all-reduce, RAdam -- with no autograd graph (the
    gradients are those autograd computes for the same loss: the loss
    backward reproduces autograd's op order, the render/TV backwards are the
    Functions' own backwards).  mode="autograd": the same kernels through the
    autograd module API (render_rays, TrainLossFn, TVFn).  mode="eager": the
    module API with eager torch sampling and loss ops (randperm, img2mse,
    sums), the op-for-op rendition of run_nerf.py."""

    def __init__(self, args, data: SyntheticBlender, device, rank=0, world=1, seed=0, mode="explicit",
                 ray_order=1):
        self.args, self.data, self.device = args, data, torch.device(device)
        self.rank, self.world = rank, world
        if mode not in ("explicit", "autograd", "eager"):
            raise ValueError(f"Trainer mode {mode!r}")
        self.seed, self.mode = seed, mode
        self.ray_order = ray_order   # functional.sample_rays order: 1 Morton (default), 0 draw order
        args.bounding_box = data.bounding_box
        torch.manual_seed(seed)                      # identical init on every rank
        (self.kw_train, self.kw_test, self.start, self.grad_vars,
         self.optimizer) = create_nerf(args, device=self.device)
        self.embed_fn = self.kw_train["embed_fn"]
        self.params = list(self.grad_vars) + list(self.embed_fn.parameters())
        self.global_step = self.start
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(1000003 * seed + 7919 * rank + 1)
        # draw_batch takes the stratified jitter and importance uniforms from
        # the device's default generator (so the explicit, autograd and
        # reference-path modes see the same numbers): after the identical
        # init, every rank but 0 re-seeds it so DP ranks do not share them
        if rank > 0 and self.device.type == "cuda":
            torch.cuda.manual_seed(1000003 * seed + 7919 * rank + 2)
        self.cpu_gen = torch.Generator().manual_seed(seed * 31 + rank)
        H, W = data.H, data.W
        jj, ii = torch.meshgrid(torch.arange(H, device=self.device), torch.arange(W, device=self.device),
                                indexing="ij")
        self.coords_full = torch.stack([jj, ii], -1).reshape(-1, 2)
        dH, dW = int(H // 2 * args.precrop_frac), int(W // 2 * args.precrop_frac)
        cj, ci = torch.meshgrid(torch.arange(H // 2 - dH, H // 2 + dH, device=self.device),
                                torch.arange(W // 2 - dW, W // 2 + dW, device=self.device), indexing="ij")
        self.coords_crop = torch.stack([cj, ci], -1).reshape(-1, 2)
        self.crop = (H // 2 - dH, W // 2 - dW, 2 * dH, 2 * dW)
        self._grads = None
        # use_batching (no_batching False, e.g. configs/scannet_scene0000.txt:6):
        # the global shuffled ray pool of run_nerf.py:505-521 over the training
        # images, consumed N_rand positions per step and reshuffled per epoch
        # (hn_sample_pool: the shuffle is a keyed bijection, nothing materialised)
        self.use_batching = not getattr(args, "no_batching", True)
        self.i_batch, self.epoch = 0, 0
        if self.use_batching and mode == "eager":
            raise NotImplementedError("Trainer(mode='eager') draws per-image batches only (no_batching)")
        if self.use_batching:
            self._pool_ids = torch.as_tensor(data.i_train).to(device=self.device, dtype=torch.int32)
            self._pool_n = int(self._pool_ids.numel()) * H * W
        # the render backward's sticky fault word (hn_device_faults) is read
        # every this many steps: one blocking copy, so a failed internal wait
        # can never leave silently wrong gradients behind for long
        self.fault_check_every = 100
        # explicit mode, one GPU: fuse the table's RAdam step into the binned
        # backward's owner pass when the step has no TV term
        self.fuse_table_step = True
        # ... and skip the coarse levels' unreachable row pairs there
        # (live_pair_mask: bitwise the same step, fewer optimizer-state bytes)
        self.skip_dead_rows = True
        # explicit mode, world > 1: reduce-scatter / sharded RAdam / all-gather
        # of the table (ShardedTableStep) instead of all-reduce + full RAdam
        self.dp_sharded = True
        # ... in this many bin-aligned segments, each exchanged as soon as the
        # backward's owner pass has formed it (1: one exchange after the whole
        # backward).  1 by default: the segmented form's RCCL overlap (segment
        # k's reduce-scatter on RCCL's stream while the owner pass forms
        # segment k+1) has run only on gloo so far; the GPU DP
        # tests and bench.py --dp-chunks select it
        self.dp_chunks = 1
        self._xchg = None
        self._owner_st = None
        # self-driving loops (bench.py): the next step's batch -- device ray
        # sampler and the jitter / importance uniforms -- is drawn on a side
        # stream as soon as this step's forward is enqueued, so it runs beside
        # the backward instead of ahead of the next forward.  The draws and
        # their order are those of draw_batch at the start of the next step
        # (bitwise the same trajectory).  Opt-in: a caller that draws its own
        # batches (draw_batch + step(i, batch)) must leave it off, or the
        # prefetch consumes the next step's random numbers first.  Measured
        # slower at config 2 (r05k: 0.996 vs 0.982 ms per step: the
        # cross-stream waits cost more than the launches they move), so off
        # unless asked for (bench.py --prefetch).
        self.prefetch = False
        # one GPU, fused table step: the MLP tensors' RAdam steps run in the
        # backward's slab reduction too (no hn_radam_step launch)
        self.fuse_mlp_step = True
        # ... and then repacks them for the next forward, which reuses the
        # render workspace (kept across steps) instead of packing again
        self._rws = None         # the render workspace
        self._rws0 = None        # an empty rank's TV-only workspace (before any render)
        self._pk = None          # (workspace, weight versions) its packed copies belong to
        self._pf = None          # (step, batch, ready event) drawn ahead
        # explicit mode: the loss value and its gradients formed by the render
        # backward's composite pre-pass (ABI 13) instead of an hn_loss_fwd_bwd
        # launch
        self.fuse_loss = True
        self._side = None
        # the backward skips the samples whose d raw is exactly zero (relu(sigma)
        # = 0: no gradient at all; hn_render_cfg.dense_bwd, ABI 14): True
        # computes them too (A/B: bench.py --dense-bwd; same results up to the
        # sign of zero)
        self.dense_bwd = False

    def _train_image(self):
        """np.random.choice(i_train) (run_nerf.py:578) from the host generator."""
        d = self.data
        return int(d.i_train[int(torch.randint(len(d.i_train), (1,), generator=self.cpu_gen))])

    def _pool_draw(self):
        """The next use_batching batch (run_nerf.py:544-555): pool positions
        [i_batch, i_batch + N_rand) of this epoch's shuffle -- with world > 1
        the global batch of world * N_rand positions, rank r taking its share --
        then i_batch advances and wraps (new epoch, new shuffle key) once the
        pool is used up.  The last batch of an epoch is short, as the
        reference's slice."""
        a, d = self.args, self.data
        gB = a.N_rand * self.world
        rem = min(gB, self._pool_n - self.i_batch)
        lo = self.i_batch + rem * self.rank // self.world
        hi = self.i_batch + rem * (self.rank + 1) // self.world
        rays, target = HF.sample_pool(d.images, d.poses, self._pool_ids, d.K, 2., 6.,
                                      _step_seed(self.seed, 0, -1 - self.epoch), lo, hi - lo)
        self.i_batch += gB
        if self.i_batch >= self._pool_n:
            self.epoch += 1
            self.i_batch = 0
        return rays, target

    def _draw_rays(self, i: int, uniforms=None):
        """The step's rays and targets: the shuffled pool (use_batching) or
        N_rand pixels of one training image (device sampler, centre crop
        before precrop_iters).  uniforms = per-ray counts of torch.rand draws
        on the default generator to make as well ([B, n] each, bitwise
        torch's: functional.torch_uniform, inside the sampler's launch),
        returned after rays and target."""
        if self.use_batching:
            rays, target = self._pool_draw()
            if uniforms:
                B = rays.shape[0]
                return (rays, target, *HF.torch_uniform([(B, n) for n in uniforms], self.device))
            return rays, target
        a, d = self.args, self.data
        img_i = self._train_image()
        crop = self.crop if i < a.precrop_iters else (0, 0, d.H, d.W)
        return HF.sample_rays(d.images[img_i], d.poses[img_i], a.N_rand, d.K, 2., 6., crop,
                              _step_seed(self.seed, self.rank, i), order=self.ray_order,
                              uniforms=[(a.N_rand, n) for n in uniforms] if uniforms else None)

    def sample_rays(self, i: int):
        """run_nerf.py:576-605 on the device: one image, N_rand pixels."""
        d, a = self.data, self.args
        img_i = self._train_image()
        coords = self.coords_crop if i < a.precrop_iters else self.coords_full
        sel = torch.randperm(coords.shape[0], device=self.device, generator=self.gen)[: a.N_rand]
        c = coords[sel]
        j, ii = c[:, 0].float(), c[:, 1].float()
        K = d.K
        dirs = torch.stack([(ii - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -torch.ones_like(ii)], -1)
        c2w = d.poses[img_i, :3, :4]
        rays_d = torch.sum(dirs[..., None, :] * c2w[:3, :3], -1)      # ray_util.py:77
        rays_o = c2w[:3, -1].expand(rays_d.shape)
        target = d.images[img_i][c[:, 0], c[:, 1]]
        return torch.stack([rays_o, rays_d], 0), target

    def loss_fn(self, rgb, extras, target, i):
        a = self.args
        mse = img2mse(rgb, target)
        mse0 = img2mse(extras["rgb0"], target) if "rgb0" in extras else None
        sp = extras["sparsity_loss"].sum() + extras["sparsity_loss0"].sum()
        tv = None
        if a.tv_loss_weight > 0 and self.rank == 0 and i <= a.tv_until:
            tv = tv_loss_levels(self.embed_fn, generator=self.cpu_gen).sum()
        loss = dp_loss(mse, mse0, sp, self.world, a.sparse_loss_weight, tv, a.tv_loss_weight)
        return loss, mse

    def _live_rows(self):
        if not hasattr(self, "_live"):
            e = self.embed_fn
            lv = live_rows(e.resolutions, e.log2_hashmap_size)
            self._live = None if lv is None else (lv[0], lv[1].to(self.device))
        return self._live

    def _live_mask(self):
        """train.live_pair_mask on the device (built once), or None when
        Trainer.skip_dead_rows is off."""
        if not self.skip_dead_rows:
            return None
        if not hasattr(self, "_livem"):
            e = self.embed_fn
            lm = live_pair_mask(e.resolutions, e.log2_hashmap_size)
            self._livem = None if lm is None else (lm[0], lm[1].to(self.device))
        return self._livem

    def finish_table_grad(self):
        """Run the backward's deferred owner pass over the bins it has not
        reduced yet (the segmented DP exchange defers it; see step()), so
        that table.grad holds the whole table gradient."""
        st, self._owner_st = self._owner_st, None
        if st is not None:
            HF.render_bwd_owner(st, 0, HF.render_bins(self._cfg, st.rays.shape[0])[0])

    def allreduce_grads(self):
        self.finish_table_grad()
        if self.world > 1:
            allreduce_grads(self.embed_fn.table, self.grad_vars, live=self._live_rows())

    def sync_optimizer_state(self):
        """With the sharded table step (world > 1): gather the table's RAdam
        moments from the ranks' shards into optimizer.state (for a checkpoint,
        run_nerf.py:663-680).  Collective: call on every rank."""
        if self._xchg is not None and self.embed_fn.table in self.optimizer.state:
            m, v = self._xchg.gather_state()
            st = self.optimizer.state[self.embed_fn.table]
            st["exp_avg"].copy_(m)
            st["exp_avg_sq"].copy_(v)

    def _fused_setup(self):
        from .render import _fusable, _linspace_cached
        kw = self.kw_train
        nq, nf, nfine = kw["network_query_fn"], kw["network_fn"], kw["network_fine"]
        if not _fusable(torch.empty(1, 11), nf, nq, kw["N_samples"], kw["N_importance"], nfine):
            raise NotImplementedError("Trainer(mode='explicit') needs the HashNeRF configuration")
        a = self.args
        self._cfg = HF.make_render_cfg(self.embed_fn.grid(), bool(kw.get("white_bkgd", False)),
                                       bool(kw.get("lindisp", False)), kw.get("perturb", 0.) > 0.,
                                       dense_bwd=self.dense_bwd)
        self._t_vals = _linspace_cached(kw["N_samples"], self.device)
        self._ws = nf.weights() + nfine.weights()
        table = self.embed_fn.table
        # world > 1 (explicit mode): the table's exchange + RAdam step sharded over
        # the ranks (ShardedTableStep); the backward writes into its buffer
        if self._xchg is not None and self._xchg.stale:
            # a rebuilt exchange seeds its shards from optimizer.state, which is
            # out of date while the previous exchange's moments are newer
            raise RuntimeError("Trainer: the sharded table moments are newer than optimizer.state; "
                               "call sync_optimizer_state() on every rank before rebuilding the step")
        self._xchg = None
        if self.world > 1 and self.dp_sharded:
            # the moments continue from the optimizer's (a resumed run's
            # checkpoint, or an earlier setup's gathered state)
            nb, shift = HF.render_bins(self._cfg, a.N_rand)
            self._xchg = ShardedTableStep(table, self._live_rows(), self.rank, self.world,
                                          state=self.optimizer.state.get(table),
                                          bins=(nb, shift) if nb else None, n_chunks=self.dp_chunks)
            self.optimizer.sharded_state = self._xchg
            self._gtable = self._xchg.grad_view()
        else:
            self._gtable = torch.zeros_like(table)
        self._pk = None          # (re)setup: the weights may have been replaced
        self._binned = HF.L.lib().hn_render_scatter_mode(self._cfg, a.N_rand) == 2
        # the ten MLP gradients: views of ONE flat buffer (the DP exchange
        # all-reduces it in place, no concatenation or copy-back)
        self._gws = HF.zeros_like_all(self._ws)
        self._gflat = self._gws[0]._base
        self._one = torch.ones((), device=self.device)
        self._gtv = None
        self._grads = True

    def draw_batch(self, i: Optional[int] = None):
        """The random inputs of step i (default: the next step, global_step + 1), drawn the way run_nerf.py:576-605 and
        render_rays draw them: the image (host generator), N_rand pixels
        without replacement (device sampler, centre crop before
        precrop_iters), the stratified jitter t_rand and importance uniforms u
        (device RNG), and the TV cubes + min vertices (rank 0, i <= tv_until).
        Returns a dict rays [B, 11], target [B, 3], t_rand, u, tv (or None)."""
        a, d, kw = self.args, self.data, self.kw_train
        i = self.global_step + 1 if i is None else i
        perturb = kw.get("perturb", 0.) > 0.
        # two draws in render_rays' order (run_nerf_helpers.py:528, then :276 via :548): the
        # autograd and reference-path modes draw them the same way, so all
        # modes see the same numbers for the same device RNG state.  On the
        # device they are torch.rand restated bit for bit and made in the
        # sampler's first launch (one launch instead of three)
        if perturb and self.device.type == "cuda":
            rays, target, t_rand, u = self._draw_rays(i, uniforms=(kw["N_samples"], kw["N_importance"]))
        else:
            rays, target = self._draw_rays(i)
            B = rays.shape[0]
            t_rand = torch.rand((B, kw["N_samples"]), device=self.device) if perturb else None
            u = (torch.rand((B, kw["N_importance"]), device=self.device) if perturb else
                 torch.linspace(0., 1., kw["N_importance"], device=self.device).expand(B, kw["N_importance"]))
        tv = None
        if a.tv_loss_weight > 0 and self.rank == 0 and i <= a.tv_until:
            tv = draw_tv_cubes(self.embed_fn.n_levels, self.embed_fn.base_resolution,
                               self.embed_fn.finest_resolution, self.cpu_gen)
        return dict(rays=rays, target=target, t_rand=t_rand, u=u, tv=tv)

    def _prefetch(self, i: int):
        """draw_batch(i) on the side stream, after the work enqueued so far on
        the current stream (the sampler's workspace is shared)."""
        cur = torch.cuda.current_stream(self.device)
        if self._side is None:
            self._side = torch.cuda.Stream(self.device)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._side.wait_event(ev)
        with torch.cuda.stream(self._side):
            b = self.draw_batch(i)
            done = torch.cuda.Event()
            done.record(self._side)
        self._pf = (i, b, done)

    def _take_prefetched(self, i: int):
        """The batch drawn ahead for step i (None if there is none): the
        current stream waits for it and takes its tensors over."""
        pf, self._pf = self._pf, None
        if pf is None or pf[0] != i:
            return None
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(pf[2])
        for k in ("rays", "target", "t_rand", "u"):
            if torch.is_tensor(pf[1][k]):
                pf[1][k].record_stream(cur)
        return pf[1]

    def _fused_forward_backward(self, i: int, batch=None):
        a = self.args
        if self._grads is None:
            self._fused_setup()
        pf = self.prefetch and batch is None and self.device.type == "cuda"
        if pf:
            batch = self._take_prefetched(i)
        if batch is None:
            batch = self.draw_batch(i)
        rays, target, t_rand, u = batch["rays"], batch["target"], batch["t_rand"], batch["u"]
        table = self.embed_fn.table
        if rays.shape[0] == 0:
            return self._empty_rank_grads(batch)
        tv = mv = cubes = None
        if batch["tv"] is not None:
            cubes, mv0 = batch["tv"]
            tv, mv = HF.tv_fwd(table, mv0, cubes, self.embed_fn.log2_hashmap_size)
        consts = (self.world, a.sparse_loss_weight, a.tv_loss_weight)
        nb = HF.L.lib().hn_render_workspace_bytes(self._cfg, rays.shape[0])
        if self._rws is None or self._rws.numel() < nb:
            self._rws, self._pk = torch.empty(nb, dtype=torch.uint8, device=self.device), None
        # the colour net of tiles without any density is skipped (the trainer never
        # returns raw rgb; with dense_bwd everything is computed, for the A/B)
        out, st = HF.render_fwd(self._cfg, rays, self._t_vals, t_rand, u, None, None, table, self._ws, True,
                                wsb=self._rws, weights_packed=self._pk is not None and self._pk == self._pack_key(),
                                skip_dead_color=not self.dense_bwd)
        self._pk = None
        if pf:
            self._prefetch(i + 1)
        loss = None
        if self.fuse_loss:
            # the loss formed by the backward's composite pre-pass (ABI 13):
            # its rgb / entropy gradients computed where they are used, its
            # value by one workgroup -- no hn_loss_fwd_bwd launch
            lo = torch.empty(4, dtype=torch.float32, device=self.device)
            loss = dict(target=target, rgb=out["rgb"], rgb0=out["rgb0"], sparsity=out["sparsity"],
                        sparsity0=out["sparsity0"], tv=tv, world=self.world, sparse_w=a.sparse_loss_weight,
                        tv_w=a.tv_loss_weight, out=lo)
            grads = {}
            # d loss / d tv_l = g * tv_w (g = 1, hn_loss_bwd's): a constant vector
            g_tv = None
            if tv is not None:
                if self._gtv is None or self._gtv.shape != tv.shape:
                    self._gtv = torch.full_like(tv, a.tv_loss_weight)
                g_tv = self._gtv
        else:
            # loss value and its input gradients in one launch (the gradients do
            # not depend on the value)
            lo, (g_rgb, g_rgb0, g_sp, g_sp0, g_tv) = HF.loss_fwd_bwd(
                out["rgb"], out["rgb0"], target, out["sparsity"], out["sparsity0"], tv, *consts, self._one)
            grads = dict(g_rgb=g_rgb, g_sparsity=g_sp, g_rgb0=g_rgb0, g_sparsity0=g_sp0)
        # the ten MLP grads (one flat buffer) are written, not accumulated:
        # no zero fill
        # the TV term's table gradient joins the render backward (records of
        # the binned owner pass, or added to the stored gradient)
        tvb = None if tv is None else (mv, cubes, g_tv)
        if self.fuse_table_step and self.world == 1 and self._binned:
            # one GPU: the table gradient (render + TV) is complete where the
            # binned owner pass forms it, so the table's RAdam step runs there
            # (run_nerf.py:642 for the embedding group) and the gradient is
            # never stored; optimizer.step() then updates the MLP groups only
            # the MLP groups' steps likewise, where the slab reduction forms
            # their gradients (optimizer.step() then has nothing left)
            mstep = [self.optimizer.take_step(p) for p in self._ws] if self.fuse_mlp_step else None
            HF.render_bwd(st, grads, None, self._gws, table_step=self.optimizer.take_step(table),
                          overwrite_mlp=True, tv=tvb, table_live=self._live_mask(), loss=loss, mlp_step=mstep,
                          repack=mstep is not None)
            if mstep is not None:
                self._pk = self._pack_key()   # the workspace holds the stepped weights' copies
            table.grad = None
        else:
            # the render backward writes every table-gradient entry (overwrite:
            # no zero fill of the 64 MiB buffer), TV included; with a segmented
            # DP exchange its owner pass runs per segment inside the exchange
            defer = self._xchg is not None and self._xchg.seg_bins is not None
            HF.render_bwd(st, grads, self._gtable, self._gws, overwrite=True, overwrite_mlp=True, tv=tvb,
                          owner_defer=defer, loss=loss)
            self._owner_st = st if defer else None
            table.grad = self._gtable
        for p, g in zip(self._ws, self._gws):
            p.grad = g
        return lo[0], lo[1]

    def _pack_key(self):
        """What the workspace's packed weights must match: the buffer and
        every weight's version counter (an in-place change of a weight, e.g.
        a checkpoint load, bumps it; the HIP optimizer's writes do not).  A
        write the version counter does not see (``p.data = ...``,
        ``p.data.copy_``, a raw-pointer write) must call invalidate_packed()."""
        return (self._rws.data_ptr(), tuple(p._version for p in self._ws))

    def invalidate_packed(self):
        """Forget the render workspace's packed MLP copies: the next forward
        packs the weights again.  Call after changing a NeRFSmall weight in a
        way its version counter does not record."""
        self._pk = None

    def _empty_rank_grads(self, batch):
        """A rank that drew no rays this step (world > 1, use_batching: the
        short last batch of an epoch holds fewer positions than ranks,
        run_nerf.py:551-555) still joins the exchange: its gradient is the TV
        term's alone (rank 0) or zero, its MSE / entropy terms empty."""
        table = self.embed_fn.table
        if self.world == 1:
            raise RuntimeError("Trainer: an empty batch on a single rank")
        self._owner_st = None
        self._gtable.zero_()
        lo = torch.zeros(2, device=self.device)
        if batch["tv"] is not None:
            cubes, mv0 = batch["tv"]
            tv, mv = HF.tv_fwd(table, mv0, cubes, self.embed_fn.log2_hashmap_size)
            w = self.args.tv_loss_weight
            lo[0] = w * tv.sum()
            g_tv = torch.full_like(tv, w)
            if self._binned:
                # the TV term alone through the binned scatter's records and exact
                # owner pass (bitwise reproducible, as a rendering rank's TV term)
                self._rws0 = HF.tv_bwd_records(self._cfg, table, mv, cubes, g_tv, self._gtable,
                                               wsb=self._rws if self._rws is not None else self._rws0)
            else:
                HF.tv_bwd(table, mv, cubes, self.embed_fn.log2_hashmap_size, g_tv, self._gtable)
        table.grad = self._gtable
        self._gflat.zero_()
        for p, g in zip(self._ws, self._gws):
            p.grad = g
        return lo[0], lo[1]

    def step(self, i: Optional[int] = None, batch=None):
        """One iteration; ``batch`` (explicit mode) = draw_batch(i) drawn by
        the caller, e.g. to feed the same inputs to a reference path.

        ``i`` is the reference loop's index (run_nerf.py:538-541: ``start + 1``
        onwards, so 1 on a fresh run, global_step + 1 after a resume); it
        defaults to exactly that.  The windows follow the reference: the
        centre crop while i < precrop_iters (steps 1..499), TV while
        i <= tv_until (1001: the weight is zeroed after the loss of step
        i > 1000 is formed, run_nerf.py:636-638), and the lr set after the
        step from the pre-increment global_step (:647-651)."""
        a = self.args
        i = self.global_step + 1 if i is None else i
        if batch is not None and self.mode != "explicit":
            raise ValueError("Trainer.step(batch=...) needs mode='explicit'")
        if self.mode == "explicit":
            loss, mse = self._fused_forward_backward(i, batch)
        else:
            self.optimizer.zero_grad(set_to_none=True)
            if self.mode == "autograd":
                rays, target = self._draw_rays(i)
                rgb, depth, acc, extras = render_ray_batch(rays, (rays.shape[0],), chunk=a.chunk, retraw=True,
                                                           **self.kw_train)
                tv = None
                if a.tv_loss_weight > 0 and self.rank == 0 and i <= a.tv_until:
                    tv = tv_loss_levels(self.embed_fn, generator=self.cpu_gen)
                loss, mse, _ = HF.train_loss(rgb, extras.get("rgb0"), target, extras["sparsity_loss"],
                                             extras.get("sparsity_loss0"), tv, self.world,
                                             a.sparse_loss_weight, a.tv_loss_weight)
            else:
                batch_rays, target = self.sample_rays(i)
                rgb, depth, acc, extras = render(self.data.H, self.data.W, self.data.K, chunk=a.chunk,
                                                 rays=batch_rays, retraw=True, near=2., far=6.,
                                                 **self.kw_train)
                loss, mse = self.loss_fn(rgb, extras, target, i)
            loss.backward()
        if self._xchg is not None and self.mode == "explicit":
            # the table: RAdam state advanced here (take_step), its exchange and
            # update sharded; the ten MLP gradients (views of one flat buffer)
            # all-reduced in place as one bucket beside the table's
            # reduce-scatter, and their RAdam steps taken in the shard's
            # hn_radam_step launch (one launch for all eleven tensors)
            table = self.embed_fn.table
            _, _, _, coeffs = self.optimizer.take_step(table)
            t_mlp = HF.TIMER.begin("xchg_mlp_allreduce")
            work = dist.all_reduce(self._gflat, async_op=True)
            mst = [self.optimizer.take_step(p) for p in self._ws]
            extra = [(p, g, m, v, c) for (p, m, v, c), g in zip(mst, self._gws)]

            def wait_mlp():
                work.wait()
                HF.TIMER.end("xchg_mlp_allreduce", t_mlp)

            st, self._owner_st = self._owner_st, None
            produce = None
            if st is not None:
                sb = self._xchg.seg_bins
                produce = lambda k: HF.render_bwd_owner(st, *sb[k])
            self._xchg.step(coeffs, produce=produce, extra=extra, pre_step=wait_mlp)
            table.grad = None
        else:
            self.allreduce_grads()
        self.optimizer.step()
        decay_steps = a.lrate_decay * 1000
        new_lr = a.lrate * (0.1 ** (self.global_step / decay_steps))
        for g in self.optimizer.param_groups:
            g["lr"] = new_lr
        self.global_step += 1
        if self.fault_check_every and self.global_step % self.fault_check_every == 0 and \
                self.device.type == "cuda":
            HF.L.check_device_faults()
        return loss, mse
