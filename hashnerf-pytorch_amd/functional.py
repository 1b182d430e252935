"""torch.autograd wrappers around the HIP C ABI (one Function per entry point).

PyTorch supplies device memory, the current HIP stream and autograd
plumbing; every byte of arithmetic on the hot path runs in the gfx950 HIP
library.  Gradient buffers are zero-initialised here and accumulated (+=) by
the kernels, mirroring the C ABI contract.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import torch

from . import _lib as L


class KernelTimer:
    """Optional HIP-event timing of the fused launches (bench.py): events are
    recorded on the same stream the kernels are enqueued on.  ``names``
    limits the timed launches (None: all); each recorded event idles the
    device for ~5 us, so bench times only what its line reports from the
    timed steps.  ``every`` = k times only every k-th call of a name (the
    sampled launches' mean; the others carry no events)."""

    def __init__(self):
        self.events = {}
        self.enabled = False
        self.names = None
        self.every = 1
        self.calls = {}

    def begin(self, name):
        if not self.enabled or (self.names is not None and name not in self.names):
            return None
        c = self.calls.get(name, 0)
        self.calls[name] = c + 1
        if c % max(self.every, 1):
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def end(self, name, start):
        if start is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.events.setdefault(name, []).append((start, e))

    def mean_ms(self, name):
        ev = self.events.get(name, [])
        return sum(s.elapsed_time(e) for s, e in ev) / max(len(ev), 1)

    def reset(self):
        self.events = {}
        self.calls = {}


TIMER = KernelTimer()

# Debug hook for parity tests: when True, the fused forward keeps its saved
# z-values / raw outputs of the last call in LAST (no effect on results).
DEBUG_KEEP = False
LAST = {}
# When True, every render backward is followed by a check of the device fault
# word (hn_device_faults: a blocking read).  The tests turn it on; trainers
# check every Trainer.fault_check_every steps instead.
CHECK_FAULTS = os.environ.get("HN_CHECK_FAULTS", "0") == "1"


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def _no_input_grad(name, *ts):
    for t in ts:
        if t is not None and t.requires_grad and torch.is_grad_enabled():
            raise NotImplementedError(
                f"hashnerf_amd.{name}: gradients w.r.t. sample positions/directions are not "
                "implemented (the reference path never needs them: rays carry no grad)")


# --------------------------------------------------------------------------
# hash encoding (embedding/hash_encoding.py:84-110)
# --------------------------------------------------------------------------
class HashEncodeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, table: torch.Tensor, grid: L.HnGrid):
        L.require_device(x, table)
        x = x.contiguous()
        n = x.shape[0]
        n_feat = grid.n_levels * grid.n_features
        feat = torch.empty((n, n_feat), dtype=torch.float32, device=x.device)
        keep = torch.empty((n,), dtype=torch.uint8, device=x.device)
        L.check(L.lib().hn_encode_fwd(grid, L.ptr(x), n, L.ptr(table.contiguous()), L.ptr(feat),
                                      L.ptr(keep), L.stream(x.device)), "encode_fwd")
        ctx.save_for_backward(x)
        ctx.grid = grid
        ctx.table_shape = table.shape
        ctx.mark_non_differentiable(keep)
        return feat, keep.bool()

    @staticmethod
    def backward(ctx, dfeat, _dkeep):
        (x,) = ctx.saved_tensors
        dtable = torch.zeros(ctx.table_shape, dtype=torch.float32, device=x.device)
        if dfeat is not None:
            dfeat = dfeat.contiguous()
            L.check(L.lib().hn_encode_bwd(ctx.grid, L.ptr(x), x.shape[0], L.ptr(dfeat), L.ptr(dtable),
                                          L.stream(x.device)), "encode_bwd")
        return None, dtable, None


def hash_encode(x, table, grid):
    _no_input_grad("hash_encode", x)
    return HashEncodeFn.apply(x, table, grid)


def sh_encode(dirs: torch.Tensor) -> torch.Tensor:
    """SHEncoder.forward, degree 4 (embedding/spherical_harmonic.py:65-103)."""
    _no_input_grad("sh_encode", dirs)
    L.require_device(dirs)
    d = dirs.reshape(-1, 3).contiguous()
    out = torch.empty((d.shape[0], 16), dtype=torch.float32, device=d.device)
    L.check(L.lib().hn_sh_fwd(L.ptr(d), d.shape[0], L.ptr(out), L.stream(d.device)), "sh_fwd")
    return out.reshape(*dirs.shape[:-1], 16)


# --------------------------------------------------------------------------
# NeRFSmall (models.py:151-174)
# --------------------------------------------------------------------------
class NeRFSmallFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w0, w1, w2, w3, w4):
        L.require_device(x, w0, w1, w2, w3, w4)
        x = x.contiguous()
        ws = [w.contiguous() for w in (w0, w1, w2, w3, w4)]
        n = x.shape[0]
        out = torch.empty((n, 4), dtype=torch.float32, device=x.device)
        nbytes = L.lib().hn_mlp_workspace_bytes()
        ws_buf = _ws(nbytes, x.device)
        L.check(L.lib().hn_mlp_fwd(L.make_mlp(ws), L.ptr(x), n, L.ptr(out), L.ptr(ws_buf), nbytes,
                                   L.stream(x.device)), "mlp_fwd")
        ctx.save_for_backward(x, *ws)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, *ws = ctx.saved_tensors
        dout = dout.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dws = [torch.zeros_like(w) for w in ws]
        nbytes = L.lib().hn_mlp_workspace_bytes()
        ws_buf = _ws(nbytes, x.device)
        L.check(L.lib().hn_mlp_bwd(L.make_mlp(ws), L.ptr(x), L.ptr(dout), x.shape[0], L.ptr(dx),
                                   L.make_mlp_grad(dws), L.ptr(ws_buf), nbytes, L.stream(x.device)),
                "mlp_bwd")
        return (dx, *dws)


# --------------------------------------------------------------------------
# raw2outputs (run_nerf_helpers.py:577-628) and sample_pdf (:264-307)
# --------------------------------------------------------------------------
class CompositeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, z, rays_d, noise, white: bool):
        L.require_device(raw, z, rays_d, noise)
        raw, z, rays_d, noise = (L.contig(t) for t in (raw, z, rays_d, noise))
        B, S = z.shape
        dev = raw.device
        rgb = torch.empty((B, 3), device=dev)
        disp, acc, depth, ent = (torch.empty((B,), device=dev) for _ in range(4))
        weights = torch.empty((B, S), device=dev)
        L.check(L.lib().hn_composite_fwd(L.ptr(raw), L.ptr(z), L.ptr(rays_d), L.ptr(noise), B, S,
                                         int(white), L.ptr(rgb), L.ptr(disp), L.ptr(acc),
                                         L.ptr(weights), L.ptr(depth), L.ptr(ent), L.stream(dev)),
                "composite_fwd")
        ctx.save_for_backward(raw, z, rays_d, noise, depth)
        ctx.set_materialize_grads(False)   # unused outputs => NULL, not zeros (0*inf)
        ctx.white = white
        return rgb, disp, acc, weights, depth, ent

    @staticmethod
    def backward(ctx, g_rgb, g_disp, g_acc, g_weights, g_depth, g_ent):
        raw, z, rays_d, noise, depth = ctx.saved_tensors
        if g_disp is not None:
            # disp = 1 / max(1e-10, depth): fold into the depth gradient
            gd = torch.where(depth > 1e-10, -g_disp / (depth * depth), torch.zeros_like(depth))
            g_depth = gd if g_depth is None else g_depth + gd
        B, S = z.shape
        d_raw = torch.empty_like(raw)
        L.check(L.lib().hn_composite_bwd(L.ptr(raw), L.ptr(z), L.ptr(rays_d), L.ptr(noise), B, S,
                                         int(ctx.white), L.ptr(L.contig(g_rgb)), L.ptr(L.contig(g_acc)),
                                         L.ptr(L.contig(g_depth)), L.ptr(L.contig(g_ent)),
                                         L.ptr(L.contig(g_weights)), L.ptr(d_raw), L.stream(raw.device)),
                "composite_bwd")
        return d_raw, None, None, None, None


def sample_pdf(bins: torch.Tensor, weights: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    L.require_device(bins, weights, u)
    bins, weights, u = bins.contiguous(), weights.detach().contiguous(), u.contiguous()
    B, nb = bins.shape
    ns = u.shape[-1]
    out = torch.empty((B, ns), device=bins.device)
    L.check(L.lib().hn_sample_pdf(L.ptr(bins), L.ptr(weights), L.ptr(u), B, nb, ns, L.ptr(out),
                                  L.stream(bins.device)), "sample_pdf")
    return out


# --------------------------------------------------------------------------
# fused render_rays (run_nerf_helpers.py:464-574)
# --------------------------------------------------------------------------
class RenderState:
    """Buffers one fused forward leaves for its backward (z values, raw
    outputs, coarse origin of each fine sample, hash features, the workspace
    holding the packed weights)."""
    __slots__ = ("cfg", "rays", "noise_c", "noise_f", "table", "ws", "z_c", "z_f", "raw_c", "raw_f",
                 "fine_src", "feat", "wsb", "nbytes", "bwd_args", "skip_dead")


def render_fwd(cfg, rays, t_vals, t_rand, u, noise_c, noise_f, table, ws, keep_feat, wsb=None,
               weights_packed=False, skip_dead_color=False):
    """hn_render_fwd (run_nerf_helpers.py:464-574, forward).  Returns the
    output dict and a RenderState (None when keep_feat is False).  wsb: the
    caller's workspace (uint8, >= workspace_bytes; default a fresh one);
    weights_packed: it already holds ws's packed copies (render_bwd with
    repack=True since the last change of ws).  skip_dead_color (ABI 14, the
    trainer): tiles whose 32 raw sigmas are all <= 0 skip the colour net --
    rgb, depth, acc, the entropies and every gradient unchanged, the raw rgb
    of those samples written as 0 -- and such fine tiles' features are not
    stored: the backward must then run with cfg.dense_bwd = 0 (render_bwd
    refuses dense_bwd = 1 on such a state)."""
    L.require_device(rays, t_vals, t_rand, u, noise_c, noise_f, table, *ws)
    rays, t_vals, t_rand, u, noise_c, noise_f = (L.contig(t) for t in (rays, t_vals, t_rand, u,
                                                                      noise_c, noise_f))
    ws = [w.contiguous() for w in ws]
    B = rays.shape[0]
    dev = rays.device
    e = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)
    out = dict(rgb=e(B, 3), depth=e(B), acc=e(B), sparsity=e(B), rgb0=e(B, 3), depth0=e(B),
               acc0=e(B), sparsity0=e(B), z_std=e(B), z_coarse=e(B, 64), z_fine=e(B, 192),
               raw_c=e(B, 64, 4), raw_f=e(B, 192, 4))
    a = L.HnRenderFwdArgs()
    a.n_rays = B
    for k, t in (("rays", rays), ("t_vals", t_vals), ("t_rand", t_rand), ("u", u),
                 ("noise_c", noise_c), ("noise_f", noise_f), ("table", table)):
        setattr(a, k, None if t is None else t.data_ptr())
    a.coarse = L.make_mlp(ws[:5])
    a.fine = L.make_mlp(ws[5:])
    for k, t in out.items():
        setattr(a, k, t.data_ptr())
    fine_src = torch.empty((B, 192), dtype=torch.uint8, device=dev)
    a.fine_src = fine_src.data_ptr()
    # hash features of every evaluated point, kept for the backward only
    # when a gradient will be taken (inference skips the 32 KB/ray store)
    feat = torch.empty((B, L.RENDER_FEAT_PER_RAY) if keep_feat else (0,), dtype=torch.float32,
                       device=dev)
    a.feat = feat.data_ptr() if keep_feat else None
    nbytes = L.lib().hn_render_workspace_bytes(cfg, B)
    if wsb is None:
        wsb = _ws(nbytes, dev)
    elif wsb.numel() * wsb.element_size() < nbytes or not wsb.is_contiguous() or wsb.device != dev:
        raise ValueError(f"hashnerf_amd.render_fwd: wsb must be a contiguous buffer of >= {nbytes} bytes on {dev}")
    else:
        nbytes = wsb.numel() * wsb.element_size()
    a.weights_packed = 1 if weights_packed else 0
    a.skip_dead_color = 1 if skip_dead_color else 0
    t0 = TIMER.begin("render_fwd")
    L.check(L.lib().hn_render_fwd(cfg, a, L.ptr(wsb), nbytes, L.stream(dev)), "render_fwd")
    TIMER.end("render_fwd", t0)
    if DEBUG_KEEP:
        LAST.update({k: out[k] for k in ("z_coarse", "z_fine", "raw_c", "raw_f")})
    st = None
    if keep_feat:
        st = RenderState()
        st.cfg, st.rays, st.noise_c, st.noise_f, st.table, st.ws = cfg, rays, noise_c, noise_f, table, ws
        st.z_c, st.z_f, st.raw_c, st.raw_f = out["z_coarse"], out["z_fine"], out["raw_c"], out["raw_f"]
        st.fine_src, st.feat, st.wsb, st.nbytes = fine_src, feat, wsb, nbytes
        st.bwd_args = None
        st.skip_dead = bool(skip_dead_color)
    return out, st


def render_bwd(st: RenderState, grads: dict, d_table, dws, overwrite: bool = False, table_step=None,
               overwrite_mlp: bool = False, tv=None, table_live=None, owner_defer: bool = False, loss=None,
               mlp_step=None, repack: bool = False):
    """hn_render_bwd: accumulates (+=) d loss / d table into d_table (or
    writes it, overwrite=True: d_table need not be zeroed) and the ten
    NeRFSmall weight gradients into dws (coarse 5, fine 5, +=; written with
    overwrite_mlp=True, dws need not be zeroed).  grads: any
    of g_rgb, g_depth, g_acc, g_sparsity, g_rgb0, g_depth0, g_acc0,
    g_sparsity0, g_raw_f (missing = 0).  table_step = (table, exp_avg,
    exp_avg_sq, coeffs) from RAdam.take_step: the binned owner pass applies
    that RAdam step to the table with this gradient (d_table may be None).
    tv = (min_vertex [L, 3] device int32, cubes, g_tv [L]) from tv_fwd and the
    loss backward: the TV term's table gradient (loss.py:11-43) joins this
    backward -- as records of the binned owner pass (so table_step stays
    fused), or added to d_table -- instead of a separate tv_bwd.
    table_live = (n_levels, int32 bitmap) from train.live_pair_mask, with
    table_step: the fused step skips the row pairs no gradient can reach
    (bitwise the same update, fewer optimizer-state bytes).
    owner_defer=True (binned scatter): the table gradient is not formed yet;
    render_bwd_owner(st, lo, hi) then writes bins [lo, hi) (render_bins
    gives their geometry), e.g. each range before its gradient exchange.
    loss (ABI 13, the trainer's step): dict(target [B, 3], out [4] device,
    rgb / rgb0 / sparsity / sparsity0 = the forward's outputs, tv [L] or
    None, world, sparse_w, tv_w) forms the training loss's upstream
    gradients in the backward itself (run_nerf.py:612-636 under
    train.dp_loss's rule; grads is not read) and writes out = loss, mse,
    mse0, entropy sum (loss_fwd's).
    mlp_step (binned scatter): the ten (p, exp_avg, exp_avg_sq, coeffs) of
    RAdam.take_step for st.ws's tensors, applied where each weight's final
    gradient is formed (the slab reduction; dws is still written); with
    repack=True the stepped weights' packed copies are then written into the
    workspace, for a next render_fwd(wsb=st.wsb, weights_packed=True)."""
    B = st.rays.shape[0]
    dev = st.rays.device
    if getattr(st, "skip_dead", False) and st.cfg.dense_bwd:
        raise ValueError("hashnerf_amd.render_bwd: the forward ran with skip_dead_color (features of tiles "
                         "without density not stored); the backward needs cfg.dense_bwd = 0")
    a = L.HnRenderBwdArgs()
    a.n_rays = B
    a.coarse = L.make_mlp(st.ws[:5])
    a.fine = L.make_mlp(st.ws[5:])
    keep = []
    names = ("g_rgb", "g_depth", "g_acc", "g_sparsity", "g_rgb0", "g_depth0", "g_acc0", "g_sparsity0",
             "g_raw_f")
    for k, t in [(n, grads.get(n)) for n in names] + [
            ("rays", st.rays), ("noise_c", st.noise_c), ("noise_f", st.noise_f), ("table", st.table),
            ("z_coarse", st.z_c), ("z_fine", st.z_f), ("raw_c", st.raw_c), ("raw_f", st.raw_f),
            ("d_table", d_table)]:
        if t is not None and k == "d_table" and not t.is_contiguous():
            raise RuntimeError("hashnerf_amd.render_bwd: d_table must be contiguous")
        t = L.contig(t)
        keep.append(t)
        setattr(a, k, None if t is None else t.data_ptr())
    a.fine_src = st.fine_src.data_ptr()
    a.feat = st.feat.data_ptr()
    a.weights_packed = 1               # same workspace and weights as the forward
    a.d_table_mode = (1 if overwrite else 0) | (2 if overwrite_mlp else 0)
    a.d_coarse = L.make_mlp_grad(dws[:5])
    a.d_fine = L.make_mlp_grad(dws[5:])
    step = None
    if table_step is not None:
        p, m, v, c = table_step
        L.require_device(p, m, v)
        step = L.HnRadamTensor()
        step.p, step.g, step.m, step.v = p.data_ptr(), None, m.data_ptr(), v.data_ptr()
        step.n = p.numel()
        for k in ("beta1", "beta2", "one_minus_beta1", "one_minus_beta2", "eps", "neg_wd_lr", "neg_step_lr",
                  "mode", "has_wd"):
            setattr(step, k, c[k])
        a.table_step = C.pointer(step)
        if table_live is not None:
            n_lv, words = table_live
            if not words.is_cuda or words.dtype != torch.int32 or not words.is_contiguous() or \
                    words.numel() < (n_lv << st.cfg.grid.log2_hashmap_size) // 64:
                raise ValueError("hashnerf_amd.render_bwd: table_live must be a contiguous device int32 "
                                 "bitmap of n_levels << (T - 6) words")
            keep.append(words)
            a.table_live = words.data_ptr()
            a.table_live_levels = n_lv
    if tv is not None:
        mv, cubes, g_tv = tv
        tva = _tv_args(st.table, mv, cubes, st.cfg.grid.log2_hashmap_size)
        keep.append(tva)
        a.tv = C.cast(C.pointer(tva), C.c_void_p)
        g_tv = g_tv.contiguous()
        keep.append(g_tv)
        a.g_tv = g_tv.data_ptr()
    a.owner_defer = 1 if owner_defer else 0
    if mlp_step is not None:
        if len(mlp_step) != 10:
            raise ValueError("hashnerf_amd.render_bwd: mlp_step needs the ten NeRFSmall tensors' steps")
        ms = (L.HnRadamTensor * 10)()
        for d, (p, m, v, c), w in zip(ms, mlp_step, st.ws):
            if p.data_ptr() != w.data_ptr():
                raise ValueError("hashnerf_amd.render_bwd: mlp_step must follow the render's weights in order")
            L.require_device(p, m, v)
            d.p, d.g, d.m, d.v, d.n = p.data_ptr(), None, m.data_ptr(), v.data_ptr(), p.numel()
            for k in ("beta1", "beta2", "one_minus_beta1", "one_minus_beta2", "eps", "neg_wd_lr", "neg_step_lr",
                      "mode", "has_wd"):
                setattr(d, k, c[k])
        a.mlp_step = ms
        a.repack = 1 if repack else 0
        keep.append(ms)
    if loss is not None:
        la = L.HnRenderLoss()
        ts = [L.contig(loss[k]) for k in ("target", "rgb", "rgb0", "sparsity", "sparsity0")]
        ltv = loss.get("tv")
        ltv = L.contig(ltv) if ltv is not None else None
        L.require_device(*ts, ltv, loss["out"])
        la.target, la.rgb, la.rgb0, la.sparsity, la.sparsity0 = (t.data_ptr() for t in ts)
        la.tv, la.n_tv = (ltv.data_ptr(), ltv.numel()) if ltv is not None else (None, 0)
        la.world, la.sparse_w, la.tv_w = float(loss["world"]), float(loss["sparse_w"]), float(loss["tv_w"])
        la.out = loss["out"].data_ptr()
        a.loss = C.pointer(la)
        keep += ts + [ltv, la]
    t0 = TIMER.begin("render_bwd")
    L.check(L.lib().hn_render_bwd(st.cfg, a, L.ptr(st.wsb), st.nbytes, L.stream(dev)), "render_bwd")
    TIMER.end("render_bwd", t0)
    # the deferred owner pass reuses these arguments (and the buffers they point to)
    st.bwd_args = (a, keep, step) if owner_defer else None
    if CHECK_FAULTS and not owner_defer:
        L.check_device_faults()


def render_bins(cfg, n_rays: int):
    """(number of bins, log2 table entries per bin) of the binned scatter
    (hn_render_bins); (0, 0) for the float-atomic schedule."""
    shift = C.c_int32(0)
    n = L.lib().hn_render_bins(cfg, n_rays, C.byref(shift))
    return int(n), int(shift.value)


def render_bwd_owner(st: RenderState, bin_lo: int, bin_hi: int):
    """hn_render_bwd_owner: the owner pass of a render_bwd(owner_defer=True)
    over bins [bin_lo, bin_hi) -- their slices of d_table written (or
    stepped, with table_step)."""
    if getattr(st, "bwd_args", None) is None:
        raise RuntimeError("hashnerf_amd.render_bwd_owner: needs a render_bwd(owner_defer=True) first")
    a = st.bwd_args[0]
    L.check(L.lib().hn_render_bwd_owner(st.cfg, a, L.ptr(st.wsb), st.nbytes, bin_lo, bin_hi,
                                        L.stream(st.rays.device)), "render_bwd_owner")
    if CHECK_FAULTS:
        L.check_device_faults()


def zeros_like_all(ts):
    """Zeroed tensors shaped like ts, views of ONE flat buffer (one fill)."""
    n = sum(t.numel() for t in ts)
    flat = torch.zeros(n, dtype=torch.float32, device=ts[0].device)
    out, off = [], 0
    for t in ts:
        out.append(flat[off:off + t.numel()].view_as(t))
        off += t.numel()
    return out


class RenderRaysFn(torch.autograd.Function):
    """Inputs: rays [B,11], t_vals [64], t_rand [B,64]|None, u [B,128],
    noise_c/noise_f |None, table, 5 coarse + 5 fine NeRFSmall weights.
    Outputs: rgb, depth, acc, sparsity, rgb0, depth0, acc0, sparsity0, z_std, raw."""

    @staticmethod
    def forward(ctx, cfg: L.HnRenderCfg, keep_feat: bool, rays, t_vals, t_rand, u, noise_c, noise_f,
                table, *ws):
        out, st = render_fwd(cfg, rays, t_vals, t_rand, u, noise_c, noise_f, table, ws, keep_feat)
        ctx.st = st
        ctx.set_materialize_grads(False)   # unused outputs => NULL, not zeros (0*inf)
        ctx.mark_non_differentiable(out["z_std"])
        return (out["rgb"], out["depth"], out["acc"], out["sparsity"], out["rgb0"], out["depth0"],
                out["acc0"], out["sparsity0"], out["z_std"], out["raw_f"])

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_acc, g_sp, g_rgb0, g_depth0, g_acc0, g_sp0, _g_zstd, g_raw):
        st = ctx.st
        if st is None:
            raise RuntimeError("hashnerf_amd.render_rays: forward ran without keeping features "
                               "(no input required grad)")
        d_table = torch.zeros_like(st.table)
        dws = zeros_like_all(st.ws)
        render_bwd(st, dict(g_rgb=g_rgb, g_depth=g_depth, g_acc=g_acc, g_sparsity=g_sp, g_rgb0=g_rgb0,
                            g_depth0=g_depth0, g_acc0=g_acc0, g_sparsity0=g_sp0, g_raw_f=g_raw),
                   d_table, dws)
        ctx.st = None
        return (None, None, None, None, None, None, None, None, d_table, *dws)


# --------------------------------------------------------------------------
# training-step driver (run_nerf.py:576-636)
# --------------------------------------------------------------------------
def _uniform_draws(shapes, dev):
    """torch.rand(shape, device=dev) for each shape, as hn_uniform_draw
    records: the default generator's seed, each draw's philox offset and
    torch's thread count for its size (ATen calc_execution_policy: 256-thread
    blocks, at most CUs x 2048 / 256 of them, 4 values per thread and call);
    the generator is advanced as the torch.rand calls would advance it.
    Returns (seed, ctypes array, output tensors)."""
    if len(shapes) > L.UNIFORM_MAX_DRAWS:
        raise ValueError(f"hashnerf_amd: at most {L.UNIFORM_MAX_DRAWS} uniform draws per launch")
    dev = torch.device(dev)
    torch.cuda.init()                          # default_generators is filled lazily
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    gen = torch.cuda.default_generators[idx]
    props = _DEV_PROPS.get(idx)
    if props is None:
        p = torch.cuda.get_device_properties(idx)
        props = _DEV_PROPS[idx] = (p.multi_processor_count,
                                   getattr(p, "max_threads_per_multi_processor", 2048))
    max_blocks = props[0] * (props[1] // 256)
    seed, off = gen.initial_seed(), gen.get_offset()
    arr = (L.HnUniformDraw * len(shapes))()
    outs = []
    for d, shape in zip(arr, shapes):
        t = torch.empty(shape, dtype=torch.float32, device=dev)
        n = t.numel()
        threads = 256 * min((n + 255) // 256, max_blocks)
        d.out, d.numel, d.threads, d.offset = t.data_ptr(), n, max(threads, 1), off
        if n:
            off += ((n - 1) // (threads * 4) + 1) * 4
        outs.append(t)
    gen.set_offset(off)
    return seed & ((1 << 64) - 1), arr, outs


_DEV_PROPS = {}


def torch_uniform(shapes, dev):
    """torch.rand(shape, device=dev) for every shape, bitwise, in one HIP
    launch (hn_uniform_philox); the default generator ends where the torch.rand
    calls would leave it."""
    seed, arr, outs = _uniform_draws(shapes, dev)
    L.check(L.lib().hn_uniform_philox(seed, arr, len(shapes), L.stream(torch.device(dev))), "uniform_philox")
    return outs


def sample_rays(image, c2w, n_rays, K, near, far, crop, seed, order=1, uniforms=None):
    """N_rand distinct pixels of one image (device, no replacement) -> the
    [n, 11] ray batch render() builds and the [n, 3] target colours.
    image [H, W, 3], c2w [3, 4] (or [4, 4]) fp32 on the device; crop =
    (y0, x0, h, w) sampling window; K the 3x3 intrinsics (host numbers).
    order=1 (hn_sample_rays_morton) lists the same drawn set in Morton order
    of its pixels -- the batch order changes the loss and its gradient only
    by float summation order -- so the fused forward's XCD-contiguous ray
    groups are spatially coherent; order=0 (hn_sample_rays) keeps the draw
    order.  Both are deterministic for a given seed.  uniforms: shapes of
    torch.rand draws to make as well (torch_uniform; with order=1 in the
    sampler's first launch), returned after rays and target."""
    L.require_device(image, c2w)
    image, c2w = image.contiguous(), c2w[:3, :4].contiguous()
    H, W = image.shape[0], image.shape[1]
    s = L.HnRaySampler()
    s.H, s.W = H, W
    s.crop_y0, s.crop_x0, s.crop_h, s.crop_w = (int(v) for v in crop)
    s.fx, s.fy, s.cx, s.cy = float(K[0][0]), float(K[1][1]), float(K[0][2]), float(K[1][2])
    s.near, s.far = float(near), float(far)
    s.seed = int(seed) & ((1 << 64) - 1)
    dev = image.device
    rays = torch.empty((n_rays, 11), dtype=torch.float32, device=dev)
    target = torch.empty((n_rays, 3), dtype=torch.float32, device=dev)
    if order == 1:
        nb = L.lib().hn_sample_rays_morton_workspace_bytes(s)
        if nb == 0:
            raise ValueError(f"sample_rays(order=1): window {s.crop_h}x{s.crop_w} too large")
        ws = _sampler_ws(dev, nb)
        if uniforms:
            useed, arr, outs = _uniform_draws(uniforms, dev)
            L.check(L.lib().hn_sample_batch_morton(s, L.ptr(image), L.ptr(c2w), n_rays, L.ptr(rays),
                                                   L.ptr(target), L.ptr(ws), nb, useed, arr, len(uniforms),
                                                   L.stream(dev)), "sample_batch_morton")
            return (rays, target, *outs)
        L.check(L.lib().hn_sample_rays_morton(s, L.ptr(image), L.ptr(c2w), n_rays, L.ptr(rays), L.ptr(target),
                                              L.ptr(ws), nb, L.stream(dev)), "sample_rays_morton")
    elif order == 0:
        L.check(L.lib().hn_sample_rays(s, L.ptr(image), L.ptr(c2w), n_rays, L.ptr(rays), L.ptr(target),
                                       L.stream(dev)), "sample_rays")
    else:
        raise ValueError(f"sample_rays: order {order!r}")
    if uniforms:
        return (rays, target, *torch_uniform(uniforms, dev))
    return rays, target


def sample_pool(images, poses, image_ids, K, near, far, seed, start, n_rays):
    """use_batching draw (run_nerf.py:505-521, 544-555): pool positions
    [start, start + n_rays) of the epoch whose shuffle key is `seed`, as the
    [n, 11] ray batch and [n, 3] targets (hn_sample_pool).  images [N, H, W, 3]
    and poses [N, 3|4, 4] on the device; image_ids the training image indices
    (device int32); K the 3x3 intrinsics (host numbers, used in float64)."""
    L.require_device(images, poses)
    images, poses = images.contiguous(), poses.contiguous()
    if image_ids.dtype != torch.int32 or not image_ids.is_cuda:
        raise TypeError("hashnerf_amd.sample_pool: image_ids must be a device int32 tensor")
    p = L.HnRayPool()
    p.n_images = int(image_ids.numel())
    p.H, p.W = int(images.shape[1]), int(images.shape[2])
    p.pose_stride = int(poses.shape[1] * poses.shape[2])
    p.fx, p.fy, p.cx, p.cy = float(K[0][0]), float(K[1][1]), float(K[0][2]), float(K[1][2])
    p.near, p.far = float(near), float(far)
    p.seed = int(seed) & ((1 << 64) - 1)
    dev = images.device
    rays = torch.empty((n_rays, 11), dtype=torch.float32, device=dev)
    target = torch.empty((n_rays, 3), dtype=torch.float32, device=dev)
    L.check(L.lib().hn_sample_pool(p, L.ptr(images), L.ptr(poses), L.ptr(image_ids.contiguous()), int(start),
                                   int(n_rays), L.ptr(rays), L.ptr(target), L.stream(dev)), "sample_pool")
    return rays, target


BLENDER_MODES = {"rgba": 0, "white": 1, "rgb": 2}


def blender_images(rgba_u8, half_res=False, mode="rgba"):
    """hn_blender_images: uint8 RGBA [n, H, W, 4] on the device -> float32
    images as load/load_blender.py:63-86 (/ 255., half_res INTER_AREA) and,
    mode="white" / "rgb", run_nerf.py:259-262's composite / channel cut."""
    if not rgba_u8.is_cuda or rgba_u8.dtype != torch.uint8 or rgba_u8.dim() != 4 or rgba_u8.shape[-1] != 4:
        raise TypeError("hashnerf_amd.blender_images: expects a device uint8 tensor [n, H, W, 4]")
    n, H, W, _ = rgba_u8.shape
    Ho, Wo = (H // 2, W // 2) if half_res else (H, W)
    m = BLENDER_MODES[mode]
    out = torch.empty((n, Ho, Wo, 4 if m == 0 else 3), dtype=torch.float32, device=rgba_u8.device)
    L.check(L.lib().hn_blender_images(L.ptr(rgba_u8.contiguous()), n, H, W, int(bool(half_res)), m, L.ptr(out),
                                      L.stream(rgba_u8.device)), "blender_images")
    return out


_SAMPLER_WS = {}


def _sampler_ws(dev, nbytes):
    """Scratch of the Morton sampler (block counts), grown on demand: one per
    (device, stream), so a batch drawn ahead on a side stream
    (Trainer.prefetch) never shares it with a draw on the current stream
    (ADVICE r05)."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0)
    ws = _SAMPLER_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        _SAMPLER_WS[key] = ws
    return ws


def loss_fwd(rgb, rgb0, target, sp, sp0, tv, world, sparse_w, tv_w):
    """hn_loss_fwd -> device [4] = loss, mse, mse0, sum of entropies."""
    L.require_device(rgb, target, sp)
    n = rgb.shape[0]
    out = torch.empty(4, dtype=torch.float32, device=rgb.device)
    L.check(L.lib().hn_loss_fwd(L.ptr(L.contig(rgb)), L.ptr(L.contig(rgb0)), L.ptr(L.contig(target)),
                                L.ptr(L.contig(sp)), L.ptr(L.contig(sp0)), n, L.ptr(L.contig(tv)),
                                0 if tv is None else tv.numel(), float(world), float(sparse_w),
                                float(tv_w), L.ptr(out), L.stream(rgb.device)), "loss_fwd")
    return out


def loss_bwd(rgb, rgb0, target, n_tv, world, sparse_w, tv_w, g_loss, has_sp0=True):
    """hn_loss_bwd -> (g_rgb, g_rgb0, g_sp, g_sp0, g_tv) for upstream g_loss (device scalar)."""
    n = rgb.shape[0]
    dev = rgb.device
    g_rgb = torch.empty_like(rgb)
    g_rgb0 = torch.empty_like(rgb) if rgb0 is not None else None
    g_sp = torch.empty(n, dtype=torch.float32, device=dev)
    g_sp0 = torch.empty(n, dtype=torch.float32, device=dev) if has_sp0 else None
    g_tv = torch.empty(n_tv, dtype=torch.float32, device=dev) if n_tv else None
    L.check(L.lib().hn_loss_bwd(L.ptr(L.contig(rgb)), L.ptr(L.contig(rgb0)), L.ptr(L.contig(target)), n,
                                n_tv, float(world), float(sparse_w), float(tv_w), L.ptr(g_loss.contiguous()),
                                L.ptr(g_rgb), L.ptr(g_rgb0), L.ptr(g_sp), L.ptr(g_sp0), L.ptr(g_tv),
                                L.stream(dev)), "loss_bwd")
    return g_rgb, g_rgb0, g_sp, g_sp0, g_tv


def loss_fwd_bwd(rgb, rgb0, target, sp, sp0, tv, world, sparse_w, tv_w, g_loss):
    """hn_loss_fwd_bwd: loss_fwd and loss_bwd in one launch -> (out [4],
    (g_rgb, g_rgb0, g_sp, g_sp0, g_tv)), bitwise the two calls' results."""
    L.require_device(rgb, target, sp)
    n = rgb.shape[0]
    dev = rgb.device
    n_tv = 0 if tv is None else tv.numel()
    out = torch.empty(4, dtype=torch.float32, device=dev)
    g_rgb = torch.empty_like(rgb)
    g_rgb0 = torch.empty_like(rgb) if rgb0 is not None else None
    g_sp = torch.empty(n, dtype=torch.float32, device=dev)
    g_sp0 = torch.empty(n, dtype=torch.float32, device=dev) if sp0 is not None else None
    g_tv = torch.empty(n_tv, dtype=torch.float32, device=dev) if n_tv else None
    L.check(L.lib().hn_loss_fwd_bwd(L.ptr(L.contig(rgb)), L.ptr(L.contig(rgb0)), L.ptr(L.contig(target)),
                                    L.ptr(L.contig(sp)), L.ptr(L.contig(sp0)), n, L.ptr(L.contig(tv)), n_tv,
                                    float(world), float(sparse_w), float(tv_w), L.ptr(out),
                                    L.ptr(g_loss.contiguous()), L.ptr(g_rgb), L.ptr(g_rgb0), L.ptr(g_sp),
                                    L.ptr(g_sp0), L.ptr(g_tv), L.stream(dev)), "loss_fwd_bwd")
    return out, (g_rgb, g_rgb0, g_sp, g_sp0, g_tv)


class TrainLossFn(torch.autograd.Function):
    """loss = (mse(rgb) + mse(rgb0)) / world + sparse_w * (sum sp + sum sp0) +
    tv_w * sum tv (run_nerf.py:612-636 under train.dp_loss's DP rule).
    Returns (loss, mse, mse0); mse/mse0 carry no gradient."""

    @staticmethod
    def forward(ctx, rgb, rgb0, target, sp, sp0, tv, world, sparse_w, tv_w):
        out = loss_fwd(rgb, rgb0, target, sp, sp0, tv, world, sparse_w, tv_w)
        ctx.save_for_backward(rgb, rgb0 if rgb0 is not None else rgb, target)
        ctx.has = (rgb0 is not None, sp0 is not None)
        ctx.n_tv = 0 if tv is None else tv.numel()
        ctx.consts = (float(world), float(sparse_w), float(tv_w))
        mse, mse0 = out[1], out[2]
        ctx.mark_non_differentiable(mse, mse0)
        return out[0], mse, mse0

    @staticmethod
    def backward(ctx, g_loss, _g_mse, _g_mse0):
        rgb, rgb0, target = ctx.saved_tensors
        has0, has_sp0 = ctx.has
        g = g_loss if g_loss is not None else torch.ones((), device=rgb.device)
        g_rgb, g_rgb0, g_sp, g_sp0, g_tv = loss_bwd(rgb, rgb0 if has0 else None, target, ctx.n_tv,
                                                    *ctx.consts, g, has_sp0)
        return g_rgb, g_rgb0, None, g_sp, g_sp0, g_tv, None, None, None


def train_loss(rgb, rgb0, target, sp, sp0, tv=None, world=1, sparse_w=0.0, tv_w=0.0):
    return TrainLossFn.apply(rgb, rgb0, target, sp, sp0, tv, world, sparse_w, tv_w)


def _tv_args(table, mv, cubes, log2T):
    a = L.HnTvArgs()
    a.n_levels = table.shape[0]
    a.log2_hashmap_size = int(log2T)
    for l, c in enumerate(cubes):
        a.cube[l] = int(c)
    a.min_vertex = mv.data_ptr()
    a.table = table.data_ptr()
    return a


def tv_fwd(table, min_vertex, cubes, log2T):
    """hn_tv_fwd: per-level TV values [L]; returns (tv, device min vertices)."""
    L.require_device(table)
    mv = min_vertex.to(dtype=torch.int32).contiguous()
    if mv.device.type == "cpu":            # no host stall: pinned + async copy
        mv = mv.pin_memory().to(table.device, non_blocking=True)
    else:
        mv = mv.to(table.device)
    tv = torch.empty(table.shape[0], dtype=torch.float32, device=table.device)
    L.check(L.lib().hn_tv_fwd(_tv_args(table, mv, cubes, log2T), L.ptr(tv), L.stream(table.device)),
            "tv_fwd")
    return tv, mv


def tv_bwd(table, mv, cubes, log2T, g_tv, dtable):
    """hn_tv_bwd: dtable += sum_l g_tv[l] d tv_l / d table."""
    g = g_tv.contiguous()
    L.check(L.lib().hn_tv_bwd(_tv_args(table, mv, cubes, log2T), L.ptr(g), L.ptr(dtable),
                              L.stream(table.device)), "tv_bwd")


def tv_bwd_records(cfg, table, mv, cubes, g_tv, d_table, wsb=None):
    """hn_render_bwd with no rays and a TV term (ABI 14): d_table = sum_l
    g_tv[l] d tv_l / d table (every entry written) through the binned
    scatter's TV records and exact owner pass -- bitwise reproducible, where
    tv_bwd's float atomics are not.  For a data-parallel rank that drew no
    rays (train.Trainer._empty_rank_grads).  wsb: workspace of >=
    hn_render_workspace_bytes(cfg, 0) bytes (default a fresh one)."""
    L.require_device(table, g_tv, d_table)
    if mv.device != table.device or mv.dtype != torch.int32 or not mv.is_contiguous():
        raise ValueError("hashnerf_amd.tv_bwd_records: min vertices must be tv_fwd's contiguous device int32 tensor")
    if not d_table.is_contiguous() or d_table.shape != table.shape:
        raise ValueError("hashnerf_amd.tv_bwd_records: d_table must be a contiguous tensor shaped like the table")
    nbytes = L.lib().hn_render_workspace_bytes(cfg, 0)
    if wsb is None or wsb.numel() * wsb.element_size() < nbytes:
        wsb = _ws(nbytes, table.device)
    a = L.HnRenderBwdArgs()
    a.n_rays = 0
    tva = _tv_args(table, mv, cubes, cfg.grid.log2_hashmap_size)
    a.tv = C.cast(C.pointer(tva), C.c_void_p)
    g = g_tv.contiguous()
    a.g_tv = g.data_ptr()
    a.d_table = d_table.data_ptr()
    a.d_table_mode = 1
    L.check(L.lib().hn_render_bwd(cfg, a, L.ptr(wsb), wsb.numel() * wsb.element_size(), L.stream(table.device)),
            "render_bwd (TV only)")
    if CHECK_FAULTS:
        L.check_device_faults()
    return wsb


class TVFn(torch.autograd.Function):
    """Per-level hash-table TV (loss.py:11-43) for all levels in one launch."""

    @staticmethod
    def forward(ctx, table, min_vertex, cubes, log2T):
        tv, mv = tv_fwd(table, min_vertex, cubes, log2T)
        ctx.save_for_backward(table, mv)
        ctx.cubes, ctx.log2T = list(cubes), int(log2T)
        return tv

    @staticmethod
    def backward(ctx, g_tv):
        table, mv = ctx.saved_tensors
        dtable = torch.zeros_like(table)
        tv_bwd(table, mv, ctx.cubes, ctx.log2T, g_tv, dtable)
        return dtable, None, None, None


def _radam_array(tensors, name):
    arr = (L.HnRadamTensor * len(tensors))()
    for d, (p, g, m, v, c) in zip(arr, tensors):
        L.require_device(p, g, m, v)
        for t in (p, g, m, v):
            if not t.is_contiguous():
                raise RuntimeError(f"hashnerf_amd.{name}: tensors must be contiguous")
        d.p, d.g, d.m, d.v = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
        d.n = p.numel()
        for k in ("beta1", "beta2", "one_minus_beta1", "one_minus_beta2", "eps", "neg_wd_lr",
                  "neg_step_lr", "mode", "has_wd"):
            setattr(d, k, c[k])
    return arr


def radam_step(tensors):
    """tensors: list of (p, g, m, v, coeff dict); one HIP launch per 16 tensors."""
    for i in range(0, len(tensors), L.RADAM_MAX_TENSORS):
        chunk = tensors[i:i + L.RADAM_MAX_TENSORS]
        arr = _radam_array(chunk, "radam_step")
        L.check(L.lib().hn_radam_step(arr, len(chunk), L.stream(chunk[0][0].device)), "radam_step")


SCATTER_MODES = {"auto": 0, "atomic": 1, "binned": 2}


def make_render_cfg(grid: L.HnGrid, white_bkgd: bool, lindisp: bool, perturb: bool,
                    n_samples: int = 64, n_importance: int = 128, scatter: str = "auto",
                    dense_bwd: bool = False) -> L.HnRenderCfg:
    """hn_render_cfg.  scatter: the backward's table-gradient scatter --
    "binned" (records + exact per-bin owner pass), "atomic" (float atomics),
    "auto" (binned where the table allows it: T <= 22).  dense_bwd: compute
    the backward of every sample, also those whose d raw is exactly zero
    (relu(sigma) = 0), which the default skips (ABI 14; same results up to
    the sign of zero)."""
    c = L.HnRenderCfg()
    c.grid = grid
    c.n_samples, c.n_importance = n_samples, n_importance
    c.white_bkgd, c.lindisp, c.perturb = int(white_bkgd), int(lindisp), int(perturb)
    c.scatter = SCATTER_MODES[scatter]
    c.dense_bwd = int(bool(dense_bwd))
    return c


def render_rays_fused(cfg, rays, t_vals, t_rand, u, noise_c, noise_f, table,
                      coarse_ws: Sequence[torch.Tensor], fine_ws: Sequence[torch.Tensor]):
    keep_feat = torch.is_grad_enabled() and any(
        t.requires_grad for t in (table, *coarse_ws, *fine_ws))
    return RenderRaysFn.apply(cfg, keep_feat, rays, t_vals, t_rand, u, noise_c, noise_f, table,
                              *coarse_ws, *fine_ws)
