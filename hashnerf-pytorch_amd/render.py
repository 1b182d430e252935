"""Volume rendering API of run_nerf_helpers.py (render, render_rays,
raw2outputs, sample_pdf, run_network, batchify, render_path) on HIP kernels.

``render_rays`` dispatches to the fused forward/backward kernels
(``functional.RenderRaysFn``) whenever the configuration is the HashNeRF one
(NetworkQuery over a 16-level HashEmbedder + SH, two NeRFSmall nets, 64+128
samples with view directions); otherwise it composes the standalone HIP ops
exactly like the reference composes eager ops.  There is no CPU path.
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np
import torch

from . import _lib as L
from . import functional as HF
from .embedding import HashEmbedder, SHEncoder
from .models import NeRFSmall
from .rays import get_ndc_rays, get_rays

img2mse = lambda x, y: torch.mean((x - y) ** 2)                     # run_nerf_helpers.py:24
mse2psnr = lambda x: -10. * torch.log(x) / torch.log(torch.tensor([10.], device=x.device))
to8b = lambda x: (255 * np.clip(x, 0, 1)).astype(np.uint8)


def batchify(fn, chunk):
    """run_nerf_helpers.py:203-210."""
    if chunk is None:
        return fn
    return lambda inputs: torch.cat([fn(inputs[i:i + chunk]) for i in range(0, inputs.shape[0], chunk)], 0)


def run_network(inputs, viewdirs, fn, embed_fn, embeddirs_fn, netchunk=1024 * 64):
    """run_nerf_helpers.py:212-227."""
    inputs_flat = torch.reshape(inputs, [-1, inputs.shape[-1]])
    embedded, keep_mask = embed_fn(inputs_flat)
    if viewdirs is not None:
        input_dirs = viewdirs[:, None].expand(inputs.shape)
        embedded_dirs = embeddirs_fn(torch.reshape(input_dirs, [-1, input_dirs.shape[-1]]))
        embedded = torch.cat([embedded, embedded_dirs], -1)
    outputs_flat = batchify(fn, netchunk)(embedded)
    outputs_flat = torch.where(keep_mask[:, None] | (torch.arange(outputs_flat.shape[-1],
                               device=outputs_flat.device) != outputs_flat.shape[-1] - 1),
                               outputs_flat, torch.zeros_like(outputs_flat))
    return torch.reshape(outputs_flat, list(inputs.shape[:-1]) + [outputs_flat.shape[-1]])


class NetworkQuery:
    """The ``network_query_fn`` closure of create_nerf (run_nerf_helpers.py:122-125),
    as an object so render_rays can see the embedders and take the fused path."""

    def __init__(self, embed_fn, embeddirs_fn, netchunk=1024 * 64):
        self.embed_fn, self.embeddirs_fn, self.netchunk = embed_fn, embeddirs_fn, netchunk

    def __call__(self, inputs, viewdirs, network_fn):
        return run_network(inputs, viewdirs, network_fn, embed_fn=self.embed_fn,
                           embeddirs_fn=self.embeddirs_fn, netchunk=self.netchunk)


def raw2outputs(raw, z_vals, rays_d, raw_noise_std=0, white_bkgd=False, pytest=False):
    """run_nerf_helpers.py:577-628 -> rgb, disp, acc, weights, depth, sparsity(entropy)."""
    noise = None
    if raw_noise_std > 0.:
        if pytest:
            np.random.seed(0)
            noise = torch.tensor(np.random.rand(*list(raw[..., 3].shape)) * raw_noise_std,
                                 dtype=torch.float32, device=raw.device)
        else:
            noise = torch.randn(raw[..., 3].shape, device=raw.device) * raw_noise_std
    rgb, disp, acc, weights, depth, ent = HF.CompositeFn.apply(raw, z_vals, rays_d, noise, bool(white_bkgd))
    return rgb, disp, acc, weights, depth, ent


def sample_pdf(bins, weights, N_samples, det=False, pytest=False):
    """run_nerf_helpers.py:264-307 (u drawn on the bins' device)."""
    B = bins.shape[0]
    if det:
        u = torch.linspace(0., 1., steps=N_samples, device=bins.device).expand(B, N_samples)
    else:
        u = torch.rand(B, N_samples, device=bins.device)
    if pytest:
        np.random.seed(0)
        u = np.broadcast_to(np.linspace(0., 1., N_samples), (B, N_samples)) if det \
            else np.random.rand(B, N_samples)
        u = torch.tensor(np.ascontiguousarray(u), dtype=torch.float32, device=bins.device)
    return HF.sample_pdf(bins, weights, u)


_LINSPACE = {}


def _linspace_cached(n, dev):
    """torch.linspace(0, 1, n) made on the CPU as the reference does (:514),
    copied to the device once (a per-call pageable copy would stall the
    host on every training step)."""
    key = (n, str(dev))
    t = _LINSPACE.get(key)
    if t is None:
        t = _LINSPACE[key] = torch.linspace(0., 1., steps=n).to(dev)
    return t


def _draw(shape, dev, pytest, fn):
    if pytest:
        np.random.seed(0)
        return torch.tensor(np.random.rand(*shape), dtype=torch.float32, device=dev)
    return fn(shape, device=dev)


def _fusable(ray_batch, network_fn, network_query_fn, N_samples, N_importance, network_fine):
    if not isinstance(network_query_fn, NetworkQuery):
        return False
    e, ed = network_query_fn.embed_fn, network_query_fn.embeddirs_fn
    return (isinstance(e, HashEmbedder) and e.n_levels == 16 and isinstance(ed, SHEncoder)
            and ed.degree == 4 and isinstance(network_fn, NeRFSmall)
            and isinstance(network_fine, NeRFSmall) and N_samples == 64 and N_importance == 128
            and ray_batch.shape[-1] > 8)


def render_rays(ray_batch, network_fn, network_query_fn, N_samples, embed_fn=None, retraw=False,
                lindisp=False, perturb=0., N_importance=0, network_fine=None, white_bkgd=False,
                raw_noise_std=0., verbose=False, pytest=False):
    """run_nerf_helpers.py:464-574.  Same arguments, same returned dict."""
    L.require_device(ray_batch)
    B = ray_batch.shape[0]
    dev = ray_batch.device
    if _fusable(ray_batch, network_fn, network_query_fn, N_samples, N_importance, network_fine):
        emb = network_query_fn.embed_fn
        t_vals = _linspace_cached(N_samples, dev)
        t_rand = _draw((B, N_samples), dev, pytest, torch.rand) if perturb > 0. else None
        if perturb == 0.:
            if pytest:
                u = torch.tensor(np.broadcast_to(np.linspace(0., 1., N_importance), (B, N_importance)),
                                 dtype=torch.float32, device=dev)
            else:
                u = torch.linspace(0., 1., N_importance, device=dev).expand(B, N_importance)
        else:
            u = _draw((B, N_importance), dev, pytest, torch.rand)
        noise_c = noise_f = None
        if raw_noise_std > 0.:
            rn = (lambda s, device: torch.randn(s, device=device))
            noise_c = _draw((B, N_samples), dev, pytest, rn) * raw_noise_std
            noise_f = _draw((B, N_samples + N_importance), dev, pytest, rn) * raw_noise_std
        cfg = HF.make_render_cfg(emb.grid(), white_bkgd, lindisp, perturb > 0.)
        (rgb, depth, acc, sp, rgb0, depth0, acc0, sp0, z_std, raw) = HF.render_rays_fused(
            cfg, ray_batch, t_vals, t_rand, u, noise_c, noise_f, emb.table, network_fn.weights(),
            network_fine.weights())
        ret = {"rgb_map": rgb, "depth_map": depth, "acc_map": acc, "sparsity_loss": sp}
        if retraw:
            ret["raw"] = raw
        ret.update({"rgb0": rgb0, "depth0": depth0, "acc0": acc0, "sparsity_loss0": sp0, "z_std": z_std})
        return ret
    return _render_rays_unfused(ray_batch, network_fn, network_query_fn, N_samples, retraw, lindisp,
                                perturb, N_importance, network_fine, white_bkgd, raw_noise_std, pytest)


def _render_rays_unfused(ray_batch, network_fn, network_query_fn, N_samples, retraw, lindisp, perturb,
                         N_importance, network_fine, white_bkgd, raw_noise_std, pytest):
    """Composition of the standalone HIP ops, op-for-op like the reference."""
    B = ray_batch.shape[0]
    dev = ray_batch.device
    rays_o, rays_d = ray_batch[:, 0:3], ray_batch[:, 3:6]
    viewdirs = ray_batch[:, -3:] if ray_batch.shape[-1] > 8 else None
    bounds = torch.reshape(ray_batch[..., 6:8], [-1, 1, 2])
    near, far = bounds[..., 0], bounds[..., 1]
    t_vals = torch.linspace(0., 1., steps=N_samples).to(dev)
    z_vals = near * (1. - t_vals) + far * t_vals if not lindisp else \
        1. / (1. / near * (1. - t_vals) + 1. / far * t_vals)
    z_vals = z_vals.expand([B, N_samples])
    if perturb > 0.:
        mids = .5 * (z_vals[..., 1:] + z_vals[..., :-1])
        upper = torch.cat([mids, z_vals[..., -1:]], -1)
        lower = torch.cat([z_vals[..., :1], mids], -1)
        t_rand = _draw(tuple(z_vals.shape), dev, pytest, torch.rand)
        z_vals = lower + (upper - lower) * t_rand
    pts = rays_o[..., None, :] + rays_d[..., None, :] * z_vals[..., :, None]
    raw = network_query_fn(pts, viewdirs, network_fn)
    rgb_map, disp_map, acc_map, weights, depth_map, sp = raw2outputs(raw, z_vals, rays_d, raw_noise_std,
                                                                     white_bkgd, pytest=pytest)
    ret = {}
    if N_importance > 0:
        rgb0, depth0, acc0, sp0 = rgb_map, depth_map, acc_map, sp
        z_mid = .5 * (z_vals[..., 1:] + z_vals[..., :-1])
        z_samples = sample_pdf(z_mid, weights[..., 1:-1], N_importance, det=(perturb == 0.),
                               pytest=pytest).detach()
        z_vals, _ = torch.sort(torch.cat([z_vals, z_samples], -1), -1)
        pts = rays_o[..., None, :] + rays_d[..., None, :] * z_vals[..., :, None]
        run_fn = network_fn if network_fine is None else network_fine
        raw = network_query_fn(pts, viewdirs, run_fn)
        rgb_map, disp_map, acc_map, weights, depth_map, sp = raw2outputs(raw, z_vals, rays_d,
                                                                         raw_noise_std, white_bkgd,
                                                                         pytest=pytest)
    ret.update({"rgb_map": rgb_map, "depth_map": depth_map, "acc_map": acc_map, "sparsity_loss": sp})
    if retraw:
        ret["raw"] = raw
    if N_importance > 0:
        ret.update({"rgb0": rgb0, "depth0": depth0, "acc0": acc0, "sparsity_loss0": sp0,
                    "z_std": torch.std(z_samples, dim=-1, unbiased=False)})
    return ret


def render(H, W, K, chunk=1024 * 32, rays=None, c2w=None, ndc=True, near=0., far=1.,
           use_viewdirs=False, c2w_staticcam=None, **kwargs):
    """run_nerf_helpers.py:310-392 -> [rgb_map, depth_map, acc_map, extras]."""
    if c2w is not None:
        rays_o, rays_d = get_rays(H, W, K, c2w)
    else:
        rays_o, rays_d = rays
    if use_viewdirs:
        viewdirs = rays_d
        if c2w_staticcam is not None:
            rays_o, rays_d = get_rays(H, W, K, c2w_staticcam)
        viewdirs = viewdirs / torch.norm(viewdirs, dim=-1, keepdim=True)
        viewdirs = torch.reshape(viewdirs, [-1, 3]).float()
    sh = rays_d.shape
    if ndc:
        rays_o, rays_d = get_ndc_rays(H, W, K[0][0], 1., rays_o, rays_d)
    rays_o = torch.reshape(rays_o, [-1, 3]).float()
    rays_d = torch.reshape(rays_d, [-1, 3]).float()
    near, far = near * torch.ones_like(rays_d[..., :1]), far * torch.ones_like(rays_d[..., :1])
    rays_ = torch.cat([rays_o, rays_d, near, far], -1)
    if use_viewdirs:
        rays_ = torch.cat([rays_, viewdirs], -1)
    return render_ray_batch(rays_, sh[:-1], chunk, **kwargs)


def render_ray_batch(rays_, out_shape, chunk=1024 * 32, **kwargs):
    """The chunk loop + output assembly of render() (run_nerf_helpers.py:370-392)
    over an already built [N, 8 or 11] ray batch (e.g. from the device sampler).
    render()-level keywords of a render_kwargs dict (ndc, near, far,
    use_viewdirs, c2w_staticcam) are already baked into the batch."""
    for k in ("ndc", "near", "far", "use_viewdirs", "c2w_staticcam"):
        kwargs.pop(k, None)
    all_ret = {}
    for i in range(0, rays_.shape[0], chunk):
        ret = render_rays(rays_[i:i + chunk], **kwargs)
        for k in ret:
            all_ret.setdefault(k, []).append(ret[k])
    all_ret = {k: (v[0] if len(v) == 1 else torch.cat(v, 0)) for k, v in all_ret.items()}
    for k in all_ret:
        all_ret[k] = torch.reshape(all_ret[k], list(out_shape) + list(all_ret[k].shape[1:]))
    k_extract = ["rgb_map", "depth_map", "acc_map"]
    return [all_ret[k] for k in k_extract] + [{k: all_ret[k] for k in all_ret if k not in k_extract}]


@torch.no_grad()
def render_path(render_poses, hwf, K, chunk, render_kwargs, gt_imgs=None, savedir=None,
                render_factor=0):
    """run_nerf_helpers.py:395-459 (evaluation): returns (rgbs, depths), depth
    normalised to [0, 1] between near and far.  With gt_imgs (and no
    render_factor) the per-image PSNRs are computed as the reference does and,
    when savedir is given, pickled to test_psnrs_avg{avg:0.2f}.pkl like
    :452-456.  The per-frame matplotlib figures (:435-449) are not written:
    plotting is outside the hot path."""
    H, W, focal = hwf
    near, far = render_kwargs["near"], render_kwargs["far"]
    if render_factor != 0:
        H, W, focal = H // render_factor, W // render_factor, focal / render_factor
    rgbs, depths, psnrs = [], [], []
    for i, c2w in enumerate(render_poses):
        rgb, depth, acc, _ = render(H, W, K, chunk=chunk, c2w=c2w[:3, :4], **render_kwargs)
        rgbs.append(rgb.cpu().numpy())
        depths.append(((depth - near) / (far - near)).cpu().numpy())
        if gt_imgs is not None and render_factor == 0:
            gt = gt_imgs[i].cpu().numpy() if torch.is_tensor(gt_imgs[i]) else gt_imgs[i]
            psnrs.append(-10. * np.log10(np.mean(np.square(rgbs[-1] - gt))))
    if gt_imgs is not None and render_factor == 0 and savedir is not None and psnrs:
        import os
        import pickle
        avg = sum(psnrs) / len(psnrs)
        with open(os.path.join(savedir, "test_psnrs_avg{:0.2f}.pkl".format(avg)), "wb") as fp:
            pickle.dump(psnrs, fp)
    render_path.last_psnrs = psnrs
    return np.stack(rgbs, 0), np.stack(depths, 0)
