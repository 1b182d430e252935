"""Losses of the training step: hash-table total variation (loss.py:11-43) and
the run_nerf.py:612-636 loss assembly."""
from __future__ import annotations

from math import exp, floor, log

import torch

from . import functional as HF
from .embedding import hash as spatial_hash


def sigma_sparsity_loss(sigmas):
    """loss.py:45-47 (Cauchy sparsity on sigma).  Imported by run_nerf.py:19
    but unused on the training path (run_nerf_helpers.py:608 is commented
    out); kept for import compatibility as plain torch ops."""
    return torch.log(1.0 + 2 * sigmas ** 2).sum(dim=-1)


def tv_cube(level, n_levels, min_resolution, max_resolution):
    """Resolution and cube edge of loss.py:13-22 (float64 math, floor, clip)."""
    b = exp((log(max_resolution) - log(min_resolution)) / (n_levels - 1))
    resolution = torch.tensor(floor(min_resolution * b ** level))
    min_cube, max_cube = min_resolution - 1, 50
    if min_cube > max_cube:
        raise ValueError("total_variation_loss: min cuboid size greater than max")
    cube = torch.floor(torch.clip(resolution / 10.0, min_cube, max_cube)).int()
    return resolution, cube


def total_variation_loss(embeddings, min_resolution, max_resolution, level, log2_hashmap_size,
                         n_levels=16, min_vertex=None, generator=None):
    """loss.py:11-43.  ``embeddings`` is ``HashEmbedder.embeddings[level]``;
    ``min_vertex`` (3 ints) replaces the torch.randint draw (:25) when given."""
    min_resolution = int(min_resolution)
    max_resolution = int(max_resolution)
    resolution, cube = tv_cube(level, n_levels, min_resolution, max_resolution)
    if min_vertex is None:
        min_vertex = torch.randint(0, int(resolution - cube), (3,), generator=generator)
    dev = embeddings.weight.device
    idx = min_vertex.to(dev) + torch.stack([torch.arange(int(cube) + 1, device=dev)] * 3, -1)
    cube_idx = torch.stack(torch.meshgrid(idx[:, 0], idx[:, 1], idx[:, 2], indexing="ij"), -1)
    e = embeddings(spatial_hash(cube_idx, log2_hashmap_size))
    tv_x = torch.pow(e[1:] - e[:-1], 2).sum()
    tv_y = torch.pow(e[:, 1:] - e[:, :-1], 2).sum()
    tv_z = torch.pow(e[:, :, 1:] - e[:, :, :-1], 2).sum()
    return (tv_x + tv_y + tv_z) / cube.to(dev)


def draw_tv_cubes(n_levels, min_resolution, max_resolution, generator=None):
    """Per-level cube edge and random min vertex, drawn like loss.py:22-25."""
    cubes, mvs = [], []
    for l in range(n_levels):
        resolution, cube = tv_cube(l, n_levels, int(min_resolution), int(max_resolution))
        cubes.append(int(cube))
        mvs.append(torch.randint(0, int(resolution - cube), (3,), generator=generator))
    return cubes, torch.stack(mvs, 0)


def tv_loss_levels(embed_fn, generator=None, min_vertex=None):
    """All 16 ``total_variation_loss`` terms of run_nerf.py:628-635 in one HIP
    forward (+ one backward) launch.  Returns the per-level values [L]; their
    sum is the reference's TV_loss."""
    cubes, mv = draw_tv_cubes(embed_fn.n_levels, embed_fn.base_resolution,
                              embed_fn.finest_resolution, generator)
    if min_vertex is not None:
        mv = min_vertex
    return HF.TVFn.apply(embed_fn.table, mv, cubes, embed_fn.log2_hashmap_size)


def training_loss(rgb, extras, target, sparse_loss_weight=1e-10):
    """run_nerf.py:612-623: mse(rgb) + mse(rgb0) + w * (sum H + sum H0)."""
    img_loss = torch.mean((rgb - target) ** 2)
    loss = img_loss
    if "rgb0" in extras:
        loss = loss + torch.mean((extras["rgb0"] - target) ** 2)
    sp = extras["sparsity_loss"].sum()
    if "sparsity_loss0" in extras:
        sp = sp + extras["sparsity_loss0"].sum()
    return loss + sparse_loss_weight * sp, img_loss
