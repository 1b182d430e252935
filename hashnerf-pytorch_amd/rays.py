"""Camera / ray helpers (ray_util.py, bbox.py, load/load_blender.py:30-35).

Host-side glue that feeds the hot path: evaluated with torch ops on the ray
device, with the reference's conventions (no +0.5 pixel centre, un-normalised
directions for training rays, world bbox padded by 1.0).
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np
import torch


def get_rays(H, W, K, c2w):
    """ray_util.py:62-80 -> rays_o, rays_d [H, W, 3] on c2w's device."""
    dev = c2w.device
    i, j = torch.meshgrid(torch.linspace(0, W - 1, W, device=dev),
                          torch.linspace(0, H - 1, H, device=dev), indexing="ij")
    i, j = i.t(), j.t()
    dirs = torch.stack([(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -torch.ones_like(i)], -1)
    rays_d = torch.sum(dirs[..., None, :] * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def get_rays_np(H, W, K, c2w):
    """ray_util.py:82-93."""
    i, j = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
    dirs = np.stack([(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -np.ones_like(i)], -1)
    rays_d = np.sum(dirs[..., np.newaxis, :] * c2w[:3, :3], -1)
    rays_o = np.broadcast_to(c2w[:3, -1], np.shape(rays_d))
    return rays_o, rays_d


def get_ndc_rays(H, W, focal, near, rays_o, rays_d):
    """ray_util.py:96-142 (forward-facing scenes), in the reference's op order
    (ox/oz and oy/oz formed once; d2 = 1 - o2)."""
    t = -(near + rays_o[..., 2]) / rays_d[..., 2]
    rays_o = rays_o + t[..., None] * rays_d
    ox_oz = rays_o[..., 0] / rays_o[..., 2]
    oy_oz = rays_o[..., 1] / rays_o[..., 2]
    o0 = -1. / (W / (2. * focal)) * ox_oz
    o1 = -1. / (H / (2. * focal)) * oy_oz
    o2 = 1. + 2. * near / rays_o[..., 2]
    d0 = -1. / (W / (2. * focal)) * (rays_d[..., 0] / rays_d[..., 2] - ox_oz)
    d1 = -1. / (H / (2. * focal)) * (rays_d[..., 1] / rays_d[..., 2] - oy_oz)
    d2 = 1 - o2
    return torch.stack([o0, o1, o2], -1), torch.stack([d0, d1, d2], -1)


def pose_spherical(theta: float, phi: float, radius: float) -> torch.Tensor:
    """load/load_blender.py:30-35: camera-to-world on a sphere."""
    t = torch.Tensor([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, radius], [0, 0, 0, 1]]).float()
    ph, th = phi / 180. * np.pi, theta / 180. * np.pi
    rp = torch.Tensor([[1, 0, 0, 0], [0, np.cos(ph), -np.sin(ph), 0],
                       [0, np.sin(ph), np.cos(ph), 0], [0, 0, 0, 1]]).float()
    rt = torch.Tensor([[np.cos(th), 0, -np.sin(th), 0], [0, 1, 0, 0],
                       [np.sin(th), 0, np.cos(th), 0], [0, 0, 0, 1]]).float()
    c2w = rt @ (rp @ t)
    return torch.Tensor(np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]])) @ c2w


def bbox_for_blender(c2ws: Sequence[torch.Tensor], H: int, W: int, focal: float,
                     near: float = 2.0, far: float = 6.0):
    """bbox.py:10-41: min/max over the 4 image-corner rays (normalised
    directions) of every camera at near and far, padded by 1.0."""
    corners = torch.tensor([[0., 0.], [W - 1., 0.], [0., H - 1.], [W - 1., H - 1.]])
    dirs = torch.stack([(corners[:, 0] - W / 2) / focal, -(corners[:, 1] - H / 2) / focal,
                        -torch.ones(4)], -1)
    lo = torch.full((3,), 100.)
    hi = torch.full((3,), -100.)
    for c2w in c2ws:
        c2w = torch.as_tensor(c2w, dtype=torch.float32).cpu()
        rd = dirs @ c2w[:3, :3].T
        rd = rd / torch.norm(rd, dim=-1, keepdim=True)
        ro = c2w[:3, -1].expand(rd.shape)
        for pts in (ro + near * rd, ro + far * rd):
            lo = torch.minimum(lo, pts.min(0).values)
            hi = torch.maximum(hi, pts.max(0).values)
    return lo - 1.0, hi + 1.0


def blender_cameras(n: int = 100, radius: float = 4.0):
    """Synthetic nerf-synthetic-style training cameras: poses on the upper
    hemisphere (elevation -30 / -60 deg alternating), as SURVEY 8(d)."""
    thetas = np.linspace(-180, 180, n + 1)[:-1]
    return [pose_spherical(float(t), -30.0 if k % 2 == 0 else -60.0, radius) for k, t in enumerate(thetas)]


CAMERA_ANGLE_X = 0.6911112070083618   # nerf-synthetic transforms_train.json


def blender_intrinsics(H: int, W: int, camera_angle_x: float = CAMERA_ANGLE_X):
    focal = .5 * W / math.tan(.5 * camera_angle_x)
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    return focal, K
