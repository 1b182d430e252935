"""Blender (nerf-synthetic) scenes for the trainer.

``load_blender_data`` mirrors load/load_blender.py:38-91 (same arguments and
return values) and ``BlenderScene`` is the trainer's dataset built from it,
with the white-background composite of run_nerf.py:259-262.  The per-pixel
arithmetic -- / 255., the half_res INTER_AREA downscale and the composite --
runs on the device (hn_blender_images); the host only decodes PNGs (PIL:
imageio and cv2 are not in this image) and reads the transforms JSON.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from . import functional as HF
from .rays import bbox_for_blender, pose_spherical


def read_rgba(path: str) -> np.ndarray:
    """A PNG as uint8 [H, W, 4] (imageio.imread of nerf-synthetic's RGBA
    PNGs).  Non-RGBA files are converted with an opaque alpha; the reference
    would take their last colour channel as alpha (load_blender.py:63 keeps
    "all 4 channels" of whatever imageio returns)."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode != "RGBA":
            im = im.convert("RGBA")
        return np.asarray(im, dtype=np.uint8).copy()


def read_blender_split(basedir: str, testskip: int = 1):
    """load_blender.py:39-60: the frames of train / val / test (every
    testskip-th of val and test), as uint8 RGBA [n, H, W, 4], float32 poses
    [n, 4, 4], the split index arrays and camera_angle_x of the last split."""
    metas = {}
    for s in ("train", "val", "test"):
        with open(os.path.join(basedir, f"transforms_{s}.json")) as fp:
            metas[s] = json.load(fp)
    imgs, poses, counts = [], [], [0]
    for s in ("train", "val", "test"):
        skip = 1 if (s == "train" or testskip == 0) else testskip
        frames = metas[s]["frames"][::skip]
        for frame in frames:
            imgs.append(read_rgba(os.path.join(basedir, frame["file_path"] + ".png")))
            poses.append(np.array(frame["transform_matrix"]))
        counts.append(counts[-1] + len(frames))
    i_split = [np.arange(counts[i], counts[i + 1]) for i in range(3)]
    return (np.stack(imgs, 0), np.stack(poses, 0).astype(np.float32), i_split,
            float(metas["test"]["camera_angle_x"]), metas)


def load_blender_data(basedir: str, half_res: bool = False, testskip: int = 1, device="cuda"):
    """load/load_blender.py:38-91 -> (imgs RGBA float32 [n, H, W, 4] on the
    device, poses [n, 4, 4] float32 numpy, render_poses [40, 4, 4],
    [H, W, focal], i_split, bounding_box)."""
    rgba, poses, i_split, camera_angle_x, metas = read_blender_split(basedir, testskip)
    H, W = rgba.shape[1:3]
    focal = .5 * W / np.tan(.5 * camera_angle_x)
    render_poses = torch.stack([pose_spherical(float(a), -30.0, 4.0)
                                for a in np.linspace(-180, 180, 40 + 1)[:-1]], 0)
    if half_res:
        H, W, focal = H // 2, W // 2, focal / 2.
    imgs = HF.blender_images(torch.from_numpy(rgba).to(device), half_res, "rgba")
    # bbox.py:10-41 over the train frames, at the (possibly halved) image size
    train_c2w = [torch.tensor(f["transform_matrix"], dtype=torch.float32) for f in metas["train"]["frames"]]
    bounding_box = bbox_for_blender(train_c2w, H, W, .5 * W / np.tan(.5 * float(metas["train"]["camera_angle_x"])))
    return imgs, poses, render_poses, [H, W, focal], i_split, bounding_box


class BlenderScene:
    """A nerf-synthetic scene on the device, shaped like train.SyntheticBlender
    (H, W, focal, K, poses, images [n, H, W, 3], i_train, bounding_box,
    test_poses / test_images): load_blender_data + run_nerf.py:259-262
    (white_bkgd composite or the RGB channels) in one device pass."""

    def __init__(self, basedir: str, device="cuda", half_res: bool = False, testskip: int = 1,
                 white_bkgd: bool = True):
        rgba, poses, i_split, camera_angle_x, metas = read_blender_split(basedir, testskip)
        H, W = rgba.shape[1:3]
        focal = .5 * W / np.tan(.5 * camera_angle_x)
        if half_res:
            H, W, focal = H // 2, W // 2, focal / 2.
        self.H, self.W, self.focal = int(H), int(W), float(focal)
        self.K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
        dev = torch.device(device)
        self.images = HF.blender_images(torch.from_numpy(rgba).to(dev), half_res,
                                        "white" if white_bkgd else "rgb")
        self.poses = torch.from_numpy(poses).to(dev)
        self.i_train, self.i_val, self.i_test = (torch.from_numpy(s) for s in i_split)
        train_c2w = [torch.tensor(f["transform_matrix"], dtype=torch.float32) for f in metas["train"]["frames"]]
        self.bounding_box = bbox_for_blender(train_c2w, self.H, self.W,
                                             .5 * W / np.tan(.5 * float(metas["train"]["camera_angle_x"])))
        self.test_poses = self.poses[self.i_test.to(dev)] if len(self.i_test) else None
        self.test_images = self.images[self.i_test.to(dev)] if len(self.i_test) else None
