"""SURVEY 8(f) #2 data semantics: the blender image preparation
(load/load_blender.py:63-86, run_nerf.py:259-262) and use_batching's ray pool
(run_nerf.py:505-521, 544-555).

CPU: the oracle against fixtures of the reference's own code
(tests/golden/make_golden.py gen_pool_rays: ray_util.get_rays_np; gen_blender_
images: the reference's numpy expressions) and the PNG-directory reader.
GPU (-m gpu): hn_blender_images against the oracle and the exact float64
means (half_res: INTER_AREA restated, cv2 absent: within 1 ulp), and
hn_sample_pool: one epoch of draws is a permutation of the pool, every ray and
target bit-exact against rays_rgb, and the next epoch reshuffles.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import golden

DEV = "cuda"


def test_oracle_pool_rays_vs_reference(oracle):
    g = golden("pool_rays")
    got = oracle.pool_rays(g["images"], g["poses"], g["i_train"], int(g["H"]), int(g["W"]), g["K"])
    np.testing.assert_array_equal(got, g["rays_rgb"])


def test_oracle_blender_images_vs_reference(oracle):
    g = golden("blender_images")
    np.testing.assert_array_equal(oracle.blender_images(g["rgba"], False, "rgba"), g["imgs"])
    np.testing.assert_array_equal(oracle.blender_images(g["rgba"], False, "white"), g["white"])
    half = oracle.blender_images(g["rgba"], True, "rgba").astype(np.float64)
    np.testing.assert_allclose(half, g["half_mean"], rtol=2 ** -23, atol=2 ** -26)
    hw = oracle.blender_images(g["rgba"], True, "white").astype(np.float64)
    m = g["half_mean"]
    np.testing.assert_allclose(hw, m[..., :3] * m[..., 3:] + (1. - m[..., 3:]), rtol=2e-7, atol=2e-7)


def _write_scene(root, n=(3, 2, 2), H=8, W=10, seed=5):
    """A nerf-synthetic-shaped directory: RGBA PNGs + transforms_*.json."""
    from PIL import Image
    g = np.random.Generator(np.random.PCG64(seed))
    k = 0
    for split, cnt in zip(("train", "val", "test"), n):
        frames = []
        for _ in range(cnt):
            arr = g.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
            os.makedirs(os.path.join(root, split), exist_ok=True)
            Image.fromarray(arr, "RGBA").save(os.path.join(root, split, f"r_{k}.png"))
            th = -180 + 37 * k
            frames.append({"file_path": f"./{split}/r_{k}", "transform_matrix": _pose(th).tolist()})
            k += 1
        with open(os.path.join(root, f"transforms_{split}.json"), "w") as f:
            json.dump({"camera_angle_x": 0.6911112070083618, "frames": frames}, f)


def _pose(theta):
    import sys
    from conftest import ROOT
    sys.path.insert(0, ROOT)
    from oracle.hashnerf_oracle import pose_spherical
    return pose_spherical(float(theta), -30.0, 4.0).numpy()


def test_png_reader_split_order(tmp_path, hn):
    from PIL import Image
    from hashnerf_pytorch_amd import data as D
    _write_scene(str(tmp_path))
    rgba, poses, i_split, cam_x, metas = D.read_blender_split(str(tmp_path), testskip=1)
    assert rgba.shape == (7, 8, 10, 4) and rgba.dtype == np.uint8
    assert [list(s) for s in i_split] == [[0, 1, 2], [3, 4], [5, 6]]
    np.testing.assert_array_equal(rgba[4], np.asarray(Image.open(tmp_path / "val" / "r_4.png")))
    assert poses.dtype == np.float32 and poses.shape == (7, 4, 4)
    _, _, i_split2, _, _ = D.read_blender_split(str(tmp_path), testskip=2)
    assert [len(s) for s in i_split2] == [3, 1, 1]      # val / test every 2nd frame


@pytest.mark.gpu
@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("mode", ["rgba", "white", "rgb"])
def test_blender_images_device(hn, oracle, half, mode):
    from hashnerf_pytorch_amd import functional as HF
    g = golden("blender_images")
    out = HF.blender_images(torch.from_numpy(g["rgba"]).to(DEV), half, mode).cpu().numpy()
    ref = oracle.blender_images(g["rgba"], half, mode)
    np.testing.assert_array_equal(out, ref)
    if not half:
        np.testing.assert_array_equal(out, {"rgba": g["imgs"], "white": g["white"], "rgb": g["imgs"][..., :3]}[mode])


@pytest.mark.gpu
def test_blender_scene_from_directory(hn, oracle, tmp_path):
    """BlenderScene: a PNG directory -> composited device images, poses,
    splits, bbox (bbox.py over the train frames), K; half_res halves H, W,
    focal."""
    from hashnerf_pytorch_amd.data import BlenderScene, load_blender_data, read_blender_split
    _write_scene(str(tmp_path))
    rgba, poses, _, _, _ = read_blender_split(str(tmp_path))
    for half in (False, True):
        sc = BlenderScene(str(tmp_path), DEV, half_res=half, white_bkgd=True)
        ref = oracle.blender_images(rgba, half, "white")
        np.testing.assert_array_equal(sc.images.cpu().numpy(), ref)
        assert (sc.H, sc.W) == ((4, 5) if half else (8, 10))
        np.testing.assert_array_equal(sc.poses.cpu().numpy(), poses)
        assert list(sc.i_train) == [0, 1, 2] and sc.test_images.shape[0] == 2
        lo, hi = oracle.bbox_for_blender([torch.from_numpy(p) for p in poses[:3]], sc.H, sc.W, sc.focal)
        np.testing.assert_allclose(sc.bounding_box[0].numpy(), lo.numpy(), rtol=0, atol=1e-6)
        np.testing.assert_allclose(sc.bounding_box[1].numpy(), hi.numpy(), rtol=0, atol=1e-6)
    imgs, poses2, render_poses, hwf, i_split, box = load_blender_data(str(tmp_path), half_res=True)
    assert imgs.shape == (7, 4, 5, 4) and hwf[:2] == [4, 5] and render_poses.shape == (40, 4, 4)
    np.testing.assert_array_equal(imgs.cpu().numpy(), oracle.blender_images(rgba, True, "rgba"))


@pytest.mark.gpu
def test_ray_pool_epoch_is_a_permutation(hn):
    from hashnerf_pytorch_amd import functional as HF
    g = golden("pool_rays")
    H, W, K = int(g["H"]), int(g["W"]), g["K"]
    images = torch.from_numpy(g["images"]).to(DEV)
    poses = torch.from_numpy(g["poses"]).to(DEV)
    ids = torch.from_numpy(g["i_train"]).to(DEV, torch.int32)
    ref = g["rays_rgb"]                                   # [N, (ro, rd, rgb), 3]
    N = ref.shape[0]
    key = {tuple(r[1].view(np.uint32)) + tuple(r[2].view(np.uint32)): q for q, r in enumerate(ref)}
    orders = []
    for seed in (11, 12):
        parts = [HF.sample_pool(images, poses, ids, K, 2., 6., seed, s, min(512, N - s)) for s in range(0, N, 512)]
        rays = torch.cat([p[0] for p in parts]).cpu().numpy()
        tgt = torch.cat([p[1] for p in parts]).cpu().numpy()
        assert rays.shape == (N, 11)
        idx = [key.get(tuple(r[3:6].view(np.uint32)) + tuple(t.view(np.uint32)), -1) for r, t in zip(rays, tgt)]
        assert -1 not in idx, "every drawn ray is a pool ray, bit-exact (get_rays_np, float64 -> float32)"
        assert sorted(idx) == list(range(N)), "one epoch draws every pool ray exactly once"
        idx = np.array(idx)
        np.testing.assert_array_equal(rays[:, 0:3], ref[idx, 0])
        assert np.all(rays[:, 6] == 2.) and np.all(rays[:, 7] == 6.)
        vd = rays[:, 3:6] / np.linalg.norm(rays[:, 3:6], axis=-1, keepdims=True)
        np.testing.assert_allclose(rays[:, 8:11], vd, rtol=1e-6, atol=1e-7)
        orders.append(idx)
    assert not np.array_equal(orders[0], orders[1]), "a new epoch key reshuffles"


@pytest.mark.gpu
def test_trainer_use_batching_pool(hn):
    """Trainer with no_batching False walks the pool N_rand positions per step,
    the last batch of an epoch short, then a new epoch (run_nerf.py:544-555)."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(16, 16, 3, DEV, seed=0)             # pool of 768 rays
    tr = Trainer(default_args(N_rand=300, log2_hashmap_size=12, no_batching=False), data, DEV)
    sizes = []
    for _ in range(4):
        b = tr.draw_batch()
        sizes.append(b["rays"].shape[0])
        tr.global_step += 1
    assert sizes == [300, 300, 168, 300] and tr.epoch == 1 and tr.i_batch == 300
    loss, _ = tr.step()
    assert torch.isfinite(loss)
