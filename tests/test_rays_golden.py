"""SURVEY 8(a) row a14 on the product side: hashnerf-pytorch_amd/rays.py
against fixtures the reference itself produced (tests/golden/make_golden.py
gen_bbox_rays: ray_util.get_rays of cams[3] at 400x400, bbox.py's
get_bbox3d_for_blenderobj over 40 pose_spherical cameras).  CPU only."""
import numpy as np
import torch

from conftest import golden


def test_product_cameras_match_golden(hn):
    g = golden("bbox_rays")
    cams = hn.rays.blender_cameras(40)               # load/load_blender.py:30-35 poses
    np.testing.assert_array_equal(np.stack([c.numpy() for c in cams]), g["cams"])


def test_product_get_rays_match_golden(hn):
    """rays.get_rays (ray_util.py:62-80): bit-exact on the same host."""
    g = golden("bbox_rays")
    H, W = int(g["H"]), int(g["W"])
    c2w = torch.from_numpy(g["cams"][3][:3, :4])
    ro, rd = hn.rays.get_rays(H, W, g["K"], c2w)
    np.testing.assert_array_equal(rd.reshape(-1, 3)[g["sel"]].numpy(), g["rays_d"])
    np.testing.assert_array_equal(ro.reshape(-1, 3)[g["sel"]].numpy(), g["rays_o"])
    # get_rays_np (ray_util.py:82-93): float32 numpy, same values up to the
    # 3-term sum order of np.sum vs torch.sum
    ro_n, rd_n = hn.rays.get_rays_np(H, W, g["K"].astype(np.float32), g["cams"][3][:3, :4])
    np.testing.assert_allclose(rd_n.reshape(-1, 3)[g["sel"]], g["rays_d"], rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(ro_n.reshape(-1, 3)[g["sel"]], g["rays_o"])


def test_product_bbox_matches_golden(hn):
    """rays.bbox_for_blender (bbox.py:10-41): corners of every camera at near /
    far, min / max, padded by 1.0."""
    g = golden("bbox_rays")
    cams = [torch.from_numpy(c) for c in g["cams"]]
    lo, hi = hn.rays.bbox_for_blender(cams, int(g["H"]), int(g["W"]), float(g["focal"]))
    np.testing.assert_allclose(lo.numpy(), g["box_min"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(hi.numpy(), g["box_max"], rtol=0, atol=1e-6)


def test_product_intrinsics(hn):
    g = golden("bbox_rays")
    focal, K = hn.rays.blender_intrinsics(int(g["H"]), int(g["W"]))
    assert focal == float(g["focal"])
    np.testing.assert_array_equal(K, g["K"])
