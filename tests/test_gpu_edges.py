"""GPU edge cases of the fused render path (run_nerf_helpers.py:464-574 via
render, :310-392) against the CPU oracle, through the C ABI:

* ragged batches -- 1 ray, a batch that leaves the forward's last 4-ray
  block partial (67), and one where some persistent backward blocks own two
  rays and others one (300 > 256 blocks);
* BASELINE configs[2] at full size (T=22, finest 1024, 8192 rays) checked
  on a 16-ray subset: rays are independent, so the full-size forward and the
  gradient of a subset loss must match the oracle on that subset;
* an empty batch: render_rays returns empty outputs and a zero gradient
  (the library returns HN_OK without launching), render() raises like the
  reference's chunk assembly.

Same checks and tolerances as test_gpu_parity.test_fused_step_vs_oracle_on_device_z:
the oracle's fine pass runs on the device's importance samples (sample_pdf's
`denom < 1e-5` threshold, run_nerf_helpers.py:303, is discontinuous), and those
samples are checked against the oracle's own.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
T = 14
BOX = (torch.tensor([-4.0, -4.0, -3.4]), torch.tensor([4.0, 4.0, 3.3]))


def _close(a, b, rtol, atol, msg):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else a
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=msg)


def _rel(a, b, tol, msg):
    a = a.detach().cpu().numpy().astype(np.float64)
    b = b.detach().cpu().numpy().astype(np.float64)
    err = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
    assert err <= tol, f"{msg}: relative error {err:.3e}"


def _setup(hn, B, seed):
    torch.manual_seed(seed)
    emb = hn.HashEmbedder(BOX, log2_hashmap_size=T, finest_resolution=512).to(DEV)
    with torch.no_grad():
        emb.table.uniform_(-0.5, 0.5)
    kw = dict(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
              input_ch=32, input_ch_views=16)
    mc, mf = hn.NeRFSmall(**kw).to(DEV), hn.NeRFSmall(**kw).to(DEV)
    focal, K = hn.rays.blender_intrinsics(100, 100)
    c2w = hn.pose_spherical(40.0 + seed, -30.0, 4.0)
    ro, rd = hn.get_rays(100, 100, K, c2w[:3, :4].to(DEV))
    sel = torch.randperm(100 * 100, device=DEV)[:B]
    rays = torch.stack([ro.reshape(-1, 3)[sel], rd.reshape(-1, 3)[sel]], 0)
    return emb, mc, mf, K, rays


def _render(hn, emb, mc, mf, K, rays):
    from importlib import import_module
    HF = import_module("hashnerf_pytorch_amd.functional")
    nq = hn.NetworkQuery(emb, hn.SHEncoder())
    HF.DEBUG_KEEP = True
    try:
        out = hn.render(100, 100, K, rays=rays, network_query_fn=nq, perturb=1., N_importance=128,
                        network_fine=mf, N_samples=64, network_fn=mc, use_viewdirs=True, white_bkgd=True,
                        ndc=False, near=2., far=6., pytest=True, retraw=True)
    finally:
        HF.DEBUG_KEEP = False
    return out, HF.LAST.get("z_fine")


@pytest.mark.parametrize("B", [1, 67, 300])
def test_fused_step_ragged_batches(hn, oracle, B):
    O = oracle
    emb, mc, mf, K, rays = _setup(hn, B, seed=B)
    (rgb, depth, acc, ex), z_fine = _render(hn, emb, mc, mf, K, rays)
    target = torch.rand(B, 3, device=DEV)
    loss, _ = hn.training_loss(rgb, ex, target, 1e-3)
    loss.backward()
    # the oracle on the same inputs; pytest=True draws t_rand and u from
    # np.random.seed(0) (run_nerf_helpers.py:531-534, :288-291)
    ro, rd = rays[0].cpu(), rays[1].cpu()
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rb = torch.cat([ro, rd, 2. * torch.ones(B, 1), 6. * torch.ones(B, 1), vd], -1)
    np.random.seed(0)
    t_rand = torch.tensor(np.random.rand(B, 64), dtype=torch.float32)
    np.random.seed(0)
    u = torch.tensor(np.random.rand(B, 128), dtype=torch.float32)
    tab = emb.table.detach().cpu().requires_grad_(True)
    wc = {k: v.detach().cpu().requires_grad_(True) for k, v in zip(O.MLP_KEYS, mc.weights())}
    wf = {k: v.detach().cpu().requires_grad_(True) for k, v in zip(O.MLP_KEYS, mf.weights())}
    ret = O.render_rays(rb, wc, wf, tab, BOX[0], BOX[1], O.level_resolutions(16, 16, 512), T,
                        t_rand=t_rand, u=u, white_bkgd=True, z_fine=z_fine.cpu())
    same = np.isclose(z_fine.cpu().numpy(), ret["z_vals"].detach().numpy(), rtol=0, atol=1e-5)
    assert same.mean() > 0.97, f"only {same.mean():.4f} of fine samples agree"
    for k, a in (("rgb_map", rgb), ("depth_map", depth), ("acc_map", acc), ("rgb0", ex["rgb0"]),
                 ("sparsity_loss", ex["sparsity_loss"]), ("sparsity_loss0", ex["sparsity_loss0"])):
        _close(a, ret[k].detach().numpy(), rtol=1e-4, atol=2e-5, msg=f"B={B} {k}")
    ref_loss = O.training_loss(ret, target.cpu(), 1e-3)
    _close(loss.item(), ref_loss.item(), rtol=1e-5, atol=1e-7, msg=f"B={B} loss")
    ref_loss.backward()
    _rel(emb.table.grad, tab.grad, 5e-4, f"B={B} table grad")
    for w_dev, w_ref in ((mc.weights(), wc), (mf.weights(), wf)):
        for p, k in zip(w_dev, O.MLP_KEYS):
            _rel(p.grad, w_ref[k].grad, 5e-4, f"B={B} {k}")


def test_empty_batch(hn):
    """render_rays on an empty batch returns empty outputs (the reference's
    eager ops do) and a zero gradient; render() itself raises KeyError on an
    empty batch exactly like the reference's chunk assembly
    (run_nerf_helpers.py:373-390: no chunk runs, all_ret stays empty)."""
    emb, mc, mf, K, rays = _setup(hn, 0, seed=5)
    assert rays.shape == (2, 0, 3)
    with pytest.raises(KeyError):
        _render(hn, emb, mc, mf, K, rays)
    nq = hn.NetworkQuery(emb, hn.SHEncoder())
    rb = torch.zeros(0, 11, device=DEV)
    ret = hn.render_rays(rb, network_fn=mc, network_query_fn=nq, N_samples=64, retraw=True, perturb=1.,
                         N_importance=128, network_fine=mf, white_bkgd=True, pytest=True)
    assert ret["rgb_map"].shape == (0, 3) and ret["depth_map"].shape == (0,) and ret["acc_map"].shape == (0,)
    assert ret["raw"].shape[0] == 0 and ret["rgb0"].shape == (0, 3)
    loss = ret["rgb_map"].sum() + ret["rgb0"].sum() + ret["sparsity_loss"].sum()
    loss.backward()
    assert emb.table.grad is None or torch.count_nonzero(emb.table.grad) == 0


def test_config3_full_size_ray_subset(hn, oracle):
    """BASELINE configs[2] shapes -- T=22 (512 MiB table), finest 1024, 8192
    rays in one fused launch pair.  Rays are independent, so a loss on a
    16-ray subset has exactly that subset's gradient: the full-size forward
    must match the oracle on those rays, and the full-size backward (the
    other 8176 rays carry zero upstream gradient) must match the oracle's
    gradient of the same subset loss."""
    O = oracle
    Tb, finest, B, n = 22, 1024, 8192, 16
    torch.manual_seed(3)
    emb = hn.HashEmbedder(BOX, log2_hashmap_size=Tb, finest_resolution=finest).to(DEV)
    with torch.no_grad():
        emb.table.uniform_(-0.5, 0.5)
    kw = dict(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
              input_ch=32, input_ch_views=16)
    mc, mf = hn.NeRFSmall(**kw).to(DEV), hn.NeRFSmall(**kw).to(DEV)
    focal, K = hn.rays.blender_intrinsics(400, 400)
    ro, rd = hn.get_rays(400, 400, K, hn.pose_spherical(-60.0, -30.0, 4.0)[:3, :4].to(DEV))
    sel = torch.randperm(400 * 400, device=DEV)[:B]
    rays = torch.stack([ro.reshape(-1, 3)[sel], rd.reshape(-1, 3)[sel]], 0)
    from importlib import import_module
    HF = import_module("hashnerf_pytorch_amd.functional")
    nq = hn.NetworkQuery(emb, hn.SHEncoder())
    HF.DEBUG_KEEP = True
    try:
        rgb, depth, acc, ex = hn.render(400, 400, K, rays=rays, network_query_fn=nq, perturb=1., N_importance=128,
                                        network_fine=mf, N_samples=64, network_fn=mc, use_viewdirs=True,
                                        white_bkgd=True, ndc=False, near=2., far=6., pytest=True, retraw=True)
    finally:
        HF.DEBUG_KEEP = False
    z_fine = HF.LAST["z_fine"]
    assert torch.isfinite(rgb).all() and torch.isfinite(ex["rgb0"]).all() and torch.isfinite(acc).all()
    sub = torch.randperm(B, generator=torch.Generator().manual_seed(1))[:n]
    target = torch.rand(n, 3, generator=torch.Generator().manual_seed(2))
    subd = sub.to(DEV)
    loss = ((rgb[subd] - target.to(DEV)) ** 2).sum() + ((ex["rgb0"][subd] - target.to(DEV)) ** 2).sum()
    loss.backward()
    np.random.seed(0)
    t_rand = torch.tensor(np.random.rand(B, 64), dtype=torch.float32)[sub]
    np.random.seed(0)
    u = torch.tensor(np.random.rand(B, 128), dtype=torch.float32)[sub]
    r_o, r_d = rays[0][subd].cpu(), rays[1][subd].cpu()
    vd = r_d / torch.norm(r_d, dim=-1, keepdim=True)
    rb = torch.cat([r_o, r_d, 2. * torch.ones(n, 1), 6. * torch.ones(n, 1), vd], -1)
    tab = emb.table.detach().cpu().requires_grad_(True)
    wc = {k: v.detach().cpu().requires_grad_(True) for k, v in zip(O.MLP_KEYS, mc.weights())}
    wf = {k: v.detach().cpu().requires_grad_(True) for k, v in zip(O.MLP_KEYS, mf.weights())}
    ret = O.render_rays(rb, wc, wf, tab, BOX[0], BOX[1], O.level_resolutions(16, 16, finest), Tb,
                        t_rand=t_rand, u=u, white_bkgd=True, z_fine=z_fine[subd].cpu())
    same = np.isclose(z_fine[subd].cpu().numpy(), ret["z_vals"].detach().numpy(), rtol=0, atol=1e-5)
    assert same.mean() > 0.97, f"only {same.mean():.4f} of fine samples agree"
    for k, a in (("rgb_map", rgb), ("depth_map", depth), ("acc_map", acc), ("rgb0", ex["rgb0"])):
        _close(a[subd], ret[k].detach().numpy(), rtol=1e-4, atol=2e-5, msg=k)
    ref = ((ret["rgb_map"] - target) ** 2).sum() + ((ret["rgb0"] - target) ** 2).sum()
    ref.backward()
    _rel(emb.table.grad, tab.grad, 5e-4, "table grad (T=22)")
    for w_dev, w_ref in ((mc.weights(), wc), (mf.weights(), wf)):
        for p, k in zip(w_dev, O.MLP_KEYS):
            _rel(p.grad, w_ref[k].grad, 5e-4, k)
