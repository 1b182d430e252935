"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU-only."""
import numpy as np
import pytest
import torch

from conftest import golden, pcg_table


def t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def test_hash_kat(oracle):
    g = golden("hash")
    for T in (12, 19, 22):
        h = oracle.spatial_hash(t(g["coords"]), T).numpy()
        np.testing.assert_array_equal(h, g[f"h{T}"])
    # (3,5,7)->329061, (1e5,2e5,3e5)->384640, (-3,-5,-7)->195227 at T=19
    assert list(g["h19"][:3]) == [329061, 384640, 195227]


@pytest.mark.parametrize("name", ["encode_t12", "encode_t12_f1024"])
def test_hash_encode_fwd_bwd(oracle, name):
    g = golden(name)
    res = oracle.level_resolutions(16, 16, int(g["finest"]))
    np.testing.assert_array_equal(np.array([float(r) for r in res], np.float32), g["resolutions"])
    tab = t(pcg_table(g["table_seed"], g["log2T"])).requires_grad_(True)
    feat, keep = oracle.hash_encode(t(g["x"]), tab, t(g["box_min"]), t(g["box_max"]), res, int(g["log2T"]))
    np.testing.assert_array_equal(feat.detach().numpy(), g["feat"])
    np.testing.assert_array_equal(keep.numpy(), g["keep"])
    assert keep.all()   # trap 3: keep_mask all-True for n_levels > 1
    (feat * t(g["dfeat"])).sum().backward()
    np.testing.assert_allclose(tab.grad.numpy(), g["grad"], rtol=1e-6, atol=1e-7)


def test_sh(oracle):
    g = golden("sh")
    np.testing.assert_array_equal(oracle.sh_encode(t(g["dirs"])).numpy(), g["out"])


def test_mlp(oracle):
    g = golden("mlp")
    w = {k: t(g["w:" + k]).clone().requires_grad_(True) for k in oracle.MLP_KEYS}
    x = t(g["x"]).clone().requires_grad_(True)
    out = oracle.nerf_small(x, w)
    np.testing.assert_allclose(out.detach().numpy(), g["out"], rtol=1e-5, atol=1e-6)
    (out * t(g["dout"])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), g["dx"], rtol=1e-5, atol=1e-6)
    for k in oracle.MLP_KEYS:
        np.testing.assert_allclose(w[k].grad.numpy(), g["g:" + k], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("white", [False, True])
def test_raw2outputs(oracle, white):
    g = golden("raw2outputs")
    s = "_w" if white else ""
    raw = t(g["raw"]).clone().requires_grad_(True)
    rgb, disp, acc, w, depth, ent = oracle.raw2outputs(raw, t(g["z"]), t(g["rays_d"]), None, white)
    np.testing.assert_array_equal(rgb.detach().numpy(), g["rgb" + s])
    np.testing.assert_array_equal(w.detach().numpy(), g["weights" + s])
    np.testing.assert_array_equal(depth.detach().numpy(), g["depth" + s])   # NaN row 0
    assert np.isnan(g["depth" + s][0])
    np.testing.assert_array_equal(ent.detach().numpy(), g["entropy" + s])
    loss = (rgb * t(g["grgb" + s])).sum() + (ent * t(g["gent" + s])).sum() + (acc * t(g["gacc" + s])).sum()
    loss.backward()
    np.testing.assert_array_equal(raw.grad.numpy(), g["draw" + s])


def test_sample_pdf(oracle):
    g = golden("sample_pdf")
    s = oracle.sample_pdf(t(g["bins"]), t(g["weights"]), t(g["u"]))
    np.testing.assert_array_equal(s.numpy(), g["samples"])
    ud = torch.linspace(0., 1., 128).expand(g["bins"].shape[0], 128)
    np.testing.assert_array_equal(oracle.sample_pdf(t(g["bins"]), t(g["weights"]), ud).numpy(),
                                  g["samples_det"])


def test_bbox_and_rays(oracle):
    g = golden("bbox_rays")
    cams = [t(c) for c in g["cams"]]
    lo, hi = oracle.bbox_for_blender(cams, int(g["H"]), int(g["W"]), float(g["focal"]))
    np.testing.assert_allclose(lo.numpy(), g["box_min"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(hi.numpy(), g["box_max"], rtol=0, atol=1e-6)
    ro, rd = oracle.get_rays(int(g["H"]), int(g["W"]), g["K"], cams[3][:3, :4])
    np.testing.assert_array_equal(rd.reshape(-1, 3)[g["sel"]].numpy(), g["rays_d"])
    np.testing.assert_array_equal(ro.reshape(-1, 3)[g["sel"]].numpy(), g["rays_o"])


@pytest.mark.parametrize("finest", [512, 1024])
def test_tv(oracle, finest):
    g = golden(f"tv_f{finest}")
    tab = t(pcg_table(g["table_seed"], g["log2T"]))
    for l in range(16):
        tl = tab[l].clone().requires_grad_(True)
        v = oracle.total_variation_loss(tl, l, t(g["min_vertex"][l]), int(g["log2T"]),
                                        finest_res=finest)
        np.testing.assert_allclose(v.item(), g["tv"][l], rtol=1e-6)
        v.backward()
        np.testing.assert_allclose(tl.grad.numpy(), g["grad"][l], rtol=1e-6, atol=1e-9)


def test_radam_trace(oracle):
    g = golden("radam")
    pa, pb = t(g["p0"]).clone(), t(g["t0"]).clone()
    sa = [torch.zeros_like(pa), torch.zeros_like(pa)]
    sb = [torch.zeros_like(pb), torch.zeros_like(pb)]
    lr = 0.01
    for step in range(8):
        oracle.radam_step(pa, t(g["ga"][step]), sa[0], sa[1], step + 1, lr, weight_decay=1e-6)
        oracle.radam_step(pb, t(g["gb"][step]), sb[0], sb[1], step + 1, lr, eps=1e-15)
        np.testing.assert_array_equal(pa.numpy(), g["pa"][step])
        np.testing.assert_array_equal(pb.numpy(), g["pb"][step])
        if step < 5:   # trap 6: no update for the first five steps
            np.testing.assert_array_equal(pa.numpy(), g["p0"])
        lr = 0.01 * (0.1 ** ((step + 1) / 500000))


def _render_inputs(g, oracle):
    tab = t(pcg_table(g["table_seed"], g["log2T"])).requires_grad_(True)
    res = oracle.level_resolutions(16, 16, int(g["finest"]))
    rays_o, rays_d = t(g["rays_o"]), t(g["rays_d"])
    viewdirs = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    B = rays_o.shape[0]
    rb = torch.cat([rays_o, rays_d, 2. * torch.ones(B, 1), 6. * torch.ones(B, 1), viewdirs], -1)
    wc = {k: t(g["wc:" + k]).clone().requires_grad_(True) for k in oracle.MLP_KEYS}
    wf = {k: t(g["wf:" + k]).clone().requires_grad_(True) for k in oracle.MLP_KEYS}
    perturb = float(g["perturb"]) > 0
    return tab, res, rb, wc, wf, (t(g["t_rand"]) if perturb else None), t(g["u"])


@pytest.mark.parametrize("name", ["render_white_perturb", "render_black_det"])
def test_render_rays_step(oracle, name):
    g = golden(name)
    tab, res, rb, wc, wf, t_rand, u = _render_inputs(g, oracle)
    ret = oracle.render_rays(rb, wc, wf, tab, t(g["box_min"]), t(g["box_max"]), res, int(g["log2T"]),
                             t_rand=t_rand, u=u, white_bkgd=bool(g["white"]))
    for k, gk in (("rgb_map", "rgb"), ("depth_map", "depth"), ("acc_map", "acc"), ("rgb0", "rgb0"),
                  ("depth0", "depth0"), ("acc0", "acc0"), ("sparsity_loss", "sparsity_loss"),
                  ("sparsity_loss0", "sparsity_loss0"), ("z_std", "z_std"), ("raw", "raw")):
        np.testing.assert_allclose(ret[k].detach().numpy(), g[gk], rtol=1e-5, atol=1e-6, err_msg=k)
    loss = oracle.training_loss(ret, t(g["target"]), float(g["sparse_w"]))
    np.testing.assert_allclose(loss.item(), g["loss"], rtol=1e-6)
    loss.backward()
    np.testing.assert_allclose(tab.grad.numpy(), g["table_grad"], rtol=1e-4, atol=1e-8)
    for tag, w in (("c", wc), ("f", wf)):
        for k in oracle.MLP_KEYS:
            np.testing.assert_allclose(w[k].grad.numpy(), g[f"g{tag}:{k}"], rtol=1e-4, atol=1e-7)


def test_ndc_rays_bitexact_vs_reference(hn):
    """rays.get_ndc_rays against ray_util.get_ndc_rays (golden, same op order)."""
    g = golden("ndc")
    o, d = hn.get_ndc_rays(int(g["H"]), int(g["W"]), float(g["focal"]), float(g["near"]),
                           torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"]))
    np.testing.assert_array_equal(o.numpy(), g["ndc_o"])
    np.testing.assert_array_equal(d.numpy(), g["ndc_d"])
