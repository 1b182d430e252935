"""The backward's two table-gradient scatters against each other and their
own properties (the embedding_dense_backward of hash_encoding.py:106 plus the
trilinear backward, summed over the coarse and fine passes of
run_nerf_helpers.py:538-558):

* binned (records per bin + exact fixed-point owner pass) vs float atomics on
  the same forward state: table gradients agree to 1e-6 relative norm (the
  atomic sums are fp32 in arbitrary order, the binned sums exact), MLP
  gradients to 1e-4 (the two schedules sum the tiles' dW in different orders);
* the binned table gradient is bitwise reproducible (integer sums), the
  atomic one is not required to be;
* d_table_mode=1 (overwrite) over garbage equals += into zeros; bit 1 does
  the same for the MLP gradients, which are bitwise reproducible too (static
  tile-to-wave map, fixed-order slab reduce);
* a small region capacity (cfg.bin_cap=64) pushes the hot bins' records
  through the shared overflow records: same gradient, no device fault;
* clumped input (a +-1 box inside the 2..6 sample range, bench config 5:
  every out-of-box sample clamps onto the box surface) spills a large share
  of the records, which the overflow holds in full;
* both against the oracle's gradient (the reference's algorithm) at
  T=19 / finest 512 with 4096 rays, the bench shape.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
BOX = (torch.tensor([-4.0, -4.0, -3.4]), torch.tensor([4.0, 4.0, 3.3]))


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float(torch.linalg.norm(a - b) / max(float(torch.linalg.norm(b)), 1e-30))


def _state(hn, B, T, seed, scatter, bin_cap=0, box=BOX, finest=512, sigma_sign=0):
    from importlib import import_module
    HF = import_module("hashnerf_pytorch_amd.functional")
    torch.manual_seed(seed)
    emb = hn.HashEmbedder(box, log2_hashmap_size=T, finest_resolution=finest).to(DEV)
    with torch.no_grad():
        emb.table.uniform_(-0.5, 0.5)
    kw = dict(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
              input_ch=32, input_ch_views=16)
    mc, mf = hn.NeRFSmall(**kw).to(DEV), hn.NeRFSmall(**kw).to(DEV)
    if sigma_sign:   # sigma = w . relu(h): all weights of one sign fix the sign of every raw sigma
        with torch.no_grad():
            for m in (mc, mf):
                w = m.sigma_net[1].weight
                w[0] = sigma_sign * w[0].abs()
    focal, K = hn.rays.blender_intrinsics(400, 400)
    ro, rd = hn.get_rays(400, 400, K, hn.pose_spherical(30.0 + seed, -30.0, 4.0)[:3, :4].to(DEV))
    sel = torch.randperm(400 * 400, device=DEV)[:B]
    ro, rd = ro.reshape(-1, 3)[sel], rd.reshape(-1, 3)[sel]
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rays = torch.cat([ro, rd, 2. * torch.ones_like(rd[:, :1]), 6. * torch.ones_like(rd[:, :1]), vd], -1)
    g = torch.Generator(device=DEV).manual_seed(seed + 1)
    t_rand = torch.rand((B, 64), device=DEV, generator=g)
    u = torch.rand((B, 128), device=DEV, generator=g)
    t_vals = torch.linspace(0., 1., 64, device=DEV)
    cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter=scatter)
    cfg.bin_cap = bin_cap
    ws = list(mc.weights()) + list(mf.weights())
    out, st = HF.render_fwd(cfg, rays, t_vals, t_rand, u, None, None, emb.table.detach(), ws, True)
    target = torch.rand((B, 3), device=DEV, generator=g)
    grads = dict(g_rgb=2. * (out["rgb"] - target) / (3 * B), g_rgb0=2. * (out["rgb0"] - target) / (3 * B),
                 g_sparsity=torch.full((B,), 1e-3, device=DEV), g_sparsity0=torch.full((B,), 1e-3, device=DEV))
    return HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads


def _bwd(HF, emb, ws, st, grads, overwrite=False, init=None, mlp_junk=False):
    d_table = torch.zeros_like(emb.table) if init is None else init.clone()
    dws = HF.zeros_like_all(ws)
    if mlp_junk:
        for d in dws:
            d.fill_(float("nan"))
    HF.render_bwd(st, grads, d_table, dws, overwrite=overwrite, overwrite_mlp=mlp_junk)
    torch.cuda.synchronize()
    HF.L.check_device_faults()
    return d_table, dws


@pytest.mark.parametrize("T,B", [(14, 300), (19, 4096)])
def test_binned_matches_atomic(hn, T, B):
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st_b, grads = _state(hn, B, T, 7, "binned")
    tb, wb = _bwd(HF, emb, ws, st_b, grads)
    *_, st_a, grads_a = _state(hn, B, T, 7, "atomic")
    ta, wa = _bwd(HF, emb, ws, st_a, grads_a)
    assert torch.count_nonzero(tb) > 0
    assert _rel(tb, ta) <= 1e-6, _rel(tb, ta)
    # same MLP backward, summed over the tiles in another order (split
    # schedule: wave 0 coarse, waves 1-3 fine) -- fp32 summation-order level
    rels = [_rel(x, y) for x, y in zip(wb, wa)]
    assert max(rels) <= 1e-4, rels


def test_binned_bitwise_reproducible_and_overwrite(hn):
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 2048, 19, 3, "binned")
    t1, _ = _bwd(HF, emb, ws, st, grads)
    t2, _ = _bwd(HF, emb, ws, st, grads)
    assert torch.equal(t1, t2), "binned table gradient changed between identical launches"
    junk = torch.full_like(emb.table, float("nan"))
    t3, _ = _bwd(HF, emb, ws, st, grads, overwrite=True, init=junk)
    assert torch.equal(t1, t3), "d_table_mode=1 must overwrite every entry"
    base = torch.randn_like(emb.table)
    t4, _ = _bwd(HF, emb, ws, st, grads, init=base)
    assert torch.equal(t4, base + t1), "d_table_mode=0 adds the gradient once"
    # d_table_mode bit 1: the MLP gradients are written over NaN garbage.  The
    # split schedule's tile-to-wave map is static and the slab reduce sums in
    # a fixed order, so this equals += into zeros bitwise
    _, w5 = _bwd(HF, emb, ws, st, grads, mlp_junk=True)
    _, w6 = _bwd(HF, emb, ws, st, grads)
    for x, y in zip(w5, w6):
        assert torch.isfinite(x).all()
        assert torch.equal(x, y)


def test_mlp_grads_bitwise_bench_shape(hn):
    """The ten NeRFSmall gradients of the binned backward are bitwise
    reproducible at the bench shape (4096 rays, T=19): every wave owns a fixed
    set of tiles (wave 0 the block's coarse units, wave w the fine part w - 1
    of each of the block's rays, in ray order), each dW block accumulates its
    tiles in that order, and the slab reduce combines the 256 x 4 slabs in a
    fixed order.  A lane-level fault of the kind round 3 saw in the forward
    (one ray's lanes 16-31 / 48-63 of a colour GEMM) would break this, where
    the former 1e-5 tolerance hid it.  Four launches."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 4096, 19, 23, "binned")
    t0, w0 = _bwd(HF, emb, ws, st, grads)
    assert all(torch.count_nonzero(x) > 0 for x in w0)
    for rep in range(3):
        t1, w1 = _bwd(HF, emb, ws, st, grads)
        assert torch.equal(t1, t0), f"repeat {rep}: table gradient"
        for k, (x, y) in enumerate(zip(w1, w0)):
            assert torch.equal(x, y), f"repeat {rep}: MLP gradient {k} differs"


def test_binned_overflow_records(hn):
    """cap 64 per (block, bin) region (sized: 256): the regions of the hot
    coarse-level bins of a 1024-ray batch spill into the shared overflow
    records; the owner pass picks them up."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 1024, 19, 5, "binned")
    t_full, _ = _bwd(HF, emb, ws, st, grads)
    *_, st_small, grads_small = _state(hn, 1024, 19, 5, "binned", bin_cap=64)
    t_small, _ = _bwd(HF, emb, ws, st_small, grads_small)
    assert _rel(t_small, t_full) <= 1e-6, _rel(t_small, t_full)


def test_binned_clumped_box(hn):
    """scannet-style box (bench config 5): samples mostly outside the box,
    the regions of the surface voxels' bins spill; binned == atomic."""
    box = (torch.tensor([-1.0, -1.0, -1.0]), torch.tensor([1.0, 1.0, 1.0]))
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st_b, grads = _state(hn, 4096, 19, 13, "binned", box=box)
    tb, wb = _bwd(HF, emb, ws, st_b, grads)
    *_, st_a, grads_a = _state(hn, 4096, 19, 13, "atomic", box=box)
    ta, wa = _bwd(HF, emb, ws, st_a, grads_a)
    assert torch.count_nonzero(tb) > 0
    assert _rel(tb, ta) <= 1e-6, _rel(tb, ta)
    rels = [_rel(x, y) for x, y in zip(wb, wa)]
    assert max(rels) <= 1e-4, rels
    # the same forward state with every region capped at 64 records (a
    # smaller layout inside the same workspace): most records spill
    st_b.cfg.bin_cap = 64
    ts, _ = _bwd(HF, emb, ws, st_b, grads)
    assert torch.equal(ts, tb), "spilled records must sum to the same (exact) gradient"


def test_forward_state_deterministic(hn):
    """Two forwards of the same seeded inputs give bitwise-equal state (the
    backward tests above compare separately built states)."""
    box = (torch.tensor([-1.0, -1.0, -1.0]), torch.tensor([1.0, 1.0, 1.0]))
    *_, s1, g1 = _state(hn, 1024, 19, 17, "binned", box=box)
    *_, s2, g2 = _state(hn, 1024, 19, 17, "binned", box=box)
    for name in ("z_f", "raw_c", "raw_f", "feat", "fine_src"):
        a, b = getattr(s1, name), getattr(s2, name)
        if name == "feat":   # compared bitwise: its ReLU mask words (ABI 10) read as floats include NaN patterns
            a, b = a.view(torch.int32), b.view(torch.int32)
        assert torch.equal(a, b), name
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k


def test_forward_deterministic_bench_shape(hn):
    """Repeated forwards at the bench shape (4096 rays, T=19) are bitwise
    equal.  Round 3 found the forward occasionally (1 in ~3-10 launches)
    giving ONE ray's points 16-31 of every tile a different colour-net result
    while the features and sigma matched: the per-tile SH GEMM on its hoisted
    operand; the SH half of color_net.0 now comes from one per-ray product in
    LDS (HN_FWD_C0SH) and 23 repeats matched (r03s).  Eight launches here."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st0, _ = _state(hn, 4096, 19, 7, "binned")
    cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter="binned")
    t_vals = torch.linspace(0., 1., 64, device=DEV)
    ref = {n: getattr(st0, n).clone() for n in ("z_f", "raw_c", "raw_f", "feat")}
    for rep in range(8):
        _, st = HF.render_fwd(cfg, rays, t_vals, t_rand, u, None, None, emb.table.detach(), ws, True)
        for n, want in ref.items():
            a, b = getattr(st, n), want
            if n == "feat":
                a, b = a.view(torch.int32), b.view(torch.int32)
            if not torch.equal(a, b):
                bad = (a != b).reshape(a.shape[0], -1).any(-1).nonzero().view(-1).tolist()
                raise AssertionError(f"repeat {rep}: {n} differs on rays {bad[:8]}")


def test_forward_deterministic_config3_shape(hn):
    """Repeated forwards at BASELINE configs[2]'s shape (T=22, finest 1024,
    8192 rays) are bitwise equal: features, ReLU mask words, z and raw of
    every ray (the round-3 fault class: one ray's colour-net lanes 16-31
    differing between launches).  Four launches."""
    B, T = 8192, 22
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st0, _ = _state(hn, B, T, 29, "binned", finest=1024)
    cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter="binned")
    t_vals = torch.linspace(0., 1., 64, device=DEV)
    ref = {n: getattr(st0, n).clone() for n in ("z_f", "raw_c", "raw_f", "feat")}
    for rep in range(4):
        _, st = HF.render_fwd(cfg, rays, t_vals, t_rand, u, None, None, emb.table.detach(), ws, True)
        for n, want in ref.items():
            a, b = getattr(st, n), want
            if n == "feat":
                a, b = a.view(torch.int32), b.view(torch.int32)
            if not torch.equal(a, b):
                bad = (a != b).reshape(a.shape[0], -1).any(-1).nonzero().view(-1).tolist()
                raise AssertionError(f"repeat {rep}: {n} differs on rays {bad[:8]}")
        del st


def test_binned_vs_oracle_bench_shape(hn, oracle):
    """T=19, finest 512, 4096 rays (BASELINE configs[1] shape): the binned
    table and MLP gradients against the oracle on a 32-ray subset of the
    loss (rays are independent, so the subset's gradient is exact)."""
    O = oracle
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, _ = _state(hn, 4096, 19, 11, "binned")
    n = 32
    sub = torch.randperm(4096, generator=torch.Generator().manual_seed(4))[:n].to(DEV)
    cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter="binned")
    fo, st = HF.render_fwd(cfg, rays, torch.linspace(0., 1., 64, device=DEV), t_rand, u, None, None,
                           emb.table.detach(), ws, True)
    g_rgb = torch.zeros((4096, 3), device=DEV)
    g_rgb0 = torch.zeros((4096, 3), device=DEV)
    g_rgb[sub] = 2. * (fo["rgb"][sub] - target[sub])
    g_rgb0[sub] = 2. * (fo["rgb0"][sub] - target[sub])
    d_table, dws = _bwd(HF, emb, ws, st, dict(g_rgb=g_rgb, g_rgb0=g_rgb0))
    tab = emb.table.detach().cpu().requires_grad_(True)
    wc = {k: v.detach().cpu().requires_grad_(True) for k, v in zip(O.MLP_KEYS, mc.weights())}
    wf = {k: v.detach().cpu().requires_grad_(True) for k, v in zip(O.MLP_KEYS, mf.weights())}
    ret = O.render_rays(rays[sub].cpu(), wc, wf, tab, BOX[0], BOX[1], O.level_resolutions(16, 16, 512), 19,
                        t_rand=t_rand[sub].cpu(), u=u[sub].cpu(), white_bkgd=True,
                        z_fine=fo["z_fine"][sub].cpu())
    same = np.isclose(fo["z_fine"][sub].cpu().numpy(), ret["z_vals"].detach().numpy(), rtol=0, atol=1e-5)
    assert same.mean() > 0.97, f"only {same.mean():.4f} of fine samples agree"
    ref = ((ret["rgb_map"] - target[sub].cpu()) ** 2).sum() + ((ret["rgb0"] - target[sub].cpu()) ** 2).sum()
    ref.backward()
    assert _rel(d_table, tab.grad) <= 5e-4, _rel(d_table, tab.grad)
    for p, w_ref in ((dws[:5], wc), (dws[5:], wf)):
        for x, k in zip(p, O.MLP_KEYS):
            assert _rel(x, w_ref[k].grad) <= 5e-4, (k, _rel(x, w_ref[k].grad))


def test_deferred_owner_ranges_bitwise(hn):
    """render_bwd(owner_defer=True) + render_bwd_owner over bin ranges (the
    data-parallel exchange's segments) writes exactly the table gradient of
    the one-call backward, range by range: bins not yet run keep the buffer's
    old contents."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 2048, 19, 9, "binned")
    ref, _ = _bwd(HF, emb, ws, st, grads, overwrite=True)
    nb, shift = HF.render_bins(st.cfg, 2048)
    assert nb == 1024 and shift == 13
    d = torch.full_like(emb.table, float("nan"))
    HF.render_bwd(st, grads, d, HF.zeros_like_all(ws), overwrite=True, owner_defer=True)
    flat, rflat, bf = d.view(-1), ref.view(-1), 2 << shift
    cuts = [0, 300, 301, 777, nb]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        HF.render_bwd_owner(st, lo, hi)
        torch.cuda.synchronize()
        assert torch.equal(flat[:hi * bf], rflat[:hi * bf]), (lo, hi)
        assert torch.isnan(flat[hi * bf:]).all()
    HF.L.check_device_faults()
    with pytest.raises(RuntimeError):
        HF.render_bwd_owner(st, 0, nb + 1)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_fused_table_step_bitwise(hn, mode):
    """The RAdam step fused into the owner pass (render_bwd(table_step=...))
    equals hn_radam_step on the gradient the same backward writes, bitwise,
    in each of RAdam's three update forms (radam.py:58-92: moments only while
    N_sma < 5 and step_size < 0, the SGD-like form, the rectified form)."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 2048, 19, 9, "binned")
    g = torch.Generator(device=DEV).manual_seed(5)
    p0 = emb.table.detach().clone()
    m0 = torch.randn(p0.shape, device=DEV, generator=g) * 1e-6
    v0 = torch.rand(p0.shape, device=DEV, generator=g) * 1e-10
    c = {"beta1": 0.9, "beta2": 0.99, "one_minus_beta1": 1 - 0.9, "one_minus_beta2": 1 - 0.99, "eps": 1e-15,
         "neg_wd_lr": 0.0, "neg_step_lr": -0.0421 * 0.01 if mode else 0.0, "mode": mode, "has_wd": 0}
    pf, mf_, vf = p0.clone(), m0.clone(), v0.clone()
    dws = HF.zeros_like_all(ws)
    HF.render_bwd(st, grads, None, dws, table_step=(pf, mf_, vf, c))
    d_table, _ = _bwd(HF, emb, ws, st, grads)
    pr, mr, vr = p0.clone(), m0.clone(), v0.clone()
    HF.radam_step([(pr, d_table, mr, vr, c)])
    torch.cuda.synchronize()
    assert torch.equal(mf_, mr) and torch.equal(vf, vr)
    assert torch.equal(pf, pr)
    if mode:
        assert not torch.equal(pf, p0)


@pytest.mark.parametrize("mode", [0, 2])
def test_fused_table_step_live_mask_bitwise(hn, mode):
    """The fused step with the live-pair bitmap (train.live_pair_mask: the
    coarse levels' row pairs outside the hashed (res+2)^3 corners are skipped)
    equals the dense hn_radam_step on the stored gradient, bitwise, when the
    dead rows' moments are zero (as they always are in training: no gradient
    ever reaches them).  Then the bitmap with one level's live pairs cleared:
    the owner sees gradient on a pair marked dead and raises fault bit 64."""
    from hashnerf_pytorch_amd.train import live_pair_mask, live_rows
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 2048, 19, 9, "binned")
    n_lv, words = live_pair_mask(emb.resolutions, 19)
    assert n_lv == 7
    words = words.to(DEV)
    _, rows = live_rows(emb.resolutions, 19)
    live = torch.zeros(16 << 19, dtype=torch.bool, device=DEV)
    live[rows.to(DEV)] = True
    live[n_lv << 19:] = True
    live = live.view(16, 1 << 19, 1)
    g = torch.Generator(device=DEV).manual_seed(5)
    p0 = emb.table.detach().clone()
    m0 = torch.randn(p0.shape, device=DEV, generator=g) * 1e-6 * live
    v0 = torch.rand(p0.shape, device=DEV, generator=g) * 1e-10 * live
    c = {"beta1": 0.9, "beta2": 0.99, "one_minus_beta1": 1 - 0.9, "one_minus_beta2": 1 - 0.99, "eps": 1e-15,
         "neg_wd_lr": 0.0, "neg_step_lr": -0.0421 * 0.01 if mode else 0.0, "mode": mode, "has_wd": 0}
    pf, mf_, vf = p0.clone(), m0.clone(), v0.clone()
    HF.render_bwd(st, grads, None, HF.zeros_like_all(ws), table_step=(pf, mf_, vf, c), table_live=(n_lv, words))
    d_table, _ = _bwd(HF, emb, ws, st, grads)
    assert torch.count_nonzero(d_table * ~live) == 0, "gradient outside train.live_rows"
    pr, mr, vr = p0.clone(), m0.clone(), v0.clone()
    HF.radam_step([(pr, d_table, mr, vr, c)])
    torch.cuda.synchronize()
    assert torch.equal(mf_, mr) and torch.equal(vf, vr)
    assert torch.equal(pf, pr)
    bad = words.clone()
    bad[(6 << 19) // 64:(7 << 19) // 64] = 0            # level 6 "dead"
    keep, HF.CHECK_FAULTS = HF.CHECK_FAULTS, False
    try:
        HF.render_bwd(st, grads, None, HF.zeros_like_all(ws), table_step=(p0.clone(), m0.clone(), v0.clone(), c),
                      table_live=(n_lv, bad))
    finally:
        HF.CHECK_FAULTS = keep
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="live mask"):
        HF.L.check_device_faults()


def test_nonfinite_gradient_raises_fault(hn):
    """A NaN upstream gradient on one ray: the reference's autograd carries it
    into embeddings[l].grad (hash_encoding.py:106); the binned owner pass's
    fixed-point sums cannot, so the scatter sets the sticky fault bit 32 and
    check_device_faults raises.  Clean inputs leave the
    word clear."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 512, 14, 21, "binned")
    _bwd(HF, emb, ws, st, grads)                      # clean: no fault (checked inside)
    bad = dict(grads)
    g = bad["g_rgb"].clone()
    g[7, 1] = float("nan")
    bad["g_rgb"] = g
    d_table = torch.zeros_like(emb.table)
    keep, HF.CHECK_FAULTS = HF.CHECK_FAULTS, False     # read the word here, not inside render_bwd
    try:
        HF.render_bwd(st, bad, d_table, HF.zeros_like_all(ws))
    finally:
        HF.CHECK_FAULTS = keep
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="non-finite"):
        HF.L.check_device_faults()
    HF.L.check_device_faults()                        # cleared by the raising read


def _tv_inputs(HF, emb, seed=3, g=1e-2):
    from importlib import import_module
    HL = import_module("hashnerf_pytorch_amd.loss")
    cubes, mv = HL.draw_tv_cubes(16, 16, 512, torch.Generator().manual_seed(seed))
    tv, mvd = HF.tv_fwd(emb.table.detach(), mv, cubes, emb.log2_hashmap_size)
    g_tv = torch.full((16,), g, device=DEV)
    return mvd, cubes, g_tv


def test_tv_records_match_tv_bwd(hn):
    """The TV term as owner-pass records (render_bwd(tv=...), VERDICT r02 item
    5) equals the render backward plus the standalone hn_tv_bwd (float
    atomics), loss.py:11-43, to fp32 summation order."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 1024, 19, 23, "binned")
    mvd, cubes, g_tv = _tv_inputs(HF, emb)
    d_a, _ = _bwd(HF, emb, ws, st, grads)
    HF.tv_bwd(emb.table.detach(), mvd, cubes, emb.log2_hashmap_size, g_tv, d_a)
    d_b = torch.zeros_like(emb.table)
    HF.render_bwd(st, grads, d_b, HF.zeros_like_all(ws), tv=(mvd, cubes, g_tv))
    torch.cuda.synchronize()
    HF.L.check_device_faults()
    tv_only = d_a - _bwd(HF, emb, ws, st, grads)[0]
    assert torch.count_nonzero(tv_only) > 0
    assert _rel(d_b, d_a) <= 1e-6, _rel(d_b, d_a)
    # TV-only difference resolved too (the render part cancels exactly: integer sums)
    assert _rel(d_b - _bwd(HF, emb, ws, st, grads)[0], tv_only) <= 1e-5


@pytest.mark.parametrize("T", [14, 19])
def test_tv_only_records_bitwise(hn, T):
    """hn_render_bwd with no rays and a TV term (ABI 14; a data-parallel rank
    that drew no rays, train.Trainer._empty_rank_grads): the TV gradient
    through the records and the exact owner pass equals hn_tv_bwd's float
    atomics (loss.py:11-43) to fp32 summation order, writes every entry
    (d_table_mode 1: a NaN-filled buffer comes back finite), is bitwise
    repeatable, and leaves the render workspace's packed weights alone."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 256, T, 29, "binned")
    mvd, cubes, g_tv = _tv_inputs(HF, emb, seed=7)
    table = emb.table.detach()
    d_a = torch.zeros_like(table)
    HF.tv_bwd(table, mvd, cubes, emb.log2_hashmap_size, g_tv, d_a)
    packed = st.wsb[:4 * 2 * 30208].clone()
    outs = []
    for _ in range(2):
        d_b = torch.full_like(table, float("nan"))
        HF.tv_bwd_records(st.cfg, table, mvd, cubes, g_tv, d_b, wsb=st.wsb)
        torch.cuda.synchronize()
        HF.L.check_device_faults()
        outs.append(d_b)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])
    assert torch.count_nonzero(d_a) > 0
    assert _rel(outs[0], d_a) <= 1e-6, _rel(outs[0], d_a)
    assert torch.equal(st.wsb[:4 * 2 * 30208], packed)
    # a fresh workspace of hn_render_workspace_bytes(cfg, 0) gives the same bits
    d_c = torch.full_like(table, float("nan"))
    HF.tv_bwd_records(st.cfg, table, mvd, cubes, g_tv, d_c)
    torch.cuda.synchronize()
    assert torch.equal(d_c, outs[0])


@pytest.mark.parametrize("mode", [1, 2])
def test_fused_table_step_with_tv_bitwise(hn, mode):
    """The fused table step with a TV term in the same owner pass equals
    hn_radam_step on the gradient the same backward (render + TV records)
    writes, bitwise."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 2048, 19, 9, "binned")
    mvd, cubes, g_tv = _tv_inputs(HF, emb, seed=5)
    g = torch.Generator(device=DEV).manual_seed(5)
    p0 = emb.table.detach().clone()
    m0 = torch.randn(p0.shape, device=DEV, generator=g) * 1e-6
    v0 = torch.rand(p0.shape, device=DEV, generator=g) * 1e-10
    c = {"beta1": 0.9, "beta2": 0.99, "one_minus_beta1": 1 - 0.9, "one_minus_beta2": 1 - 0.99, "eps": 1e-15,
         "neg_wd_lr": 0.0, "neg_step_lr": -0.0421 * 0.01, "mode": mode, "has_wd": 0}
    pf, mf_, vf = p0.clone(), m0.clone(), v0.clone()
    HF.render_bwd(st, grads, None, HF.zeros_like_all(ws), table_step=(pf, mf_, vf, c), tv=(mvd, cubes, g_tv))
    d_table = torch.zeros_like(emb.table)
    HF.render_bwd(st, grads, d_table, HF.zeros_like_all(ws), tv=(mvd, cubes, g_tv))
    pr, mr, vr = p0.clone(), m0.clone(), v0.clone()
    HF.radam_step([(pr, d_table, mr, vr, c)])
    torch.cuda.synchronize()
    HF.L.check_device_faults()
    assert torch.equal(mf_, mr) and torch.equal(vf, vr)
    assert torch.equal(pf, pr)


@pytest.mark.parametrize("perturb", [True, False])
def test_fine_z_sort_structure(hn, perturb):
    """sort(cat(z_vals, z_samples)) (run_nerf_helpers.py:551) in the forward
    (merge_sort_z: bitonic importance run merged with the sorted coarse run):
    every ray's fine z is non-decreasing, each coarse index appears exactly
    once in fine_src at its own value, and the 128 others are tagged 255; on a
    tie a coarse sample comes first (the rank sort's index order)."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, _ = _state(hn, 2048, 19, 23, "binned")
    if not perturb:   # det sampling: u = linspace, many exact ties between the rays' samples
        cfg = HF.make_render_cfg(emb.grid(), True, False, False, scatter="binned")
        t_vals = torch.linspace(0., 1., 64, device=DEV)
        u = torch.linspace(0., 1., 128, device=DEV).expand(2048, 128).contiguous()
        _, st = HF.render_fwd(cfg, rays, t_vals, None, u, None, None, emb.table.detach(), ws, True)
    zf, zc, src = st.z_f.cpu(), st.z_c.cpu(), st.fine_src.cpu().long()
    assert (zf[:, 1:] >= zf[:, :-1]).all()
    coarse = src < 64
    assert (coarse.sum(1) == 64).all() and ((src == 255) | coarse).all()
    pos = torch.full((zf.shape[0], 64), -1, dtype=torch.long)
    rows = torch.arange(zf.shape[0])[:, None].expand_as(src)
    pos[rows[coarse], src[coarse]] = torch.arange(192).expand_as(src)[coarse]
    assert (pos >= 0).all()
    assert torch.equal(torch.gather(zf, 1, pos), zc)
    # coarse first on ties: no importance sample equal to a coarse value sits before it
    prev = torch.cat([torch.full((zf.shape[0], 1), -1.0), zf[:, :-1]], 1)
    prev_tag = torch.cat([torch.zeros((zf.shape[0], 1), dtype=torch.long), src[:, :-1]], 1)
    assert not ((prev == zf) & coarse & (prev_tag == 255)).any()


@pytest.mark.parametrize("sign", [-1, 1])
def test_skip_extremes_match_dense(hn, sign):
    """Exact-zero skipping at its two ends (ABI 14 hn_render_cfg.dense_bwd):
    every raw sigma <= 0 (sign -1: no sample has a weight, every d raw is 0,
    the work lists are empty) and every raw sigma >= 0 (sign +1: nearly
    nothing to skip).  The skipping backward equals the dense one: the table
    gradient bitwise (exact integer sums), the ten NeRFSmall gradients within
    1e-5 (per-wave grouping), all exact zeros for sign -1; no device fault."""
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 1024, 16, 23, "binned",
                                                                     sigma_sign=sign)
    sig = torch.cat([st.raw_c[..., 3].reshape(-1), st.raw_f[..., 3].reshape(-1)])
    if sign < 0:
        assert bool((sig <= 0).all())
    else:
        assert float((sig > 0).float().mean()) > 0.9
    res = {}
    for dense in (1, 0):
        st.cfg.dense_bwd = dense
        res[dense] = _bwd(HF, emb, ws, st, grads)
    st.cfg.dense_bwd = 0
    (td, wd), (ts, wsk) = res[1], res[0]
    assert torch.equal(td + 0.0, ts + 0.0), "table gradient: skipping changed it"
    for k, (a, b) in enumerate(zip(wd, wsk)):
        if sign < 0:
            assert torch.count_nonzero(a) == 0 and torch.count_nonzero(b) == 0, f"gradient {k} not zero"
        else:
            rel = float((a.double() - b.double()).norm() / a.double().norm().clamp_min(1e-30))
            assert rel <= 1e-5, f"gradient {k}: skipped vs dense relative {rel:.3e}"
    if sign < 0:
        assert torch.count_nonzero(ts) == 0
    else:
        assert torch.count_nonzero(ts) > 0
