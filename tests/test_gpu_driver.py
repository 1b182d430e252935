"""GPU tests of the training-step driver kernels (hn_sample_rays, hn_loss_*)
against the eager torch formulation of run_nerf.py:576-636 and ray_util.py.

* sampler: pixels distinct and inside the crop window; rays equal get_rays'
  rays of those pixels (rtol 1e-6: the same fp32 expressions; torch's
  3-term sum order is not specified) and targets equal the image pixels.
* loss: gradients bit-exact against torch autograd of the eager expression
  (same op order); the loss value within 1e-6 relative (fp64 vs pairwise
  fp32 reductions).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cam(hn):
    H = W = 64
    focal, K = hn.rays.blender_intrinsics(H, W)
    c2w = hn.pose_spherical(30.0, -30.0, 4.0)[:3, :4].float().to(DEV)
    g = torch.Generator().manual_seed(0)
    img = torch.rand((H, W, 3), generator=g).to(DEV)
    return H, W, K, c2w, img


@pytest.mark.parametrize("crop", [None, (16, 8, 32, 40)])
def test_sample_rays_matches_get_rays(hn, crop):
    from hashnerf_pytorch_amd import functional as HF
    H, W, K, c2w, img = _cam(hn)
    crop = crop or (0, 0, H, W)
    n = 1000 if crop[2] * crop[3] >= 1000 else crop[2] * crop[3]
    rays, target = HF.sample_rays(img, c2w, n, K, 2.0, 6.0, crop, seed=12345)
    rays_o, rays_d = hn.get_rays(H, W, K, c2w)
    # recover the pixel of each ray from its target colour position: compare
    # against every pixel's ray via the direction (unique per pixel)
    d_all = rays_d.reshape(-1, 3)
    dist = torch.cdist(rays[:, 3:6], d_all)
    pix = dist.argmin(1)
    assert pix.unique().numel() == n, "pixels drawn without replacement"
    py, px = pix // W, pix % W
    y0, x0, h, w = crop
    assert bool(((py >= y0) & (py < y0 + h) & (px >= x0) & (px < x0 + w)).all())
    torch.testing.assert_close(rays[:, 3:6], d_all[pix], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(rays[:, 0:3], rays_o.reshape(-1, 3)[pix], rtol=0, atol=0)
    assert torch.equal(rays[:, 6], torch.full((n,), 2.0, device=DEV))
    assert torch.equal(rays[:, 7], torch.full((n,), 6.0, device=DEV))
    vd = d_all[pix] / torch.norm(d_all[pix], dim=-1, keepdim=True)
    torch.testing.assert_close(rays[:, 8:11], vd, rtol=1e-6, atol=1e-6)
    assert torch.equal(target, img.reshape(-1, 3)[pix])


def test_sample_rays_full_window_is_a_permutation(hn):
    from hashnerf_pytorch_amd import functional as HF
    H, W, K, c2w, img = _cam(hn)
    rays, target = HF.sample_rays(img, c2w, H * W, K, 2.0, 6.0, (0, 0, H, W), seed=7)
    # every pixel exactly once: the targets are a permutation of the image
    a = target.cpu().numpy()
    b = img.reshape(-1, 3).cpu().numpy()
    assert np.array_equal(np.sort(a.view(np.uint32).view("V12").ravel()),
                          np.sort(b.view(np.uint32).view("V12").ravel()))
    r2, _ = HF.sample_rays(img, c2w, 256, K, 2.0, 6.0, (0, 0, H, W), seed=8)
    assert not torch.equal(rays[:256], r2), "seed changes the sample"


def _morton(row, col):
    key = np.zeros_like(row)
    for b in range(16):
        key |= ((row >> b) & 1) << (2 * b + 1) | ((col >> b) & 1) << (2 * b)
    return key


@pytest.mark.parametrize("crop,n", [((0, 0, 64, 64), 1000), ((16, 8, 32, 40), 700), ((0, 0, 64, 64), 1)])
def test_morton_sampler_same_draw_in_morton_order(hn, crop, n):
    """order=1 (hn_sample_rays_morton) returns exactly the draw of order=0
    (hn_sample_rays) for the same seed, listed in Morton order of the
    window-relative (row, col), deterministically."""
    from hashnerf_pytorch_amd import functional as HF
    H, W, K, c2w, img = _cam(hn)
    r0, t0 = HF.sample_rays(img, c2w, n, K, 2.0, 6.0, crop, seed=4242, order=0)
    r1, t1 = HF.sample_rays(img, c2w, n, K, 2.0, 6.0, crop, seed=4242, order=1)
    r1b, _ = HF.sample_rays(img, c2w, n, K, 2.0, 6.0, crop, seed=4242, order=1)
    assert torch.equal(r1, r1b), "deterministic"
    d_all = hn.get_rays(H, W, K, c2w)[1].reshape(-1, 3)
    p0 = torch.cdist(r0[:, 3:6], d_all).argmin(1).cpu().numpy()
    p1 = torch.cdist(r1[:, 3:6], d_all).argmin(1).cpu().numpy()
    assert np.array_equal(np.sort(p0), np.sort(p1)), "same set of pixels"
    y0, x0 = crop[0], crop[1]
    keys = _morton(p1 // W - y0, p1 % W - x0)
    assert np.all(np.diff(keys) > 0), "Morton order"
    # each ray keeps its own target colour
    order = np.argsort(p0)
    inv = np.argsort(p1)
    assert torch.equal(t0[torch.from_numpy(order).to(DEV)], t1[torch.from_numpy(inv).to(DEV)])


@pytest.mark.parametrize("world,tv", [(1, False), (2, True)])
def test_fused_loss_matches_eager(hn, world, tv):
    from hashnerf_pytorch_amd import functional as HF
    from hashnerf_pytorch_amd.train import dp_loss
    g = torch.Generator().manual_seed(3)
    B = 1000
    mk = lambda *s: torch.rand(s, generator=g).to(DEV).requires_grad_(True)
    rgb, rgb0, sp, sp0 = mk(B, 3), mk(B, 3), mk(B), mk(B)
    tvv = mk(16) if tv else None
    target = torch.rand((B, 3), generator=g).to(DEV)
    sw, tw = 1e-3, 1e-2
    loss, mse, mse0 = HF.train_loss(rgb, rgb0, target, sp, sp0, tvv, world, sw, tw)
    grads = torch.autograd.grad(loss, [rgb, rgb0, sp, sp0] + ([tvv] if tv else []))
    # eager reference: img2mse + dp_loss, as train.Trainer(fused=False) computes it
    m = torch.mean((rgb - target) ** 2)
    m0 = torch.mean((rgb0 - target) ** 2)
    ref = dp_loss(m, m0, sp.sum() + sp0.sum(), world, sw, tvv.sum() if tv else None, tw)
    rgrads = torch.autograd.grad(ref, [rgb, rgb0, sp, sp0] + ([tvv] if tv else []))
    for a, b in zip(grads, rgrads):
        assert torch.equal(a, b)
    torch.testing.assert_close(loss, ref, rtol=1e-6, atol=0)
    torch.testing.assert_close(mse, m.detach(), rtol=1e-6, atol=0)
    torch.testing.assert_close(mse0, m0.detach(), rtol=1e-6, atol=0)


@pytest.mark.parametrize("world,tv,B", [(1, False, 1000), (2, True, 4096), (1, True, 3)])
def test_loss_fwd_bwd_one_launch_bitwise(hn, world, tv, B):
    """hn_loss_fwd_bwd (the trainer's single launch) = hn_loss_fwd + hn_loss_bwd, bitwise."""
    from hashnerf_pytorch_amd import functional as HF
    g = torch.Generator().manual_seed(5)
    mk = lambda *s: torch.rand(s, generator=g).to(DEV)
    rgb, rgb0, sp, sp0, target = mk(B, 3), mk(B, 3), mk(B), mk(B), mk(B, 3)
    tvv = mk(5000) if tv else None       # n_tv > 3 B for the small batch: the grid covers it
    one = torch.ones((), device=DEV)
    consts = (world, 1e-3, 1e-2)
    out_a = HF.loss_fwd(rgb, rgb0, target, sp, sp0, tvv, *consts)
    g_a = HF.loss_bwd(rgb, rgb0, target, 0 if tvv is None else tvv.numel(), *consts, one)
    out_b, g_b = HF.loss_fwd_bwd(rgb, rgb0, target, sp, sp0, tvv, *consts, one)
    assert torch.equal(out_a, out_b)
    for a, b in zip(g_a, g_b):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)


def test_trainer_explicit_matches_autograd(hn):
    """The explicit launch sequence (mode="explicit") and the autograd module
    API (mode="autograd") give the same loss and gradients for the same seeds
    (rays, jitter, TV cubes): same kernels, only the float-atomic order of the
    table gradient differs."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(64, 64, 4, DEV, seed=0)
    res = {}
    for mode in ("explicit", "autograd"):
        args = default_args(N_rand=512, log2_hashmap_size=14, tv_loss_weight=1e-4, tv_until=10,
                            sparse_loss_weight=1e-3)
        tr = Trainer(args, data, DEV, mode=mode)
        tr.fuse_table_step = False           # keep the table gradient to compare
        torch.manual_seed(123)
        loss, mse = tr.step()
        res[mode] = (float(loss.detach()), float(mse), tr.embed_fn.table.grad.clone(),
                     [p.grad.clone() for p in tr.kw_train["network_fn"].weights() +
                      tr.kw_train["network_fine"].weights()])
    le, me, te, we = res["explicit"]
    la, ma, ta, wa = res["autograd"]
    assert abs(le - la) <= 1e-6 * abs(la) and me == ma
    assert float((te - ta).norm() / ta.norm()) < 1e-5
    for x, y in zip(we, wa):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-8)


@pytest.mark.gpu
def test_trainer_step_index_follows_reference_loop(hn):
    """Trainer.step() without an index uses the reference loop's
    i = global_step + 1 (run_nerf.py:538-541), so TV is on through i <= tv_until
    and the precrop window covers i < precrop_iters, also after a resume."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(32, 32, 2, DEV, seed=0)
    args = default_args(N_rand=64, log2_hashmap_size=12, tv_loss_weight=1e-4, tv_until=2)
    tr = Trainer(args, data, DEV)
    assert tr.global_step == 0 and args.tv_until == 2
    assert tr.draw_batch()["tv"] is not None          # i = 1
    tr.step()                                         # i = 1
    tr.step()                                         # i = 2 (last TV step)
    assert tr.global_step == 2
    assert tr.draw_batch()["tv"] is None              # i = 3 > tv_until
    assert default_args().tv_until == 1001            # run_nerf.py:636-638: TV through i = 1001


@pytest.mark.parametrize("tv", [0.0, 1e-4])
def test_trainer_fused_table_step_bitwise(hn, tv):
    """the trainer path that fuses the table's RAdam step into the
    binned owner pass (take_step -> render_bwd(table_step) -> step() of the
    MLP groups only) against the unfused path (gradient stored, hn_radam_step)
    from the same seed: table, moments and step counters bitwise equal after
    8 steps (the update starts at step 6, N_sma >= 5), without and with a TV
    term (whose gradient joins the owner pass as records, so the fused branch
    is taken in both)."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(64, 64, 4, DEV, seed=0)
    res = {}
    for fuse in (True, False):
        args = default_args(N_rand=512, log2_hashmap_size=14, tv_loss_weight=tv, tv_until=10 ** 6,
                            sparse_loss_weight=1e-3)
        tr = Trainer(args, data, DEV, seed=3)
        tr.fuse_table_step = fuse
        torch.manual_seed(11)
        for _ in range(8):
            tr.step()
        t = tr.embed_fn.table
        st = tr.optimizer.state[t]
        ws = tr.kw_train["network_fn"].weights() + tr.kw_train["network_fine"].weights()
        res[fuse] = (t.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(), st["step"],
                     [p.detach().clone() for p in ws], [tr.optimizer.state[p]["step"] for p in ws])
    a, b = res[True], res[False]
    for k in range(3):
        assert torch.equal(a[k], b[k]), k
    assert a[3] == b[3] == 8
    for x, y in zip(a[4], b[4]):
        assert torch.equal(x, y)
    assert a[5] == b[5] == [8] * 10


@pytest.mark.gpu
def test_device_fault_word_clear_after_fused_steps(hn):
    """The render backward's bounded waits never run out in a normal step:
    the sticky fault word (hn_device_faults) reads 0 after a few fused steps."""
    import ctypes as C
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(64, 64, 2, DEV, seed=0)    # precrop window 32x32 >= 300 rays
    tr = Trainer(default_args(N_rand=300, log2_hashmap_size=12), data, DEV)
    for _ in range(3):
        tr.step()
    w = C.c_int32(-1)
    assert hn._lib.lib().hn_device_faults(C.byref(w), 0) == 0
    assert w.value == 0
    hn._lib.check_device_faults()


@pytest.mark.parametrize("batching", [True, False], ids=["per_image", "pool"])
def test_trainer_prefetch_same_trajectory(hn, batching):
    """Trainer.prefetch: the next step's batch (device sampler, jitter and
    importance uniforms, TV cubes; or the use_batching pool) drawn on a side
    stream beside the backward gives bitwise the trajectory of drawing it at
    the step's start -- the same draws in the same order -- over 7 steps
    across the precrop boundary (precrop_iters 4) with TV through step 5."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(48, 48, 3, DEV, seed=0)
    res = {}
    for pf in (False, True):
        args = default_args(N_rand=256, log2_hashmap_size=13, tv_loss_weight=1e-4, tv_until=5,
                            precrop_iters=4, sparse_loss_weight=1e-3, no_batching=batching)
        tr = Trainer(args, data, DEV, seed=5)
        tr.prefetch = pf
        torch.manual_seed(17)
        losses = [float(tr.step()[0]) for _ in range(7)]
        ws = tr.kw_train["network_fn"].weights() + tr.kw_train["network_fine"].weights()
        res[pf] = (losses, tr.embed_fn.table.detach().clone(), [p.detach().clone() for p in ws])
    a, b = res[False], res[True]
    assert a[0] == b[0]
    assert torch.equal(a[1], b[1])
    for x, y in zip(a[2], b[2]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("world,tv", [(1, True), (2, False)])
def test_fused_loss_backward_matches_separate(hn, world, tv):
    """ABI 13: render_bwd(loss=...) forms the loss's gradients in its
    composite pre-pass and reduces the loss value there.  Against
    hn_loss_fwd_bwd + render_bwd(grads) on the same forward (4096 rays,
    T=19): the table and MLP gradients are bitwise equal (the same op forms),
    the loss value agrees to 1e-6 (fp64 sums, another thread count).  world=2
    applies the DP rule."""
    from hashnerf_pytorch_amd import functional as HF
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(200, 200, 4, DEV, seed=0, scene="procedural")
    args = default_args(N_rand=4096, log2_hashmap_size=19, tv_loss_weight=1e-3 if tv else 0.0,
                        tv_until=10 ** 6, sparse_loss_weight=1e-3)
    tr = Trainer(args, data, DEV, seed=1)
    tr._fused_setup()
    torch.manual_seed(3)
    b = tr.draw_batch(600)
    table = tr.embed_fn.table
    tvv = tvb = None
    if b["tv"] is not None:
        cubes, mv0 = b["tv"]
        tvv, mv = HF.tv_fwd(table, mv0, cubes, tr.embed_fn.log2_hashmap_size)
        tvb = (mv, cubes, torch.full_like(tvv, args.tv_loss_weight))
    consts = (world, args.sparse_loss_weight, args.tv_loss_weight)
    out, st = HF.render_fwd(tr._cfg, b["rays"], tr._t_vals, b["t_rand"], b["u"], None, None, table, tr._ws, True)
    lo_a, (g_rgb, g_rgb0, g_sp, g_sp0, g_tv) = HF.loss_fwd_bwd(out["rgb"], out["rgb0"], b["target"],
                                                               out["sparsity"], out["sparsity0"], tvv, *consts,
                                                               torch.ones((), device=DEV))
    if tvv is not None:
        assert torch.equal(g_tv, tvb[2])
    res = []
    for fused in (False, True):
        d_table = torch.empty_like(table)
        dws = HF.zeros_like_all(tr._ws)
        lo_b = torch.empty(4, device=DEV)
        grads = dict(g_rgb=g_rgb, g_sparsity=g_sp, g_rgb0=g_rgb0, g_sparsity0=g_sp0)
        loss = None if not fused else dict(
            target=b["target"], rgb=out["rgb"], rgb0=out["rgb0"], sparsity=out["sparsity"],
            sparsity0=out["sparsity0"], tv=tvv, world=world, sparse_w=args.sparse_loss_weight,
            tv_w=args.tv_loss_weight, out=lo_b)
        HF.render_bwd(st, {} if fused else grads, d_table, dws, overwrite=True, overwrite_mlp=True, tv=tvb,
                      loss=loss)
        torch.cuda.synchronize()
        res.append((d_table, dws, lo_b))
    assert torch.equal(res[0][0], res[1][0])
    for x, y in zip(res[0][1], res[1][1]):
        assert torch.equal(x, y)
    torch.testing.assert_close(res[1][2], lo_a, rtol=1e-6, atol=0)


def test_trainer_fused_loss_same_trajectory(hn):
    """Trainer.fuse_loss (ABI 13, the default) against the separate loss
    kernel: 8 steps (TV through step 5, the fused table
    step) leave table, moments and MLP weights bitwise equal; the losses agree
    to 1e-6."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(64, 64, 4, DEV, seed=0)
    res = {}
    for fl in (False, True):
        args = default_args(N_rand=512, log2_hashmap_size=14, tv_loss_weight=1e-4, tv_until=5,
                            sparse_loss_weight=1e-3)
        tr = Trainer(args, data, DEV, seed=3)
        tr.fuse_loss = fl
        torch.manual_seed(11)
        losses = [float(tr.step()[0]) for _ in range(8)]
        t = tr.embed_fn.table
        st = tr.optimizer.state[t]
        ws = tr.kw_train["network_fn"].weights() + tr.kw_train["network_fine"].weights()
        res[fl] = (losses, t.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone(),
                   [p.detach().clone() for p in ws])
    a, b = res[False], res[True]
    np.testing.assert_allclose(b[0], a[0], rtol=1e-6)
    for k in (1, 2, 3):
        assert torch.equal(a[k], b[k]), k
    for x, y in zip(a[4], b[4]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("shapes", [[(4096, 64), (4096, 128)], [(1000, 7)], [(3, 2_500_001), (17,)],
                                    [(8192, 64), (0, 5), (8192, 128)]])
def test_uniform_philox_matches_torch_rand(hn, shapes):
    """functional.torch_uniform (hn_uniform_philox, ABI 13) = torch.rand on
    the default generator, bit for bit, and leaves the generator's offset
    where the torch.rand calls leave it: the trainer's two draws, a ragged
    size, one big enough that torch's threads loop (components 1-3 and later
    Philox calls used), an empty draw between two."""
    from hashnerf_pytorch_amd import functional as HF
    torch.cuda.init()
    gen = torch.cuda.default_generators[torch.cuda.current_device()]
    torch.cuda.manual_seed(1234)
    torch.rand(5, device=DEV)                  # a nonzero starting offset
    off0 = gen.get_offset()
    ref = [torch.rand(s, device=DEV) for s in shapes]
    off_ref = gen.get_offset()
    gen.set_offset(off0)
    got = HF.torch_uniform(shapes, DEV)
    assert gen.get_offset() == off_ref
    for r, g in zip(ref, got):
        assert r.shape == g.shape and torch.equal(r, g)
    assert torch.equal(torch.rand(9, device=DEV), (gen.set_offset(off_ref), torch.rand(9, device=DEV))[1])


def test_sample_batch_morton_draws(hn):
    """sample_rays(uniforms=...) (hn_sample_batch_morton): the same rays and
    targets as hn_sample_rays_morton and the same numbers as two torch.rand
    calls after it, from one launch pair."""
    from hashnerf_pytorch_amd import functional as HF
    from hashnerf_pytorch_amd.train import SyntheticBlender
    d = SyntheticBlender(200, 200, 2, DEV, seed=0)
    args = (d.images[0], d.poses[0], 4096, d.K, 2., 6., (0, 0, 200, 200), 77)
    torch.cuda.manual_seed(9)
    r0, t0 = HF.sample_rays(*args)
    a = torch.rand((4096, 64), device=DEV)
    b = torch.rand((4096, 128), device=DEV)
    torch.cuda.manual_seed(9)
    r1, t1, a1, b1 = HF.sample_rays(*args, uniforms=[(4096, 64), (4096, 128)])
    for x, y in ((r0, r1), (t0, t1), (a, a1), (b, b1)):
        assert torch.equal(x, y)


def test_trainer_fused_mlp_step_same_trajectory(hn):
    """Trainer.fuse_mlp_step (ABI 13: the ten NeRFSmall RAdam steps applied in
    the backward's slab reduction, hn_render_bwd_args.mlp_step, and the
    stepped weights repacked for the next forward, which then skips its
    packing) against optimizer.step()'s hn_radam_step launch and the forward's
    own packing: 8 steps (the first five in RAdam's no-update mode, TV through
    step 5; a weight scaled in place after step 6, which must be repacked)
    leave the table, every weight and every moment bitwise equal."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    data = SyntheticBlender(64, 64, 4, DEV, seed=0)
    res = {}
    for fm in (False, True):
        args = default_args(N_rand=512, log2_hashmap_size=14, tv_loss_weight=1e-4, tv_until=5,
                            sparse_loss_weight=1e-3)
        tr = Trainer(args, data, DEV, seed=3)
        tr.fuse_mlp_step = fm
        torch.manual_seed(11)
        losses = [float(tr.step()[0]) for _ in range(6)]
        with torch.no_grad():
            tr._ws[3].mul_(0.5)             # the packed copies are stale now
        losses += [float(tr.step()[0]) for _ in range(2)]
        ws = tr.kw_train["network_fn"].weights() + tr.kw_train["network_fine"].weights()
        st = [tr.optimizer.state[p] for p in ws]
        res[fm] = (losses, tr.embed_fn.table.detach().clone(), [p.detach().clone() for p in ws],
                   [s["exp_avg"].clone() for s in st], [s["exp_avg_sq"].clone() for s in st],
                   [int(s["step"]) for s in st])
    a, b = res[False], res[True]
    assert a[0] == b[0] and a[5] == b[5]
    assert torch.equal(a[1], b[1])
    for k in (2, 3, 4):
        for x, y in zip(a[k], b[k]):
            assert torch.equal(x, y), k


def test_zero_gradient_skip_bitwise(hn):
    """Exact-zero skipping (ABI 14, hn_render_cfg.dense_bwd = 0, the default):
    a sample with relu(sigma) = 0 has alpha = 0 and weight 0, so raw2outputs'
    backward (run_nerf_helpers.py:577-628) gives it d raw = 0 exactly, and its
    MLP backward and table-gradient records are exact zeros.  The backward
    skips the MLP units whose 64 samples all have d raw = 0, the scatter reads
    no feature grads for such samples and writes no all-zero record.  After
    1000 training steps on the procedural chair (empty space learned: most
    samples have sigma <= 0) the table gradient and the ten NeRFSmall
    gradients of one batch equal those of the dense backward bitwise, up to
    the sign of zero (x + 0.0 normalises -0.0) for the table (exact integer
    sums), and within 1e-5 for the NeRFSmall gradients (the MLP backward's
    balanced unit lists give the two forms different per-wave groupings of the
    same products); each form is bitwise repeatable, and a large share of
    the units was skipped."""
    from hashnerf_pytorch_amd import functional as HF
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    # bench.py's configs[1] workload (400 x 400, 100 views, T=19, 4096 rays)
    data = SyntheticBlender(400, 400, 100, DEV, seed=0, scene="procedural")
    tr = Trainer(default_args(N_rand=4096, log2_hashmap_size=19, tv_loss_weight=1e-6), data, DEV, seed=0)
    for _ in range(1000):
        tr.step()
    tr.fuse_table_step = False
    batch = tr.draw_batch(2000)
    out = {}
    HF.DEBUG_KEEP = True
    try:
        for dense in (1, 0, 0):
            # the dense form's forward stores every tile's features (skip_dead_color off)
            tr._cfg.dense_bwd = dense
            tr.dense_bwd = bool(dense)
            tr._fused_forward_backward(2000, batch)
            torch.cuda.synchronize()
            HF.L.check_device_faults()
            g = [tr.embed_fn.table.grad] + [p.grad for p in tr._ws]
            out.setdefault(dense, []).append([x.detach().clone() + 0.0 for x in g])
        raw_f = HF.LAST["raw_f"][..., 3]
    finally:
        HF.DEBUG_KEEP = False
    skipped = (raw_f <= 0).view(-1, 3, 64).all(-1).float().mean().item()
    assert skipped > 0.3, f"only {skipped:.2f} of the fine units have no gradient"
    dense, sk, sk2 = out[1][0], out[0][0], out[0][1]
    assert torch.count_nonzero(dense[0]) > 0
    assert torch.equal(dense[0], sk[0]), "table gradient: skipping changed it"
    for k, (a, b, c) in enumerate(zip(dense, sk, sk2)):
        rel = float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))
        assert rel <= 1e-5, f"gradient {k}: skipped vs dense relative {rel:.3e}"
        assert torch.equal(b, c), f"gradient {k}: not repeatable"
