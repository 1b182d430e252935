"""Data-parallel semantics on CPU with world_size=2 over gloo.

(1) allreduce_grads sums the hash-table gradient and the flattened MLP
    gradients across ranks.
(2) The per-rank loss rule (train.dp_loss: MSE / world, entropy sums not
    scaled, TV on one rank) makes the SUM-all-reduced gradient equal to the
    reference loss gradient over the global batch (run_nerf.py:612-636).
    Checked with the CPU oracle as the renderer (test infrastructure only).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(B=24, T=12):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import hashnerf_oracle as O
    g = torch.Generator().manual_seed(7)
    box = (torch.tensor([-4.0, -4.0, -3.4]), torch.tensor([4.0, 4.0, 3.3]))
    tab = (torch.rand(16, 2 ** T, 2, generator=g) * 2 - 1) * 0.5
    wc = O.init_nerf_small(g)
    wf = O.init_nerf_small(g)
    c2w = O.pose_spherical(20.0, -30.0, 4.0)
    focal = 0.5 * 100 / np.tan(0.5 * 0.6911112070083618)
    K = np.array([[focal, 0, 50.0], [0, focal, 50.0], [0, 0, 1]])
    ro, rd = O.get_rays(100, 100, K, c2w[:3, :4])
    sel = torch.randperm(100 * 100, generator=g)[:B]
    ro, rd = ro.reshape(-1, 3)[sel], rd.reshape(-1, 3)[sel]
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rb = torch.cat([ro, rd, 2 * torch.ones(B, 1), 6 * torch.ones(B, 1), vd], -1)
    t_rand = torch.rand(B, 64, generator=g)
    u = torch.rand(B, 128, generator=g)
    target = torch.rand(B, 3, generator=g)
    mv = torch.stack([torch.randint(0, 5, (3,), generator=g) for _ in range(16)])
    return O, box, tab, wc, wf, rb, t_rand, u, target, mv, T


def _grads(O, box, tab, wc, wf, rb, t_rand, u, target, mv, T, loss_fn):
    tab = tab.clone().requires_grad_(True)
    wc = {k: v.clone().requires_grad_(True) for k, v in wc.items()}
    wf = {k: v.clone().requires_grad_(True) for k, v in wf.items()}
    ret = O.render_rays(rb, wc, wf, tab, box[0], box[1], O.level_resolutions(16, 16, 512), T,
                        t_rand=t_rand, u=u, white_bkgd=True)
    tv = sum(O.total_variation_loss(tab[l], l, mv[l], T) for l in range(16))
    loss = loss_fn(ret, target, tv)
    loss.backward()
    return tab, [wc[k] for k in O.MLP_KEYS] + [wf[k] for k in O.MLP_KEYS]


def _worker(rank, world, port, out_path, T=12):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd.train import allreduce_grads, dp_loss, live_rows
    O, box, tab, wc, wf, rb, t_rand, u, target, mv, T = _scene(T=T)
    B = rb.shape[0]
    sl = slice(rank * B // world, (rank + 1) * B // world)

    def loss_fn(ret, tgt, tv):
        mse = torch.mean((ret["rgb_map"] - tgt) ** 2)
        mse0 = torch.mean((ret["rgb0"] - tgt) ** 2)
        ent = ret["sparsity_loss"].sum() + ret["sparsity_loss0"].sum()
        return dp_loss(mse, mse0, ent, world, 1e-3, tv if rank == 0 else None, 1e-2)

    tab_g, mlp = _grads(O, box, tab, wc, wf, rb[sl], t_rand[sl], u[sl], target[sl], mv, T, loss_fn)
    # T=16: levels 0-3 go through the compacted live-row bucket
    allreduce_grads(tab_g, mlp, live=live_rows(O.level_resolutions(16, 16, 512), T))
    if rank == 0:
        torch.save({"table": tab_g.grad, "mlp": [p.grad for p in mlp]}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_grads_sums(tmp_path):
    port = _free_port()
    mp.spawn(_allreduce_worker, args=(2, port, str(tmp_path / "ar.pt")), nprocs=2, join=True)
    got = torch.load(tmp_path / "ar.pt", weights_only=True)
    assert torch.equal(got["table"], torch.full((3, 8, 2), 3.0))
    assert torch.equal(got["mlp"][0], torch.full((4, 5), 30.0))
    assert torch.equal(got["mlp"][1], torch.full((7,), 300.0))


def _allreduce_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd.train import allreduce_grads
    table = torch.nn.Parameter(torch.zeros(3, 8, 2))
    table.grad = torch.full((3, 8, 2), float(rank + 1))
    ps = [torch.nn.Parameter(torch.zeros(4, 5)), torch.nn.Parameter(torch.zeros(7))]
    ps[0].grad = torch.full((4, 5), 10.0 * (rank + 1))
    ps[1].grad = torch.full((7,), 100.0 * (rank + 1))
    allreduce_grads(table, ps)
    if rank == 0:
        torch.save({"table": table.grad, "mlp": [p.grad for p in ps]}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("T", [12, 16])
def test_dp_gradient_equals_global_batch(tmp_path, T):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path / "dp.pt"), T), nprocs=2, join=True)
    got = torch.load(tmp_path / "dp.pt", weights_only=True)
    O, box, tab, wc, wf, rb, t_rand, u, target, mv, T = _scene(T=T)

    def ref_loss(ret, tgt, tv):   # run_nerf.py:612-636 on the whole batch
        return (torch.mean((ret["rgb_map"] - tgt) ** 2) + torch.mean((ret["rgb0"] - tgt) ** 2)
                + 1e-3 * (ret["sparsity_loss"].sum() + ret["sparsity_loss0"].sum()) + 1e-2 * tv)

    tab_g, mlp = _grads(O, box, tab, wc, wf, rb, t_rand, u, target, mv, T, ref_loss)
    ref = tab_g.grad
    err = (got["table"] - ref).norm() / ref.norm()
    assert err < 1e-5, err
    for a, p in zip(got["mlp"], mlp):
        e = (a - p.grad).norm() / p.grad.norm()
        assert e < 1e-5, e


def test_live_rows_cover_every_gradient():
    """The rows allreduce_grads leaves out (train.live_rows) carry no gradient:
    render + TV backward of the oracle with samples outside the bbox (clamped
    corners, hash_encoding.py:66-76) and TV cubes at the far corner of the grid."""
    import sys
    sys.path.insert(0, ROOT)
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd.train import live_rows
    O, box, tab, wc, wf, rb, t_rand, u, target, mv, T = _scene(T=16)
    res = O.level_resolutions(16, 16, 512)
    mv = torch.stack([torch.tensor([int(r) - int(O.tv_cube(l, 16, 16, 512)[1]) - 1] * 3) for l, r in enumerate(res)])

    def loss_fn(ret, tgt, tv):
        return (torch.mean((ret["rgb_map"] - tgt) ** 2) + 1e-3 * ret["sparsity_loss"].sum() + 1e-2 * tv)

    tab_g, _ = _grads(O, box, tab, wc, wf, rb, t_rand, u, target, mv, T, loss_fn)
    n_lv, rows = live_rows(res, T)
    assert n_lv == 4
    head = tab_g.grad[:n_lv].reshape(-1, 2)
    dead = torch.ones(head.shape[0], dtype=torch.bool)
    dead[rows] = False
    assert head[~dead].abs().sum() > 0
    assert torch.count_nonzero(head[dead]) == 0


def test_live_pair_mask_matches_live_rows():
    """train.live_pair_mask (hn_render_bwd_args.table_live) sets exactly the
    pairs (R >> 1) of the rows live_rows returns, at T=19 / finest 512 (levels
    0-6) and T=22 / finest 1024 (levels 0-8)."""
    import sys
    sys.path.insert(0, ROOT)
    import hn_loader
    hn_loader.load()
    import numpy as np
    from hashnerf_pytorch_amd.embedding import level_resolutions
    from hashnerf_pytorch_amd.train import live_pair_mask, live_rows
    for T, fin, want in ((19, 512, 7), (22, 1024, 9)):
        _, res = level_resolutions(16, 16, fin)
        n_lv, rows = live_rows(res, T)
        n2, words = live_pair_mask(res, T)
        assert n_lv == n2 == want and words.dtype == torch.int32 and words.numel() == n_lv << (T - 6)
        bits = np.unpackbits(words.numpy().view(np.uint8), bitorder="little").astype(bool)
        expect = np.zeros(n_lv << (T - 1), dtype=bool)
        expect[rows.numpy() >> 1] = True
        assert np.array_equal(bits, expect)


def _toy_step(tensors):
    """A per-element stand-in for hn_radam_step (test infrastructure): the
    sharded step's index math does not depend on the update's form, and
    p, m, v stay untouched where g = m = v = 0 (the dead rows), as RAdam's do."""
    for p, g, m, v, c in tensors:
        m.mul_(c["beta1"]).add_(g)
        v.mul_(c["beta2"]).addcmul_(g, g)
        p.sub_(c["lr"] * m / (v.sqrt() + 1.0))


def _sharded_worker(rank, world, port, out_path, n_chunks=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd.train import ShardedTableStep
    L_, R, F_ = 4, 64, 2
    g0 = torch.Generator().manual_seed(11)
    rows = torch.tensor([0, 3, 5, 17, 40, 63, 64 + 2, 64 + 9, 64 + 33], dtype=torch.int64)   # levels 0-1 sparse
    live = (2, rows)
    dead = torch.ones(2 * R, dtype=torch.bool)
    dead[rows] = False
    p0 = torch.randn(L_, R, F_, generator=g0)
    m0 = torch.randn(L_, R, F_, generator=g0)
    v0 = torch.rand(L_, R, F_, generator=g0)
    m0[:2] = m0[:2].reshape(-1, F_).masked_fill(dead[:, None], 0).view(2, R, F_)
    v0[:2] = v0[:2].reshape(-1, F_).masked_fill(dead[:, None], 0).view(2, R, F_)
    c = {"beta1": 0.9, "beta2": 0.99, "lr": 0.05}

    def grads(step):
        out = []
        for r in range(world):
            g = torch.randn(L_, R, F_, generator=torch.Generator().manual_seed(100 * step + r))
            g[:2] = g[:2].reshape(-1, F_).masked_fill(dead[:, None], 0).view(2, R, F_)
            out.append(g)
        return out

    def run(emulate):
        # n_chunks > 1: bins of 16 rows (32 floats), the exchange in bin-aligned
        # segments, each segment's gradient formed just before its exchange (the
        # trainer's deferred owner pass) over a gradient buffer holding NaN
        table = torch.nn.Parameter(p0.clone())
        bins = (L_ * R // 16, 4) if n_chunks > 1 else None
        xs = ShardedTableStep(table, live, rank, world, state={"exp_avg": m0, "exp_avg_sq": v0},
                              stepper=_toy_step, bins=bins, n_chunks=n_chunks, emulate=emulate)
        # default on host tensors: the production calls (reduce_scatter_tensor
        # with async_op, in-place all_gather_into_tensor), as an RCCL run makes them
        assert xs.coll.emulate == bool(emulate)
        assert len(xs.segs) == (3 if n_chunks > 1 else 1)
        for step in range(3):
            g = grads(step)[rank]
            if n_chunks > 1:
                xs.grad_view().fill_(float("nan"))

                def produce(k, g=g):
                    lo, hi = xs.seg_bins[k]
                    xs.grad_view().view(-1)[lo * 32:hi * 32] = g.reshape(-1)[lo * 32:hi * 32]
                xs.step(c, produce=produce)
            else:
                xs.grad_view().copy_(g)
                xs.step(c)
        assert xs.stale
        m, v = xs.gather_state()
        assert not xs.stale
        return table.detach().clone(), m, v

    p_n, m_n, v_n = run(None)     # production collectives
    p_e, m_e, v_e = run(True)     # the emulation (gloo on device tensors)
    # reference: the summed gradient, the dense update over the whole table
    pr, mr, vr = p0.clone(), m0.clone(), v0.clone()
    for step in range(3):
        _toy_step([(pr, sum(grads(step)), mr, vr, c)])
    if rank == 0:
        torch.save({"p": p_n, "m": m_n, "v": v_n, "pe": p_e, "me": m_e, "ve": v_e,
                    "pr": pr, "mr": mr, "vr": vr}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_chunks", [1, 3])
def test_sharded_table_step_matches_dense(tmp_path, n_chunks):
    """train.ShardedTableStep through train.Collectives: the production calls
    (reduce_scatter_tensor with async_op, in-place all_gather_into_tensor) on
    gloo, and the emulation into the same out-tensors and offsets, give
    bitwise the same result; 3 steps from loaded moments (a resumed run) leave
    the table and the gathered moments equal to the summed-gradient dense
    update; the dead coarse rows stay untouched.  n_chunks=3: the same in
    bin-aligned segments, each formed (produce) right before its exchange."""
    port = _free_port()
    mp.spawn(_sharded_worker, args=(2, port, str(tmp_path / "sh.pt"), n_chunks), nprocs=2, join=True)
    got = torch.load(tmp_path / "sh.pt", weights_only=True)
    for k in ("p", "m", "v"):   # production calls and emulation: bitwise the same step
        assert torch.equal(got[k], got[k + "e"]), k
    torch.testing.assert_close(got["p"], got["pr"], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(got["m"], got["mr"], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(got["v"], got["vr"], rtol=1e-6, atol=1e-7)


def test_sharded_state_dict_refuses_stale_moments():
    """RAdam.state_dict() raises while a sharded table step holds newer
    moments than the optimizer (a checkpoint would silently keep stale ones)."""
    import sys
    import types
    sys.path.insert(0, ROOT)
    import hn_loader
    hn = hn_loader.load()
    p = torch.nn.Parameter(torch.zeros(4))
    opt = hn.RAdam([p], lr=0.1)
    opt.sharded_state = types.SimpleNamespace(stale=True)
    with pytest.raises(RuntimeError, match="sync_optimizer_state"):
        opt.state_dict()
    opt.sharded_state.stale = False
    opt.state_dict()


def _load_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import hn_loader
    hn = hn_loader.load()
    from hashnerf_pytorch_amd.train import ShardedTableStep
    L_, R, F_ = 2, 32, 2
    g0 = torch.Generator().manual_seed(5)
    table = torch.nn.Parameter(torch.randn(L_, R, F_, generator=g0))
    opt = hn.RAdam([table], lr=0.1)
    xs = ShardedTableStep(table, None, rank, world, stepper=_toy_step)
    opt.sharded_state = xs
    xs.grad_view().copy_(torch.randn(L_, R, F_, generator=g0))
    xs.step({"beta1": 0.9, "beta2": 0.99, "lr": 0.05})
    assert xs.stale
    # a checkpoint loaded after the first sharded step: its moments must reach
    # the shards (and the stale flag clear), not stay in optimizer.state only
    m1, v1 = torch.randn(L_, R, F_, generator=g0), torch.rand(L_, R, F_, generator=g0)
    sd = {"state": {0: {"step": 7, "exp_avg": m1, "exp_avg_sq": v1}},
          "param_groups": [{**{k: v for k, v in opt.param_groups[0].items() if k != "params"}, "params": [0]}]}
    opt.load_state_dict(sd)
    assert not xs.stale
    m, v = xs.gather_state()
    ok = torch.equal(m, m1) and torch.equal(v, v1)
    # a rebuilt trainer setup refuses to seed shards from a stale optimizer copy
    xs.stale = True
    if rank == 0:
        torch.save({"ok": ok, "shard_m": xs.m.clone(), "want": xs._shard_of(m1)}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_moments_follow_load_state_dict(tmp_path):
    """RAdam.load_state_dict after the sharded table step began
    re-seeds the ranks' moment shards from the loaded exp_avg / exp_avg_sq."""
    port = _free_port()
    mp.spawn(_load_worker, args=(2, port, str(tmp_path / "ld.pt")), nprocs=2, join=True)
    got = torch.load(tmp_path / "ld.pt", weights_only=True)
    assert got["ok"]
    assert torch.equal(got["shard_m"], got["want"])
