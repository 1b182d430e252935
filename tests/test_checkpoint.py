"""Checkpoint format (run_nerf.py:663-680 save, run_nerf_helpers.py create_nerf
reload): a checkpoint written with the reference's keys is reloaded by
create_nerf(ft_path=...) with weights, hash table, global step and optimizer
state restored.  CPU-only (no kernel launches)."""
import torch

from conftest import ROOT  # noqa: F401


def _args(hn, tmp_path, **over):
    from hashnerf_pytorch_amd.train import default_args
    a = default_args(log2_hashmap_size=10, **over)
    a.bounding_box = (torch.tensor([-1.5, -1.5, -1.0]), torch.tensor([1.5, 1.5, 1.0]))
    a.basedir, a.expname = str(tmp_path), "exp"
    return a


def test_checkpoint_round_trip_reference_keys(hn, tmp_path):
    from hashnerf_pytorch_amd.create import create_nerf
    torch.manual_seed(0)
    kw, _, start, grad_vars, opt = create_nerf(_args(hn, tmp_path), device="cpu")
    assert start == 0
    with torch.no_grad():
        kw["embed_fn"].table.add_(torch.randn_like(kw["embed_fn"].table))
        for p in grad_vars:
            p.add_(torch.randn_like(p))
    # one optimizer step's state (step counters, moments) without a GPU:
    for group in opt.param_groups:
        for p in group["params"]:
            st = opt.state[p]
            st["step"] = 3
            st["exp_avg"] = torch.full_like(p, 0.5)
            st["exp_avg_sq"] = torch.full_like(p, 0.25)
    ckpt = tmp_path / "exp" / "000100.tar"
    ckpt.parent.mkdir()
    torch.save({"global_step": 100,
                "network_fn_state_dict": kw["network_fn"].state_dict(),
                "network_fine_state_dict": kw["network_fine"].state_dict(),
                "embed_fn_state_dict": kw["embed_fn"].state_dict(),
                "optimizer_state_dict": opt.state_dict()}, ckpt)
    sd = kw["embed_fn"].state_dict()
    assert list(sd) == [f"embeddings.{l}.weight" for l in range(16)]   # the reference's keys

    torch.manual_seed(1)
    kw2, _, start2, grad_vars2, opt2 = create_nerf(_args(hn, tmp_path, no_reload=False), device="cpu")
    assert start2 == 100
    assert torch.equal(kw2["embed_fn"].table, kw["embed_fn"].table)
    for a, b in zip(grad_vars2, grad_vars):
        assert torch.equal(a, b)
    for group in opt2.param_groups:
        for p in group["params"]:
            assert opt2.state[p]["step"] == 3
            assert torch.equal(opt2.state[p]["exp_avg"], torch.full_like(p, 0.5))
    # ft_path takes precedence over the experiment directory
    kw3, _, start3, _, _ = create_nerf(_args(hn, tmp_path, no_reload=False, ft_path=str(ckpt)), device="cpu")
    assert start3 == 100 and torch.equal(kw3["embed_fn"].table, kw["embed_fn"].table)


def _reference_layout_state(kw, grad_vars, T, step=7):
    """An optimizer state dict in the reference's layout (run_nerf_helpers.py:132-135):
    group 0 = the ten NeRFSmall weights, group 1 = the 16 per-level
    nn.Embedding weights [2^T, 2], each with its own moments."""
    import torch.nn as nn

    from hashnerf_pytorch_amd.radam import RAdam
    levels = [nn.Parameter(torch.zeros(2 ** T, 2)) for _ in range(16)]
    mlp = [nn.Parameter(torch.zeros_like(p)) for p in grad_vars]
    ref = RAdam([{"params": mlp, "weight_decay": 1e-6}, {"params": levels, "eps": 1e-15}],
                lr=0.01, betas=(0.9, 0.99))
    g = torch.Generator().manual_seed(5)
    for p in mlp + levels:
        ref.state[p] = {"step": step, "exp_avg": torch.randn(p.shape, generator=g),
                        "exp_avg_sq": torch.rand(p.shape, generator=g)}
    return ref.state_dict()


def test_optimizer_state_reference_layout_loads(hn, tmp_path):
    """a reference checkpoint's optimizer state (16 embedding
    params) loads into the stacked-table optimizer, and this optimizer's state
    dict is written in the reference's layout (so the reference can resume)."""
    from hashnerf_pytorch_amd.create import create_nerf
    torch.manual_seed(0)
    T = 10
    kw, _, _, grad_vars, opt = create_nerf(_args(hn, tmp_path), device="cpu")
    sd = _reference_layout_state(kw, grad_vars, T)
    assert [len(g["params"]) for g in sd["param_groups"]] == [10, 16]
    opt.load_state_dict(sd)
    table = kw["embed_fn"].table
    st = opt.state[table]
    assert st["step"] == 7 and st["exp_avg"].shape == table.shape
    for l in range(16):
        assert torch.equal(st["exp_avg"][l], sd["state"][10 + l]["exp_avg"])
        assert torch.equal(st["exp_avg_sq"][l], sd["state"][10 + l]["exp_avg_sq"])
    for i, p in enumerate(grad_vars):
        assert torch.equal(opt.state[p]["exp_avg"], sd["state"][i]["exp_avg"])
    # written back in the reference's layout, bit-identical
    out = opt.state_dict()
    assert [len(g["params"]) for g in out["param_groups"]] == [10, 16]
    assert out["param_groups"][1]["eps"] == 1e-15 and out["param_groups"][0]["weight_decay"] == 1e-6
    for i in range(26):
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(out["state"][i][k], sd["state"][i][k]), (i, k)
        assert out["state"][i]["step"] == 7
    # and it survives torch.save / torch.load(weights_only=True)
    path = tmp_path / "opt.tar"
    torch.save(out, path)
    back = torch.load(path, weights_only=True)
    kw2, _, _, _, opt2 = create_nerf(_args(hn, tmp_path), device="cpu")
    opt2.load_state_dict(back)
    assert torch.equal(opt2.state[kw2["embed_fn"].table]["exp_avg"], st["exp_avg"])


def test_optimizer_state_layout_mismatch_raises(hn, tmp_path):
    from hashnerf_pytorch_amd.create import create_nerf
    kw, _, _, grad_vars, opt = create_nerf(_args(hn, tmp_path), device="cpu")
    sd = _reference_layout_state(kw, grad_vars, 10)
    sd["param_groups"][1]["params"] = sd["param_groups"][1]["params"][:15]
    import pytest
    with pytest.raises(ValueError):
        opt.load_state_dict(sd)
