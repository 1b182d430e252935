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
