"""One rank of the device data-parallel test (tests/test_gpu_dp.py).

Started by the test as a child process (RANK / WORLD_SIZE / MASTER_* in the
environment), one per rank, all on cuda:0, torch.distributed over gloo.  The
rank runs the HIP explicit-mode Trainer's forward + backward on ITS slice of a
global batch the test drew (train.Trainer._fused_forward_backward, the step's
launch sequence), all-reduces the gradients (Trainer.allreduce_grads: the
SUM exchange of run_nerf.py:640-642 under SURVEY 8e's loss rule), and rank 0
saves the reduced gradients.
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(batch_path, out_path):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    spec = torch.load(batch_path, weights_only=True)
    dev = torch.device("cuda", 0)
    data = SyntheticBlender(spec["H"], spec["W"], spec["n_img"], dev, seed=0)
    args = default_args(**spec["args"])
    tr = Trainer(args, data, dev, rank=rank, world=world, seed=0)
    tr.fuse_table_step = False
    b = spec["ranks"][rank]
    batch = dict(rays=b["rays"].to(dev), target=b["target"].to(dev), t_rand=b["t_rand"].to(dev),
                 u=b["u"].to(dev), tv=(b["tv_cubes"], b["tv_mv"]) if "tv_mv" in b else None)
    loss, _ = tr._fused_forward_backward(spec["i"], batch)
    tr.allreduce_grads()
    torch.cuda.synchronize()
    from hashnerf_pytorch_amd import _lib
    _lib.check_device_faults()
    if rank == 0:
        ws = tr.kw_train["network_fn"].weights() + tr.kw_train["network_fine"].weights()
        torch.save({"table": tr.embed_fn.table.grad.cpu(), "mlp": [p.grad.cpu() for p in ws],
                    "loss": loss.detach().cpu()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def train(out_path, sharded, steps, resume_at=0):
    """`steps` training steps of the explicit trainer on this rank's own draws,
    the table exchange sharded (reduce-scatter / shard RAdam / all-gather) or
    all-reduced; rank 0 saves the table, its RAdam moments and the MLP weights.
    resume_at > 0: after that many steps the moments are gathered into the
    optimizer (a checkpoint's state, run_nerf.py:663-680) and the sharded
    exchange is rebuilt from it, as a resumed run builds it (create_nerf's
    reload, run_nerf_helpers.py:158-168)."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    dev = torch.device("cuda", 0)
    data = SyntheticBlender(64, 64, 4, dev, seed=0)
    args = default_args(N_rand=256, log2_hashmap_size=14, tv_loss_weight=1e-4, tv_until=4, sparse_loss_weight=1e-3)
    tr = Trainer(args, data, dev, rank=rank, world=world, seed=0)
    tr.dp_sharded = sharded
    # the uninterrupted sharded run exchanges in 4 bin-aligned segments (each
    # reduce-scattered right after the owner pass forms it); the resumed run
    # in one (Trainer's default)
    tr.dp_chunks = 4 if not resume_at else 1
    for k in range(steps):
        if resume_at and k == resume_at:
            tr.sync_optimizer_state()
            tr.optimizer.state_dict()          # refuses stale moments: must not raise now
            tr._grads = tr._xchg = None        # the next step rebuilds the exchange from optimizer.state
        tr.step()
    tr.sync_optimizer_state()
    torch.cuda.synchronize()
    from hashnerf_pytorch_amd import _lib
    _lib.check_device_faults()
    if rank == 0:
        t = tr.embed_fn.table
        st = tr.optimizer.state[t]
        ws = tr.kw_train["network_fn"].weights() + tr.kw_train["network_fine"].weights()
        torch.save({"table": t.detach().cpu(), "m": st["exp_avg"].cpu(), "v": st["exp_avg_sq"].cpu(),
                    "step": st["step"], "mlp": [p.detach().cpu() for p in ws]}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def train_pool(out_path, steps, emulate, tv=True):
    """use_batching (the global shuffled ray pool, run_nerf.py:505-555) on a
    pool whose epoch ends in a batch of ONE position for two ranks: rank 1
    draws no rays that step and must still join the exchange.
    emulate: "1" = gloo's emulated collectives, "0" = the production
    reduce_scatter_tensor / all_gather_into_tensor calls on device tensors."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd.train import ShardedTableStep, SyntheticBlender, Trainer, default_args
    dev = torch.device("cuda", 0)
    # 1 image of 7 x 19 = 133 rays = 2 x 66 + 1: every second step's batch is
    # 1 ray (rank 0 draws none, rank 1 the one: train._pool_draw's split)
    data = SyntheticBlender(7, 19, 1, dev, seed=0)
    # (the empty rank's TV term goes through the binned records: bitwise
    # reproducible, so the comparisons run with it)
    args = default_args(N_rand=66, log2_hashmap_size=14, tv_loss_weight=1e-4 if tv else 0.0, tv_until=10 ** 6,
                        sparse_loss_weight=1e-3, no_batching=False)
    tr = Trainer(args, data, dev, rank=rank, world=world, seed=0)
    if emulate is not None:
        tr._fused_setup()
        tr._xchg.coll.emulate = emulate
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    from hashnerf_pytorch_amd import _lib
    _lib.check_device_faults()
    tr.sync_optimizer_state()
    if rank == 0:
        t = tr.embed_fn.table
        torch.save({"table": t.detach().cpu(), "finite": bool(torch.isfinite(t).all()), "step": tr.global_step},
                   out_path)
    dist.barrier()
    dist.destroy_process_group()


def probe(out_path):
    """gloo's reduce_scatter_tensor (async) and all_gather_into_tensor on
    device tensors against their definition: rank 0 saves what it got."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    inp = torch.arange(4 * world, dtype=torch.float32, device=dev) + 100 * rank
    out = torch.full((4,), -1.0, device=dev)
    dist.reduce_scatter_tensor(out, inp, async_op=True).wait()
    want = sum(torch.arange(4 * world, dtype=torch.float32) + 100 * r for r in range(world))[4 * rank:4 * rank + 4]
    g = torch.full((4 * world,), -1.0, device=dev)
    dist.all_gather_into_tensor(g, out)
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"rs": out.cpu(), "rs_want": want, "ag": g.cpu(),
                    "ag_want": sum(torch.arange(4 * world, dtype=torch.float32) + 100 * r for r in range(world))},
                   out_path)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    if sys.argv[1] == "probe":
        probe(sys.argv[2])
    elif sys.argv[1] == "train_pool":
        em = {"-": None, "1": True, "0": False}[sys.argv[4]]
        train_pool(sys.argv[2], int(sys.argv[3]), em, len(sys.argv) <= 5 or sys.argv[5] == "1")
    elif sys.argv[1] == "train":
        train(sys.argv[2], sys.argv[3] == "1", int(sys.argv[4]), int(sys.argv[5]) if len(sys.argv) > 5 else 0)
    else:
        main(sys.argv[1], sys.argv[2])
