"""Fraction of samples / MLP tiles / scatter units whose gradient is exactly
zero in the bench's trained regime: a sample whose raw sigma is <= 0 has
alpha = 0 and weight 0, so raw2outputs' backward gives it d raw = 0 exactly
(run_nerf_helpers.py:577-628: relu(sigma), w = alpha * T), and the MLP
backward turns that into zero feature and weight-gradient contributions.
Runs bench.py's trainer (procedural chair, --pretrain steps) and prints one
JSON line per config.   usage: python scripts/zero_grad_frac.py [config ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import hn_loader  # noqa: E402

hn_loader.load()
from hashnerf_pytorch_amd import functional as HF  # noqa: E402
from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args  # noqa: E402


def run(cfg_id, pretrain=1000, steps=4):
    cfg = bench.CONFIGS[cfg_id]
    dev = torch.device("cuda", 0)
    targs = default_args(N_rand=cfg["N_rand"], log2_hashmap_size=cfg["log2_hashmap_size"],
                         finest_res=cfg["finest_res"], tv_loss_weight=cfg["tv_loss_weight"],
                         tv_until=cfg.get("tv_until", 1001), white_bkgd=cfg.get("white_bkgd", True),
                         sparse_loss_weight=cfg.get("sparse_loss_weight", 1e-10),
                         no_batching=cfg.get("no_batching", True))
    data = SyntheticBlender(400, 400, 100, dev, seed=0, scene="procedural")
    if "bbox" in cfg:
        data.bounding_box = tuple(torch.tensor(v) for v in cfg["bbox"])
    tr = Trainer(targs, data, dev, seed=0)
    for _ in range(pretrain):
        tr.step()
    acc = {}
    HF.DEBUG_KEEP = True
    for _ in range(steps):
        tr.step()
        rc, rf = HF.LAST["raw_c"][..., 3], HF.LAST["raw_f"][..., 3]
        zc, zf = rc <= 0, rf <= 0
        stats = {
            "coarse_samples": zc.float().mean().item(),
            "fine_samples": zf.float().mean().item(),
            "coarse_tiles": zc.view(-1, 2, 32).all(-1).float().mean().item(),
            "fine_tiles": zf.view(-1, 6, 32).all(-1).float().mean().item(),
            "fine_units_of_64": zf.view(-1, 3, 64).all(-1).float().mean().item(),
            "rays": (zc.all(-1) & zf.all(-1)).float().mean().item(),
        }
        for k, v in stats.items():
            acc[k] = acc.get(k, 0.0) + v / steps
    HF.DEBUG_KEEP = False
    return {"config": cfg_id, "pretrain": pretrain, "zero_sigma_fraction": {k: round(v, 4) for k, v in acc.items()}}


if __name__ == "__main__":
    for c in [int(a) for a in sys.argv[1:]] or [2]:
        print(json.dumps(run(c)), flush=True)
