"""Diagnostic: dump the rays and fine-pass sample depths of one bench-config
training batch (after a few training steps) to gpurun_out/points.npz, for
offline modelling of the table-gradient atomic requests."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hn_loader  # noqa: E402

hn_loader.load()
from hashnerf_pytorch_amd import functional as HF  # noqa: E402
from hashnerf_pytorch_amd.render import render_ray_batch  # noqa: E402
from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args  # noqa: E402

dev = torch.device("cuda")
# usage: python scripts/dump_points.py [train_steps] [scene: uniform | procedural]
args = default_args(N_rand=4096, log2_hashmap_size=19, finest_res=512, tv_loss_weight=1e-6, tv_until=10 ** 9)
scene = sys.argv[2] if len(sys.argv) > 2 else "uniform"
data = SyntheticBlender(400, 400, 100, dev, seed=0, scene=scene)
tr = Trainer(args, data, dev)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    tr.step()
rays, _ = HF.sample_rays(data.images[3], data.poses[3], 4096, data.K, 2., 6., (0, 0, 400, 400), 99)
HF.DEBUG_KEEP = True
with torch.no_grad():
    render_ray_batch(rays, (4096,), chunk=args.chunk, retraw=True, **tr.kw_train)
HF.DEBUG_KEEP = False
os.makedirs("gpurun_out", exist_ok=True)
bb = data.bounding_box
np.savez("gpurun_out/points.npz", rays=rays.cpu().numpy(), z_fine=HF.LAST["z_fine"].cpu().numpy(),
         box_min=np.asarray(bb[0]), box_max=np.asarray(bb[1]))
print("saved", HF.LAST["z_fine"].shape)
