"""Diagnostic: stage-by-stage comparison of the HIP render path with the CPU
oracle on a golden fixture (coarse raw/weights, importance samples, fine raw).
Writes gpurun_out/diag_<name>.npz for offline analysis."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hn_loader  # noqa: E402
from conftest import golden, pcg_table  # noqa: E402
from oracle import hashnerf_oracle as O  # noqa: E402

hn = hn_loader.load()
from hashnerf_pytorch_amd import functional as HF  # noqa: E402

DEV = "cuda"
name = sys.argv[1] if len(sys.argv) > 1 else "render_black_det"
g = golden(name)
B = g["rays_o"].shape[0]
T = int(g["log2T"])
tab = torch.from_numpy(pcg_table(g["table_seed"], T))
box = (torch.from_numpy(g["box_min"]), torch.from_numpy(g["box_max"]))
res = O.level_resolutions(16, 16, int(g["finest"]))
wc = {k: torch.from_numpy(g["wc:" + k]) for k in O.MLP_KEYS}
wf = {k: torch.from_numpy(g["wf:" + k]) for k in O.MLP_KEYS}
rays_o, rays_d = torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"])
vd = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
rb = torch.cat([rays_o, rays_d, 2. * torch.ones(B, 1), 6. * torch.ones(B, 1), vd], -1)
perturb = float(g["perturb"]) > 0
t_rand = torch.from_numpy(g["t_rand"]) if perturb else None
u = torch.from_numpy(g["u"])
white = bool(g["white"])
ret = O.render_rays(rb, wc, wf, tab, box[0], box[1], res, T, t_rand=t_rand, u=u, white_bkgd=white)

# GPU, stage by stage (standalone HIP ops, fed the ORACLE's inputs at each stage)
emb = hn.HashEmbedder(box, log2_hashmap_size=T, finest_resolution=int(g["finest"])).to(DEV)
with torch.no_grad():
    emb.table.copy_(tab)
kw = dict(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
          input_ch=32, input_ch_views=16)
mc = hn.NeRFSmall(**kw).to(DEV)
mc.load_state_dict({k: v for k, v in wc.items()})
mf = hn.NeRFSmall(**kw).to(DEV)
mf.load_state_dict({k: v for k, v in wf.items()})
sh = hn.SHEncoder()
z0 = ret["z_vals0"].to(DEV)
pts0 = rays_o.to(DEV)[:, None] + rays_d.to(DEV)[:, None] * z0[..., None]
with torch.no_grad():
    raw0 = hn.run_network(pts0, vd.to(DEV), mc, emb, sh)
    o0 = hn.raw2outputs(raw0, z0, rays_d.to(DEV), 0, white)
    w0_oracle = ret["weights0"].detach()
    zmid = .5 * (ret["z_vals0"][..., 1:] + ret["z_vals0"][..., :-1])
    zs_gpu_own = HF.sample_pdf(zmid.to(DEV), o0[3][..., 1:-1], u.to(DEV))
    zs_gpu_orw = HF.sample_pdf(zmid.to(DEV), w0_oracle[..., 1:-1].to(DEV), u.to(DEV))
    zf = ret["z_vals"].to(DEV)
    ptsf = rays_o.to(DEV)[:, None] + rays_d.to(DEV)[:, None] * zf[..., None]
    rawf = hn.run_network(ptsf, vd.to(DEV), mf, emb, sh)
    of = hn.raw2outputs(rawf, zf, rays_d.to(DEV), 0, white)
np.savez(os.path.join(ROOT, "gpurun_out", f"diag_{name}.npz"),
         raw0_gpu=raw0.cpu().numpy(), raw0_orc=ret["raw0"].detach().numpy(),
         w0_gpu=o0[3].cpu().numpy(), w0_orc=w0_oracle.numpy(),
         zs_gpu_own=zs_gpu_own.cpu().numpy(), zs_gpu_orw=zs_gpu_orw.cpu().numpy(),
         zs_orc=ret["z_samples"].detach().numpy(),
         rawf_gpu=rawf.cpu().numpy(), rawf_orc=ret["raw"].detach().numpy(),
         entf_gpu=of[5].cpu().numpy(), entf_orc=ret["sparsity_loss"].detach().numpy(),
         wf_gpu=of[3].cpu().numpy(), wf_orc=ret["weights"].detach().numpy())
print("saved", name)
