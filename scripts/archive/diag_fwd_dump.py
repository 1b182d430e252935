"""Diagnostic: one render forward of tests/test_gpu_scatter.py's bench-shape
state; saves the saved state (bitwise) to an .npz for comparing two builds."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
import hn_loader
hn = hn_loader.load()
from test_gpu_scatter import _state, _bwd
HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, 4096, 19, 7, "binned")
d_table, dws = _bwd(HF, emb, ws, st, grads)
out = {k: getattr(st, k).detach().cpu().view(torch.int32).numpy() for k in ("feat", "raw_c", "raw_f", "z_f")}
out["d_table"] = d_table.cpu().view(torch.int32).numpy()
for i, w in enumerate(dws):
    out[f"dw{i}"] = w.cpu().view(torch.int32).numpy()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1])
