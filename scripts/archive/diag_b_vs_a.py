"""Diagnostic: the binned vs atomic backward of tests/test_gpu_scatter.py,
repeated in one process; per-tensor MLP-gradient differences each time."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import hn_loader
hn = hn_loader.load()
from test_gpu_scatter import _state, _bwd, _rel
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    HF, emb, mc, mf, ws, rays, t_rand, u, target, st_b, grads = _state(hn, 4096, 19, 7, "binned")
    tb, wb = _bwd(HF, emb, ws, st_b, grads)
    *_, st_a, grads_a = _state(hn, 4096, 19, 7, "atomic")
    ta, wa = _bwd(HF, emb, ws, st_a, grads_a)
    tb2, wb2 = _bwd(HF, emb, ws, st_b, grads)
    ta2, wa2 = _bwd(HF, emb, ws, st_a, grads_a)
    print(rep, "table b/a %.2e" % _rel(tb, ta),
          "mlp b/a", ["%.1e" % _rel(x, y) for x, y in zip(wb, wa)],
          "b/b2 max %.1e" % max(_rel(x, y) for x, y in zip(wb, wb2)),
          "a/a2 max %.1e" % max(_rel(x, y) for x, y in zip(wa, wa2)), flush=True)
