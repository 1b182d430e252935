"""Diagnostic: two identical render forwards with the stored-mask build; report
where the feature cache (features | ReLU mask words) differs."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import hn_loader
hn = hn_loader.load()
from test_gpu_scatter import _state
box = (torch.tensor([-1.0, -1.0, -1.0]), torch.tensor([1.0, 1.0, 1.0]))
*_, s1, _ = _state(hn, 1024, 19, 17, "binned", box=box)
*_, s2, _ = _state(hn, 1024, 19, 17, "binned", box=box)
a, b = s1.feat.view(torch.int32), s2.feat.view(torch.int32)
d = (a != b).nonzero()
print("differing words:", d.shape[0], "of", a.numel())
if d.shape[0]:
    ray, col = d[:, 0], d[:, 1]
    feat = col < 8192
    print("in features:", int(feat.sum()), "in masks:", int((~feat).sum()))
    m = col[~feat] - 8192
    tile, word, lane = m // 192, (m % 192) // 64, m % 64
    for name, v in (("ray", ray[~feat]), ("tile", tile), ("word", word), ("lane", lane)):
        u, c = torch.unique(v, return_counts=True)
        print(name, list(zip(u.tolist()[:20], c.tolist()[:20])))
    i = (~feat).nonzero()[:8, 0]
    for j in i.tolist():
        r, cc = int(ray[j]), int(col[j])
        print(r, cc, hex(int(a[r, cc]) & 0xffffffff), hex(int(b[r, cc]) & 0xffffffff))
for name in ("z_f", "raw_c", "raw_f", "fine_src"):
    print(name, torch.equal(getattr(s1, name), getattr(s2, name)))
