"""Diagnostic: identical render forwards (tests/test_gpu_scatter.py _state at
the bench shape) compared bitwise -- feature cache (features | ReLU mask
words), z, raw, outputs and the packed weights in the workspace."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import hn_loader
hn = hn_loader.load()
from test_gpu_scatter import _state
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
sched = sys.argv[3] if len(sys.argv) > 3 else "binned"
ref = None
for rep in range(reps):
    *_, st, _ = _state(hn, B, 19, 7, sched)
    torch.cuda.synchronize()
    cur = dict(rays=st.rays.clone(), feat=st.feat.view(torch.int32).clone(), z_f=st.z_f.clone(), raw_c=st.raw_c.clone(),
               raw_f=st.raw_f.clone(), z_c=st.z_c.clone(), src=st.fine_src.clone(),
               packed=st.wsb.view(torch.int32)[:2 * 30208].clone())
    if ref is None:
        ref = cur
        continue
    out = []
    for k, v in cur.items():
        d = (v.view(-1) != ref[k].view(-1)) if k != "feat" else None
        if k == "feat":
            a, b = v, ref[k]
            diff = (a != b).nonzero()
            if diff.shape[0]:
                ray, col = diff[:, 0], diff[:, 1]
                feat = col < 8192
                m = col[~feat] - 8192
                out.append(f"feat {int(feat.sum())} mask {int((~feat).sum())} rays {torch.unique(ray).numel()}")
                if (~feat).any():
                    tile, word, lane = m // 192, (m % 192) // 64, m % 64
                    out.append(f" mask tiles {torch.unique(tile).tolist()[:8]} words {torch.unique(word).tolist()} "
                               f"lanes {torch.unique(lane).tolist()[:12]}")
                    for rr in torch.unique(ray[~feat]).tolist()[:3]:
                        sel = (~feat) & (ray == rr)
                        mm = col[sel] - 8192
                        out.append(f" ray {rr}: lanes {sorted(set((mm % 64).tolist()))} words {sorted(set(((mm % 192) // 64).tolist()))} rows {sorted(set((mm // 64).tolist()))}")
                        rc = (cur["raw_c"][rr] - ref["raw_c"][rr]).abs()
                        out.append(f" ray {rr}: raw_c |d| max {float(rc.max()):.3e} at pts {sorted(set((rc.amax(-1) > 0).nonzero().view(-1).tolist()))}")
                    j = int((~feat).nonzero()[0, 0])
                    r, c = int(ray[j]), int(col[j])
                    out.append(f" e.g. ray {r} col {c}: {int(a[r, c]) & 0xffffffff:#x} vs {int(b[r, c]) & 0xffffffff:#x}")
                if feat.any():
                    j = int(feat.nonzero()[0, 0])
                    r, c = int(ray[j]), int(col[j])
                    out.append(f" feat e.g. ray {r} col {c}: {a[r, c].view(torch.float32)} vs {b[r, c].view(torch.float32)}")
        elif int(d.sum()):
            out.append(f"{k} {int(d.sum())}")
    print(rep, "identical" if not out else " | ".join(out), flush=True)
