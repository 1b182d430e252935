"""Diagnostic: record statistics of the binned table-gradient scatter for the
bench workload (procedural chair after --pretrain steps): records per launch,
per-(block, bin) region fill against the capacity, overflow records, and the
records per level.  Reads the workspace layout of hn_render.hip (bin_geom)."""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

G_END, W_END, BLOCKS, OVF = 30208, 9344, 256, 1 << 20


def bin_geom(T, n):
    shift = min(14, T + 4)
    nbins = 1 << (T + 4 - shift)
    rpb = (n + BLOCKS - 1) // BLOCKS
    avg = rpb * 192 * 4 * 2.0 ** (shift - T)
    cap = (int(avg) + 128 + 63) & ~63
    return shift, nbins, cap


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pretrain", type=int, default=1000)
    ap.add_argument("--n-rand", type=int, default=4096)
    ap.add_argument("--log2T", type=int, default=19)
    ap.add_argument("--finest", type=int, default=512)
    a = ap.parse_args()
    import hn_loader
    hn_loader.load()
    from hashnerf_pytorch_amd import functional as HF
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    dev = torch.device("cuda", 0)
    targs = default_args(N_rand=a.n_rand, log2_hashmap_size=a.log2T, finest_res=a.finest, tv_until=10 ** 9)
    data = SyntheticBlender(400, 400, 100, dev, seed=0, scene="procedural")
    tr = Trainer(targs, data, dev, seed=0)
    for _ in range(a.pretrain):
        tr.step()
    cap_st = {}
    orig = HF.render_bwd

    def grab(st, *args, **kw):
        cap_st["st"] = st
        return orig(st, *args, **kw)

    HF.render_bwd = grab
    tr.step()
    torch.cuda.synchronize()
    st = cap_st["st"]
    n, T = a.n_rand, a.log2T
    shift, nbins, cap = bin_geom(T, n)
    off = 2 * G_END + BLOCKS * 2 * W_END + n * 64 * 32 + n * 256 * 4
    nrec = BLOCKS * nbins * cap + OVF
    ws = st.wsb.view(torch.int32)
    idx0 = off + 4 * nrec
    cnt = ws[idx0 + nrec: idx0 + nrec + BLOCKS * nbins].cpu().numpy().astype(np.int64).reshape(nbins, BLOCKS)
    n_ovf = int(ws[idx0 + nrec + BLOCKS * nbins].item())
    tot = int(cnt.sum())
    print(f"B={n} T={T} shift={shift} nbins={nbins} cap={cap} records={tot} ({tot / n:.0f}/ray) "
          f"overflow_count={n_ovf} regions>cap={(cnt > cap).sum()} max={cnt.max()} mean={cnt.mean():.1f}")
    bins_per_level = max(1, (1 << T) >> shift)
    lv = cnt.sum(1).reshape(-1, bins_per_level).sum(1) if nbins >= 16 else None
    if lv is not None:
        print("records per level:", " ".join(str(int(x)) for x in lv))
        mx = cnt.max(1).reshape(-1, bins_per_level).max(1)
        print("max region fill per level:", " ".join(str(int(x)) for x in mx))
    HF.L.check_device_faults()
    print("no device faults")


if __name__ == "__main__":
    main()
