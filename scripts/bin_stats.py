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

G_END, W_END, BLOCKS = 30208, 9344, 256


def bin_geom(T, n):
    shift = min(13, T + 4)
    nbins = 1 << (T + 4 - shift)
    rpb = (n + BLOCKS - 1) // BLOCKS
    avg = rpb * 192 * 4 * 2.0 ** (shift - T)
    cap = (int(avg) + 128 + 63) & ~63
    if ((cap >> 6) & 1) == 0:   # an odd multiple of 64 (hn_render.hip bin_geom)
        cap += 64
    return shift, nbins, cap


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pretrain", type=int, default=1000)
    ap.add_argument("--n-rand", type=int, default=4096)
    ap.add_argument("--log2T", type=int, default=19)
    ap.add_argument("--finest", type=int, default=512)
    ap.add_argument("--quick", action="store_true", help="counts only (no owner / precision study)")
    ap.add_argument("--dups", action="store_true", help="records vs distinct entries per region / bin, per level")
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
    off = 2 * G_END + BLOCKS * 4 * W_END + n * 64 * 32 + n * 256 * 4
    off += n * 192 * 32                       # fine feature grads (binned schedule)
    tv_per_block = (16 * 26 * 51 * 51 + BLOCKS - 1) // BLOCKS     # hn_render.hip kTvRecPerBlock
    ovf_per_block = (3 * n + BLOCKS - 1) // BLOCKS * 64 * 64 + tv_per_block
    nrec = BLOCKS * nbins * cap + BLOCKS * ovf_per_block   # regions + overflow lists (hn_render.hip bin_records)
    ws = st.wsb.view(torch.int32)
    idx0 = off + 4 * nrec
    cnt = ws[idx0 + nrec: idx0 + nrec + BLOCKS * nbins].cpu().numpy().astype(np.int64).reshape(nbins, BLOCKS)
    n_ovf = int(ws[idx0 + nrec + BLOCKS * (nbins + 16)].item())
    tot = int(cnt.sum())
    print(f"B={n} T={T} shift={shift} nbins={nbins} cap={cap} records={tot} ({tot / n:.0f}/ray) "
          f"overflow_count={n_ovf} regions>cap={(cnt > cap).sum()} max={cnt.max()} mean={cnt.mean():.1f}")
    bins_per_level = max(1, (1 << T) >> shift)
    lv = cnt.sum(1).reshape(-1, bins_per_level).sum(1) if nbins >= 16 else None
    if lv is not None:
        print("records per level:", " ".join(str(int(x)) for x in lv))
        mx = cnt.max(1).reshape(-1, bins_per_level).max(1)
        print("max region fill per level:", " ".join(str(int(x)) for x in mx))
        spill = np.maximum(cnt - cap, 0).sum(1).reshape(-1, bins_per_level).sum(1)
        print("spilled records per level:", " ".join(str(int(x)) for x in spill))
    if a.dups:
        # merge potential: per level, records vs distinct entry words inside
        # one producer's region of a bin (what an in-block merge could fold),
        # and inside a whole bin over all producers (the owner's view)
        idx_i = off + 4 * nrec
        wr = ws[idx_i: idx_i + nbins * BLOCKS * cap].view(nbins, BLOCKS, cap).to(torch.int64) & 0xffffffff
        cm = torch.from_numpy(np.minimum(cnt, cap)).to(wr.device)
        valid = torch.arange(cap, device=wr.device)[None, None, :] < cm[:, :, None]
        big = torch.iinfo(torch.int64).max
        srt, _ = torch.sort(torch.where(valid, wr, big), dim=2)
        newv = torch.ones_like(srt, dtype=torch.bool)
        newv[:, :, 1:] = srt[:, :, 1:] != srt[:, :, :-1]
        dist_region = ((newv & (srt != big)).sum(2)).sum(1).cpu().numpy()      # per bin
        flat = torch.where(valid, wr, big).reshape(nbins, -1)
        sb, _ = torch.sort(flat, dim=1)
        nb_ = torch.ones_like(sb, dtype=torch.bool)
        nb_[:, 1:] = sb[:, 1:] != sb[:, :-1]
        dist_bin = (nb_ & (sb != big)).sum(1).cpu().numpy()
        recs = np.minimum(cnt, cap).sum(1)
        per = lambda x: x.reshape(-1, bins_per_level).sum(1)
        print("level: records (in regions) / distinct per producer region / distinct per bin")
        for l, (r_, d1, d2) in enumerate(zip(per(recs), per(dist_region), per(dist_bin))):
            print(f"  {l:2d}: {int(r_):9d} {int(d1):9d} ({r_ / max(d1, 1):.2f}x) {int(d2):9d} ({r_ / max(d2, 1):.2f}x)")
        print(f"  all: {int(recs.sum())} {int(dist_region.sum())} ({recs.sum() / dist_region.sum():.2f}x) "
              f"{int(dist_bin.sum())} ({recs.sum() / dist_bin.sum():.2f}x)")
    if a.quick:
        HF.L.check_device_faults()
        return
    # owner-pass simulation on a few bins: chunks of 1024 flattened records ->
    # 2048 items (entry, owner (e >> 5) & 15); per owner batches of 64 items;
    # the claim rounds a batch needs = max items per tag slot (hashed entry)
    vals_i = off
    aos = os.environ.get("HN_REC_AOS", "0") != "0"   # the library build setting (-DHN_REC_AOS)
    idx_i = off + 4 * nrec
    wsi = ws
    sel, tmask = (1 << shift) - 1, (1 << T) - 1
    for b in (0, nbins // 2, nbins - 1, nbins - 2):
        c = np.minimum(cnt[b], cap)
        recs = []
        for p in range(BLOCKS):
            r = (b * BLOCKS + p) * cap + np.arange(int(c[p]))
            # records in groups of 4 (4 value quads, then 4 words: HN_REC_AOS)
            wi = vals_i + (r >> 2) * 20 + 16 + (r & 3) if aos else idx_i + r
            recs.append(wsi[torch.from_numpy(wi).to(wsi.device)].cpu().numpy().view(np.uint32))
        w = np.concatenate(recs)
        e0 = (w & 0x0fffffff) & sel
        d = ((np.uint32(1) << (w >> 28)) - 1) & tmask
        e1 = e0 ^ d
        rounds, batches, maxmult = 0, 0, 0
        for ch in range(0, len(w), 1024):
            ea, eb = e0[ch:ch + 1024], e1[ch:ch + 1024]
            items = np.concatenate([np.stack([ea, eb], 1).reshape(-1)])
            own = (items >> 5) & 15
            for o in range(16):
                it = items[own == o]
                for q in range(0, len(it), 64):
                    bt = it[q:q + 64]
                    slot = ((bt.astype(np.uint64) * 0x9E3779B1) & 0xffffffff) >> 24
                    m = np.bincount(slot.astype(np.int64)).max()
                    rounds += m
                    batches += 1
                    maxmult = max(maxmult, np.bincount(bt.astype(np.int64)).max())
        print(f"bin {b}: records {len(w)} distinct entries {len(np.unique(np.concatenate([e0, e1])))} "
              f"batches {batches} rounds {rounds} ({rounds / max(batches, 1):.1f}/batch) max same-entry per batch {maxmult}")
    # fixed-point accumulation study: per bin, scale from the max |record
    # value| (exponent E): int64 units of 2^(E - 42); error of the rounded
    # fixed-point sums vs exact (float64) sums, and vs fp32 sequential sums
    vals_all = ws.view(torch.float32)
    for b in (0, nbins // 4, nbins // 2, nbins - 1):
        c = np.minimum(cnt[b], cap)
        wl, vl = [], []
        for p in range(BLOCKS):
            r0 = (b * BLOCKS + p) * cap
            wl.append(wsi[idx_i + r0: idx_i + r0 + int(c[p])].cpu().numpy().view(np.uint32))
            vl.append(vals_all[vals_i + 4 * r0: vals_i + 4 * (r0 + int(c[p]))].cpu().numpy().reshape(-1, 4))
        w, v = np.concatenate(wl), np.concatenate(vl)
        if len(w) == 0:
            continue
        e0 = (w & 0x0fffffff) & sel
        e1 = e0 ^ (((np.uint32(1) << (w >> 28)) - 1) & tmask)
        ent = np.concatenate([2 * e0, 2 * e0 + 1, 2 * e1, 2 * e1 + 1]).astype(np.int64)
        x = np.concatenate([v[:, 0], v[:, 1], v[:, 2], v[:, 3]])
        exact = np.zeros(2 << shift)
        np.add.at(exact, ent, x.astype(np.float64))
        f32 = np.zeros(2 << shift, np.float32)
        np.add.at(f32, ent, x)
        E = int(np.floor(np.log2(np.abs(x).max())))
        q = np.rint(x.astype(np.float64) * 2.0 ** (42 - E)).astype(np.int64)
        acc = np.zeros(2 << shift, np.int64)
        np.add.at(acc, ent, q)
        fx = (acc.astype(np.float64) * 2.0 ** (E - 42)).astype(np.float32)
        nz = exact != 0
        rel = lambda a: np.abs(a[nz] - exact[nz]) / np.abs(exact[nz])
        rf, rq = rel(f32), rel(fx)
        print(f"bin {b}: maxexp {E} nonzero {nz.sum()} |g| min {np.abs(exact[nz]).min():.2e} median "
              f"{np.median(np.abs(exact[nz])):.2e} | rel err fp32 median {np.median(rf):.1e} p99.9 "
              f"{np.quantile(rf, .999):.1e} max {rf.max():.1e} | fixed64 median {np.median(rq):.1e} p99.9 "
              f"{np.quantile(rq, .999):.1e} max {rq.max():.1e}; entries with fixed64 err > fp32 max: "
              f"{(rq > rf.max()).sum()}")
    HF.L.check_device_faults()
    print("no device faults")


if __name__ == "__main__":
    main()
