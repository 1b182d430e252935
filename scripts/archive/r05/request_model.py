"""Diagnostic: model the memory-side float-atomic requests of the backward's
table-gradient scatter on recorded samples (gpurun_out/points.npz from
scripts/dump_points.py), for alternative merge schemes.

Lane layout of the scatter (hn_render.hip scatter_level_x): per (tile, group
of 16 points, level) there are 4 atomic wave-instructions (corner row jk);
lane (point p, x offset xi, feature f) adds to entry h(x + xi, y_j, z_k),
feature f, when p heads a run of samples in one voxel.  Memory-side cost of
one instruction (microbenchmark scripts/atomic_coalesce.hip): lanes in one
64-B segment coalesce, a dword hit by several lanes costs one extra request
per extra lane -> per segment: max multiplicity over its dwords.

  usage: python scripts/request_model.py [n_rays]
"""
import sys
from collections import Counter

import numpy as np

PY, PZ = np.uint32(2654435761), np.uint32(805459861)


def cells(pts, bmin, bmax, log2T=19, L=16, base=16, finest=512):
    b = np.exp((np.log(np.float32(finest)) - np.log(np.float32(base))) / (L - 1))
    out = []
    xc = np.clip(pts, bmin, bmax)
    for l in range(L):
        res = np.floor(np.float32(base) * np.float32(b) ** l)
        gs = ((bmax - bmin) / res).astype(np.float32)
        out.append(np.floor((xc - bmin) / gs).astype(np.int64).astype(np.uint32))
    return out   # [L] x [n, 3]


def instr_cost(addrs):
    """addrs: dword addresses of the active lanes of one instruction."""
    seg = Counter()
    per = Counter(addrs)
    for a, m in per.items():
        s = a >> 4
        seg[s] = max(seg[s], m)
    return sum(seg.values()), len(set(a >> 4 for a in addrs))


def model(rays, z, bmin, bmax, log2T=19):
    mask = np.uint32((1 << log2T) - 1)
    tot = Counter()
    for r in range(rays.shape[0]):
        o, d = rays[r, 0:3], rays[r, 3:6]
        pts = (o[None, :] + d[None, :] * z[r][:, None]).astype(np.float32)
        cl = cells(pts, bmin, bmax, log2T)
        for l in range(16):
            c = cl[l]
            row0 = l << log2T
            for t0 in range(0, 192, 32):
                segs = set()
                for p in range(t0, t0 + 32):
                    x, y, zz = (int(v) for v in c[p])
                    for j in (0, 1):
                        for k in (0, 1):
                            hy = np.uint32((y + j) * int(PY) & 0xffffffff)
                            hz = np.uint32((zz + k) * int(PZ) & 0xffffffff)
                            for xi in (0, 1):
                                e = int((np.uint32(x + xi) ^ hy ^ hz) & mask)
                                segs.add((row0 + e) >> 3)
                tot["union_32pt_bound"] += len(segs)
            for g0 in range(0, 192, 16):
                cg = c[g0:g0 + 16]
                heads = [0] + [p for p in range(1, 16) if (cg[p] != cg[p - 1]).any()]
                # x-adjacent successor head: its x-offset-0 corners are this
                # head's x-offset-1 corners (same dwords)
                xadj = set()
                for a, b2 in zip(heads, heads[1:]):
                    if cg[b2][0] == cg[a][0] + 1 and cg[b2][1] == cg[a][1] and cg[b2][2] == cg[a][2]:
                        xadj.add(b2)
                for j in (0, 1):
                    for k in (0, 1):
                        cur, xm = [], []
                        for p in heads:
                            x, y, zz = (int(v) for v in cg[p])
                            hy = np.uint32((y + j) * int(PY) & 0xffffffff)
                            hz = np.uint32((zz + k) * int(PZ) & 0xffffffff)
                            for xi in (0, 1):
                                e = int((np.uint32(x + xi) ^ hy ^ hz) & mask)
                                for f in (0, 1):
                                    adr = ((row0 + e) * 2 + f)
                                    cur.append(adr)
                                    if not (xi == 0 and p in xadj):
                                        xm.append(adr)
                        # general neighbour give (prev head, any distance), y/z rows,
                        # chain-free + x-step duplicate merge
                        gm = []
                        for idx, p in enumerate(heads):
                            x, y, zz = (int(v) for v in cg[p])
                            give_row = False
                            xdup = False
                            if idx > 0:
                                q = heads[idx - 1]
                                dx, dy, dz = (int(cg[p][a]) - int(cg[q][a]) for a in range(3))
                                if dx == 0 and 0 <= j + dy <= 1 and 0 <= k + dz <= 1 and (dy or dz):
                                    give_row = True
                                if dx == 1 and dy == 0 and dz == 0:
                                    xdup = True
                            if give_row and idx + 1 < len(heads):
                                r2 = heads[idx + 1]
                                ex, ey, ez = (int(cg[r2][a]) - int(cg[p][a]) for a in range(3))
                                # p receives into row (j,k) from r2 when r2's row (j-ey, k-ez) maps here
                                if ex == 0 and (ey or ez) and 0 <= j - ey <= 1 and 0 <= k - ez <= 1:
                                    give_row = False
                            if give_row:
                                continue
                            hy = np.uint32((y + j) * int(PY) & 0xffffffff)
                            hz = np.uint32((zz + k) * int(PZ) & 0xffffffff)
                            for xi in (0, 1):
                                if xi == 0 and xdup:
                                    continue
                                e = int((np.uint32(x + xi) ^ hy ^ hz) & mask)
                                for f in (0, 1):
                                    gm.append((row0 + e) * 2 + f)
                        tot["general_give_merge"] += instr_cost(gm)[0] if gm else 0
                        # parity rule: heads with odd head index give their shared y/z
                        # rows to the previous head (chain-free by construction)
                        pg = []
                        for idx, p in enumerate(heads):
                            x, y, zz = (int(v) for v in cg[p])
                            if idx & 1:
                                q = heads[idx - 1]
                                dx, dy, dz = (int(cg[p][a]) - int(cg[q][a]) for a in range(3))
                                if dx == 0 and (dy or dz) and abs(dy) <= 1 and abs(dz) <= 1 and \
                                        0 <= j + dy <= 1 and 0 <= k + dz <= 1:
                                    continue
                            hy = np.uint32((y + j) * int(PY) & 0xffffffff)
                            hz = np.uint32((zz + k) * int(PZ) & 0xffffffff)
                            for xi in (0, 1):
                                e = int((np.uint32(x + xi) ^ hy ^ hz) & mask)
                                for f in (0, 1):
                                    pg.append((row0 + e) * 2 + f)
                        tot["parity_give_yz"] += instr_cost(pg)[0] if pg else 0
                        a1, dd = instr_cost(cur)
                        a2, _ = instr_cost(xm)
                        tot["current"] += a1
                        tot["x_adjacent_merged"] += a2
                        tot["all_dups_merged"] += dd
                        tot["instructions"] += 1
                segs = set()
                for p in heads:
                    x, y, zz = (int(v) for v in cg[p])
                    for j in (0, 1):
                        for k in (0, 1):
                            hy = np.uint32((y + j) * int(PY) & 0xffffffff)
                            hz = np.uint32((zz + k) * int(PZ) & 0xffffffff)
                            for xi in (0, 1):
                                e = int((np.uint32(x + xi) ^ hy ^ hz) & mask)
                                segs.add((row0 + e) >> 3)
                tot["union_16pt_bound"] += len(segs)
    return tot


def main():
    d = np.load("gpurun_out/points.npz")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    rays, z = d["rays"][:n], d["z_fine"][:n]
    t = model(rays, z, d["box_min"].astype(np.float32), d["box_max"].astype(np.float32))
    for k, v in t.items():
        print(f"{k:20s} {v / n:9.1f} per ray")


if __name__ == "__main__":
    main()
