"""Diagnostic: how many memory-side atomic requests would the table-gradient
scatter save if sample runs inside one voxel were merged over longer spans
than today's 16-point DPP row?  Replays recorded samples
(gpurun_out/points.npz from scripts/dump_points.py) through the scatter's
lane layout (see scripts/request_model.py for the cost model):

  group : runs merged inside each 16-point group (today);
  tile  : runs continue across the two groups of a 32-point tile (the
          group-0 tail run is issued with group 1);
  ray   : runs continue across the ray's 192 samples.

  usage: python scripts/request_model_runs.py [n_rays]
"""
import sys

import numpy as np

from request_model import PY, PZ, cells, instr_cost


def cost(c, row0, mask, span):
    """Requests of one ray at one level when runs merge within `span` points;
    instructions stay per 16-point group and hold the heads that start there."""
    tot = 0
    for s0 in range(0, 192, span):
        seg = c[s0:s0 + span]
        heads = [0] + [p for p in range(1, len(seg)) if (seg[p] != seg[p - 1]).any()]
        for g0 in range(0, len(seg), 16):
            hg = [p for p in heads if g0 <= p < g0 + 16]
            if not hg:
                continue
            for j in (0, 1):
                for k in (0, 1):
                    adr = []
                    for p in hg:
                        x, y, zz = (int(v) for v in seg[p])
                        hy = np.uint32((y + j) * int(PY) & 0xffffffff)
                        hz = np.uint32((zz + k) * int(PZ) & 0xffffffff)
                        for xi in (0, 1):
                            e = int((np.uint32(x + xi) ^ hy ^ hz) & mask)
                            adr += [(row0 + e) * 2, (row0 + e) * 2 + 1]
                    tot += instr_cost(adr)[0]
    return tot


def main():
    d = np.load("gpurun_out/points.npz")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    rays, z = d["rays"][:n], d["z_fine"][:n]
    bmin, bmax = d["box_min"].astype(np.float32), d["box_max"].astype(np.float32)
    mask = np.uint32((1 << 19) - 1)
    tot = {"group": 0, "tile": 0, "ray": 0}
    per_level = {k: np.zeros(16) for k in tot}
    for r in range(n):
        o, dd = rays[r, 0:3], rays[r, 3:6]
        pts = (o[None, :] + dd[None, :] * z[r][:, None]).astype(np.float32)
        cl = cells(pts, bmin, bmax)
        for l in range(16):
            for name, span in (("group", 16), ("tile", 32), ("ray", 192)):
                c = cost(cl[l], l << 19, mask, span)
                tot[name] += c
                per_level[name][l] += c
    for k, v in tot.items():
        print(f"{k:6s} {v / n:8.1f} requests/ray  ({v / tot['group']:.3f})")
    print("per level (group):", np.round(per_level["group"] / n, 1).tolist())
    print("per level (ray):  ", np.round(per_level["ray"] / n, 1).tolist())


if __name__ == "__main__":
    main()
