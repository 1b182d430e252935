"""Calibration of the short PSNR gate (tests/test_psnr.py) from the paired
400-iteration runs of scripts/gpu_psnr_short_cal.sh: for each candidate
statistic (mean over a tail window of the paired per-evaluation differences
PSNR_hip - PSNR_ref), its spread over seeds at the reference learning rate
(lr x 1) and its shift under a deliberate regression (the HIP side at lr x 0.7).

    python scripts/psnr_short_cal.py gpurun_out/psnr_short_r04i [out.json]
"""
import glob
import json
import os
import sys

import numpy as np


def stat(curve, frac):
    n = curve[-1]["iter"]
    tail = [c for c in curve if c["iter"] > (1. - frac) * n]
    return float(np.mean([c["diff"] for c in tail]))


def main():
    d = sys.argv[1]
    runs = {}
    for f in sorted(glob.glob(os.path.join(d, "short_lr*_seed*.json"))):
        name = os.path.basename(f)[len("short_lr"):-len(".json")]
        lr, seed = name.split("_seed")
        runs.setdefault(lr, {})[int(seed)] = json.load(open(f))
    out = {"source": d, "windows": {}}
    for frac in (1.0, 0.5, 0.25):
        row = {}
        for lr, by_seed in sorted(runs.items()):
            xs = [stat(r["curve"], frac) for _, r in sorted(by_seed.items())]
            row[lr] = dict(n=len(xs), mean=round(float(np.mean(xs)), 4), std=round(float(np.std(xs, ddof=1)), 4)
                           if len(xs) > 1 else None, min=round(min(xs), 4), max=round(max(xs), 4),
                           per_seed=[round(x, 4) for x in xs])
        out["windows"][str(frac)] = row
        print(f"tail {frac}: " + "  ".join(f"lr x{lr}: mean {v['mean']:+.3f} std {v['std']} "
                                           f"[{v['min']:+.3f}, {v['max']:+.3f}]" for lr, v in row.items()))
    finals = {lr: [round(r["final"]["psnr_hip"], 3) for _, r in sorted(b.items())] for lr, b in runs.items()}
    out["final_psnr_hip"] = finals
    print("final HIP PSNR (median over the run's tail):", finals)
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
