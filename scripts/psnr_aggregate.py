"""PSNR@5k parity over paired seeds (tests/test_psnr.py runs written with
HN_PSNR_OUT): for each seed the HIP trainer and the reference path train
from the same initial parameters on the same inputs; the metric's bar
(PSNR within +-0.1 dB at equal iterations) is applied to the
mean of the per-seed differences of the tail-median PSNRs.

  usage: python scripts/psnr_aggregate.py OUT.json RUN_seed0.json RUN_seed1.json ...
"""
import json
import sys

import numpy as np

TOL_DB = 0.1
out_path, runs = sys.argv[1], [json.load(open(p)) for p in sys.argv[2:]]
per = [dict(seed=r.get("seed", 0), psnr_hip=r["final"]["psnr_hip"], psnr_ref=r["final"]["psnr_ref"],
            diff=r["final"]["diff"]) for r in runs]
d = np.array([p["diff"] for p in per])
agg = dict(iters=runs[0]["iters"], H=runs[0]["H"], W=runs[0]["W"], N_rand=runs[0]["N_rand"],
           n_train=runs[0]["n_train"], scene=runs[0]["scene"], tol_db=TOL_DB, n_seeds=len(per),
           mean_psnr_hip=round(float(np.mean([p["psnr_hip"] for p in per])), 4),
           mean_psnr_ref=round(float(np.mean([p["psnr_ref"] for p in per])), 4),
           mean_diff=round(float(d.mean()), 4), std_diff=round(float(d.std(ddof=1)), 4) if len(d) > 1 else None,
           per_seed=per, runs=runs)
json.dump(agg, open(out_path, "w"), indent=1)
print(json.dumps({k: v for k, v in agg.items() if k != "runs"}))
assert abs(agg["mean_diff"]) <= TOL_DB, agg["mean_diff"]
