"""PSNR@5k parity over paired seeds (tests/test_psnr.py runs written with
HN_PSNR_OUT): for each seed the HIP trainer and the reference path train
from the same initial parameters on the same inputs; the metric's bar
(PSNR within +-0.1 dB at equal iterations) is applied to the
mean over seeds of each run's tail-mean paired difference (the mean, over the
evaluations of the last 20 % of the run, of PSNR_hip - PSNR_ref at the same
iteration), with its 95 % confidence interval (Student t, n - 1 dof): parity
is shown when the whole interval lies inside +-0.1 dB.

  usage: python scripts/psnr_aggregate.py OUT.json RUN_seed0.json RUN_seed1.json ...
"""
import json
import sys

import numpy as np
from scipy import stats

TOL_DB = 0.1
out_path, runs = sys.argv[1], [json.load(open(p)) for p in sys.argv[2:]]
per = [dict(seed=r.get("seed", 0), psnr_hip=r["final"]["psnr_hip"], psnr_ref=r["final"]["psnr_ref"],
            diff_median=r["final"]["diff"], diff=r["final"].get("diff_mean", r["final"]["diff"]),
            diff_pmed=r["final"].get("diff_pmed"))
       for r in runs]
d = np.array([p["diff"] for p in per])
n = len(d)
mean = float(d.mean())
sd = float(d.std(ddof=1)) if n > 1 else float("nan")
se = sd / np.sqrt(n) if n > 1 else float("nan")
half = float(stats.t.ppf(0.975, n - 1) * se) if n > 1 else float("nan")
agg = dict(iters=runs[0]["iters"], H=runs[0]["H"], W=runs[0]["W"], N_rand=runs[0]["N_rand"],
           n_train=runs[0]["n_train"], n_test=runs[0].get("n_test"), scene=runs[0]["scene"], tol_db=TOL_DB,
           statistic="mean over seeds of the tail-mean paired difference PSNR_hip - PSNR_ref",
           n_seeds=n, mean_psnr_hip=round(float(np.mean([p["psnr_hip"] for p in per])), 4),
           mean_psnr_ref=round(float(np.mean([p["psnr_ref"] for p in per])), 4),
           mean_diff=round(mean, 4), std_diff=round(sd, 4), se_diff=round(se, 4),
           ci95=[round(mean - half, 4), round(mean + half, 4)],
           parity_shown=bool(n > 1 and abs(mean) + half <= TOL_DB),
           per_seed=per, runs=runs)
# secondary statistic (reported, not the bar): per run, the median over the
# tail evaluations of the paired differences (robust to one evaluation's spike)
dp = np.array([p["diff_pmed"] for p in per if p["diff_pmed"] is not None])
if len(dp) > 1:
    se2 = float(dp.std(ddof=1)) / np.sqrt(len(dp))
    h2 = float(stats.t.ppf(0.975, len(dp) - 1) * se2)
    agg["secondary_paired_median"] = dict(n=len(dp), mean=round(float(dp.mean()), 4), se=round(se2, 4),
                                          ci95=[round(float(dp.mean()) - h2, 4), round(float(dp.mean()) + h2, 4)])
json.dump(agg, open(out_path, "w"), indent=1)
print(json.dumps({k: v for k, v in agg.items() if k not in ("runs", "per_seed")}))
