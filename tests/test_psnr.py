"""PSNR parity at equal iterations (BASELINE metric "PSNR@5k iters"; SURVEY
8(d): "PSNR within +-0.1 of reference at equal iterations").

nerf-synthetic is not in the image, so both runs train on a procedural chair
(``train.procedural_field``: box/sphere SDF density, textured albedo) whose
views are rendered on the device by dense quadrature.  Two trainings start
from the SAME initial parameters and consume the SAME inputs every step (one
``Trainer.draw_batch`` per step: image, pixels, jitter, importance uniforms,
TV cubes):

* HIP path: ``Trainer`` (explicit mode) -- fused render fwd/bwd, fused loss,
  TV, RAdam kernel, the lr decay of run_nerf.py:647-651;
* reference path: the oracle (our pinned restatement of run_nerf_helpers /
  hash_encoding / loss / radam) evaluated with eager torch ops --
  on the GPU, because 5k reference iterations on the host would take a day;
  its numbers are still those of the reference's algorithm, pinned on the CPU
  by tests/test_oracle_golden.py.

Both are then evaluated on held-out views (deterministic sampling, the test
kwargs of create_nerf) with the reference's per-image PSNR averaged
(run_nerf_helpers.py:430-455).  The trajectories are not bit-identical (MFMA
vs BLAS summation order, atomic order), so the check is the statistical one
the metric states: |PSNR_hip - PSNR_ref| <= 0.1 dB at 5k iterations, averaged
over paired seeds, PSNR being the median over the evaluations in the last 20 %
of a run (one evaluation swings with the optimizer's step noise).  HN_PSNR_SEEDS=k adds k HIP-only runs
at other seeds, to show how far two equally good runs land apart.

HN_PSNR_REF_CACHE=run.json re-runs only the HIP side of a seed against the
reference curve of an earlier paired run (the reference path depends on the
seed alone; scripts/gpu_psnr_seq.sh checks it by re-running one seed in full).

The gate the GPU suite runs (test_psnr_short_gate) is short: 4 paired seeds of 400 iterations at 100x100 (50 views), each
evaluated every 25 iterations; its statistic is the mean over the seeds of
each run's mean paired difference PSNR_hip - PSNR_ref over its 16
evaluations.  Calibration (scripts/gpu_psnr_short_cal.sh r04i, 6 seeds each,
profiles/r04/psnr_short_cal_r04i.json): a run's statistic has mean -0.008 dB
and std 0.275 dB at the reference learning rate, and mean -0.683 dB (std
0.448) with the HIP side's lr x 0.7 (a deliberate regression).  Over 4 seeds
the mean's std is 0.137 dB, so the band |mean| <= 0.3 dB (TOL_DB_SHORT4)
passes parity ~97 % of the time for a trajectory-changing code edit and fails
the lr x 0.7 regression ~95 % of the time; each run alone is held to 1.0 dB
(~3.6 sigma).

test_psnr_parity_equal_iterations is the configurable single run
(HN_PSNR_ITERS etc.; skipped unless HN_PSNR_ITERS is set):
HN_PSNR_ITERS=5000 HN_PSNR_EVERY=100 HN_PSNR_RES=200 HN_PSNR_NTRAIN=100
HN_PSNR_OUT=path gives one paired run at 5k iterations (HN_PSNR_SEED picks
its seed) and writes the curve as JSON.  The "@5k" figure is the mean over
paired seeds, checked against +-0.1 dB by scripts/psnr_aggregate.py
(scripts/gpu_psnr_seq.sh; profiles/r03/psnr_5k_r03y.json): one paired run
alone is checked against 0.37 dB (TOL_DB_RUN), 3 standard deviations of the
paired difference of single runs (0.124 dB over 23 seeds).
"""
import json
import math
import os
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_DB = 0.1          # at 5k iterations: the metric's bar, on the mean over paired seeds (its 95 %
                      # confidence interval, scripts/psnr_aggregate.py)
TOL_DB_RUN = 0.37     # one paired run at 5k iterations: 3 sigma of the paired difference over the
                      # 23 paired seeds of round 3 (mean +0.021 dB, std 0.124 dB,
                      # profiles/r03/psnr_5k_r03y.json); the 0.1 dB bar is carried by the mean
TOL_DB_SHORT = 0.75   # a single configurable short run (test_psnr_parity_equal_iterations)
TOL_DB_SHORT4 = 0.3   # the short gate: |mean over 4 paired seeds| (calibration above)
TOL_DB_SHORT1 = 1.0   # ... and each of its runs alone
# seeds of the short gate: those whose 400-iteration HIP PSNR clears the
# floor by >= 1 dB in the calibration (final_psnr_hip at lr x 1, seeds 0-5:
# 13.98, 12.65, 12.59, 13.06, 15.16, 13.82 dB; profiles/r04/psnr_short_cal_r04i.json):
# seeds 0, 3, 4, 5 (13.06-15.16 dB).  Their calibrated statistics: lr x 1
# +0.118 / +0.011 / -0.100 / +0.128 (mean +0.039 dB, inside the 0.3 dB band),
# lr x 0.7 -1.454 / -0.625 / -0.839 / -0.607 (mean -0.881 dB: fails it)
SHORT_SEEDS = (0, 3, 4, 5)
FLOOR_DB_SHORT = 12.0  # a short run's last HIP evaluation must clear this: the untrained
                       # (all-white) prediction scores 9.07 dB on its 4 test views; the HIP
                       # path reaches 12.59-15.16 dB at iteration 400 over seeds 0-5 at the
                       # reference lr (13.06-15.16 on SHORT_SEEDS)


def _oracle_trainer(O, tr, dev):
    """Reference-path state initialised from the HIP trainer's parameters."""
    tab = tr.embed_fn.table.detach().clone().requires_grad_(True)
    wc = {k: w.detach().clone().requires_grad_(True)
          for k, w in zip(O.MLP_KEYS, tr.kw_train["network_fn"].weights())}
    wf = {k: w.detach().clone().requires_grad_(True)
          for k, w in zip(O.MLP_KEYS, tr.kw_train["network_fine"].weights())}
    params = [(tab, 0.0, 1e-15)] + [(p, 1e-6, 1e-8) for p in list(wc.values()) + list(wf.values())]
    state = [(torch.zeros_like(p), torch.zeros_like(p)) for p, _, _ in params]
    return tab, wc, wf, params, state


def _oracle_step(O, ref, i, batch, args, box, res, T, lr):
    """run_nerf.py:608-651 on the oracle: render_rays + loss (+ TV while
    i <= tv_until) + backward + RAdam (radam.py:58-92)."""
    tab, wc, wf, params, state = ref
    ret = O.render_rays(batch["rays"], wc, wf, tab, box[0], box[1], res, T,
                        t_rand=batch["t_rand"], u=batch["u"], white_bkgd=True)
    loss = O.training_loss(ret, batch["target"], args.sparse_loss_weight)
    if batch["tv"] is not None:
        _, mv = batch["tv"]
        tv = sum(O.total_variation_loss(tab[l], l, mv[l], T, finest_res=args.finest_res)
                 for l in range(16))
        loss = loss + args.tv_loss_weight * tv
    for p, _, _ in params:
        p.grad = None
    loss.backward()
    with torch.no_grad():
        for (p, wd, eps), (m, v) in zip(params, state):
            O.radam_step(p, p.grad, m, v, i, lr, weight_decay=wd, eps=eps)
    return float(torch.mean((ret["rgb_map"].detach() - batch["target"]) ** 2))


@torch.no_grad()
def _eval_oracle(O, ref, data, box, res, T, chunk=4096):
    tab, wc, wf, _, _ = ref
    psnrs = []
    for c2w, gt in zip(data.test_poses, data.test_images):
        ro, rd = O.get_rays(data.H, data.W, data.K, c2w[:3, :4].cpu())
        ro, rd = ro.reshape(-1, 3).to(DEV), rd.reshape(-1, 3).to(DEV)
        vd = rd / torch.norm(rd, dim=-1, keepdim=True)
        rb = torch.cat([ro, rd, 2. * torch.ones_like(rd[:, :1]), 6. * torch.ones_like(rd[:, :1]), vd], -1)
        rgb = torch.cat([O.render_rays(rb[k:k + chunk], wc, wf, tab, box[0], box[1], res, T,
                                       white_bkgd=True)["rgb_map"] for k in range(0, rb.shape[0], chunk)])
        psnrs.append(-10. * math.log10(float(torch.mean((rgb.reshape(gt.shape) - gt) ** 2))))
    return float(np.mean(psnrs)), psnrs


@torch.no_grad()
def _eval_hip(hn, tr, data):
    hwf = (data.H, data.W, data.focal)
    kw = dict(tr.kw_test, near=2., far=6.)
    hn.render_path(data.test_poses, hwf, data.K, 4096, kw, gt_imgs=data.test_images)
    ps = list(hn.render_path.last_psnrs)
    return float(np.mean(ps)), ps


_DATA = {}


def _paired_run(hn, oracle, iters, every, H, n_train, n_test, seed, tail_frac, lr_scale=1.0, cpath=None,
                seeds_extra=0):
    """One paired training run (HIP trainer and reference path from the same
    initial parameters and inputs); returns the run's record."""
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
    O = oracle
    W = H
    args = default_args(N_rand=1024, H=H, W=W, n_train=n_train)
    key = (H, n_train, n_test)
    if key not in _DATA:
        _DATA.clear()
        _DATA[key] = SyntheticBlender(H, W, n_train, DEV, scene="procedural", n_test=n_test)
    data = _DATA[key]
    tr = Trainer(args, data, DEV, seed=seed)
    ref_lrate = args.lrate
    tr.args.lrate = ref_lrate * lr_scale        # (tr.args is args)
    for g in tr.optimizer.param_groups:
        g["lr"] *= lr_scale
    box = tuple(torch.as_tensor(t, dtype=torch.float32).to(DEV) for t in data.bounding_box)
    res = O.level_resolutions(16, 16, args.finest_res)
    T = args.log2_hashmap_size
    ref = _oracle_trainer(O, tr, DEV)
    # HN_PSNR_REF_CACHE=run.json: the reference path's curve from an earlier
    # paired run at the same seed and settings.  The reference path is a
    # function of the seed alone (its initial parameters and every batch come
    # from the same Trainer streams, and nothing it runs is library code), so
    # its PSNR at an iteration is the same number on every library version;
    # only the HIP side is re-run.  (A paired run of the same seed checks this:
    # scripts/psnr_aggregate.py compares the curves of runs sharing a seed.)
    cache = None
    if cpath:
        cache = json.load(open(cpath))
        for key, want in (("seed", seed), ("iters", iters), ("H", H), ("W", W), ("n_train", n_train),
                          ("n_test", n_test), ("N_rand", args.N_rand)):
            assert cache.get(key) == want, f"reference cache {cpath}: {key} {cache.get(key)} != {want}"
        cache = {c["iter"]: c["psnr_ref"] for c in cache["curve"]}
    curve = []
    t_hip = t_ref = 0.0
    lr = lr0 = ref_lrate                       # the reference path's own lr
    for i in range(1, iters + 1):                  # the reference loop's index (run_nerf.py:538-541)
        batch = tr.draw_batch(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step(i, batch)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if cache is None:
            _oracle_step(O, ref, i, batch, args, box, res, T, lr)
        torch.cuda.synchronize()
        t_hip += t1 - t0
        t_ref += time.perf_counter() - t1
        lr = lr0 * (0.1 ** ((i - 1) / (args.lrate_decay * 1000)))   # run_nerf.py:647-651
        assert abs(lr * lr_scale - tr.optimizer.param_groups[0]["lr"]) <= 1e-12 * max(lr, 1.0)
        if (i % every == 0 and (i > (1. - tail_frac) * iters or i % (5 * every) == 0)) or i == iters:
            ph, _ = _eval_hip(hn, tr, data)
            pr = cache[i] if cache is not None else _eval_oracle(O, ref, data, box, res, T)[0]
            curve.append(dict(iter=i, psnr_hip=round(ph, 4), psnr_ref=round(pr, 4),
                              diff=round(ph - pr, 4)))
            print(f"iter {i}: PSNR hip {ph:.3f}  ref {pr:.3f}  diff {ph - pr:+.3f}", flush=True)
    # the statistic: median PSNR over the evaluations in the last 20 % (or
    # HN_PSNR_TAIL) of the run (a single evaluation swings with the optimizer's
    # step noise)
    tail = [c for c in curve if c["iter"] > (1. - tail_frac) * iters] or curve[-1:]
    med = lambda k: round(float(np.median([c[k] for c in tail])), 4)
    mean = lambda k: round(float(np.mean([c[k] for c in tail])), 4)
    stat = dict(psnr_hip=med("psnr_hip"), psnr_ref=med("psnr_ref"), n_evals=len(tail),
                from_iter=tail[0]["iter"], mean_hip=mean("psnr_hip"), mean_ref=mean("psnr_ref"))
    stat["diff"] = round(stat["psnr_hip"] - stat["psnr_ref"], 4)
    # the lower-variance statistic the multi-seed aggregate uses: the mean over
    # the tail evaluations of the paired (same-iteration) differences
    stat["diff_mean"] = mean("diff")
    # secondary, robust to single-evaluation spikes: the median over the tail
    # evaluations of the paired differences
    stat["diff_pmed"] = med("diff")
    # scale of the bar: the HIP path alone at other seeds (other images,
    # pixels, jitter and init) -- how far two equally good runs land apart
    spread = []
    for sd in range(seed + 1, seed + seeds_extra + 1):
        t2 = Trainer(args, data, DEV, seed=sd)
        ps = []
        for i in range(1, iters + 1):
            t2.step(i)
            if i % every == 0 and i > (1. - tail_frac) * iters:
                ps.append(_eval_hip(hn, t2, data)[0])
        spread.append(round(float(np.median(ps)), 4))
    if spread:
        stat["hip_other_seeds"] = spread
    tol = TOL_DB_RUN if iters >= 5000 else TOL_DB_SHORT
    out = dict(iters=iters, seed=seed, H=H, W=W, N_rand=args.N_rand, n_train=n_train, n_test=n_test, tail=tail_frac,
               ref_cache=cpath or None,
               scene="procedural chair (train.procedural_field)", tol_db=tol, final=stat, curve=curve,
               ms_per_iter_hip=round(1e3 * t_hip / iters, 3),
               ms_per_iter_ref_eager_gpu=round(1e3 * t_ref / iters, 3))
    print(json.dumps(out["final"]), flush=True)
    return out


def test_psnr_parity_equal_iterations(hn, oracle):
    """The configurable single paired run (HN_PSNR_* in the module
    docstring); the GPU suite's gate is test_psnr_short_gate."""
    if "HN_PSNR_ITERS" not in os.environ:
        pytest.skip("set HN_PSNR_ITERS (e.g. 5000) for a configurable paired run")
    iters = int(os.environ["HN_PSNR_ITERS"])
    every = int(os.environ.get("HN_PSNR_EVERY", str(max(iters // 8, 1))))
    # HN_PSNR_LR_SCALE (calibration only): the HIP side trains at a scaled
    # learning rate -- a deliberate regression that shows what size of PSNR
    # loss the gate catches
    out = _paired_run(hn, oracle, iters, every, int(os.environ.get("HN_PSNR_RES", "100")),
                      int(os.environ.get("HN_PSNR_NTRAIN", "50")), int(os.environ.get("HN_PSNR_NTEST", "4")),
                      int(os.environ.get("HN_PSNR_SEED", "0")), float(os.environ.get("HN_PSNR_TAIL", "0.2")),
                      float(os.environ.get("HN_PSNR_LR_SCALE", "1")), os.environ.get("HN_PSNR_REF_CACHE"),
                      int(os.environ.get("HN_PSNR_SEEDS", "0")))
    path = os.environ.get("HN_PSNR_OUT")
    if path:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    stat = out["final"]
    assert out["curve"][-1]["psnr_hip"] > (FLOOR_DB_SHORT if out["iters"] < 5000 else 12.0), \
        "the HIP path did not learn the scene"
    assert abs(stat["diff_mean"]) <= out["tol_db"], out


def test_psnr_short_gate(hn, oracle):
    """The short gate in one test (no state shared between tests, so -k
    selection, xdist or reordering cannot skip its band): for each of the 4
    seeds one paired run of 400 iterations evaluated every 25 -- its statistic
    is the mean paired difference over the 16 evaluations, held to 1.0 dB
    alone, and its last HIP evaluation must clear the floor -- then
    |mean over the seeds| <= 0.3 dB (calibration: module docstring)."""
    per = {}
    for seed in SHORT_SEEDS:
        out = _paired_run(hn, oracle, 400, 25, 100, 50, 4, seed, 1.0)
        d = out["final"]["diff_mean"]
        per[seed] = d
        assert out["curve"][-1]["psnr_hip"] > FLOOR_DB_SHORT, ("the HIP path did not learn the scene", seed)
        assert abs(d) <= TOL_DB_SHORT1, (seed, out["final"])
    m = float(np.mean([per[s] for s in SHORT_SEEDS]))
    print(f"short PSNR gate: per-seed {per}, mean {m:+.3f} dB", flush=True)
    assert abs(m) <= TOL_DB_SHORT4, (m, per)
