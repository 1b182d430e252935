"""Headline benchmark: training rays/s (fwd+bwd) of the HashNeRF step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|3|4|5]

N = 1 runs BASELINE.json configs[1] (chair, N_rand 4096, 64+128 samples,
L=16 F=2 T=2^19 finest 512) on one MI355X.  N > 1 is launched by torchrun
(one process per GPU, RCCL): data-parallel over rays, per-rank N_rand fixed
(weak scaling), one SUM all-reduce of hash + MLP grads per step.

A step is one full training iteration: on-device ray sampling from a
synthetic 400x400 image set resident in HBM, fused render forward, loss
(MSE fine+coarse, entropy sparsity, TV), fused backward, gradient
all-reduce (N > 1), RAdam step, lr decay.  Rank 0 prints one JSON line.
--config 1 is BASELINE configs[0] (configs/chair.txt verbatim on the CPU
PyTorch path): the oracle's training step (the CPU restatement of the
reference, oracle/) at N_rand 1024, T=2^19, finest 512, precrop window, on
the host cores; it touches no GPU.
TV follows the reference's schedule (run_nerf.py:636-638: through i = 1001),
so the timed steps after the 1000 untimed ones have none -- except config 3,
whose BASELINE entry asks for the TV term on every step.  With one GPU and no
TV term the table's RAdam step runs fused into the backward's owner pass.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # configs/chair.txt:1-19 verbatim: N_rand 1024, 64+128, precrop 500 @ 0.5,
    # lrate 0.01 (README.md:20), T=19, finest 512; the reference's pure-PyTorch
    # CPU path (BASELINE configs[0]: "plumbing, no GPU")
    1: dict(workload="configs/chair.txt on the CPU PyTorch path: N_rand=1024, 64+128, T19 finest512, "
                     "precrop 0.5 (BASELINE configs[0])",
            N_rand=1024, log2_hashmap_size=19, finest_res=512, tv_loss_weight=1e-6),
    2: dict(workload="chair 1xMI355X N_rand=4096 64+128 L16 F2 T19 finest512 (BASELINE configs[1])",
            N_rand=4096, log2_hashmap_size=19, finest_res=512, tv_loss_weight=1e-6),
    3: dict(workload="lego T22 finest1024 N_rand=8192 TV on (BASELINE configs[2])",
            N_rand=8192, log2_hashmap_size=22, finest_res=1024, tv_loss_weight=1e-6, tv_until=10 ** 9),
    4: dict(workload="hotdog DP, N_rand=8192 per GPU (BASELINE configs[3])",
            N_rand=8192, log2_hashmap_size=19, finest_res=512, tv_loss_weight=1e-6),
    # scannet_scene0000.txt: white_bkgd False; the bbox is the mesh bounds
    # (load/load_scannet.py:105), far tighter than the sample range, so most
    # samples are out of the box (extrapolated weights, SURVEY trap 3)
    # use_batching (no_batching False, configs/scannet_scene0000.txt:6): the
    # global shuffled pool of every training ray (run_nerf.py:505-521, 544-555)
    5: dict(workload="scannet-style unbounded scene: bbox +-1 inside the 2..6 sample range, black bkgd, "
                     "sparse_loss_weight 1e-3, use_batching ray pool, N_rand=4096 per GPU, 64+128 "
                     "(BASELINE configs[4])",
            N_rand=4096, log2_hashmap_size=19, finest_res=512, tv_loss_weight=1e-6,
            white_bkgd=False, sparse_loss_weight=1e-3, bbox=((-1., -1., -1.), (1., 1., 1.)), no_batching=False),
}
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
ATOMIC_PEAK_GREQ = round(1.3e12 / 64 / 1e9, 1)   # float atomics: 1.3 TB/s of 64-B requests
PT_BYTES = 16 * 8 * 8          # one point: 16 levels x 8 corners x (2 x fp32)
UNIQUE_PTS = 192               # per ray (the 64 coarse points recur in the fine pass)
# per ray 192 unique points gathered + scatter-added, + 36 B ray I/O
PATH_BYTES_PER_RAY = UNIQUE_PTS * PT_BYTES * 2 + 36
# the backward launch's algorithmic bytes are the scatter-add half: it reads
# the forward's saved features, it does not re-gather the table
BWD_BYTES_PER_RAY = UNIQUE_PTS * PT_BYTES            # bwd launch: scatter-add
FWD_BYTES_PER_RAY = UNIQUE_PTS * PT_BYTES            # fwd kernel: gather
# SURVEY 8(d) FLOPs: NeRFSmall 18,688 FLOP per point forward, 37,376 backward;
# 64 coarse + 192 fine evaluations per ray.  The backward kernel recomputes
# the forward, so it carries both.
MLP_FWD_FLOP_PER_RAY = 256 * 18688
MLP_BWD_FLOP_PER_RAY = 256 * (18688 + 37376)
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA
N_SIMDS = 1024                   # 256 CUs x 4 SIMDs
# the kernels of one hn_render_bwd launch, per table-gradient scatter
BWD_KERNELS = {"atomic": ("render_comp_bwd_kernel", "render_bwd_kernel", "slab_reduce_kernel"),
               # binned: the dW slab reduction runs inside scatter_bins_kernel (HN_SC_SLAB)
               # render_lists_kernel (round 6): the exact-zero skipping's work lists
               "binned": ("render_comp_bwd_kernel", "render_lists_kernel", "render_bwd_kernel",
                          "scatter_bins_kernel", "ovf_place_kernel", "bin_reduce_kernel")}


def measured_traffic(cfg_id, n_rand_override, scene, pretrain, scatter):
    """HBM-side bytes per hn_render_bwd launch from the last PMC passes of the
    same workload (scripts/gpu_pmc.sh -> profiles/traffic_config<N>_<scene>_p<pretrain>_<scatter>.json):
    2 x FETCH_SIZE + WRITE_SIZE summed over the launch's kernels.  PMC
    counters need their own rocprofv3 passes, so bench.py cannot collect
    them live; None when no file matches this workload."""
    path = os.path.join(ROOT, "profiles", f"traffic_config{cfg_id}_{scene}_p{pretrain}_{scatter}.json")
    if n_rand_override or not os.path.exists(path):
        return None, None, None, {}
    t = json.load(open(path))
    ks = t.get("kernels", {})
    # ovf_place_kernel returns at once without spills; render_lists_kernel runs only
    # with exact-zero skipping (and files of older libraries lack it)
    kern = [k for k in BWD_KERNELS[scatter] if k not in ("ovf_place_kernel", "render_lists_kernel") or k in ks]
    if not all(k in ks and "fetch_bytes" in ks[k] for k in kern):
        return None, None, None, ks
    return (sum(ks[k]["fetch_bytes"] + ks[k]["write_bytes"] for k in kern), t.get("source"),
            sum(ks[k].get("atomic_requests", 0.0) for k in kern) or None, ks)


def mfma_busy(ks, kernel, source):
    """MFMA-pipe busy fraction of one kernel from the same PMC file:
    SQ_VALU_MFMA_BUSY_CYCLES (summed over all SIMDs; 32 cycles per
    v_mfma_f32_32x32x16_bf16, 64 per v_mfma_f32_32x32x2_f32) over the SIMD
    cycles of the dispatch, GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs;
    MI355X_MICROARCH.md 'DVFS give-back') x 1024 SIMDs."""
    e = ks.get(kernel, {})
    busy, grbm = e.get("mfma_busy_cycles"), e.get("grbm_gui_active")
    if not busy or not grbm:
        return None
    return {"busy_frac": round(busy / (N_SIMDS * grbm / 8.0), 4), "mfma_busy_cycles": busy,
            "grbm_gui_active": grbm, "source": source}


def _oracle_trainer(cfg, seed=0):
    """The oracle's training state and one training step on the host
    (test infrastructure: the CPU restatement of the reference path, oracle/):
    returns step(i, n_rays, precrop) -> None.  Synthetic blender-style
    cameras at 400 x 400, uniform targets, the config's table size, loss terms
    (sparsity weight, TV while i <= tv_until, bbox and background), fwd + bwd
    + RAdam with the reference's lr decay (run_nerf.py:647-651)."""
    import numpy as np

    from oracle import hashnerf_oracle as O

    T, finest = cfg["log2_hashmap_size"], cfg["finest_res"]
    white = cfg.get("white_bkgd", True)
    sparse_w = cfg.get("sparse_loss_weight", 1e-10)
    tv_w, tv_until = cfg["tv_loss_weight"], cfg.get("tv_until", 1001)
    g = torch.Generator().manual_seed(seed)
    box = tuple(torch.tensor(v) for v in cfg["bbox"]) if "bbox" in cfg else \
        (torch.tensor([-4.02, -4.02, -3.34]), torch.tensor([4.02, 4.02, 3.24]))
    tab = ((torch.rand(16, 2 ** T, 2, generator=g) * 2 - 1) * 1e-4).requires_grad_(True)
    wc = {k: v.requires_grad_(True) for k, v in O.init_nerf_small(g).items()}
    wf = {k: v.requires_grad_(True) for k, v in O.init_nerf_small(g).items()}
    params = [tab] + list(wc.values()) + list(wf.values())
    state = [(torch.zeros_like(p), torch.zeros_like(p)) for p in params]
    res = O.level_resolutions(16, 16, finest)
    H = W = 400
    focal = .5 * W / np.tan(.5 * 0.6911112070083618)
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    lrate, decay = 0.01, cfg.get("lrate_decay", 10)

    def step(i, n, precrop=False):
        c2w = O.pose_spherical(float(i * 37 % 360 - 180), -30.0, 4.0)
        ro, rd = O.get_rays(H, W, K, c2w[:3, :4])
        if precrop:   # run_nerf.py:586-595: the centre 2dH x 2dW window, precrop_frac 0.5
            dH = dW = int(H // 2 * 0.5)
            ro, rd = ro[H // 2 - dH:H // 2 + dH, W // 2 - dW:W // 2 + dW], rd[H // 2 - dH:H // 2 + dH, W // 2 - dW:W // 2 + dW]
        ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
        sel = torch.randperm(ro.shape[0], generator=g)[:n]   # without replacement (:600)
        ro, rd = ro[sel], rd[sel]
        vd = rd / torch.norm(rd, dim=-1, keepdim=True)
        rb = torch.cat([ro, rd, 2 * torch.ones(n, 1), 6 * torch.ones(n, 1), vd], -1)
        ret = O.render_rays(rb, wc, wf, tab, box[0], box[1], res, T,
                            t_rand=torch.rand(n, 64, generator=g),
                            u=torch.rand(n, 128, generator=g), white_bkgd=white)
        loss = O.training_loss(ret, torch.rand(n, 3, generator=g), sparse_w)
        if tv_w and i <= tv_until:
            for l in range(16):                        # run_nerf.py:628-635, loss.py:22-25
                r, cube = O.tv_cube(l, 16, 16, finest)
                mv = torch.randint(0, int(r - cube), (3,), generator=g)
                loss = loss + tv_w * O.total_variation_loss(tab[l], l, mv, T, finest_res=finest)
        for p in params:
            p.grad = None
        loss.backward()
        lr = lrate * (0.1 ** ((i - 1) / (decay * 1000)))   # set after the previous step (:647-651)
        with torch.no_grad():
            for p, (m, v) in zip(params, state):
                O.radam_step(p, p.grad, m, v, i, lr, weight_decay=1e-6 if p is not tab else 0.0,
                             eps=1e-15 if p is tab else 1e-8)

    return step


def cpu_baseline(cfg, steps=3, n_rays=None, warm_rays=256):
    """Oracle (torch-CPU restatement of the reference) training step on the
    config's own shape: n_rays = the config's N_rand rays per step (SURVEY
    8(d): >= 3 timed steps at each config's B, after one warm-up step), same
    table size, the config's loss terms (sparsity weight, TV on every step for
    config 3, the bbox and background), fwd + bwd + RAdam.  The warm-up step
    runs warm_rays rays (the same code path; it only pays first-call costs).
    The timed steps are numbered past the TV window, as the GPU's timed steps
    follow 1000 pretraining steps."""
    threads = torch.get_num_threads()
    n_rays = n_rays or cfg["N_rand"]
    T, finest = cfg["log2_hashmap_size"], cfg["finest_res"]
    tv = cfg.get("tv_until", 1001) > 1001
    step = _oracle_trainer(cfg)
    step(1001, warm_rays)                     # warm-up (first-call costs)
    t0 = time.perf_counter()
    for i in range(steps):
        step(1002 + i, n_rays)
    dt = time.perf_counter() - t0
    return {"value": round(steps * n_rays / dt, 2), "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"{steps} oracle training steps x {n_rays} rays (the config's B; T=2^{T}, finest {finest}, "
                      f"64+128, fwd+bwd+RAdam{', TV' if tv else ''}) on {threads} host threads after a "
                      f"{warm_rays}-ray warm-up step, {dt:.1f} s"}


def bench_config1(args):
    """BASELINE configs[0]: configs/chair.txt verbatim on the CPU PyTorch path
    (the oracle: the reference's algorithm restated in torch-CPU eager ops, as
    the reference runs it on a CPU).  Steps 1..K of a fresh run: N_rand 1024
    from the 200 x 200 precrop window (i < precrop_iters = 500), TV on
    (i <= 1001), RAdam (no update before step 6), lr decay; one warm-up step
    first.  Prints one JSON line; no GPU is touched."""
    cfg = dict(CONFIGS[1], lrate_decay=500)          # configs/chair.txt:10
    threads = torch.get_num_threads()
    B = args.n_rand or cfg["N_rand"]
    step = _oracle_trainer(cfg)
    t0 = time.perf_counter()
    step(1, B, precrop=True)                         # warm-up: the run's first step
    warm = time.perf_counter() - t0
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(2 + i, B, precrop=True)
    dt = time.perf_counter() - t0
    value = args.steps * B / dt
    line = {
        "metric": "training rays/sec (fwd+bwd) on chair; PSNR@5k iters",
        "value": round(value, 2), "unit": "rays/s", "n_gpus": 0, "steps": args.steps, "warmup": 1,
        "ms_per_step": round(dt * 1e3 / args.steps, 1), "higher_is_better": True, "scaling": "none",
        "vs_baseline": None, "dtype": "fp32", "device": f"cpu ({threads} threads)",
        "data": "synthetic: blender-style 400x400 cameras, uniform targets (no dataset in the image)",
        "config": {"workload": cfg["workload"], "rays_per_step": B, "samples_per_ray": "64+128",
                   "log2_hashmap_size": 19, "finest_res": 512, "precrop": "steps 1..499, frac 0.5",
                   "lrate_decay": 500, "parallelism": "none"},
        "path": "oracle/hashnerf_oracle.py: the reference's hot path restated op for op in torch-CPU "
                "(pinned by reference-made golden fixtures, tests/test_oracle_golden.py)",
        "roofline": None,
        "cpu_baseline": {"value": round(value, 2), "unit": "rays/s", "cores": threads, "kind": "port",
                         "sample": f"{args.steps} training steps x {B} rays after a {warm:.1f} s warm-up step"},
    }
    print(json.dumps(line), flush=True)


def optimizer_bytes(tr):
    """HBM bytes the fused table RAdam step must move per launch: p, m and v
    (fp32) read and written for every table parameter it steps -- the dense
    levels whole, the coarse levels' live row pairs only (train.live_pair_mask,
    Trainer.skip_dead_rows)."""
    e = tr.embed_fn
    T, L_, F_ = e.log2_hashmap_size, e.n_levels, 2
    total = L_ * (1 << T) * F_
    lm = tr._live_mask()
    if lm is not None:
        n_lv, words = lm
        import numpy as np
        live_pairs = int(np.unpackbits(words.cpu().numpy().view(np.uint8)).sum())
        total = (L_ - n_lv) * (1 << T) * F_ + live_pairs * 2 * F_
    return total * 4 * 3 * 2


# the data-parallel exchange's phases, timed with HIP events on the compute
# stream (train.ShardedTableStep.step, Trainer.step): reduce-scatter issue to
# wait, the one hn_radam_step launch (table shard + NeRFSmall tensors), the
# all-gather, and the NeRFSmall gradients' all-reduce (issued before the
# reduce-scatter, waited before the step)
XCHG_TIMERS = ("xchg_reduce_scatter", "xchg_step", "xchg_all_gather", "xchg_mlp_allreduce")
# DESIGN.md 7's model of the exchange on one MI355X node: ring collectives
# over xGMI (7 links x ~153 GB/s per GPU, the prompt's figure); each of the
# reduce-scatter and the all-gather moves (N - 1) / N of the vector per rank.
# Bounds: one link's bandwidth (a single ring) and all seven.
XGMI_LINK_GBS = 153.0
XGMI_LINKS = 7


def predicted_exchange_ms(vec_bytes, world):
    """(one-link, seven-link) lower bounds on reduce-scatter + all-gather (ms)."""
    b = 2.0 * (world - 1) / world * vec_bytes
    return (round(b / (XGMI_LINK_GBS * 1e9) * 1e3, 4), round(b / (XGMI_LINKS * XGMI_LINK_GBS * 1e9) * 1e3, 4))


def exchange_report(tr, world, mine, worst, backend):
    """The N > 1 line's exchange fields: the bytes and each phase's time
    (this rank, and the max over ranks), against DESIGN.md 7's prediction."""
    x = tr._xchg
    vec = x.exchange_bytes() if x is not None else None
    mlp = 4 * sum(p.numel() for p in tr._ws)
    rep = {"backend": backend, "segments": len(x.segs) if x is not None else None,
           "exchange_bytes": {"reduce_scatter_in": vec, "all_gather_out": vec, "mlp_allreduce": mlp},
           "rank0_ms": {k.replace("xchg_", ""): round(v, 4) for k, v in zip(XCHG_TIMERS, mine)},
           "max_over_ranks_ms": {k.replace("xchg_", ""): round(v, 4) for k, v in zip(XCHG_TIMERS, worst)},
           "timer": "HIP events on the compute stream around each phase (issue to completion), "
                    "the same kernel-steps loop as the launch times"}
    if vec:
        one, seven = predicted_exchange_ms(vec, world)
        rep["predicted_rs_plus_ag_ms"] = {"one_link": one, "seven_links": seven,
                                          "model": f"2 x (N-1)/N x {vec} B over {XGMI_LINK_GBS} GB/s xGMI links"}
        rep["measured_rs_plus_ag_ms"] = round(worst[0] + worst[2], 4)
    return rep


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`python bench.py --gpus N` (N > 1) outside torchrun: start torchrun with
    N ranks on this node as a CHILD process (one process per GPU, this same
    command line in each) and return its exit code.  Runs before anything
    touches the GPU in this process (no torch.cuda call, no exec)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); N > 1 outside torchrun starts torchrun with N ranks")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=None, choices=sorted(CONFIGS))
    ap.add_argument("--n-rand", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # the default workload is the chair stand-in in its trained regime: 1000
    # untimed steps first (~2 s), so the timed steps see the sample
    # distribution of most of a 5k-iteration run rather than of the first
    # precrop steps of an untrained network
    ap.add_argument("--scene", default="procedural", choices=("uniform", "procedural"),
                    help="uniform: random targets; procedural: train.procedural_field chair images")
    ap.add_argument("--pretrain", type=int, default=1000,
                    help="untimed training steps before warmup")
    ap.add_argument("--kernel-steps", type=int, default=5,
                    help="steps after the timed region whose launches are timed with HIP events (roofline)")
    ap.add_argument("--cpu-steps", type=int, default=3,
                    help="timed oracle steps of the CPU baseline, each at the config's N_rand")
    ap.add_argument("--ray-order", type=int, default=1, choices=(0, 1),
                    help="batch order from the sampler: 1 Morton order of the pixels, 0 draw order")
    ap.add_argument("--dense-table-step", action="store_true",
                    help="A/B: the fused table step over every row (no live-pair mask)")
    ap.add_argument("--dp-chunks", type=int, default=1,
                    help="N > 1: segments of the sharded table exchange, each reduce-scattered as soon as "
                         "the owner pass has formed it (1: one exchange after the backward)")
    ap.add_argument("--prefetch", action="store_true",
                    help="A/B: draw the next step's batch on a side stream beside the backward")
    ap.add_argument("--separate-loss", action="store_true",
                    help="A/B: the loss in its own hn_loss_fwd_bwd launch instead of the backward's pre-pass")
    ap.add_argument("--separate-mlp-step", action="store_true",
                    help="A/B: the MLP RAdam step in its own hn_radam_step launch")
    ap.add_argument("--dense-bwd", action="store_true",
                    help="A/B: the backward also computes the samples whose d raw is exactly zero "
                         "(hn_render_cfg.dense_bwd; the default skips them, same results)")
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for N>1 (nccl = RCCL; gloo only for rehearsals)")
    args = ap.parse_args()

    if args.config == 1:                      # the CPU path: no GPU touched
        if (args.gpus or 1) > 1:
            raise SystemExit("bench.py --config 1 is the CPU path (one process)")
        return bench_config1(args)
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # same per-GPU workload at every N (weak scaling); --config 4 selects the
    # 8192-rays-per-GPU DP configuration of BASELINE configs[3]
    cfg_id = args.config or 2
    cfg = dict(CONFIGS[cfg_id])
    if args.n_rand:
        cfg["N_rand"] = args.n_rand
    # one process per GPU.  RCCL needs a device of its own per rank: refuse
    # before the process group exists (and before any HIP call: the device
    # count comes from the environment / driver query only) rather than let
    # ranks share a device.  gloo rehearsals may stack ranks on one GPU.
    n_dev = torch.cuda.device_count()
    if world > 1 and args.backend == "nccl" and world > n_dev:
        print(f"bench.py: --backend nccl with WORLD_SIZE={world} ranks but {n_dev} visible GPU(s): "
              f"one GPU per rank is required (use --backend gloo for a single-GPU rehearsal)",
              file=sys.stderr, flush=True)
        sys.exit(3)
    local_dev = local % max(n_dev, 1)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    import hn_loader
    hn = hn_loader.load()
    from hashnerf_pytorch_amd import functional as HF
    from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args

    targs = default_args(N_rand=cfg["N_rand"], log2_hashmap_size=cfg["log2_hashmap_size"],
                         finest_res=cfg["finest_res"], tv_loss_weight=cfg["tv_loss_weight"],
                         tv_until=cfg.get("tv_until", 1001), white_bkgd=cfg.get("white_bkgd", True),
                         sparse_loss_weight=cfg.get("sparse_loss_weight", 1e-10),
                         no_batching=cfg.get("no_batching", True))
    t_data = time.perf_counter()
    data = SyntheticBlender(400, 400, 100, dev, seed=0, scene=args.scene)
    t_data = time.perf_counter() - t_data
    if "bbox" in cfg:
        data.bounding_box = tuple(torch.tensor(v) for v in cfg["bbox"])
    tr = Trainer(targs, data, dev, rank=rank, world=world, seed=0, ray_order=args.ray_order)
    tr.skip_dead_rows = not args.dense_table_step
    tr.dp_chunks = args.dp_chunks
    # --prefetch: the next step's rays and uniforms drawn on a side stream
    # beside the backward (the same draws; Trainer.prefetch).  Off by default:
    # measured slower (r05k: 0.996 vs 0.982 ms per step) -- the cross-stream
    # waits cost more than the ~20 us of sampler and RNG launches they move
    tr.prefetch = args.prefetch
    tr.fuse_loss = not args.separate_loss
    tr.fuse_mlp_step = not args.separate_mlp_step
    tr.dense_bwd = args.dense_bwd

    for _ in range(args.pretrain):
        tr.step()                             # reference loop index global_step + 1
    for _ in range(args.warmup):
        tr.step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed region carries no event records (an event pair idles the
    # device ~10 us): the kernels' launch times come from the steps after it
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, mse = tr.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    HF.L.check_device_faults()                # after the timed region: one blocking read
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    # ONE timer for every launch time in the line: HIP events on the launch
    # stream around the forward and the backward launches (the deferred owner
    # pass of world > 1 included) of args.kernel_steps further steps, the same
    # training loop continuing; the committed rocprofv3 kernel-trace summary of
    # the same command agrees with them (profiles/)
    HF.TIMER.reset()
    HF.TIMER.names = {"render_fwd", "render_bwd", "render_bwd_owner"} | set(XCHG_TIMERS)
    HF.TIMER.every = 1
    HF.TIMER.enabled = True
    for _ in range(args.kernel_steps):
        tr.step()
    torch.cuda.synchronize()
    HF.TIMER.enabled = False
    fwd_ms = HF.TIMER.mean_ms("render_fwd")
    bwd_ms = HF.TIMER.mean_ms("render_bwd") + HF.TIMER.mean_ms("render_bwd_owner")
    # N > 1: each rank's exchange phases (same timer), then their max over ranks
    xchg = None
    if world > 1:
        xt = torch.tensor([HF.TIMER.mean_ms(k) for k in XCHG_TIMERS], device=dev)
        xmax = xt.clone()
        dist.all_reduce(xmax, op=dist.ReduceOp.MAX)
        xchg = exchange_report(tr, world, xt.tolist(), xmax.tolist(), args.backend)
    # diagnostic, after the timed region: the host's time to enqueue one step
    # (Python + ctypes; the device runs concurrently) -- at or above
    # ms_per_step the host, not the GPU, would set the step rate
    host = []
    for _ in range(5):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        tr.step()
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    host_ms = 1e3 * sorted(host)[len(host) // 2]
    # what the exact-zero skips had to work with, from one more step's raw
    # sigmas (a sample with raw sigma <= 0 has alpha = 0: no gradient, and its
    # colour enters no output).  Lower bounds of the skipped shares: the
    # kernels' own marks also count samples whose d raw vanishes otherwise
    HF.DEBUG_KEEP = True
    tr.step()
    HF.DEBUG_KEEP = False
    dc, df = HF.LAST["raw_c"][..., 3] <= 0, HF.LAST["raw_f"][..., 3] <= 0
    sparsity = {
        "coarse_units_without_density": round(dc.all(-1).float().mean().item(), 4),
        "fine_units_without_density": round(df.view(-1, 3, 64).all(-1).float().mean().item(), 4),
        "tiles_without_density": round(torch.cat([dc.view(-1, 32), df.view(-1, 32)]).all(-1).float().mean().item(), 4),
        "samples_without_density": round(torch.cat([dc.reshape(-1), df.reshape(-1)]).float().mean().item(), 4),
        "skips": "" if args.dense_bwd else
        "MLP-backward units and scatter units without gradient, zero records, and the forward's colour net "
        "on tiles without density (hn_render_cfg.dense_bwd = 0, skip_dead_color): every output and "
        "gradient as computed densely (tests/test_gpu_driver.py::test_zero_gradient_skip_bitwise)"}
    B = cfg["N_rand"]
    value = world * B * args.steps / dt
    if rank == 0:
        scatter = "binned" if HF.L.lib().hn_render_scatter_mode(tr._cfg, B) == 2 else "atomic"
        traffic, traffic_src, atomics, pmc = measured_traffic(cfg_id, args.n_rand, args.scene, args.pretrain,
                                                              scatter)
        bwd_gbs = B * BWD_BYTES_PER_RAY / (bwd_ms * 1e-3) / 1e9 if bwd_ms > 0 else 0.0
        fwd_gbs = B * FWD_BYTES_PER_RAY / (fwd_ms * 1e-3) / 1e9 if fwd_ms > 0 else 0.0
        path_gbs = value / world * PATH_BYTES_PER_RAY / 1e9
        line = {
            "metric": "training rays/sec (fwd+bwd) on chair; PSNR@5k iters",
            "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3 / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            # encoding, composite, losses, optimizer and every accumulation in f32; the
            # NeRFSmall GEMMs run on the bf16 MFMA with f32 operands split into bf16
            # parts: 3 in the forward (f32-accurate), 2 (~2^-17) in the gradients
            "dtype": "fp32 (MLP GEMMs split-bf16 MFMA: 3 parts fwd, 2 parts grads)",
            "data": ("synthetic: 100 blender-style 400x400 cameras, " +
                     ("uniform random targets" if args.scene == "uniform" else
                      f"procedural chair images (train.procedural_field, rendered in {t_data:.1f} s)") +
                     (f", timed after {args.pretrain} untimed training steps" if args.pretrain else "")),
            "config": {"workload": cfg["workload"], "rays_per_gpu": B, "global_batch": B * world,
                       "samples_per_ray": "64+128", "log2_hashmap_size": cfg["log2_hashmap_size"],
                       "finest_res": cfg["finest_res"], "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm",
                         "kernel": "render_bwd (hn_render_bwd launch: " + " + ".join(BWD_KERNELS[scatter]) + ")",
                         "achieved": round(bwd_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(bwd_gbs / HBM_PEAK_GBS, 4),
                         "traffic": round(traffic) if traffic else None,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes": B * BWD_BYTES_PER_RAY,
                         "bytes_per_ray": BWD_BYTES_PER_RAY, "bytes_per_ray_meaning":
                             "192 unique points x 16 levels x 8 corners x 8 B scatter-added",
                         "launch_ms": round(bwd_ms, 4), "scatter": scatter,
                         "timer": f"HIP events on the launch stream, {args.kernel_steps} steps after the timed region "
                                  "(the same timer for every launch time in this line)",
                         # the forward's gather and the whole step, same peak
                         "fwd_gather": {"kernel": "render_fwd_kernel", "bytes_per_ray": FWD_BYTES_PER_RAY,
                                        "launch_ms": round(fwd_ms, 4), "achieved": round(fwd_gbs, 1),
                                        "frac": round(fwd_gbs / HBM_PEAK_GBS, 4)},
                         "path": {"bytes_per_ray": PATH_BYTES_PER_RAY, "achieved": round(path_gbs, 1),
                                  "frac": round(path_gbs / HBM_PEAK_GBS, 4),
                                  "meaning": "gather + scatter-add + ray I/O per ray x rays/s (whole step)"}},
            "host_enqueue_ms": round(host_ms, 3),
            "kernels": {"render_fwd_ms": round(fwd_ms, 4), "render_fwd_GBs": round(fwd_gbs, 1),
                        "render_bwd_ms": round(bwd_ms, 4),
                        "path_GBs": round(path_gbs, 1), "path_frac": round(path_gbs / HBM_PEAK_GBS, 4)},
            # MFMA: the NeRFSmall GEMMs of the forward (render_fwd_kernel) and of
            # the MLP backward (render_bwd_kernel: forward recompute + backward)
            "mfma": {"peak_TFLOPs": BF16_DENSE_PEAK_TFLOPS, "peak_meaning": "bf16 dense MFMA",
                     "render_fwd_kernel": dict(
                         alg_TFLOPs=round(B * MLP_FWD_FLOP_PER_RAY / (fwd_ms * 1e-3) / 1e12, 1) if fwd_ms > 0 else None,
                         alg_frac=round(B * MLP_FWD_FLOP_PER_RAY / (fwd_ms * 1e-3) / 1e12 / BF16_DENSE_PEAK_TFLOPS, 4)
                         if fwd_ms > 0 else None,
                         pmc=mfma_busy(pmc, "render_fwd_kernel", traffic_src)),
                     "render_bwd_kernel": dict(alg_flop_per_ray=MLP_BWD_FLOP_PER_RAY,
                                               pmc=mfma_busy(pmc, "render_bwd_kernel", traffic_src))},
            "mlp_math": ("NeRFSmall GEMMs on v_mfma_f32_32x32x16_bf16 with f32 operands split into bf16 "
                         "parts: 3 parts in the forward (f32-accurate), 2 in the data/weight gradients"),
            "loss": round(float(loss.item()), 6),
        }
        opt_b = optimizer_bytes(tr) if (world == 1 and tr.fuse_table_step and scatter == "binned") else 0
        if opt_b:
            # the fused table RAdam inside the launch (owner pass): p, m, v read
            # and written on every live row pair -- mandated by the reference's
            # dense optimizer (radam.py:58-92), reported as its own algorithmic
            # term beside the scatter-add bytes ("reported separately")
            alg2 = B * BWD_BYTES_PER_RAY + opt_b
            gbs2 = alg2 / (bwd_ms * 1e-3) / 1e9 if bwd_ms > 0 else 0.0
            line["roofline"].update(
                optimizer_bytes=opt_b, optimizer_bytes_meaning=(
                    "fused table RAdam: p, m, v (3 x 4 B) read + written per live table parameter "
                    f"({opt_b // 24:,} of {16 * 2 ** cfg['log2_hashmap_size'] * 2:,})"),
                with_optimizer={"algorithmic_bytes": alg2, "achieved": round(gbs2, 1),
                                "frac": round(gbs2 / HBM_PEAK_GBS, 4),
                                "traffic_ratio": round(traffic / alg2, 3) if traffic else None})
        if scatter == "atomic" and atomics:
            # the binding resource of the atomic scatter: memory-side float-atomic
            # requests (TCC_EA0_ATOMIC, same PMC passes) per second, against
            # MI355X_MICROARCH.md 'Global float atomics': ~1.3 TB/s of added bytes =
            # 64-B memory-side requests at ~20.3 G/s chip-wide
            rate = atomics / (bwd_ms * 1e-3) / 1e9
            line["roofline"].update(atomic_requests=round(atomics), atomic_Greq_per_s=round(rate, 2),
                                    atomic_peak_Greq_per_s=ATOMIC_PEAK_GREQ,
                                    atomic_frac=round(rate / ATOMIC_PEAK_GREQ, 3))
        line["sparsity"] = sparsity
        if xchg is not None:
            line["exchange"] = xchg
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, steps=args.cpu_steps)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
