"""Generate golden fixtures by running the REFERENCE's own Python on CPU.

Run in the survey container only (``/root/reference`` must exist):

    python tests/golden/make_golden.py

The reference is imported read-only through the non-invasive shim described
in SURVEY.md 8(c) (kornia stub, BOX_OFFSETS created on CPU, two shipped
ImportErrors bridged); nothing from the reference is copied.  Inputs are
drawn from numpy PCG64 streams so every fixture is reproducible, and each
fixture stores inputs + reference outputs as small ``.npz`` files next to
this script.  ``tests/test_oracle_golden.py`` pins ``oracle/`` against them.
"""
from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    kornia = types.ModuleType("kornia")

    def create_meshgrid(H, W, normalized_coordinates=True, device=None, dtype=torch.float32):
        xs = torch.linspace(0, W - 1, W, dtype=dtype)
        ys = torch.linspace(0, H - 1, H, dtype=dtype)
        if normalized_coordinates:
            xs = (xs / (W - 1) - 0.5) * 2
            ys = (ys / (H - 1) - 0.5) * 2
        gy, gx = torch.meshgrid(ys, xs, indexing="ij")
        return torch.stack([gx, gy], -1)[None]

    kornia.create_meshgrid = create_meshgrid
    sys.modules.setdefault("kornia", kornia)
    orig = torch.tensor

    def cpu_tensor(*a, **kw):
        if kw.get("device") == "cuda":
            kw["device"] = "cpu"
        return orig(*a, **kw)

    torch.tensor = cpu_tensor
    try:
        he = importlib.import_module("embedding.hash_encoding")
    finally:
        torch.tensor = orig
    sh = importlib.import_module("embedding.spherical_harmonic")
    he.SHEncoder = sh.SHEncoder
    importlib.import_module("embedding.embedder").get_embedder = None
    ref = types.SimpleNamespace(
        rnh=importlib.import_module("run_nerf_helpers"), he=he, sh=sh,
        models=importlib.import_module("models"), loss=importlib.import_module("loss"),
        radam=importlib.import_module("radam"), bbox=importlib.import_module("bbox"),
        ray_util=importlib.import_module("ray_util"),
        blender_pose=None)
    return ref


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def pose_spherical(theta, phi, radius):
    # load/load_blender.py:30-35 (load_blender imports imageio/cv2: absent here).
    t = torch.Tensor([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, radius], [0, 0, 0, 1]]).float()
    ph, th = phi / 180. * np.pi, theta / 180. * np.pi
    rp = torch.Tensor([[1, 0, 0, 0], [0, np.cos(ph), -np.sin(ph), 0],
                       [0, np.sin(ph), np.cos(ph), 0], [0, 0, 0, 1]]).float()
    rt = torch.Tensor([[np.cos(th), 0, -np.sin(th), 0], [0, 1, 0, 0],
                       [np.sin(th), 0, np.cos(th), 0], [0, 0, 0, 1]]).float()
    c2w = rt @ (rp @ t)
    return torch.Tensor(np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]])) @ c2w


CAM_ANGLE_X = 0.6911112070083618


def cameras(n=40):
    thetas = np.linspace(-180, 180, n + 1)[:-1]
    return [pose_spherical(float(t), -30.0 if k % 2 == 0 else -60.0, 4.0) for k, t in enumerate(thetas)]


def gen_hash(ref):
    g = rng(1)
    coords = np.concatenate([
        np.array([[3, 5, 7], [100000, 200000, 300000], [-3, -5, -7], [0, 0, 0], [512, 512, 512],
                  [1023, 0, 1], [-1, 2 ** 20, 7]], dtype=np.int64),
        g.integers(-2 ** 24, 2 ** 24, size=(256, 3), dtype=np.int64)], 0)
    out = {"coords": coords}
    for T in (12, 19, 22):
        out[f"h{T}"] = ref.he.hash(torch.from_numpy(coords)[:, None, :], T)[:, 0].numpy()
    save("hash", **out)


def make_embedder(ref, box, T, finest, table_seed):
    emb = ref.he.HashEmbedder(bounding_box=box, log2_hashmap_size=T, finest_resolution=finest)
    g = rng(table_seed)
    tab = (g.random((16, 2 ** T, 2), dtype=np.float32) * 2 - 1) * 0.5
    with torch.no_grad():
        for l in range(16):
            emb.embeddings[l].weight.copy_(torch.from_numpy(tab[l]))
    return emb, tab


def gen_encode(ref):
    box = (torch.tensor([-1.5, -1.2, -1.0]), torch.tensor([1.3, 1.1, 1.25]))
    for T, finest, name in ((12, 512, "encode_t12"), (12, 1024, "encode_t12_f1024")):
        emb, tab = make_embedder(ref, box, T, finest, 7)
        g = rng(11)
        n = 500
        lo, hi = box[0].numpy(), box[1].numpy()
        x = g.uniform(lo, hi, size=(n, 3)).astype(np.float32)
        x[:20] = g.uniform(lo - 0.6, hi + 0.6, size=(20, 3)).astype(np.float32)   # trap 3
        x[20] = hi
        x[21] = lo
        x[22] = [hi[0], lo[1], 0.0]
        xt = torch.from_numpy(x)
        feat, keep = emb(xt)
        dfeat = torch.from_numpy(g.standard_normal(feat.shape).astype(np.float32))
        (feat * dfeat).sum().backward()
        grad = np.stack([emb.embeddings[l].weight.grad.numpy() for l in range(16)], 0)
        save(name, box_min=box[0].numpy(), box_max=box[1].numpy(), log2T=T, finest=finest,
             table_seed=7, x=x, feat=feat.detach().numpy(), keep=keep.numpy(), dfeat=dfeat.numpy(),
             grad=grad, resolutions=np.array([float(r) for r in
                                               [torch.floor(emb.base_resolution * emb.b ** i)
                                                for i in range(16)]], dtype=np.float32))


def gen_sh(ref):
    g = rng(3)
    d = g.standard_normal((300, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    d[0] = [0, 0, 1]
    d[1] = [1, 0, 0]
    out = ref.sh.SHEncoder()(torch.from_numpy(d))
    save("sh", dirs=d, out=out.numpy())


def make_mlps(ref, seed):
    torch.manual_seed(seed)
    kw = dict(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3,
              hidden_dim_color=64, input_ch=32, input_ch_views=16)
    return ref.models.NeRFSmall(**kw), ref.models.NeRFSmall(**kw)


def mlp_weights(m):
    return {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}


def gen_mlp(ref):
    m, _ = make_mlps(ref, 0)
    g = rng(5)
    x = g.standard_normal((333, 48)).astype(np.float32)
    xt = torch.from_numpy(x).requires_grad_(True)
    out = m(xt)
    dout = torch.from_numpy(g.standard_normal(out.shape).astype(np.float32))
    (out * dout).sum().backward()
    arrays = {"x": x, "out": out.detach().numpy(), "dout": dout.numpy(), "dx": xt.grad.numpy()}
    for k, v in m.named_parameters():
        arrays["w:" + k] = v.detach().numpy()
        arrays["g:" + k] = v.grad.numpy()
    save("mlp", **arrays)


def gen_raw2outputs(ref):
    g = rng(9)
    B, S = 40, 64
    raw = g.standard_normal((B, S, 4)).astype(np.float32) * 2
    raw[0, :, 3] = -1.0                      # all-zero sigma after relu -> NaN depth
    raw[1, :, 3] = 50.0                      # opaque
    z = np.sort(g.uniform(2, 6, size=(B, S)).astype(np.float32), -1)
    d = g.standard_normal((B, 3)).astype(np.float32)
    out = {}
    for white in (False, True):
        rawt = torch.from_numpy(raw).requires_grad_(True)
        rgb, disp, acc, w, depth, ent = ref.rnh.raw2outputs(rawt, torch.from_numpy(z), torch.from_numpy(d),
                                                           0, white)
        grgb = torch.from_numpy(g.standard_normal(rgb.shape).astype(np.float32))
        gent = torch.from_numpy(g.standard_normal(ent.shape).astype(np.float32))
        gacc = torch.from_numpy(g.standard_normal(acc.shape).astype(np.float32))
        loss = (rgb * grgb).sum() + (ent * gent).sum() + (acc * gacc).sum()
        loss.backward()
        sfx = "_w" if white else ""
        out.update({"rgb" + sfx: rgb.detach().numpy(), "disp" + sfx: disp.detach().numpy(),
                    "acc" + sfx: acc.detach().numpy(), "weights" + sfx: w.detach().numpy(),
                    "depth" + sfx: depth.detach().numpy(), "entropy" + sfx: ent.detach().numpy(),
                    "grgb" + sfx: grgb.numpy(), "gent" + sfx: gent.numpy(), "gacc" + sfx: gacc.numpy(),
                    "draw" + sfx: rawt.grad.numpy()})
    save("raw2outputs", raw=raw, z=z, rays_d=d, **out)


def gen_sample_pdf(ref):
    g = rng(13)
    B = 50
    bins = np.sort(g.uniform(2, 6, size=(B, 63)).astype(np.float32), -1)
    w = g.random((B, 62), dtype=np.float32) ** 4
    w[0] = 0.0
    w[1, 10] = 1.0
    u = g.random((B, 128), dtype=np.float32)
    # u must be given: monkeypatch torch.rand for the single draw inside sample_pdf.
    orig = torch.rand
    torch.rand = lambda *a, **k: torch.from_numpy(u)
    try:
        s = ref.rnh.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), 128, det=False)
    finally:
        torch.rand = orig
    sdet = ref.rnh.sample_pdf(torch.from_numpy(bins), torch.from_numpy(w), 128, det=True)
    save("sample_pdf", bins=bins, weights=w, u=u, samples=s.numpy(), samples_det=sdet.numpy())


def scene(ref, H=40, W=40):
    focal = .5 * W / np.tan(.5 * CAM_ANGLE_X)
    cams = cameras()
    meta = {"camera_angle_x": CAM_ANGLE_X,
            "frames": [{"transform_matrix": c.numpy().tolist()} for c in cams]}
    box = ref.bbox.get_bbox3d_for_blenderobj(meta, H, W, near=2.0, far=6.0)
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    return cams, box, K, focal


def gen_bbox_rays(ref):
    H = W = 400
    cams, box, K, focal = scene(ref, H, W)
    ro, rd = ref.ray_util.get_rays(H, W, K, cams[3][:3, :4])
    sel = rng(17).integers(0, H * W, size=256)
    save("bbox_rays", cams=np.stack([c.numpy() for c in cams]), H=H, W=W, focal=focal,
         box_min=box[0].numpy(), box_max=box[1].numpy(), K=K, sel=sel,
         rays_o=ro.reshape(-1, 3)[sel].numpy(), rays_d=rd.reshape(-1, 3)[sel].numpy())


def gen_render(ref, name, T=14, finest=512, B=64, white=True, perturb=1.0, seed=21,
               sparse_w=1e-3):
    H = W = 40
    cams, box, K, focal = scene(ref, H, W)
    emb, tab = make_embedder(ref, box, T, finest, seed)
    shenc = ref.sh.SHEncoder()
    mc, mf = make_mlps(ref, seed)
    g = rng(seed)
    pose = cams[5][:3, :4]
    ro, rd = ref.ray_util.get_rays(H, W, K, pose)
    sel = g.choice(H * W, size=B, replace=False)
    rays_o = ro.reshape(-1, 3)[sel]
    rays_d = rd.reshape(-1, 3)[sel]
    target = torch.from_numpy(g.random((B, 3), dtype=np.float32))
    nq = lambda inputs, viewdirs, fn: ref.rnh.run_network(inputs, viewdirs, fn, embed_fn=emb,
                                                          embeddirs_fn=shenc, netchunk=65536)
    kw = dict(network_query_fn=nq, perturb=perturb, N_importance=128, network_fine=mf,
              N_samples=64, network_fn=mc, embed_fn=emb, use_viewdirs=True, white_bkgd=white,
              raw_noise_std=0., ndc=False, lindisp=False, near=2., far=6., pytest=True)
    rgb, depth, acc, extras = ref.rnh.render(H, W, K, chunk=32768, rays=torch.stack([rays_o, rays_d], 0),
                                              retraw=True, **kw)
    loss = torch.mean((rgb - target) ** 2) + torch.mean((extras["rgb0"] - target) ** 2)
    loss = loss + sparse_w * (extras["sparsity_loss"].sum() + extras["sparsity_loss0"].sum())
    loss.backward()
    # the pytest hooks (run_nerf_helpers.py:531-534, 279-287) use np.random.seed(0)
    np.random.seed(0)
    t_rand = np.random.rand(B, 64).astype(np.float32)
    if perturb > 0:
        np.random.seed(0)
        u = np.random.rand(B, 128).astype(np.float32)
    else:   # det=True under pytest: np.linspace cast to fp32 (:283-287)
        u = np.broadcast_to(np.linspace(0., 1., 128), (B, 128)).astype(np.float32)
    grad = np.stack([emb.embeddings[l].weight.grad.numpy() for l in range(16)], 0)
    arrays = dict(box_min=box[0].numpy(), box_max=box[1].numpy(), log2T=T, finest=finest,
                  table_seed=seed, white=white, perturb=perturb, sparse_w=sparse_w,
                  rays_o=rays_o.numpy(), rays_d=rays_d.numpy(), target=target.numpy(),
                  t_rand=t_rand, u=u, rgb=rgb.detach().numpy(), depth=depth.detach().numpy(),
                  acc=acc.detach().numpy(), loss=loss.detach().numpy(),
                  table_grad=grad)
    for k in ("rgb0", "depth0", "acc0", "sparsity_loss", "sparsity_loss0", "z_std", "raw"):
        arrays[k] = extras[k].detach().numpy()
    for tag, m in (("c", mc), ("f", mf)):
        for k, v in m.named_parameters():
            arrays[f"w{tag}:{k}"] = v.detach().numpy()
            arrays[f"g{tag}:{k}"] = v.grad.numpy()
    save(name, **arrays)


def gen_ndc(ref):
    """ray_util.get_ndc_rays on LLFF-like forward-facing rays (run_nerf_helpers.py:349)."""
    H, W, focal = 30, 40, 35.0
    g = rng(31)
    ro = torch.from_numpy(g.normal(0, 0.3, (200, 3)).astype(np.float32))
    ro[:, 2] += 0.5
    rd = torch.from_numpy(g.normal(0, 0.2, (200, 3)).astype(np.float32))
    rd[:, 2] = -1.0 + rd[:, 2] * 0.1
    o, d = ref.ray_util.get_ndc_rays(H, W, focal, 1.0, ro, rd)
    save("ndc", H=H, W=W, focal=focal, near=1.0, rays_o=ro.numpy(), rays_d=rd.numpy(),
         ndc_o=o.numpy(), ndc_d=d.numpy())


def gen_render_image(ref, T=12, finest=256, H=12, W=14, seed=23):
    """render() over a whole image from c2w (run_nerf_helpers.py:310-392, the
    render_path inner call, :418) with a chunk smaller than the image, det
    sampling (pytest hooks), white background."""
    cams, box, K, focal = scene(ref, H, W)
    emb, tab = make_embedder(ref, box, T, finest, seed)
    shenc = ref.sh.SHEncoder()
    mc, mf = make_mlps(ref, seed)
    nq = lambda inputs, viewdirs, fn: ref.rnh.run_network(inputs, viewdirs, fn, embed_fn=emb,
                                                          embeddirs_fn=shenc, netchunk=65536)
    kw = dict(network_query_fn=nq, perturb=0., N_importance=128, network_fine=mf,
              N_samples=64, network_fn=mc, embed_fn=emb, use_viewdirs=True, white_bkgd=True,
              raw_noise_std=0., ndc=False, lindisp=False, near=2., far=6., pytest=True)
    pose = cams[7][:3, :4]
    with torch.no_grad():
        rgb, depth, acc, extras = ref.rnh.render(H, W, K, chunk=50, c2w=pose, **kw)
    arrays = dict(box_min=box[0].numpy(), box_max=box[1].numpy(), log2T=T, finest=finest,
                  table_seed=seed, H=H, W=W, K=K, c2w=pose.numpy(), rgb=rgb.numpy(),
                  depth=depth.numpy(), acc=acc.numpy(), rgb0=extras["rgb0"].numpy())
    for tag, m in (("c", mc), ("f", mf)):
        for k, v in m.named_parameters():
            arrays[f"w{tag}:{k}"] = v.detach().numpy()
    save("render_image", **arrays)


def gen_tv(ref):
    T = 12
    box = (torch.tensor([-1., -1., -1.]), torch.tensor([1., 1., 1.]))
    for finest in (512, 1024):
        emb, tab = make_embedder(ref, box, T, finest, 31)
        mins, vals, grads = [], [], []
        torch.manual_seed(123)
        orig = torch.randint
        rec = []

        def randint(*a, **k):
            r = orig(*a, **k)
            rec.append(r.clone())
            return r

        ref.loss.torch.randint = randint
        try:
            for l in range(16):
                emb.zero_grad()
                v = ref.loss.total_variation_loss(emb.embeddings[l], emb.base_resolution,
                                                  emb.finest_resolution, l, T, n_levels=16)
                v.backward()
                vals.append(v.item())
                grads.append(emb.embeddings[l].weight.grad.numpy().copy())
        finally:
            ref.loss.torch.randint = orig
        save(f"tv_f{finest}", log2T=T, finest=finest, table_seed=31, min_vertex=np.stack(rec),
             tv=np.array(vals, dtype=np.float32), grad=np.stack(grads))


def gen_radam(ref):
    g = rng(41)
    p0 = g.standard_normal((20,)).astype(np.float32)
    t0 = g.standard_normal((30,)).astype(np.float32) * 1e-4
    pa = torch.nn.Parameter(torch.from_numpy(p0.copy()))
    pb = torch.nn.Parameter(torch.from_numpy(t0.copy()))
    opt = ref.radam.RAdam([{"params": [pa], "weight_decay": 1e-6}, {"params": [pb], "eps": 1e-15}],
                          lr=0.01, betas=(0.9, 0.99))
    ga, gb, pas, pbs = [], [], [], []
    for step in range(8):
        opt.zero_grad()
        a = g.standard_normal(20).astype(np.float32)
        b = g.standard_normal(30).astype(np.float32) * 1e-3
        pa.grad = torch.from_numpy(a.copy())
        pb.grad = torch.from_numpy(b.copy())
        opt.step()
        for gr in opt.param_groups:
            gr["lr"] = 0.01 * (0.1 ** ((step + 1) / 500000))
        ga.append(a); gb.append(b)
        pas.append(pa.detach().numpy().copy()); pbs.append(pb.detach().numpy().copy())
    save("radam", p0=p0, t0=t0, ga=np.stack(ga), gb=np.stack(gb), pa=np.stack(pas), pb=np.stack(pbs))


def gen_pool_rays(ref):
    """use_batching's ray pool (run_nerf.py:509-515): get_rays_np (the
    reference's ray_util.py:82-93, called here) of every training image, the
    rays_rgb stacking / transposition / reshape / float32 cast of those lines
    restated with the same numpy calls (run_nerf.py imports configargparse /
    imageio, absent here).  3 training images of 20 x 24 among 5 (i_train =
    0, 2, 3), cameras as make_golden.cameras, K in float64 as load_blender."""
    H, W = 20, 24
    focal = .5 * W / np.tan(.5 * CAM_ANGLE_X)
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    poses = np.stack([c.numpy() for c in cameras(5)]).astype(np.float32)
    images = rng(31).random((5, H, W, 3), dtype=np.float32)
    i_train = np.array([0, 2, 3])
    rays = np.stack([ref.ray_util.get_rays_np(H, W, K, p) for p in poses[:, :3, :4]], 0)
    rays_rgb = np.concatenate([rays, images[:, None]], 1)
    rays_rgb = np.transpose(rays_rgb, [0, 2, 3, 1, 4])
    rays_rgb = np.stack([rays_rgb[i] for i in i_train], 0)
    rays_rgb = np.reshape(rays_rgb, [-1, 3, 3]).astype(np.float32)
    save("pool_rays", H=H, W=W, K=K, poses=poses, images=images, i_train=i_train, rays_rgb=rays_rgb)


def gen_blender_images(ref):
    """Blender image preparation on a synthetic RGBA array (no PNGs needed):
    load/load_blender.py:63 `(np.array(imgs) / 255.).astype(np.float32)`, and
    run_nerf.py:259-262 `images[..., :3] * images[..., -1:] + (1. - images[...,
    -1:])` at full resolution, with the reference's own numpy expressions.
    half_res (:78-86) calls cv2.resize(INTER_AREA), and cv2 is not in the
    image: the fixture holds the exact (float64) 2 x 2 means of the float32
    pixels instead, and the float64 composite of those means; a float32
    INTER_AREA sum is within 1 ulp of them (tests/test_blender_data.py)."""
    g = rng(37)
    rgba = g.integers(0, 256, size=(3, 6, 8, 4), dtype=np.uint8)
    rgba[0, 0, 0] = (255, 0, 0, 0)          # fully transparent
    rgba[0, 0, 1] = (10, 20, 30, 255)       # opaque
    imgs = (np.array(rgba) / 255.).astype(np.float32)
    white = imgs[..., :3] * imgs[..., -1:] + (1. - imgs[..., -1:])
    f = imgs.astype(np.float64)
    half_mean = 0.25 * (f[:, 0::2, 0::2] + f[:, 0::2, 1::2] + f[:, 1::2, 0::2] + f[:, 1::2, 1::2])
    save("blender_images", rgba=rgba, imgs=imgs, white=white, half_mean=half_mean)


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    if len(sys.argv) > 1:            # regenerate selected fixtures only, e.g. `ndc render_image`
        for name in sys.argv[1:]:
            globals()["gen_" + name](ref)
        return
    gen_hash(ref)
    gen_encode(ref)
    gen_sh(ref)
    gen_mlp(ref)
    gen_raw2outputs(ref)
    gen_sample_pdf(ref)
    gen_bbox_rays(ref)
    gen_tv(ref)
    gen_radam(ref)
    gen_render(ref, "render_white_perturb", white=True, perturb=1.0, seed=21)
    gen_render(ref, "render_black_det", white=False, perturb=0.0, seed=22, T=13, finest=1024)
    gen_ndc(ref)
    gen_render_image(ref)


if __name__ == "__main__":
    main()
