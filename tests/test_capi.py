"""CPU-side checks of the C ABI boundary: the library loads without a GPU, it
exports every symbol include/hashnerf_amd.h declares, the ctypes struct
layouts match the header, and argument validation fails loudly (no compute
call is made)."""
import ctypes as C
import os
import re

import pytest
import torch

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "hashnerf_amd.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|size_t|const char\*)\s+(hn_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol(hn):
    lib = hn._lib.lib()
    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
        assert n in hn._lib.SIGNATURES, f"ctypes signature missing for {n}"
    assert lib.hn_abi_version() == hn._lib.ABI_VERSION == 14


def test_struct_sizes_match_header(hn):
    L = hn._lib
    assert C.sizeof(L.HnGrid) == 16 + 24 + 32 * 12
    assert C.sizeof(L.HnMlp) == 5 * 8
    assert C.sizeof(L.HnRenderCfg) == C.sizeof(L.HnGrid) + 8 * 4
    assert L.lib().hn_mlp_workspace_bytes() == L.MLP_PACKED_FLOATS * 4


def test_struct_layouts_match_compiled_header(hn, tmp_path):
    """Every field offset of every ABI struct, as gcc lays out the header,
    equals the ctypes mirror's offset (catches a field added on one side)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    L = hn._lib
    structs = {"hn_grid": L.HnGrid, "hn_mlp": L.HnMlp, "hn_mlp_grad": L.HnMlpGrad,
               "hn_render_cfg": L.HnRenderCfg, "hn_render_fwd_args": L.HnRenderFwdArgs,
               "hn_render_bwd_args": L.HnRenderBwdArgs, "hn_tv_args": L.HnTvArgs,
               "hn_ray_sampler": L.HnRaySampler, "hn_ray_pool": L.HnRayPool,
               "hn_radam_tensor": L.HnRadamTensor, "hn_render_loss": L.HnRenderLoss,
               "hn_uniform_draw": L.HnUniformDraw}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hashnerf_amd.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in cls._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for cname, cls in structs.items():
        assert got[(cname, "sizeof")] == C.sizeof(cls), cname
        for f in cls._fields_:
            assert got[(cname, f[0])] == getattr(cls, f[0]).offset, (cname, f[0])


def test_argument_validation_without_gpu(hn):
    L = hn._lib
    lib = L.lib()
    g = L.make_grid(16, 2, 19, [-1] * 3, [1] * 3, [[0.1] * 3] * 16)
    # n == 0 is a no-op; NULL pointers and bad shapes are rejected before any launch
    assert lib.hn_encode_fwd(g, None, 0, None, None, None, None) == 0
    assert lib.hn_encode_fwd(g, None, 10, None, None, None, None) == 1
    g.n_features = 4
    assert lib.hn_encode_fwd(g, None, 10, None, None, None, None) == 2
    assert lib.hn_sample_pdf(None, None, None, 4, 300, 8, None, None) == 2
    cfg = L.HnRenderCfg()
    cfg.grid = L.make_grid(8, 2, 19, [-1] * 3, [1] * 3, [[0.1] * 3] * 8)
    a = L.HnRenderFwdArgs()
    a.n_rays = 4
    assert lib.hn_render_fwd(cfg, a, None, 0, None) == 2   # L != 16
    assert lib.hn_status_string(3).decode() == "workspace too small"
    # ray pool: empty batch is a no-op, positions past the pool and bad shapes are rejected
    p = L.HnRayPool()
    p.n_images, p.H, p.W, p.pose_stride = 2, 4, 4, 16
    assert lib.hn_sample_pool(p, None, None, None, 0, 0, None, None, None) == 0
    assert lib.hn_sample_pool(p, None, None, None, 0, 8, None, None, None) == 1
    x = C.c_void_p(16)   # never dereferenced: validation happens before any launch
    assert lib.hn_sample_pool(p, x, x, x, 30, 8, x, x, None) == 2    # 30 + 8 > 2 * 4 * 4
    p.pose_stride = 9
    assert lib.hn_sample_pool(p, x, x, x, 0, 8, x, x, None) == 2
    # blender images: odd size with half_res, bad mode
    assert lib.hn_blender_images(x, 1, 5, 4, 1, 1, x, None) == 2
    assert lib.hn_blender_images(x, 1, 4, 4, 0, 3, x, None) == 2
    assert lib.hn_blender_images(None, 0, 4, 4, 1, 1, None, None) == 0
    # torch.rand restatement (ABI 13): argument checks return before any launch
    d = (L.HnUniformDraw * 5)()
    assert lib.hn_uniform_philox(1, d, 5, None) == 2                   # more than HN_UNIFORM_MAX_DRAWS
    assert lib.hn_uniform_philox(1, None, 1, None) == 1
    d[0].numel, d[0].threads, d[0].offset = 8, 256, 2                  # offset not a multiple of 4
    assert lib.hn_uniform_philox(1, d, 1, None) == 2
    d[0].offset, d[0].out = 4, None
    assert lib.hn_uniform_philox(1, d, 1, None) == 1                   # no output
    d[0].numel = 0
    assert lib.hn_uniform_philox(1, d, 1, None) == 0                   # nothing to draw


def test_bins_and_deferred_owner_validation_without_gpu(hn):
    """ABI 12: hn_render_bins reports the binned scatter's geometry (host
    arithmetic only), and hn_render_bwd_owner rejects a call that did not
    defer its owner pass, a bad bin range or missing buffers before any
    launch."""
    L = hn._lib
    lib = L.lib()
    HF = hn.functional
    box = (torch.tensor([-1.5, -1.5, -1.5]), torch.tensor([1.5, 1.5, 1.5]))
    for T, finest, want in ((19, 512, (1024, 13)), (22, 1024, (8192, 13)), (14, 512, (32, 13))):
        emb = hn.HashEmbedder(box, log2_hashmap_size=T, finest_resolution=finest)
        cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter="binned")
        assert HF.render_bins(cfg, 4096) == want, (T, HF.render_bins(cfg, 4096))
        cfg_a = HF.make_render_cfg(emb.grid(), True, False, True, scatter="atomic")
        assert HF.render_bins(cfg_a, 4096) == (0, 0)
    shift = C.c_int32(-1)
    assert lib.hn_render_bins(None, 4096, C.byref(shift)) == 0
    emb = hn.HashEmbedder(box, log2_hashmap_size=19, finest_resolution=512)
    cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter="binned")
    a = L.HnRenderBwdArgs()
    a.n_rays = 4096
    x = C.c_void_p(16)   # never dereferenced: validation happens before any launch
    ws = lib.hn_render_workspace_bytes(cfg, 4096)
    assert lib.hn_render_bwd_owner(cfg, None, x, ws, 0, 1, None) == 1          # no args
    assert lib.hn_render_bwd_owner(cfg, a, None, ws, 0, 1, None) == 1          # no workspace
    assert lib.hn_render_bwd_owner(cfg, a, x, ws, 0, 1, None) == 2             # owner_defer not set
    a.owner_defer = 1
    assert lib.hn_render_bwd_owner(cfg, a, x, ws, 0, 1, None) == 1             # neither d_table nor table_step
    a.d_table = 16
    assert lib.hn_render_bwd_owner(cfg, a, x, ws - 4, 0, 1, None) == 3         # workspace too small
    assert lib.hn_render_bwd_owner(cfg, a, x, ws, 0, 1025, None) == 2          # past the last bin
    assert lib.hn_render_bwd_owner(cfg, a, x, ws, 7, 3, None) == 2             # reversed range
    assert lib.hn_render_bwd_owner(cfg, a, x, ws, 5, 5, None) == 0             # empty range: no-op


def test_zero_ray_backward_validation_without_gpu(hn):
    """ABI 14: hn_render_bwd with n_rays == 0 is a no-op without a TV term;
    with one it is the TV-only records path, which checks its arguments
    before any launch (needs g_tv and d_table, the binned scatter, no owner
    deferral); hn_render_cfg.dense_bwd must be 0 or 1."""
    L = hn._lib
    lib = L.lib()
    HF = hn.functional
    box = (torch.tensor([-1.5, -1.5, -1.5]), torch.tensor([1.5, 1.5, 1.5]))
    emb = hn.HashEmbedder(box, log2_hashmap_size=19, finest_resolution=512)
    cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter="binned")
    x = C.c_void_p(16)   # never dereferenced: validation happens before any launch
    a = L.HnRenderBwdArgs()
    a.n_rays = 0
    assert lib.hn_render_bwd(cfg, a, None, 0, None) == 0                        # nothing to do
    tva = L.HnTvArgs()
    tva.n_levels, tva.log2_hashmap_size = 16, 19
    for l in range(16):
        tva.cube[l] = 8
    tva.min_vertex = tva.table = 16
    a.tv = C.cast(C.pointer(tva), C.c_void_p)
    ws = lib.hn_render_workspace_bytes(cfg, 0)
    assert lib.hn_render_bwd(cfg, a, x, ws, None) == 1                          # no g_tv / d_table
    a.g_tv, a.d_table, a.d_table_mode = 16, 16, 1
    assert lib.hn_render_bwd(cfg, a, x, ws - 4, None) == 3                      # workspace too small
    a.owner_defer = 1
    assert lib.hn_render_bwd(cfg, a, x, ws, None) == 2                          # no deferred owner here
    a.owner_defer = 0
    tva.cube[3] = 51
    assert lib.hn_render_bwd(cfg, a, x, ws, None) == 2                          # cube past the records' bound
    tva.cube[3] = 8
    cfg_a = HF.make_render_cfg(emb.grid(), True, False, True, scatter="atomic")
    assert lib.hn_render_bwd(cfg_a, a, x, ws, None) == 2                        # float-atomic schedule: hn_tv_bwd
    cfg.dense_bwd = 4
    assert lib.hn_render_bwd(cfg, a, x, ws, None) == 2                          # dense_bwd is 0 or 1


def test_product_path_refuses_cpu_tensors(hn):
    emb = hn.HashEmbedder((torch.tensor([-1., -1, -1]), torch.tensor([1., 1, 1])), log2_hashmap_size=12)
    with pytest.raises(RuntimeError, match="ROCm"):
        emb(torch.zeros(4, 3))
    with pytest.raises(RuntimeError, match="ROCm"):
        hn.SHEncoder()(torch.zeros(4, 3))


def test_state_dict_round_trip_reference_keys(hn, oracle):
    emb = hn.HashEmbedder((torch.tensor([-1., -1, -1]), torch.tensor([1., 1, 1])), log2_hashmap_size=10)
    sd = emb.state_dict()
    assert list(sd) == [f"embeddings.{l}.weight" for l in range(16)]
    assert sd["embeddings.3.weight"].shape == (1024, 2)
    emb2 = hn.HashEmbedder((torch.tensor([-1., -1, -1]), torch.tensor([1., 1, 1])), log2_hashmap_size=10)
    emb2.load_state_dict(sd)
    assert torch.equal(emb2.table, emb.table)
    # the level views behave like nn.Embedding (used by the TV loss)
    idx = torch.tensor([0, 5, 1023])
    assert torch.equal(emb.embeddings[3](idx), emb.table[3][idx])


def test_grid_sizes_bitexact_with_reference_formula(hn, oracle):
    box = (torch.tensor([-4.0249, -4.0249, -3.3366]), torch.tensor([4.0249, 4.0249, 3.2414]))
    for finest in (512, 1024):
        emb = hn.HashEmbedder(box, log2_hashmap_size=12, finest_resolution=finest)
        res = oracle.level_resolutions(16, 16, finest)
        assert [float(r) for r in emb.resolutions] == [float(r) for r in res]
        gs = oracle.grid_sizes(box[0], box[1], res)
        g = emb.grid()
        for l in range(16):
            for a in range(3):
                assert C.c_float(gs[l, a].item()).value == g.grid_size[l][a]


def test_render_bwd_refuses_dense_after_skipping_forward(hn):
    """A forward with skip_dead_color (the trainer's) stores no features for
    fine tiles without density; functional.render_bwd refuses a dense_bwd = 1
    backward of such a state before any launch (ABI 14 hn_render_fwd_args)."""
    HF = hn.functional
    box = (torch.tensor([-1.5, -1.5, -1.5]), torch.tensor([1.5, 1.5, 1.5]))
    emb = hn.HashEmbedder(box, log2_hashmap_size=14, finest_resolution=64)
    st = HF.RenderState()
    st.cfg = HF.make_render_cfg(emb.grid(), True, False, True, scatter="binned")
    st.rays = torch.zeros((4, 11))
    st.skip_dead = True
    st.cfg.dense_bwd = 1
    with pytest.raises(ValueError, match="dense_bwd"):
        HF.render_bwd(st, {}, None, [])
