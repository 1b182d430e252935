"""Digest of one fused forward + backward at the bench shape (4096 rays,
T=19, seeded inputs) with the library HN_LIB_PATH selects: sha256 of the
table gradient, the ten MLP gradients and the forward state, so that variant
libraries that must be bitwise equal can be compared across processes.
  usage: HN_LIB_PATH=... python scripts/variant_digest.py [B] [T] [finest]"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hn_loader  # noqa: E402

hn = hn_loader.load()
from test_gpu_scatter import _bwd, _state  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T = int(sys.argv[2]) if len(sys.argv) > 2 else 19
fin = int(sys.argv[3]) if len(sys.argv) > 3 else 512
HF, emb, mc, mf, ws, rays, t_rand, u, target, st, grads = _state(hn, B, T, 31, "binned", finest=fin)
h = lambda *ts: hashlib.sha256(b"".join(t.detach().contiguous().cpu().numpy().tobytes() for t in ts)).hexdigest()[:16]
f0 = h(st.z_f, st.raw_c, st.raw_f, st.feat)   # the forward state before the backward runs
tab, dws = _bwd(HF, emb, ws, st, grads)
f1 = h(st.z_f, st.raw_c, st.raw_f, st.feat)
print(f"fwd {f0} table {h(tab)} mlp {h(*dws)}" + ("" if f1 == f0 else f" CHANGED-BY-BWD {f1}"))
if os.environ.get("HN_DIGEST_PARTS"):
    print("  parts z_f %s raw_c %s raw_f %s feat %s" % (h(st.z_f), h(st.raw_c), h(st.raw_f), h(st.feat)))
