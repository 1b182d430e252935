"""Digest of a training trajectory with the library HN_LIB_PATH selects: the
bench's trainer (procedural chair, one config) for N steps, then sha256 of
the table, its RAdam moments and the NeRFSmall weights (zeros normalised:
x + 0.0 maps -0.0 to +0.0, the only difference exact-zero skips can make),
plus the last step's loss.  Variant libraries whose results must be bitwise
equal print the same line.   usage: HN_LIB_PATH=... python scripts/traj_digest.py [steps] [config]"""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import hn_loader  # noqa: E402

hn_loader.load()
from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
cfg = bench.CONFIGS[int(sys.argv[2]) if len(sys.argv) > 2 else 2]
dev = torch.device("cuda", 0)
targs = default_args(N_rand=cfg["N_rand"], log2_hashmap_size=cfg["log2_hashmap_size"], finest_res=cfg["finest_res"],
                     tv_loss_weight=cfg["tv_loss_weight"], tv_until=cfg.get("tv_until", 1001),
                     white_bkgd=cfg.get("white_bkgd", True), sparse_loss_weight=cfg.get("sparse_loss_weight", 1e-10),
                     no_batching=cfg.get("no_batching", True))
data = SyntheticBlender(400, 400, 100, dev, seed=0, scene="procedural")
if "bbox" in cfg:
    data.bounding_box = tuple(torch.tensor(v) for v in cfg["bbox"])
tr = Trainer(targs, data, dev, seed=0)
for _ in range(steps):
    loss, _ = tr.step()
torch.cuda.synchronize()
t = tr.embed_fn.table
st = tr.optimizer.state[t]
ws = tr.kw_train["network_fn"].weights() + tr.kw_train["network_fine"].weights()
h = lambda *ts: hashlib.sha256(b"".join((x.detach() + 0.0).contiguous().cpu().numpy().tobytes() for x in ts)).hexdigest()[:16]
print(f"steps {steps} table {h(t)} moments {h(st['exp_avg'], st['exp_avg_sq'])} mlp {h(*ws)} loss {float(loss):.9g}")
