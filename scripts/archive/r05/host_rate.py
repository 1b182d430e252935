"""Host-side enqueue time per training step (no synchronisation inside the
loop) against the GPU step time: whether a short timed window is host-bound."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import hn_loader
hn_loader.load()
from hashnerf_pytorch_amd.train import SyntheticBlender, Trainer, default_args
dev = torch.device("cuda", 0)
args = default_args(N_rand=4096, log2_hashmap_size=19, finest_res=512, tv_loss_weight=1e-6, tv_until=1001)
data = SyntheticBlender(400, 400, 100, dev, seed=0, scene="procedural")
tr = Trainer(args, data, dev, seed=0)
for _ in range(1010):
    tr.step()
torch.cuda.synchronize()
for n in (20, 200):
    t0 = time.perf_counter()
    host = []
    for _ in range(n):
        h0 = time.perf_counter()
        tr.step()
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"steps {n}: host enqueue {1e3 * (t1 - t0) / n:.3f} ms/step (first {1e3 * host[0]:.3f}, median "
          f"{1e3 * sorted(host)[n // 2]:.3f}), wall incl. drain {1e3 * (t2 - t0) / n:.3f} ms/step", flush=True)
