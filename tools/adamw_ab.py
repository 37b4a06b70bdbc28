"""A/B the AdamW sweep of libsvla builds at 1.5 G parameters (bytes: 28 per parameter), interleaved:
python tools/adamw_ab.py lib1.so lib2.so ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

n = 1_500_000_000
dev = "cuda"
master = torch.randn(n, device=dev)
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
grad = torch.randn(n, device=dev).to(torch.bfloat16)
param = master.to(torch.bfloat16)
libs = [(os.path.basename(p), L.load(os.path.abspath(p))) for p in sys.argv[1:]]
best = {}
for rnd in range(4):
    for tag, cd in libs:
        L._lib = cd
        K.adamw(master, param, grad, m, v, 1e-5, 0.9, 0.999, 1e-8, 0.0, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for s in range(3):
            K.adamw(master, param, grad, m, v, 1e-5, 0.9, 0.999, 1e-8, 0.0, s + 2)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / 3
        best[tag] = min(best.get(tag, 1e9), t)
for tag, t in best.items():
    print(f"{tag:24s} {t:8.2f} ms  {28 * n / t / 1e9:6.2f} TB/s", flush=True)
