"""A/B the GELU HBM passes (svla_gelu_rows) of libsvla builds at the step's shapes -- SigLIP fc1 (8192 x 4304: mode 0
forward, mode 2 backward) and BEiT fc1 (18464 x 4096, mode 1) -- isolated, interleaved, best of 5; outputs compared
bitwise with the first build: python tools/gelu_rows_ab.py lib1.so [lib2.so ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spatialvla_amd import _lib as L
from spatialvla_amd import kernels as K

dev = "cuda"
torch.manual_seed(0)
BF = torch.bfloat16
cases = {}
for name, (M, N, mode) in {"siglip_fwd": (8192, 4304, 0), "siglip_bwd": (8192, 4304, 2),
                           "beit_fwd": (18464, 4096, 1)}.items():
    x = (torch.randn(M, N, device=dev) * 2).to(BF)
    pre = (torch.randn(M, N, device=dev) * 2).to(BF) if mode == 2 else None
    y = torch.empty_like(x)
    nbytes = x.numel() * 2 * (3 if mode == 2 else 2)
    cases[name] = (mode, x, pre, y, nbytes)
libs = [(os.path.basename(p), L.load(os.path.abspath(p))) for p in sys.argv[1:]]
best, outs = {}, {}
for rnd in range(5):
    for tag, lib in libs:
        L._lib = lib
        for name, (mode, x, pre, y, nb) in cases.items():
            K.gelu_rows(mode, x, y, pre=pre)
            if rnd == 0:
                outs[(name, tag)] = y.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                K.gelu_rows(mode, x, y, pre=pre)
            e1.record()
            e1.synchronize()
            best[(name, tag)] = min(best.get((name, tag), 1e9), e0.elapsed_time(e1) / 10)
t0 = libs[0][0]
for name, (mode, x, pre, y, nb) in cases.items():
    for tag, _ in libs:
        same = torch.equal(outs[(name, tag)].view(torch.int16), outs[(name, t0)].view(torch.int16))
        ms = best[(name, tag)]
        print(f"{name:11s} {tag:24s} {ms * 1e3:8.1f} us  {nb / ms / 1e9:5.2f} TB/s  bitwise_equal={same}", flush=True)
