"""Attention forward time vs key tiles per block at one full round of blocks (B*Hkv*ceil(L/64) = 256 blocks), to
split the per-block fixed cost from the per-tile cost: python tools/attn_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K

BF = torch.bfloat16
dev = "cuda"
for D, Hq, Hkv, cap in ((256, 8, 4, 50.0), (72, 16, 16, 0.0)):
    for n in (1, 2, 4, 8):
        Lq = 64 * n
        B = max(1, 256 // ((Hq // (2 if Hq != Hkv else 1)) * n)) if Hq != Hkv else max(1, 256 // (Hq * n))
        W = (Hq + 2 * Hkv) * D
        qkv = torch.randn(B * Lq, W, device=dev).to(BF)
        a = K.attn_args(B, Lq, Hq, Hkv, D, qkv[:, :Hq * D], W, qkv[:, Hq * D:(Hq + Hkv) * D], W,
                        qkv[:, (Hq + Hkv) * D:], W, 1 / 16, cap, None, 0)
        out = torch.empty(B * Lq, Hq * D, dtype=BF, device=dev)
        lse = torch.empty(B, Hq, Lq, device=dev)
        K.attn_fwd(a, out, lse)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                K.attn_fwd(a, out, lse)
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
        fl = 4.0 * B * Hq * Lq * Lq * D
        print(f"D={D} tiles/block={n} B={B} L={Lq}: {best:7.1f} us  {fl / best * 1e-6:7.1f} TF", flush=True)
