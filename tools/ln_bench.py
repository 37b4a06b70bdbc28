"""Isolated LayerNorm forward (svla_layernorm_fwd) on the training step's BEiT / SigLIP shapes, graph-replayed:
python tools/ln_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import kernels as K  # noqa: E402
from tools.prefill_gemm_bench import timed  # noqa: E402

for M, H in ((18464, 1024), (8192, 1152), (577, 1024), (256, 1152)):
    x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    w, b = torch.randn(H, device="cuda").to(torch.bfloat16), torch.randn(H, device="cuda").to(torch.bfloat16)
    y = torch.empty_like(x)
    mean, rstd = torch.empty(M, device="cuda"), torch.empty(M, device="cuda")
    us = timed(lambda: K.layernorm_fwd(x, w, b, 1e-6, y, mean, rstd))
    print(f"M={M} H={H}: {us:.1f} us, {2 * M * H * 2 / us / 1e6:.2f} TB/s", flush=True)
