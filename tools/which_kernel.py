"""Launch one GEMM shape under the default dispatch (for a kernel trace: which kernel does variant 0 pick).
python tools/which_kernel.py geglu M I K | plain M N K"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import kernels as K  # noqa: E402

kind, M, N, Kd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
if kind == "geglu":
    wg, wu = (torch.randn(N, Kd, device="cuda") * 0.03).to(torch.bfloat16), (torch.randn(N, Kd, device="cuda") * 0.03).to(torch.bfloat16)
    h, g, u = (torch.empty(M, N, dtype=torch.bfloat16, device="cuda") for _ in range(3))
    for _ in range(3):
        K.linear_geglu_fwd(x, wg, wu, h, g, u)
else:
    w = (torch.randn(N, Kd, device="cuda") * 0.03).to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    for _ in range(3):
        K.linear_fwd(x, [w], y)
torch.cuda.synchronize()
print("ok")
