"""Fixed vs per-k-tile cost of a GEMM variant: graph-replayed time over a K sweep at fixed M x N.
SVLA_VARIANTS=0,13 python tools/gemm_ksweep.py M N"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import kernels as K  # noqa: E402
from tools.prefill_gemm_bench import timed  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("SVLA_VARIANTS", "0,13").split(",")]
M, N = int(sys.argv[1]), int(sys.argv[2])
for Kd in (64, 256, 1024, 4096):
    x = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, Kd, device="cuda") * 0.03).to(torch.bfloat16)
    y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    res = {}
    for v in VARIANTS:
        K.gemm_variant = v
        res[f"v{v}"] = round(timed(lambda: K.linear_fwd(x, [w], y)), 2)
    K.gemm_variant = 0
    print(json.dumps({"M": M, "N": N, "K": Kd, "us": res}), flush=True)
# an empty kernel's replay time for scale
z = torch.zeros(16, device="cuda")
print(json.dumps({"fill_16_us": round(timed(lambda: z.fill_(1.0)), 2)}), flush=True)
