"""A/B of the B=1 prefill GEMM shapes (BEiT-L/16 at 384^2: 577 tokens; SigLIP at 224^2: 256 tokens) on one MI355X:
auto dispatch (variant 0) against 8-phase + stream-K for every sub-wave grid (variant 8).  Graph-replayed launches,
mean time per launch; checks the two variants agree (fp32 accumulation, different K split -> small differences)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import kernels as K  # noqa: E402

BF = torch.bfloat16
VARIANTS = [int(v) for v in os.environ.get("SVLA_VARIANTS", "0,8").split(",")]
SHAPES = [("beit_qkv", 577, 3072, 1024), ("beit_o", 577, 1024, 1024), ("beit_fc1", 577, 4096, 1024),
          ("beit_fc2", 577, 1024, 4096), ("siglip_qkv", 256, 3456, 1152), ("siglip_o", 256, 1152, 1152),
          ("siglip_fc1", 256, 4304, 1152), ("siglip_fc2", 256, 1152, 4304)]


def timed(fn, reps=50):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    torch.manual_seed(0)
    for name, M, N, Kd in SHAPES:
        x = torch.randn(M, Kd, device="cuda").to(BF)
        w = (torch.randn(N, Kd, device="cuda") * 0.03).to(BF)
        res = {}
        outs = {}
        for v in VARIANTS:
            K.gemm_variant = v
            y = torch.empty(M, N, dtype=BF, device="cuda")
            res[v] = round(timed(lambda: K.linear_fwd(x, [w], y)), 2)
            outs[v] = y.float()
        K.gemm_variant = 0
        rel = {v: float((outs[0] - outs[v]).norm() / outs[0].norm()) for v in VARIANTS}
        print(json.dumps({"shape": name, "M": M, "N": N, "K": Kd, "us": {f"v{v}": res[v] for v in VARIANTS},
                          "rel_diff": rel}), flush=True)


if __name__ == "__main__":
    main()
