"""The Gemma2 projections of the B=1 prefill (configs[1]: 299 prompt tokens, SpatialVLA-4B widths) per GEMM variant:
q|k|v with the RoPE epilogue, o, gate|up with the GeGLU epilogue, down.  Graph-replayed launches, mean us per launch,
with the rel-L2 difference of each variant's output from variant 0's (fp32 accumulation, other K splits).
SVLA_VARIANTS=0,1,3,8 python tools/gemma_prefill_gemm_bench.py [M]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import _lib as L  # noqa: E402
from spatialvla_amd import kernels as K  # noqa: E402
from tools.prefill_gemm_bench import timed  # noqa: E402

BF = torch.bfloat16
VARIANTS = [int(v) for v in os.environ.get("SVLA_VARIANTS", "0,1,3,8").split(",")]
H, I, D, HQ, HKV = 2304, 9216, 256, 8, 4


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 299
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(M, H, device=dev).to(BF)
    wq = (torch.randn(HQ * D, H, device=dev) * 0.03).to(BF)
    wk = (torch.randn(HKV * D, H, device=dev) * 0.03).to(BF)
    wv = (torch.randn(HKV * D, H, device=dev) * 0.03).to(BF)
    wo = (torch.randn(H, HQ * D, device=dev) * 0.03).to(BF)
    wg = (torch.randn(I, H, device=dev) * 0.03).to(BF)
    wu = (torch.randn(I, H, device=dev) * 0.03).to(BF)
    wd = (torch.randn(H, I, device=dev) * 0.03).to(BF)
    a = torch.randn(M, HQ * D, device=dev).to(BF)
    hm = torch.randn(M, I, device=dev).to(BF)
    pos = torch.arange(M, device=dev, dtype=torch.float32)[:, None]
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=dev, dtype=torch.float32) / D))
    cos, sin = torch.cos(pos * inv).to(BF).contiguous(), torch.sin(pos * inv).to(BF).contiguous()
    qkv = torch.empty(M, (HQ + 2 * HKV) * D, dtype=BF, device=dev)
    o = torch.empty(M, H, dtype=BF, device=dev)
    h, g, u = (torch.empty(M, I, dtype=BF, device=dev) for _ in range(3))
    dn = torch.empty(M, H, dtype=BF, device=dev)
    cases = [
        ("qkv_rope", 2 * M * H * (HQ + 2 * HKV) * D, (H * (HQ + 2 * HKV) * D) * 2,
         lambda: K.linear_fwd(x, [wq, wk, wv], qkv, kind=L.EPI_ROPE, rope=(cos, sin, M, D, (HQ + HKV) * D)), qkv),
        ("o", 2 * M * HQ * D * H, H * HQ * D * 2, lambda: K.linear_fwd(a, [wo], o), o),
        ("gate_up_geglu", 2 * M * H * 2 * I, 2 * I * H * 2, lambda: K.linear_geglu_fwd(x, wg, wu, h, g, u), h),
        ("down", 2 * M * I * H, H * I * 2, lambda: K.linear_fwd(hm, [wd], dn), dn),
    ]
    total = {v: 0.0 for v in VARIANTS}
    for name, flop, wbytes, fn, out in cases:
        res, outs = {}, {}
        for v in VARIANTS:
            K.gemm_variant = v
            res[v] = round(timed(fn), 2)
            total[v] += res[v]
            outs[v] = out.float().clone()
        K.gemm_variant = 0
        rel = {f"v{v}": float((outs[0] - outs[v]).norm() / outs[0].norm()) for v in VARIANTS}
        floor = max(flop / 2.5e15, wbytes / 8e12) * 1e6
        print(json.dumps({"shape": name, "M": M, "us": {f"v{v}": res[v] for v in VARIANTS}, "floor_us": round(floor, 2),
                          "rel_diff": rel}), flush=True)
    print(json.dumps({"layer_total_us": {f"v{v}": round(t, 1) for v, t in total.items()}}), flush=True)
    # hipBLASLt through torch.mm on the same operands, no epilogue (the library's time for the plain product)
    wqkv, wgu = torch.cat([wq, wk, wv]), torch.cat([wg, wu])
    lib = {"qkv": timed(lambda: torch.mm(x, wqkv.t(), out=qkv)), "o": timed(lambda: torch.mm(a, wo.t(), out=o)),
           "gate_up": timed(lambda: torch.mm(x, wgu.t())), "down": timed(lambda: torch.mm(hm, wd.t(), out=dn))}
    print(json.dumps({"torch_mm_us": {k: round(v, 2) for k, v in lib.items()},
                      "total": round(sum(lib.values()), 1)}), flush=True)


if __name__ == "__main__":
    main()
