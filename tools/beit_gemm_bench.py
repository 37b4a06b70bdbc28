"""The ZoeDepth BEiT-L GEMMs of the training step's frozen depth forward (B=32 x 577 tokens = 18464 rows) with their
epilogues, per dispatch variant, beside torch.matmul (hipBLASLt, plain product) on the same operands.
python tools/beit_gemm_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import kernels as K, _lib as L  # noqa: E402

BF = torch.bfloat16
M = 32 * 577


def timed(f, reps=20):
    for _ in range(3):
        f()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        f()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[reps // 2]


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g).to(BF)
    cases = [("qkv BIAS", 3072, 1024, L.EPI_BIAS), ("o BIAS_SCALE_RESID", 1024, 1024, L.EPI_BIAS_SCALE_RESID),
             ("fc1 BIAS", 4096, 1024, L.EPI_BIAS), ("fc1 BIAS_GELU_ERF", 4096, 1024, L.EPI_BIAS_GELU_ERF),
             ("fc2 BIAS_SCALE_RESID", 1024, 4096, L.EPI_BIAS_SCALE_RESID), ("fc2 STORE", 1024, 4096, L.EPI_STORE)]
    for name, n, k, kind in cases:
        x, w, b, cs, res = r(M, k), r(n, k) * 0.02, r(n), r(n), r(M, n)
        out = torch.empty(M, n, dtype=BF, device="cuda")
        kw = {}
        if kind in (L.EPI_BIAS, L.EPI_BIAS_GELU_ERF, L.EPI_BIAS_SCALE_RESID):
            kw["bias"] = b
        if kind == L.EPI_BIAS_SCALE_RESID:
            kw.update(colscale=cs, in0=res)
        row = []
        for v in [int(s) for s in os.environ.get("SVLA_VARIANTS", "0,1,3,8").split(",")]:
            K.gemm_variant = v
            try:
                ms = timed(lambda: K.linear_fwd(x, [w], out, kind=kind, **kw))
                row.append(f"v{v} {ms * 1e3:6.1f} us")
            except Exception as e:  # noqa: BLE001
                row.append(f"v{v} n/a")
        K.gemm_variant = 0
        t = timed(lambda: x @ w.T)
        fl = 2.0 * M * n * k
        print(f"{name:22s} M={M} N={n:5d} K={k:5d}  " + "  ".join(row) + f"  torch {t * 1e3:6.1f} us "
              f"({fl / t / 1e9:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
