"""fp8 vs bf16 GEMM on the Gemma2 forward projection shapes (B=32, M=9984): time per launch, TFLOP/s against the
bf16 (2.5 PF) and fp8 (5 PF) dense peaks; quantisation pass cost alongside."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
M = 9984
SHAPES = [("qkv", 4096, 2304, False), ("o", 2304, 2048, False), ("gate/up", 18432, 2304, True),
          ("down", 2304, 9216, False), ("square 8k", 8192, 8192, False)]


def timeit(fn, reps=10):
    for _ in range(3): fn()
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps): fn()
        e1.record(); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


for name, n, k, geglu in SHAPES:
    m = 8192 if name == "square 8k" else M
    x = torch.randn(m, k, device="cuda").to(BF)
    w = (torch.randn(n, k, device="cuda") * 0.02).to(BF)
    xq, xs = K.quant_fp8_rows(x)
    wq, ws = K.quant_fp8_rows(w)
    if geglu:
        I = n // 2
        h = torch.empty(m, I, dtype=BF, device="cuda"); g = torch.empty_like(h); u = torch.empty_like(h)
        f8 = lambda: K.gemm_fp8(xq, xs, wq, ws, h, kind=L.EPI_GEGLU, geglu_I=I, out1=g, out2=u)
        b16 = lambda: K.linear_geglu_fwd(x, w[:I], w[I:], h, g, u)
    else:
        out = torch.empty(m, n, dtype=BF, device="cuda")
        f8 = lambda: K.gemm_fp8(xq, xs, wq, ws, out)
        b16 = lambda: K.linear_fwd(x, [w], out)
    q = lambda: K.quant_fp8_rows(x, xq, xs)
    t8, t16, tq = timeit(f8), timeit(b16), timeit(q)
    fl = 2.0 * m * n * k
    print(f"{name:10s} M={m} N={n} K={k}: fp8 {t8:.3f} ms {fl / t8 / 1e9:7.1f} TF ({fl / t8 / 5e12:.3f} of 5 PF)"
          f" | bf16 {t16:.3f} ms {fl / t16 / 1e9:7.1f} TF | act quant {tq * 1e3:.1f} us | speedup {t16 / t8:.2f}x",
          flush=True)
