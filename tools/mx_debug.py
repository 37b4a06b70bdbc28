"""MX GEMM bring-up checks: python tools/mx_debug.py -> rel-L2 of svla_gemm_mxfp8 against the dequantised fp32
product under controlled block-scale patterns (uniform, A-only, B-only, one k-block, per lane-half), small shapes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K

BF = torch.bfloat16
dev = "cuda"


def deq(q, sc):
    X = sc.exponents()
    r, k = q.shape
    return (q.float().view(r, k // 32, 32) * torch.exp2(X.float())[..., None]).view(r, k)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


def run(name, x, w):
    xq, xs = K.quant_mx_rows(x.to(BF))
    wq, ws = K.quant_mx_rows(w.to(BF))
    out = torch.empty(x.shape[0], w.shape[0], dtype=BF, device=dev)
    K.gemm_mxfp8(xq, xs, wq, ws, out)
    ex = deq(xq, xs) @ deq(wq, ws).T
    rowq, rs = K.quant_fp8_rows(x.to(BF))
    print(f"{name:40s} {tuple(x.shape)}x{tuple(w.shape)}: rel {rel(out, ex):.3e}  "
          f"xs exps [{int(xs.exponents().min())}, {int(xs.exponents().max())}] "
          f"ws exps [{int(ws.exponents().min())}, {int(ws.exponents().max())}]", flush=True)


torch.manual_seed(0)
for m, n, k in ((256, 256, 128), (256, 256, 256), (512, 256, 1024), (624, 4096, 2304)):
    x = torch.randn(m, k, device=dev)
    w = torch.randn(n, k, device=dev)
    run("uniform", x, w)
    sA = torch.exp2(torch.randint(-6, 7, (m, k // 32), device=dev).float())
    sB = torch.exp2(torch.randint(-6, 7, (n, k // 32), device=dev).float())
    run("A blocks vary", (x.view(m, -1, 32) * sA[..., None]).view(m, k), w)
    run("B blocks vary", x, (w.view(n, -1, 32) * sB[..., None]).view(n, k))
    xk = x.clone(); xk[:, 32:64] *= 256
    run("A k-block 1 x256", xk, w)
    xr = x.clone(); xr[1::2] *= 256
    run("A odd rows x256", xr, w)
    wr = w.clone(); wr[1::2] *= 256
    run("B odd rows x256", x, wr)
