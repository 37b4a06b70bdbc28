"""One fp8 GEMM shape repeated, for rocprofv3 passes: python tools/fp8_pmc_one.py row|mx|bf16 M N K [iters]
row: svla_gemm_fp8 (row scales), mx: svla_gemm_mxfp8 (OCP MX block scales), bf16: svla_gemm_bf16 (reference)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

arm, M, N, Kd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
bf = torch.bfloat16
x = torch.randn(M, Kd, device="cuda").to(bf)
w = (torch.randn(N, Kd, device="cuda") * 0.02).to(bf)
out = torch.empty(M, N, dtype=bf, device="cuda")
if arm == "row":
    xq, xs = K.quant_fp8_rows(x); wq, ws = K.quant_fp8_rows(w)
    f = lambda: K.gemm_fp8(xq, xs, wq, ws, out)  # noqa: E731
elif arm == "mx":
    xq, xs = K.quant_mx_rows(x); wq, ws = K.quant_mx_rows(w)
    f = lambda: K.gemm_mxfp8(xq, xs, wq, ws, out)  # noqa: E731
else:
    A, B = K._operand([x], L.LAYOUT_KC), K._operand([w], L.LAYOUT_KC)
    f = lambda: K.gemm(M, N, Kd, A, B, [out], [0], N, K._epi())  # noqa: E731
for _ in range(3):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(iters):
    f()
e1.record(); e1.synchronize()
ms = e0.elapsed_time(e1) / iters
print(f"{arm} {M}x{N}x{Kd}: {ms:.3f} ms {2e-9 * M * N * Kd / ms:.1f} TF", flush=True)
