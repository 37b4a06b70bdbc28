"""One GEMM shape, repeated: our kernel (arm "svla") or torch.matmul/hipBLASLt (arm "torch"), for rocprofv3 PMC passes.
python tools/gemm_pmc_one.py svla|torch M N K [iters]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

arm, M, N, Kd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
lay = os.environ.get("SVLA_LAYOUT", "nt")  # nt: x @ W^T, nn: dY @ W (dgrad), tn: dY^T @ X (wgrad)
bf = torch.bfloat16
a = torch.randn(M, Kd, device="cuda").to(bf) if lay != "tn" else torch.randn(Kd, M, device="cuda").to(bf)
b = torch.randn(N, Kd, device="cuda").to(bf) if lay == "nt" else torch.randn(Kd, N, device="cuda").to(bf)
c = torch.empty(M, N, device="cuda", dtype=bf)
A = K._operand([a], L.LAYOUT_KC if lay != "tn" else L.LAYOUT_RC)
B = K._operand([b], L.LAYOUT_KC if lay == "nt" else L.LAYOUT_RC)
ref = {"nt": lambda: torch.matmul(a, b.T, out=c), "nn": lambda: torch.matmul(a, b, out=c),
       "tn": lambda: torch.matmul(a.T, b, out=c)}[lay]
f = (lambda: K.gemm(M, N, Kd, A, B, [c], [0], N, K._epi())) if arm == "svla" else ref
for _ in range(iters):
    f()
torch.cuda.synchronize()
print("done", arm, M, N, Kd)
