"""One GEMM shape, repeated: our kernel (arm "svla") or torch.matmul/hipBLASLt (arm "torch"), for rocprofv3 PMC passes.
python tools/gemm_pmc_one.py svla|torch M N K [iters]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

arm, M, N, Kd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16)
b = torch.randn(N, Kd, device="cuda").to(torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
A, B = K._operand([a], L.LAYOUT_KC), K._operand([b], L.LAYOUT_KC)
f = (lambda: K.gemm(M, N, Kd, A, B, [c], [0], N, K._epi())) if arm == "svla" else (lambda: torch.matmul(a, b.T, out=c))
for _ in range(iters):
    f()
torch.cuda.synchronize()
print("done", arm, M, N, Kd)
