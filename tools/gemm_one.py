"""Run one GEMM shape a few times with one variant (for rocprofv3 counter passes):
python tools/gemm_one.py VARIANT "shape name" [reps]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L
from tools.gemm_bench import SHAPES, BF

v, name = int(sys.argv[1]), sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
_, m, n, k, lay = next(s for s in SHAPES if s[0] == name)
a = torch.randn(m, k, device="cuda").to(BF) if lay != "tn" else torch.randn(k, m, device="cuda").to(BF)
b = torch.randn(n, k, device="cuda").to(BF) if lay == "nt" else torch.randn(k, n, device="cuda").to(BF)
A = K._operand([a], L.LAYOUT_KC if lay != "tn" else L.LAYOUT_RC)
B = K._operand([b], L.LAYOUT_KC if lay == "nt" else L.LAYOUT_RC)
c = torch.empty(m, n, dtype=BF, device="cuda")
L.lib().svla_gemm_set_variant(v)
for _ in range(reps):
    K.gemm(m, n, k, A, B, [c], [0], n, K._epi())
torch.cuda.synchronize()
print("done", name, v)
