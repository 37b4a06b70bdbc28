"""Where does each output of the 4-wave kernel land?  One 256x256 tile (variant 3), integer-valued operands:
for the first rows/cols of the tile print the reference coordinates of the value found there."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L
M = N = 256
Kd = int(sys.argv[1]) if len(sys.argv) > 1 else 64
a = torch.zeros(M, Kd, device="cuda"); b = torch.zeros(N, Kd, device="cuda")
a[torch.arange(M), 0] = torch.arange(M, device="cuda").float()   # C[m][n] = m * 1 + 1000-coded n below
a[:, 1] = 1.0
b[:, 0] = 1.0
b[torch.arange(N), 1] = (torch.arange(N, device="cuda").float() * 0 + 0)
# C[m][n] = m + 256 * n  needs exact bf16: use two k terms with small ints
a = torch.zeros(M, Kd, device="cuda"); b = torch.zeros(N, Kd, device="cuda")
a[:, 0] = torch.arange(M, device="cuda").float(); b[:, 0] = 1.0     # m
a[:, 1] = 1.0; b[:, 1] = torch.arange(N, device="cuda").float()     # + n ... encode n in a second output
a16, b16 = a.to(torch.bfloat16), b.to(torch.bfloat16)
c = torch.empty(M, N, dtype=torch.float32, device="cuda")
cb = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
A, B = K._operand([a16], L.LAYOUT_KC), K._operand([b16], L.LAYOUT_KC)
K.gemm(M, N, Kd, A, B, [cb], [0], N, K._epi(), variant=3)
ref = a16.float() @ b16.float().T
print("max err", (cb.float() - ref).abs().max().item())
# second run: only m (to decode rows), only n (cols)
a2 = torch.zeros_like(a16); a2[:, 0] = torch.arange(M, device="cuda").to(torch.bfloat16); b2 = torch.zeros_like(b16); b2[:, 0] = 1
K.gemm(M, N, Kd, K._operand([a2], L.LAYOUT_KC), K._operand([b2], L.LAYOUT_KC), [cb], [0], N, K._epi(), variant=3)
rows = cb.float().clone()
a3 = torch.zeros_like(a16); a3[:, 0] = 1; b3 = torch.zeros_like(b16); b3[:, 0] = torch.arange(N, device="cuda").to(torch.bfloat16)
K.gemm(M, N, Kd, K._operand([a3], L.LAYOUT_KC), K._operand([b3], L.LAYOUT_KC), [cb], [0], N, K._epi(), variant=3)
cols = cb.float().clone()
torch.set_printoptions(linewidth=250)
print("row ids at out[0:8, 0:20]\n", rows[0:8, 0:20].int().cpu())
print("col ids at out[0:8, 0:20]\n", cols[0:8, 0:20].int().cpu())
print("row ids at out[16:20, 0:20]\n", rows[16:20, 0:20].int().cpu())
print("col ids at out[0:4, 120:140]\n", cols[0:4, 120:140].int().cpu())
