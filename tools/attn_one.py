"""One attention shape, fwd (and optionally bwd) repeated, for rocprofv3 passes:
python tools/attn_one.py gemma2|siglip [fwd|bwd] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K
from tools.attn_bench import SHAPES, BF

name = sys.argv[1] if len(sys.argv) > 1 else "gemma2"
what = sys.argv[2] if len(sys.argv) > 2 else "fwd"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
_, B, Lq, Hq, Hkv, D, scale, cap, prefix = next(s for s in SHAPES if s[0] == name)
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
W = (Hq + 2 * Hkv) * D
qkv = torch.randn(B * Lq, W, device=dev, generator=g).to(BF)
q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
cls = bias = None
if prefix == "bias":
    bias = torch.zeros(Hq, Lq, (Lq + 7) // 8 * 8, dtype=BF, device=dev)
    bias[:, :, :Lq] = torch.randn(Hq, Lq, Lq, device=dev, generator=g).to(BF)
elif prefix is not None:
    cls = torch.zeros(B, Lq, dtype=torch.uint8, device=dev)
    cls[:, prefix:] = 1
a = K.attn_args(B, Lq, Hq, Hkv, D, q, qkv.stride(0), k, qkv.stride(0), v, qkv.stride(0), scale, cap, cls, 0,
                bias=bias)
out = torch.empty(B * Lq, Hq * D, dtype=BF, device=dev)
lse = torch.empty(B, Hq, Lq, device=dev)
do = torch.randn(B * Lq, Hq * D, device=dev, generator=g).to(BF)
dqkv = torch.empty_like(qkv)
ld = dqkv.stride(0)
K.attn_fwd(a, out, lse)
for _ in range(reps):
    if what == "fwd":
        K.attn_fwd(a, out, lse)
    else:
        K.attn_bwd(a, out, do, lse, dqkv[:, :Hq * D], ld, dqkv[:, Hq * D:(Hq + Hkv) * D], ld, dqkv[:, (Hq + Hkv) * D:], ld)
torch.cuda.synchronize()
print("ok")
