"""BEiT attention forward (B=32, L=577, 16 heads, D=64) with and without the relative position bias, one or more
libsvla builds, best of 5 rounds of 20 launches: python tools/beit_attn_probe.py [lib1.so ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
B, Lq, H, D = int(os.environ.get("B", 32)), 577, 16, 64
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
qkv = torch.randn(B * Lq, 3 * H * D, device=dev, generator=g).to(BF)
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
bias = torch.zeros(H, Lq, (Lq + 7) // 8 * 8, dtype=BF, device=dev)
bias[:, :, :Lq] = torch.randn(H, Lq, Lq, device=dev, generator=g).to(BF)
fl = 4.0 * B * H * Lq * Lq * D
paths = sys.argv[1:] or [L.LIB_PATH]
libs = [(os.path.basename(p).replace("libsvla_", "").replace(".so", ""), L.load(os.path.abspath(p))) for p in paths]
res, outs = {}, {}
for rnd in range(5):
    for tag, cd in libs:
        L._lib = cd
        for bname, bb in (("bias", bias), ("nobias", None)):
            a = K.attn_args(B, Lq, H, H, D, q, qkv.stride(0), k, qkv.stride(0), v, qkv.stride(0), 0.125, 0.0, None, 0,
                            bias=bb)
            out = torch.empty(B * Lq, H * D, dtype=BF, device=dev)
            lse = torch.empty(B, H, Lq, device=dev)
            K.attn_fwd(a, out, lse)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                K.attn_fwd(a, out, lse)
            e1.record()
            e1.synchronize()
            t = e0.elapsed_time(e1) / 20 * 1e3
            key = (tag, bname)
            res[key] = min(res.get(key, 1e30), t)
            if rnd == 0:
                outs[key] = out.float().clone()
for (tag, bname), t in res.items():
    ref = outs[(libs[0][0], bname)]
    e = float((outs[(tag, bname)] - ref).norm() / ref.norm())
    print(f"beit {bname:7s} {tag:10s} {t:8.1f} us {fl / t * 1e-6:7.1f} TF ({fl / t * 1e-6 / 2500:.3f})  vs first {e:.1e}",
          flush=True)
