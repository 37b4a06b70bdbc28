"""Time svla_attn_fwd / svla_attn_bwd at the training shapes (B=32) for one or more libsvla builds, interleaved in
one process, best of N rounds; outputs of every build are checked against the first one.
python tools/attn_bench.py [lib1.so lib2.so ...]   (default: the in-tree spatialvla_amd/libsvla.so)

FLOPs: fwd 4*B*Hq*L^2*D (QK^T and PV), bwd 2.5x fwd (S recompute, dP, dV, dK, dQ)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
SHAPES = [  # name, B, L, Hq, Hkv, D, scale, softcap, prefix (None: no key classes)
    ("gemma2", 32, 312, 8, 4, 256, 1 / 16, 50.0, 299),
    ("siglip", 32, 256, 16, 16, 72, 72 ** -0.5, 0.0, None),
    ("beit", 32, 577, 16, 16, 64, 0.125, 0.0, "bias"),  # ZoeDepth BEiT-L at 384^2: relative position bias, fwd only
]


def main():
    paths = sys.argv[1:] or [L.LIB_PATH]
    libs = [(os.path.basename(p).replace("libsvla_", "").replace(".so", ""), L.load(os.path.abspath(p)))
            for p in paths]
    dev = "cuda"
    for name, B, Lq, Hq, Hkv, D, scale, cap, prefix in SHAPES:
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
        do = torch.randn(B * Lq, Hq * D, device=dev, generator=g).to(BF)
        fl = 4.0 * B * Hq * Lq * Lq * D
        res, outs = {}, {}
        for rnd in range(5):
            for tag, cd in libs:
                L._lib = cd
                a = K.attn_args(B, Lq, Hq, Hkv, D, q, qkv.stride(0), k, qkv.stride(0), v, qkv.stride(0), scale, cap,
                                cls, 0, bias=bias)
                out = torch.empty(B * Lq, Hq * D, dtype=BF, device=dev)
                lse = torch.empty(B, Hq, Lq, device=dev)
                dqkv = torch.zeros_like(qkv)
                ld = dqkv.stride(0)
                fwd = lambda: K.attn_fwd(a, out, lse)  # noqa: E731
                bwd = (lambda: None) if bias is not None else lambda: K.attn_bwd(a, out, do, lse, dqkv[:, :Hq * D], ld,  # noqa: E731
                                         dqkv[:, Hq * D:(Hq + Hkv) * D], ld, dqkv[:, (Hq + Hkv) * D:], ld)
                fwd(); bwd()
                torch.cuda.synchronize()
                ts = []
                for f in (fwd, bwd):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(20):
                        f()
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) / 20 * 1e3)
                prev = res.get(tag, (1e30, 1e30))
                res[tag] = (min(prev[0], ts[0]), min(prev[1], ts[1]))
                if rnd == 0:
                    outs[tag] = (out.float().clone(), dqkv.float().clone())
        ref = outs[libs[0][0]]
        for tag, _ in libs:
            tf, tb = res[tag]
            o, dg = outs[tag]
            eo = float((o - ref[0]).norm() / ref[0].norm())
            eg = float((dg - ref[1]).norm() / ref[1].norm())
            print(f"{name:7s} {tag:10s} fwd {tf:8.1f} us {fl / tf * 1e-6:7.1f} TF ({fl / tf * 1e-6 / 2500:.3f})   "
                  f"bwd {tb:8.1f} us {2.5 * fl / tb * 1e-6:7.1f} TF ({2.5 * fl / tb * 1e-6 / 2500:.3f})   "
                  f"vs {libs[0][0]}: out {eo:.1e} grads {eg:.1e}", flush=True)


if __name__ == "__main__":
    main()
