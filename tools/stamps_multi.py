"""k-loop stamps of several diagnostic gemm4 builds (-DG4_STAMPS=1, optionally -DG4_ABL=n) in ONE process:
python tools/stamps_multi.py lib1.so [lib2.so ...] -- M,N,K[,layout] [M,N,K ...]
Per build and shape: ticks per data-parallel k-tile, per stream-K k-tile, epilogue per tile, and the kernel's wall."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from spatialvla_amd import kernels as K, _lib as L

sep = sys.argv.index("--")
libs = [(os.path.basename(p), L.load(os.path.abspath(p), strict=False)) for p in sys.argv[1:sep]]
shapes = []
for s in sys.argv[sep + 1:]:
    f = s.split(",")
    shapes.append((int(f[0]), int(f[1]), int(f[2]), f[3] if len(f) > 3 else "nt"))
BF = torch.bfloat16
for M, N, Kd, lay in shapes:
    a = torch.randn(M, Kd, device="cuda").to(BF) if lay != "tn" else torch.randn(Kd, M, device="cuda").to(BF)
    b = torch.randn(N, Kd, device="cuda").to(BF) if lay == "nt" else torch.randn(Kd, N, device="cuda").to(BF)
    c = torch.empty(M, N, device="cuda", dtype=BF)
    A = K._operand([a], L.LAYOUT_KC if lay != "tn" else L.LAYOUT_RC)
    B = K._operand([b], L.LAYOUT_KC if lay == "nt" else L.LAYOUT_RC)
    for tag, lib in libs:
        L._lib = lib
        f = lambda: K.gemm(M, N, Kd, A, B, [c], [0], N, K._epi())  # noqa: E731
        for _ in range(3):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record(); e1.synchronize()
        ms = e0.elapsed_time(e1) / 10
        buf = np.zeros((16384, 4, 14), dtype=np.uint64)
        fn = lib.svla_diag_g4_stamps
        fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        torch.cuda.synchronize()
        lib.svla_diag_g4_stamps_clear()
        f(); torch.cuda.synchronize()
        assert fn(buf.ctypes.data, buf.nbytes) == 0
        s = buf.astype(np.float64)
        s = s[s[:, 0, 7] > 0]
        tot = s[:, :, 7].max(1)  # per block: the slowest wave
        order = np.argsort(tot)
        pb = lambda b: (f"total {tot[b]:.0f} = dp k-tiles {s[b, 0, 13]:.0f}, sk k-tiles {s[b, 0, 12]:.0f} in "
                        f"{s[b, 0, 11]:.0f}, tiles {s[b, 0, 6]:.0f}, epilogue {s[b, 0, 5]:.0f}")
        print(f"    blocks {len(s)}: total ticks min {tot.min():.0f} median {np.median(tot):.0f} max {tot.max():.0f}; "
              f"slowest block: {pb(order[-1])}; median block: {pb(order[len(order) // 2])}", flush=True)
        nt = s[..., 6].sum(0)[0]
        ml = s[..., 3] + s[..., 4]
        sk_t, sk_n, dp_n = s[..., 11], s[..., 12], s[..., 13]
        kl = s[..., 3].sum() / max((dp_n + sk_n).sum(), 1)
        print(f"{M}x{N}x{Kd} {lay} {tag:22s} {ms:.3f} ms {2e-9 * M * N * Kd / ms:7.1f} TF | k-loop {kl:6.0f} ticks/k-tile"
              f" | dp {(ml - sk_t).sum() / max(dp_n.sum(), 1):6.0f}/k-tile ({dp_n[:, 0].sum():.0f}), sk"
              f" {sk_t.sum() / max(sk_n.sum(), 1):6.0f}/k-tile ({sk_n[:, 0].sum():.0f}) | epilogue/tile"
              f" {s[..., 5].sum() / 4 / nt:6.0f} | waits top {s[..., 0].mean() / s[..., 3].mean():.3f} RB1"
              f" {s[..., 1].mean() / s[..., 3].mean():.3f} RB2 {s[..., 2].mean() / s[..., 3].mean():.3f}"
              f" | block mean {s[..., 7].mean():.0f} max {s[..., 7].max():.0f}", flush=True)
