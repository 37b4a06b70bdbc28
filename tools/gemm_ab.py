"""A/B two libsvla builds in ONE process (interleaved rounds, best of N per arm): python tools/gemm_ab.py libA.so
libB.so [shape-name filters].  Shapes from tools/gemm_bench.py; both builds share kernels.gemm's stream-K workspace."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L
from tools.gemm_bench import SHAPES, BF

libs = []
for path in sys.argv[1:3]:
    cd = L.load(os.path.abspath(path), strict=False)
    libs.append((os.path.basename(path), cd, None))  # kernels.gemm passes its (zero-kept) workspace per call
sel = sys.argv[3:]
for name, m, n, k, lay in SHAPES:
    if sel and not any(x in name for x in sel):
        continue
    a = torch.randn(m, k, device="cuda").to(BF) if lay != "tn" else torch.randn(k, m, device="cuda").to(BF)
    b = torch.randn(n, k, device="cuda").to(BF) if lay == "nt" else torch.randn(k, n, device="cuda").to(BF)
    A = K._operand([a], L.LAYOUT_KC if lay != "tn" else L.LAYOUT_RC)
    B = K._operand([b], L.LAYOUT_KC if lay == "nt" else L.LAYOUT_RC)
    c = torch.empty(m, n, dtype=BF, device="cuda")
    best = {}
    outs = {}
    for rnd in range(5):
        for tag, cd, _ in libs:
            L._lib = cd
            f = lambda: K.gemm(m, n, k, A, B, [c], [0], n, K._epi())  # noqa: E731
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record(); e1.synchronize()
            best[tag] = min(best.get(tag, 1e9), e0.elapsed_time(e1) / 10)
            outs[tag] = c.clone()
    t = list(best)
    same = torch.equal(outs[t[0]], outs[t[1]])
    print(f"{name:16s} " + "  ".join(f"{x}: {best[x]:.3f} ms {2e-9 * m * n * k / best[x]:7.1f} TF" for x in t)
          + f"  ratio {best[t[0]] / best[t[1]]:.3f} bitwise_equal={same}", flush=True)
