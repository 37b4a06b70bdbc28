"""Time several libsvla builds (one GEMM variant each) in ONE process, interleaved, best of N, next to torch:
python tools/gemm_multi.py VARIANT lib1.so lib2.so ... -- [shape-name filters]."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L
from tools.gemm_bench import SHAPES, BF

args = sys.argv[1:]
variant = int(args[0])
paths = args[1:args.index("--")] if "--" in args else args[1:]
sel = args[args.index("--") + 1:] if "--" in args else []
libs = []
for path in paths:
    cd = L.load(os.path.abspath(path))
    libs.append((os.path.basename(path).replace("libsvla_", "").replace(".so", ""), cd, None))
K.gemm_variant = variant
for name, m, n, k, lay in SHAPES:
    if sel and not any(x in name for x in sel):
        continue
    a = torch.randn(m, k, device="cuda").to(BF) if lay != "tn" else torch.randn(k, m, device="cuda").to(BF)
    b = torch.randn(n, k, device="cuda").to(BF) if lay == "nt" else torch.randn(k, n, device="cuda").to(BF)
    A = K._operand([a], L.LAYOUT_KC if lay != "tn" else L.LAYOUT_RC)
    B = K._operand([b], L.LAYOUT_KC if lay == "nt" else L.LAYOUT_RC)
    at, bt = (a if lay != "tn" else a.T), (b.T if lay == "nt" else b)
    c = torch.empty(m, n, dtype=BF, device="cuda")
    ref = (at.float() @ bt.float())
    best, errs = {}, {}
    arms = [(t, cd) for t, cd, _ in libs] + [("torch", None)]
    for rnd in range(4):
        for tag, cd in arms:
            if cd is not None:
                L._lib = cd
                f = lambda: K.gemm(m, n, k, A, B, [c], [0], n, K._epi())  # noqa: E731
            else:
                f = lambda: at @ bt  # noqa: E731
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record(); e1.synchronize()
            best[tag] = min(best.get(tag, 1e9), e0.elapsed_time(e1) / 10)
            if cd is not None and rnd == 0:
                errs[tag] = ((c.float() - ref).norm() / ref.norm()).item()
    print(f"{name:16s} " + " ".join(f"{t}:{2e-9 * m * n * k / best[t]:6.0f}" for t, _ in arms)
          + "  maxerr %.1e" % max(errs.values()), flush=True)
