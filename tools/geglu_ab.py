"""Cost of the fused GeGLU epilogue on the Gemma2 gate|up projection (B=32: 9984 x 18432 x 2304): the GEGLU launch
(h, g, u written) against a plain STORE of the same 9984 x 18432 product, same operands, one process, best of 3
rounds of 5 launches.  python tools/geglu_ab.py [lib.so ...]  (each extra library is loaded in turn)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
M, Kd, I = 9984, 2304, 9216


def timeit(fn, reps=5):
    fn(); torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps): fn()
        e1.record(); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best * 1e3


def main():
    libs = sys.argv[1:] or [None]
    g0 = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, Kd, device="cuda", generator=g0).to(BF)
    wg = (torch.randn(I, Kd, device="cuda", generator=g0) * 0.05).to(BF)
    wu = (torch.randn(I, Kd, device="cuda", generator=g0) * 0.05).to(BF)
    w = torch.cat([wg, wu])
    h, g, u = (torch.empty(M, I, dtype=BF, device="cuda") for _ in range(3))
    c = torch.empty(M, 2 * I, dtype=BF, device="cuda")
    ref = None
    for path in libs:
        if path is not None:
            L._lib = L.load(os.path.abspath(path), strict=False)
        A, B = K._operand([x], L.LAYOUT_KC), K._operand([w], L.LAYOUT_KC)
        store = lambda: K.gemm(M, 2 * I, Kd, A, B, [c], [0], 2 * I, K._epi())
        geglu = lambda: K.linear_geglu_fwd(x, wg, wu, h, g, u)
        ts, tg = timeit(store), timeit(geglu)
        geglu(); torch.cuda.synchronize()
        hh = h.float()
        if ref is None:
            gf = (x.float() @ wg.float().T).to(BF).float()
            uf = (x.float() @ wu.float().T).to(BF).float()
            ref = (torch.nn.functional.gelu(gf, approximate="tanh").to(BF).float() * uf).to(BF).float()
            del gf, uf
        diff = (hh != ref).float().mean().item()
        rel = ((hh - ref).norm() / ref.norm()).item()
        print(f"{path or 'default'}: STORE {ts:7.1f} us  GEGLU {tg:7.1f} us  epilogue cost {tg - ts:6.1f} us "
              f"({(tg / ts - 1) * 100:5.1f} %)  h vs torch: rel {rel:.2e} differing {diff:.2e}", flush=True)


if __name__ == "__main__":
    main()
