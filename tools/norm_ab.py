"""A/B two libsvla builds on the HBM-pass kernels at the 4B shape -- the Gemma2 RMSNorm kernels (rows = 32 x 312,
N = 2304) and the lm_head softcap + statistics pass (9984 x 265408) -- interleaved rounds in one process, best of 5
per arm, outputs compared bitwise: python tools/norm_ab.py libA.so libB.so"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spatialvla_amd import _lib as L
from spatialvla_amd import kernels as K

R, N = 9984, 2304
BF = torch.bfloat16
dev = "cuda"
torch.manual_seed(0)
r = lambda *s: torch.randn(*s, device=dev).to(BF)  # noqa: E731
x, res, y, dy, dres = r(R, N), r(R, N), r(R, N), r(R, N), r(R, N)
w1, w2 = r(N) * 0.1, r(N) * 0.1
rs1, rs2 = torch.rand(R, device=dev) + 0.5, torch.rand(R, device=dev) + 0.5
outs = {}


V = 265408
LDV = (V + 63) // 64 * 64
logits = torch.empty(R, LDV, dtype=BF, device=dev)
logits.view(-1)[:].copy_((torch.randn(R * LDV // 64, device=dev) * 8).repeat_interleave(64).to(BF))  # 5.3 GB
stats = torch.empty(R, (V + 127) // 128, 3, device=dev)
small = (torch.randn(512, LDV, device=dev) * 8).to(BF)
# the special values that send a lane to the softcap pass's per-element path: NaN, a +-0 group max, ties, +-inf
small[0, 5] = float("nan")
small[1, 128:256] = -small[1, 128:256].abs()
small[1, 130], small[1, 200], small[1, 131] = 0.0, -0.0, 0.0
small[2, 256:384] = -small[2, 256:384].abs() - 1
small[2, 300] = -0.0
small[3, :128] = 2.5
small[4, 9], small[4, 700], small[5, 3], small[5, 4] = 7.0, float("inf"), float("-inf"), 1e30
small[6, 512:640] = float("-inf")
small[7, V - 3] = float("nan")
gsig = r(8192, 4304)
part = torch.randn(624, 2304, device=dev)
cs1, cs2, cs3 = (torch.empty(n, dtype=BF, device=dev) for n in (4304, 1152, 2304))


def softcap_small():
    t = small.clone()
    st = torch.empty(512, (V + 127) // 128, 3, device=dev)
    K.softcap_ce_rows(t, V, st, 30.0)
    return t, st


def cases():
    o1, o2 = torch.empty_like(x), torch.empty_like(x)
    rstd = torch.empty(R, device=dev)
    dw1, dw2 = torch.empty(N, dtype=BF, device=dev), torch.empty(N, dtype=BF, device=dev)
    return {
        "rms_fwd": (lambda: K.rmsnorm_fwd(x, w1, 1e-6, o1, rstd), (o1, rstd)),
        "add_rms_fwd": (lambda: K.add_rmsnorm_fwd(res, x, w1, 1e-6, o1, rstd), (o1, rstd)),
        "add_rmsnorm2_train": (lambda: K.add_rmsnorm2_fwd_train(res, y, w1, w2, 1e-6, 1e-6, o1, o2, rs1, rs2),
                               (o1, o2, rs1, rs2)),
        "rms_bwd": (lambda: K.rmsnorm_bwd(x, w1, rs1, dy, dres, o1, dw1), (o1, dw1)),
        "rms_bwd2": (lambda: K.rmsnorm2_bwd(x, w2, rs2, dy, dres, y, w1, rs1, o1, o2, dw2, dw1), (o1, o2, dw1, dw2)),
        "softcap_rows": (lambda: K.softcap_ce_rows(logits, V, stats, 30.0), None),
        "colsum_bf16_4304": (lambda: K.colsum_bf16(gsig, cs1), (cs1,)),  # SigLIP fc1 bias gradient
        "colsum_bf16_1152": (lambda: K.colsum_bf16(gsig[:, :1152], cs2), (cs2,)),
        "colsum_f32_2304": (lambda: K.colsum_f32(part, cs3), (cs3,)),  # norm-weight partial planes
    }


libs = [(os.path.basename(p), L.load(os.path.abspath(p))) for p in sys.argv[1:3]]
best = {}
for rnd in range(5):
    for tag, lib in libs:
        L._lib = lib
        for name, (f, res_t) in cases().items():
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20 if name != "softcap_rows" else 3):
                f()
            e1.record()
            e1.synchronize()
            best[(name, tag)] = min(best.get((name, tag), 1e9),
                                    e0.elapsed_time(e1) / (20 if name != "softcap_rows" else 3) * 1e3)
            if rnd == 0:
                outs[(name, tag)] = [t.clone() for t in res_t] if res_t is not None else list(softcap_small())
ta, tb = libs[0][0], libs[1][0]
for name in cases():
    same = all(torch.equal(a.contiguous().view(torch.uint8), b.contiguous().view(torch.uint8))  # bitwise, NaN incl.
               for a, b in zip(outs[(name, ta)], outs[(name, tb)]))
    print(f"{name:20s} {ta}: {best[(name, ta)]:7.1f} us  {tb}: {best[(name, tb)]:7.1f} us  "
          f"ratio {best[(name, ta)] / best[(name, tb)]:.3f}  bitwise_equal={same}", flush=True)
