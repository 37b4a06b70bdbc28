"""Dispatch A/B of the training step's epilogue GEMMs: product dispatch (v0) vs the 4-wave kernel forced (v3), one
process, best of 3 rounds of 5 launches.  python tools/epi_ab.py [name filters]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
dev = "cuda"


def r(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(BF)


def timeit(fn, reps=5):
    fn(); torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps): fn()
        e1.record(); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


def case_fwd(M, N, Kd, kind, **kw):
    x, w = r(M, Kd), r(N, Kd, sc=0.02)
    out = torch.empty(M, N, dtype=BF, device=dev)
    extra = {}
    if kind in (L.EPI_BIAS, L.EPI_BIAS_GELU, L.EPI_BIAS_RESID, L.EPI_BIAS_GELU_ERF, L.EPI_BIAS_SCALE_RESID):
        extra["bias"] = r(N, sc=0.1)
    if kind == L.EPI_BIAS_GELU:
        extra["out1"] = torch.empty(M, N, dtype=BF, device=dev)
    if kind in (L.EPI_BIAS_RESID, L.EPI_BIAS_SCALE_RESID):
        extra["in0"] = r(M, N)
    if kind == L.EPI_BIAS_SCALE_RESID:
        extra["colscale"] = r(N, sc=0.1)
    if kind == L.EPI_ROPE:
        pos = torch.arange(1, 313, device=dev).float()
        inv = 1.0 / (10000 ** (torch.arange(0, 256, 2, device=dev).float() / 256))
        fr = pos[:, None] * inv[None]
        cos, sin = fr.cos().to(BF).contiguous(), fr.sin().to(BF).contiguous()
        extra["rope"] = (cos, sin, 312, 256, 3072)
    return lambda: K.linear_fwd(x, [w], out, kind=kind, **extra), out


def case_dgrad_gelu(M, N, Kd):
    dy, w, pre = r(M, Kd), r(Kd, N, sc=0.02), r(M, N)
    out = torch.empty(M, N, dtype=BF, device=dev)
    return lambda: K.linear_dgrad(dy, [w], out, kind=L.EPI_GELU_BWD, in0=pre), out


CASES = [
    ("siglip qkv BIAS", lambda: case_fwd(8192, 3456, 1152, L.EPI_BIAS)),
    ("siglip o BIAS_RESID", lambda: case_fwd(8192, 1152, 1152, L.EPI_BIAS_RESID)),
    ("siglip fc1 BIAS_GELU", lambda: case_fwd(8192, 4304, 1152, L.EPI_BIAS_GELU)),
    ("siglip fc2 BIAS_RESID", lambda: case_fwd(8192, 1152, 4304, L.EPI_BIAS_RESID)),
    ("siglip fc1 dgrad GELU_BWD", lambda: case_dgrad_gelu(8192, 4304, 1152)),
    ("beit qkv BIAS", lambda: case_fwd(18464, 3072, 1024, L.EPI_BIAS)),
    ("beit o SCALE_RESID", lambda: case_fwd(18464, 1024, 1024, L.EPI_BIAS_SCALE_RESID)),
    ("beit fc1 GELU_ERF", lambda: case_fwd(18464, 4096, 1024, L.EPI_BIAS_GELU_ERF)),
    ("beit fc2 SCALE_RESID", lambda: case_fwd(18464, 1024, 4096, L.EPI_BIAS_SCALE_RESID)),
    ("gemma qkv ROPE", lambda: case_fwd(9984, 4096, 2304, L.EPI_ROPE)),
    ("gemma o wgrad", None),
    ("projector BIAS", lambda: case_fwd(8192, 2304, 1152, L.EPI_BIAS)),
]

sel = sys.argv[1:]
for name, mk in CASES:
    if sel and not any(s in name for s in sel):
        continue
    if mk is None:  # o_proj weight gradient: dy[M, 2304]^T x attn[M, 2048]
        dy, xa = r(9984, 2304), r(9984, 2048)
        dw = torch.empty(2304, 2048, dtype=BF, device=dev)
        fn, out = (lambda: K.linear_wgrad(dy, xa, [dw])), dw
    else:
        fn, out = mk()
    res = {}
    for v in (0, 3, 0, 3):
        K.gemm_variant = v
        t = timeit(fn)
        res[v] = min(res.get(v, 1e30), t)
        outs = out.clone()
        res[f"o{v}"] = outs
    K.gemm_variant = 0
    d = (res["o0"].float() - res["o3"].float()).norm() / res["o0"].float().norm().clamp_min(1e-30)
    print(f"{name:26s} v0 {res[0] * 1e3:8.1f} us  v3 {res[3] * 1e3:8.1f} us  v3/v0 {res[3] / res[0]:.3f}  rel {d:.1e}",
          flush=True)
