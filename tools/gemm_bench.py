"""Microbenchmark of svla_gemm_bf16 on the SpatialVLA-4B GEMM shapes (B=32, M=9984), with torch.matmul
(hipBLASLt) on the same operands as a yardstick.  Prints one line per shape: TFLOP/s and % of 2.5 PF."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
M = 9984
SHAPES = [  # name, M, N, K, layouts
    ("qkv fwd", M, 4096, 2304, "nt"), ("o fwd", M, 2304, 2048, "nt"), ("gate/up fwd", M, 18432, 2304, "nt"),
    ("down fwd", M, 2304, 9216, "nt"), ("down dgrad", M, 9216, 2304, "nn"), ("gate/up dgrad", M, 2304, 18432, "nn"),
    ("gate/up wgrad", 18432, 2304, M, "tn"), ("down wgrad", 2304, 9216, M, "tn"),
    ("lm_head fwd", M, 265408, 2304, "nt"), ("siglip fc1 fwd", 8192, 4304, 1152, "nt"),
    ("siglip qkv fwd", 8192, 3456, 1152, "nt"), ("siglip o fwd", 8192, 1152, 1152, "nt"),
    ("siglip fc2 fwd", 8192, 1152, 4304, "nt"), ("siglip fc2 dgrad", 8192, 4304, 1152, "nn"),
    ("siglip fc1 wgrad", 4304, 1152, 8192, "tn"), ("siglip o wgrad", 1152, 1152, 8192, "tn"),
    ("qkv wgrad", 4096, 2304, M, "tn"), ("o dgrad", M, 2048, 2304, "nn"), ("o wgrad", 2304, 2048, M, "tn"),
    ("qkv dgrad", M, 2304, 4096, "nn"),
    ("square 4k", 4096, 4096, 4096, "nt"), ("square 8k", 8192, 8192, 8192, "nt"),
]


def run(name, m, n, k, lay, reps=10):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    if lay == "nt":
        a = torch.randn(m, k, device=dev, generator=g).to(BF); b = torch.randn(n, k, device=dev, generator=g).to(BF)
        A, B = K._operand([a], L.LAYOUT_KC), K._operand([b], L.LAYOUT_KC)
        ref = lambda: a @ b.T
    elif lay == "nn":
        a = torch.randn(m, k, device=dev, generator=g).to(BF); b = torch.randn(k, n, device=dev, generator=g).to(BF)
        A, B = K._operand([a], L.LAYOUT_KC), K._operand([b], L.LAYOUT_RC)
        ref = lambda: a @ b
    else:
        a = torch.randn(k, m, device=dev, generator=g).to(BF); b = torch.randn(k, n, device=dev, generator=g).to(BF)
        A, B = K._operand([a], L.LAYOUT_RC), K._operand([b], L.LAYOUT_RC)
        ref = lambda: a.T @ b
    c = torch.empty(m, n, dtype=BF, device=dev)
    f = lambda: K.gemm(m, n, k, A, B, [c], [0], n, K._epi())
    for fn in (f, ref):
        for _ in range(2): fn()
    torch.cuda.synchronize()
    variants = [int(v) for v in os.environ.get("SVLA_VARIANTS", "0").split(",")]
    arms = [(f"v{v}", v, f) for v in variants] + [("torch", None, ref)]
    best = {}
    for rnd in range(3):  # interleaved rounds in one process; report the best of 3 per arm
        for tag, v, fn in arms:
            if v is not None:
                K.gemm_variant = v
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps): fn()
            e1.record(); e1.synchronize()
            ms = e0.elapsed_time(e1) / reps
            best[tag] = min(best.get(tag, 1e30), ms)
    r = ref().float()
    errs = []
    for v in variants:
        K.gemm_variant = v
        c.fill_(float("nan")); f(); torch.cuda.synchronize()
        errs.append(f"{((c.float() - r).norm() / r.norm()).item():.1e}")
    K.gemm_variant = 0
    cols = "  ".join(f"{t} {best[t]:7.3f} ms {2.0 * m * n * k / best[t] / 1e9:7.1f} TF" for t, _, _ in arms)
    print(f"{name:16s} M={m:6d} N={n:6d} K={k:6d} {cols}  relerr {'/'.join(errs)}", flush=True)


def stamps(m, n, k, lay="nt"):
    """Diagnostic build 12 (SVLA_GEMM_DIAG bit 3): per-wave s_memtime at every barrier of block 0."""
    dev = "cuda"
    if lay == "nt":
        a = torch.randn(m, k, device=dev).to(BF); b = torch.randn(n, k, device=dev).to(BF)
        A, B = K._operand([a], L.LAYOUT_KC), K._operand([b], L.LAYOUT_KC)
    elif lay == "nn":
        a = torch.randn(m, k, device=dev).to(BF); b = torch.randn(k, n, device=dev).to(BF)
        A, B = K._operand([a], L.LAYOUT_KC), K._operand([b], L.LAYOUT_RC)
    else:
        a = torch.randn(k, m, device=dev).to(BF); b = torch.randn(k, n, device=dev).to(BF)
        A, B = K._operand([a], L.LAYOUT_RC), K._operand([b], L.LAYOUT_RC)
    c = torch.zeros(m, n, dtype=BF, device=dev)
    for _ in range(3):
        K.gemm(m, n, k, A, B, [c], [0], n, K._epi())
    torch.cuda.synchronize()
    nst = (k + 31) // 32
    raw = c.view(-1).view(torch.int64)[: 8 * (2 * nst + 4)].cpu().view(8, 2 * nst + 4)[:, : 2 * nst + 1]
    d = (raw[:, 1:] - raw[:, :-1]).float()
    print(f"stamps {lay} M={m} N={n} K={k}: phase-a mean {d[:, 0::2].mean():.0f}  phase-b mean {d[:, 1::2].mean():.0f} "
          f"(s_memtime ticks); first stage {d[:, :2].tolist()[0]}, per-wave mean {d.mean(1).tolist()}")


if __name__ == "__main__":
    if os.environ.get("SVLA_STAMPS"):
        stamps(9984, 18432, 2304)
        stamps(9984, 9216, 2304, "nn")
        stamps(18432, 2304, 9984, "tn")
        sys.exit(0)
    sel = sys.argv[1:]
    for s in SHAPES:
        if not sel or any(x in s[0] for x in sel):
            run(*s)
