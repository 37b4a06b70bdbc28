"""Time the training step's weak GEMM shapes (STORE epilogue) under every dispatch variant and torch (hipBLASLt).
python tools/gemm_shapes.py  -> TFLOP/s per (shape, arm)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
# (M, N, K, layout A, layout B): 'K' = [rows][K] (KC), 'R' = [K][rows] (RC)
SH = [(8192, 1152, 1152, "K", "K"), (8192, 1152, 1152, "K", "R"), (1152, 1152, 8192, "R", "R"),
      (8192, 4304, 1152, "K", "K"), (8192, 4304, 1152, "K", "R"), (8192, 1152, 4304, "K", "K"),
      (8192, 1152, 4304, "K", "R"), (1152, 4304, 8192, "R", "R"), (4304, 1152, 8192, "R", "R"),
      (8192, 3456, 1152, "K", "K"), (8192, 1152, 3456, "K", "R"), (3456, 1152, 8192, "R", "R"),
      (9984, 4096, 2304, "K", "K"), (4096, 2304, 9984, "R", "R"), (9984, 2304, 4096, "K", "R"),
      (9984, 2048, 2304, "K", "R"), (2304, 2048, 9984, "R", "R"), (9984, 2304, 2048, "K", "K")]
if os.environ.get("BIG"):
    SH = [(9984, 2304, 9216, "K", "K"), (2304, 9216, 9984, "R", "R"), (9984, 9216, 2304, "K", "R"),
          (18432, 2304, 9984, "R", "R"), (9984, 2304, 18432, "K", "R")]
L.lib()
for M, N, Kd, la, lb in SH:
    a = torch.randn(M, Kd, device="cuda").to(BF) if la == "K" else torch.randn(Kd, M, device="cuda").to(BF)
    b = torch.randn(N, Kd, device="cuda").to(BF) if lb == "K" else torch.randn(Kd, N, device="cuda").to(BF)
    A = K._operand([a], L.LAYOUT_KC if la == "K" else L.LAYOUT_RC)
    B = K._operand([b], L.LAYOUT_KC if lb == "K" else L.LAYOUT_RC)
    at = a if la == "K" else a.T
    bt = b.T if lb == "K" else b
    c = torch.empty(M, N, dtype=BF, device="cuda")
    res = {}
    for rnd in range(3):
        for arm in (0, 1, 2, 3, 4, "torch"):
            if arm == "torch":
                f = lambda: at @ bt  # noqa: E731
            else:
                L.lib().svla_gemm_set_variant(arm)
                f = lambda: K.gemm(M, N, Kd, A, B, [c], [0], N, K._epi())  # noqa: E731
            f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                f()
            e1.record(); e1.synchronize()
            res[arm] = min(res.get(arm, 1e9), e0.elapsed_time(e1) / 10)
    L.lib().svla_gemm_set_variant(0)
    fl = 2.0 * M * N * Kd
    print(f"{M}x{N}x{Kd} {la}{lb}  " + "  ".join(f"{arm}:{fl / (t * 1e-3) / 1e12:6.0f}" for arm, t in res.items()),
          flush=True)
