"""Per-wave wait cycles of the gemm4 k-loop (diagnostic build -DG4_STAMPS=1): python tools/gemm_stamps.py lib.so M N K"""
import ctypes, os, sys
# usage: python tools/gemm_stamps.py lib.so M N K [layout nt|nn|tn]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from spatialvla_amd import kernels as K, _lib as L

lib = L.load(os.path.abspath(sys.argv[1]))
L._lib = lib
M, N, Kd = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
lay = sys.argv[5] if len(sys.argv) > 5 else "nt"
a = torch.randn(M, Kd, device="cuda").to(torch.bfloat16) if lay != "tn" else torch.randn(Kd, M, device="cuda").to(torch.bfloat16)
b = torch.randn(N, Kd, device="cuda").to(torch.bfloat16) if lay == "nt" else torch.randn(Kd, N, device="cuda").to(torch.bfloat16)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
A = K._operand([a], L.LAYOUT_KC if lay != "tn" else L.LAYOUT_RC)
B = K._operand([b], L.LAYOUT_KC if lay == "nt" else L.LAYOUT_RC)
K.gemm_variant = 0
for _ in range(5):
    K.gemm(M, N, Kd, A, B, [c], [0], N, K._epi())
torch.cuda.synchronize()
buf = np.zeros((16384, 4, 14), dtype=np.uint64)
fn = lib.svla_diag_g4_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0
tiles = ((M + 255) // 256) * ((N + 255) // 256)
s = buf[:16384].astype(np.float64)
s = s[s[:, 0, 7] > 0]
nt = s[..., 6].sum(0)[0]
print(f"blocks {len(s)}, tiles {nt:.0f}: per tile (ticks) prologue {s[..., 4].sum() / 4 / nt:.0f}, k-loop "
      f"{s[..., 3].sum() / 4 / nt:.0f}, epilogue {s[..., 5].sum() / 4 / nt:.0f} (write+barrier "
      f"{s[..., 8].sum() / 4 / nt:.0f}, read+epi+store {s[..., 9].sum() / 4 / nt:.0f}, end barrier "
      f"{s[..., 10].sum() / 4 / nt:.0f}); per block total {s[..., 7].mean():.0f}")
for w in range(4):
    print(f"  wave {w}: write {s[:, w, 8].sum() / nt:.0f} read/store {s[:, w, 9].sum() / nt:.0f} endbar {s[:, w, 10].sum() / nt:.0f}")
tot = s[..., 3].mean()
print(f"{M}x{N}x{Kd}: k-loop mean {tot:.0f} ticks/wave; share waiting at top-lgkm {s[..., 0].mean() / tot:.3f}, "
      f"RB1 {s[..., 1].mean() / tot:.3f}, RB2 {s[..., 2].mean() / tot:.3f}; per wave (RB1, RB2): "
      f"{[(round(s[:, w, 1].mean() / tot, 3), round(s[:, w, 2].mean() / tot, 3)) for w in range(4)]}")

ml = s[..., 3] + s[..., 4]  # whole mainloop (prologue + k-loop) per wave
sk_t, sk_n, dp_n = s[..., 11], s[..., 12], s[..., 13]
print(f"data-parallel: {dp_n[:, 0].sum():.0f} k-tiles, {(ml - sk_t).sum() / max(dp_n.sum(), 1):.0f} ticks per k-tile; "
      f"stream-K: {sk_n[:, 0].sum():.0f} k-tiles, {sk_t.sum() / max(sk_n.sum(), 1):.0f} ticks per k-tile; "
      f"block total mean {s[..., 7].mean():.0f} max {s[..., 7].max():.0f}; mainloop share {ml.mean() / s[..., 7].mean():.3f}, "
      f"epilogue share {s[..., 5].mean() / s[..., 7].mean():.3f}")
