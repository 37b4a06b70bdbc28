"""Phase cycles of attn_fwd32_kernel (diagnostic build -DATT32_STAMPS=1, spatialvla_amd/libsvla_att.so) at the Gemma2
training shape: python tools/att32_stamps.py -> per-block medians / means of prologue, tile-top waits, phases A-D
(summed over the 5 key tiles), epilogue, total (s_memtime cycles, wave 0 of each block)."""
import ctypes
import os
import sys

import numpy as np

os.environ["SVLA_ATTN32"] = "1"  # the 32x32x16 forward is opt-in

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from spatialvla_amd import kernels as K, _lib as L  # noqa: E402
from tools.attn_bench import SHAPES, BF  # noqa: E402


def main():
    L._lib = L.load(os.path.join(os.path.dirname(L.LIB_PATH), "libsvla_att.so"))
    _, B, Lq, Hq, Hkv, D, scale, cap, prefix = SHAPES[0]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(1)
    qkv = torch.randn(B * Lq, (Hq + 2 * Hkv) * D, device=dev, generator=g).to(BF)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    cls = torch.zeros(B, Lq, dtype=torch.uint8, device=dev)
    cls[:, prefix:] = 1
    a = K.attn_args(B, Lq, Hq, Hkv, D, q, qkv.stride(0), k, qkv.stride(0), v, qkv.stride(0), scale, cap, cls, 0)
    out = torch.empty(B * Lq, Hq * D, dtype=BF, device=dev)
    lse = torch.empty(B, Hq, Lq, device=dev)
    for _ in range(3):
        K.attn_fwd(a, out, lse)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    K.attn_fwd(a, out, lse)
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros((4096, 8), dtype=np.uint64)
    fn = L._lib.svla_diag_att32_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    nblk = ((Lq + 63) // 64) * (Hq // 2) * B
    st = buf[:nblk].astype(np.float64)
    names = ["prologue", "tile-top waits", "A: QK0", "B: QK1+sm0", "C: PV0+sm1", "D: PV1", "epilogue", "total"]
    print(f"kernel {e0.elapsed_time(e1) * 1e3:.1f} us, {nblk} blocks")
    for i, n in enumerate(names):
        print(f"{n:16s} median {np.median(st[:, i]):10.0f}  mean {st[:, i].mean():10.0f}  max {st[:, i].max():10.0f}")


if __name__ == "__main__":
    main()
