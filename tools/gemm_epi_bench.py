"""Cost of the heavy GEMM epilogues on their training shapes (B=32): the lm_head with SOFTCAP_CE vs a plain store,
the q|k|v projection with ROPE vs a plain store; one process, best of 3 rounds of 5 launches."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K, _lib as L

BF = torch.bfloat16
M = 9984


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


x = torch.randn(M, 2304, device="cuda").to(BF)
# q|k|v + RoPE
w = (torch.randn(4096, 2304, device="cuda") * 0.02).to(BF)
out = torch.empty(M, 4096, dtype=BF, device="cuda")
pos = torch.arange(1, 313, device="cuda").float()
inv = 1.0 / (10000 ** (torch.arange(0, 256, 2, device="cuda").float() / 256))
fr = pos[:, None] * inv[None]
cos, sin = fr.cos().to(BF).contiguous(), fr.sin().to(BF).contiguous()
t0 = timeit(lambda: K.linear_fwd(x, [w], out))
t1 = timeit(lambda: K.linear_fwd(x, [w], out, kind=L.EPI_ROPE, rope=(cos, sin, 312, 256, 3072)))
K.gemm_variant = 3  # 4-wave kernel
t1b = timeit(lambda: K.linear_fwd(x, [w], out, kind=L.EPI_ROPE, rope=(cos, sin, 312, 256, 3072)))
ref4 = out.clone()
K.gemm_variant = 0
K.linear_fwd(x, [w], out, kind=L.EPI_ROPE, rope=(cos, sin, 312, 256, 3072))
same = torch.equal(out, ref4)
fl = 2.0 * M * 4096 * 2304
print(f"qkv   store {t0:.3f} ms ({fl / t0 / 1e9:.0f} TF)   rope {t1:.3f} ms ({fl / t1 / 1e9:.0f} TF)   "
      f"rope on the 4-wave kernel {t1b:.3f} ms (bitwise equal: {same})", flush=True)
# lm_head + softcap CE partials
V = 265347
Vp = (V + 63) // 64 * 64
wl = (torch.randn(V, 2304, device="cuda") * 0.02).to(BF)
logits = torch.empty(M, Vp, dtype=BF, device="cuda")
stats = torch.empty(M, (V + 127) // 128, 3, dtype=torch.float32, device="cuda")
t2 = timeit(lambda: K.gemm(M, V, 2304, K._operand([x], L.LAYOUT_KC), K._operand([wl], L.LAYOUT_KC), [logits], [0], Vp,
                           K._epi()))
t3 = timeit(lambda: K.gemm(M, V, 2304, K._operand([x], L.LAYOUT_KC), K._operand([wl], L.LAYOUT_KC), [logits], [0], Vp,
                           K._epi(L.EPI_SOFTCAP_CE, cap=30.0, row_stats=stats)))
sc = lambda: K.gemm(M, V, 2304, K._operand([x], L.LAYOUT_KC), K._operand([wl], L.LAYOUT_KC), [logits], [0], Vp,  # noqa
                    K._epi(L.EPI_SOFTCAP_CE, cap=30.0, row_stats=stats))
ref_l, ref_s = logits.clone(), stats.clone()
K.gemm_variant = 4  # never the 4-wave kernel: the 8-phase kernel's LDS epilogue
t4 = timeit(sc)
l8, s8 = logits.clone(), stats.clone()
K.gemm_variant = 0
fl = 2.0 * M * V * 2304
print(f"lm_head store {t2:.3f} ms ({fl / t2 / 1e9:.0f} TF)   softcap_ce {t3:.3f} ms ({fl / t3 / 1e9:.0f} TF)   "
      f"softcap_ce 8-phase {t4:.3f} ms; logits equal {torch.equal(ref_l[:, :V], l8[:, :V])}, max |dstats| "
      f"{(ref_s[..., :2] - s8[..., :2]).abs().max().item():.3e}, argmax equal "
      f"{torch.equal(ref_s[..., 2].view(torch.int32), s8[..., 2].view(torch.int32))}", flush=True)
