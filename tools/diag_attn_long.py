import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
from test_kernels_gpu import _r, _ref_attn
from harness import rel_l2
from spatialvla_amd import kernels as Kn
BF = torch.bfloat16
cuda = "cuda"
def case(D, Hq, Hkv, Lk, Lq, window, cap, pad, fresh):
    torch.manual_seed(11)
    B, cap_rows = 2, Lk + 7
    kd = Hkv * D
    kc = _r(B, cap_rows, kd); vc = _r(B, cap_rows, kd); qfull = _r(B, Lk, Hq * D)
    P = Lk - Lq - 5
    cls = torch.full((B, cap_rows), 2, dtype=torch.uint8, device=cuda)
    cls[:, :P] = 0; cls[:, P:Lk] = 1
    if pad: cls[1, 3] = 2
    qkv = torch.cat([qfull.view(B * Lk, -1), kc[:, :Lk].reshape(B * Lk, kd), vc[:, :Lk].reshape(B * Lk, kd)], 1)
    c2 = cls[:, :Lk].contiguous()
    a = Kn.attn_args(B, Lk, Hq, Hkv, D, qkv[:, :Hq * D], qkv.stride(0), qkv[:, Hq * D:Hq * D + kd], qkv.stride(0), qkv[:, Hq * D + kd:], qkv.stride(0), 1 / 16, cap, c2, window)
    full = torch.empty(B * Lk, Hq * D, dtype=BF, device=cuda)
    Kn.attn_fwd(a, full, torch.empty(B, Hq, Lk, device=cuda))
    ref = _ref_attn(qfull.view(B, Lk, Hq, D), kc[:, :Lk].view(B, Lk, Hkv, D), vc[:, :Lk].view(B, Lk, Hkv, D), 1 / 16, cap, cls[:, :Lk], window)
    o = full.view(B, Lk, Hq, D)
    print(Lk, window, "pad", pad, "total", round(rel_l2(o, ref), 4), "last rows per head b0", [round(rel_l2(o[0, -1, h], ref[0, -1, h]), 3) for h in range(Hq)], "b1", [round(rel_l2(o[1, -1, h], ref[1, -1, h]), 3) for h in range(Hq)], "row0", round(rel_l2(o[:, 0], ref[:, 0]), 3), "rowP", round(rel_l2(o[:, P-1], ref[:, P-1]), 3), flush=True)
for args in [(256, 8, 4, 4500, 1, 4096, 50.0, True, 0), (256, 8, 4, 4500, 1, 4096, 50.0, False, 0), (256, 8, 4, 4500, 1, 0, 50.0, True, 0), (256, 8, 4, 1000, 2, 0, 50.0, True, 0), (256, 8, 4, 4500, 1, 4096, 0.0, False, 0)]:
    case(*args)
