"""Which E8M0 block scale does v_mfma_scale_f32_32x32x64_f8f6f4 apply to each byte of a lane's fragment?
python tools/mx_probe.py -> for every tile-k position p of one 128-k tile: A = B = one-hot e4m3 1.0 at p (every row),
A's block scales 2^b for block b = 0..3 (byte b of each row's dword), B's 2^0; D = 2^(applied block).  With the
intended map (lane half h of k-half hf holds tile bytes 64 hf + 32 h .. +31 and uses scale byte 2 hf + h) D = 2^(p//32)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from spatialvla_amd import kernels as K

dev = "cuda"
M = N = 256
Kd = 128
res = []
for p in range(Kd):
    a = torch.zeros(M, Kd, dtype=torch.uint8, device=dev)
    a[:, p] = 0x38  # e4m3 1.0
    sa = K.MXScales(M, Kd, dev)
    sb = K.MXScales(N, Kd, dev)
    sa.buf.view(-1, 4)[:] = torch.tensor([127, 128, 129, 130], dtype=torch.uint8, device=dev)
    sb.buf.fill_(127)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    K.gemm_mxfp8(a.view(torch.float8_e4m3fn), sa, a.view(torch.float8_e4m3fn), sb, out)
    v = out.float()
    vals = sorted(set(round(x, 3) for x in v.flatten().tolist()))
    res.append((p, vals[:4]))
for p, vals in res:
    print(p, p // 32, vals)
# row map: one-hot at k = 0, A's scales 2^(r % 4) for row r (all blocks), B's 2^(c % 2) for column c
a = torch.zeros(M, Kd, dtype=torch.uint8, device=dev)
a[:, 0] = 0x38
sa = K.MXScales(M, Kd, dev)
sb = K.MXScales(N, Kd, dev)
r = torch.arange(M, device=dev)
sa.buf.view(-1, 4)[:M] = (127 + r % 4).to(torch.uint8)[:, None]
sb.buf.view(-1, 4)[:N] = (127 + r[:N] % 2).to(torch.uint8)[:, None]
out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
K.gemm_mxfp8(a.view(torch.float8_e4m3fn), sa, a.view(torch.float8_e4m3fn), sb, out)
exp = torch.exp2((r % 4).float())[:, None] * torch.exp2((r[:N] % 2).float())[None, :]
bad = (out.float() != exp).nonzero()
print("row/col map: mismatches", bad.shape[0], "first", bad[:8].tolist(), "values", out.float()[:6, :4].tolist())
