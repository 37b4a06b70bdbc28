"""Bias-gradient column sums (svla_colsum_bf16) at the SigLIP shapes: one launch (workspace NULL) vs the row-split
path (workspace), interleaved rounds, best of 5; outputs compared to the fp32 sum.  python tools/colsum_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spatialvla_amd import _lib as L

dev = "cuda"
torch.manual_seed(0)
lib = L.lib()
S = torch.cuda.current_stream().cuda_stream
best = {}
for M, N, ld in [(8192, 4304, 4304), (8192, 1152, 1152), (8192, 3456, 3456), (8192, 1152, 4304)]:
    x = torch.randn(M, ld, device=dev).to(torch.bfloat16)
    out = torch.empty(N, dtype=torch.bfloat16, device=dev)
    nb = int(lib.svla_colsum_bf16_workspace_bytes(M, N))
    ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device=dev)
    ref = x[:, :N].float().sum(0)
    for rnd in range(5):
        for arm, wp in (("single", None), ("split", ws.data_ptr() if nb else None)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                L.check(lib.svla_colsum_bf16(M, N, x.data_ptr(), ld, out.data_ptr(), 0, wp, S), "colsum")
            e1.record()
            e1.synchronize()
            k = (M, N, ld, arm)
            best[k] = min(best.get(k, 1e9), e0.elapsed_time(e1) / 20 * 1e3)
            err = ((out.float() - ref).norm() / ref.norm()).item()
            assert err < 5e-3, (k, err)
    print(f"M={M} N={N} ld={ld}: single {best[(M, N, ld, 'single')]:6.1f} us  split {best[(M, N, ld, 'split')]:6.1f} us"
          f"  (workspace {nb} B)", flush=True)
