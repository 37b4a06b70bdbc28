"""A/B the lm_head softcap + statistics pass of several libsvla builds at the 4B shape (9984 x 265408, in place),
interleaved, best of 5 per build; outputs on a special-value sample compared bitwise with the first build:
python tools/softcap_ab.py lib1.so lib2.so ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spatialvla_amd import _lib as L
from spatialvla_amd import kernels as K

R, V = 9984, 265408
dev = "cuda"
torch.manual_seed(0)
logits = torch.empty(R, V, dtype=torch.bfloat16, device=dev)
logits.view(-1)[:].copy_((torch.randn(R * V // 64, device=dev) * 8).repeat_interleave(64).to(torch.bfloat16))
stats = torch.empty(R, (V + 127) // 128, 3, device=dev)
small = (torch.randn(64, V, device=dev) * 8).to(torch.bfloat16)
small[0, 5], small[7, V - 3] = float("nan"), float("nan")
small[1, 128:256] = -small[1, 128:256].abs()
small[1, 130], small[1, 200] = 0.0, -0.0
small[3, :128] = 2.5
small[4, 700], small[5, 3] = float("inf"), float("-inf")
libs = [(os.path.basename(p), L.load(os.path.abspath(p))) for p in sys.argv[1:]]
best, outs = {}, {}
for rnd in range(5):
    for tag, lib in libs:
        L._lib = lib
        if rnd == 0:
            t = small.clone()
            st = torch.empty(64, (V + 127) // 128, 3, device=dev)
            K.softcap_ce_rows(t, V, st, 30.0)
            outs[tag] = (t.view(torch.uint8), st.view(torch.uint8))
        K.softcap_ce_rows(logits, V, stats, 30.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            K.softcap_ce_rows(logits, V, stats, 30.0)
        e1.record()
        e1.synchronize()
        best[tag] = min(best.get(tag, 1e9), e0.elapsed_time(e1) / 3)
t0 = libs[0][0]
for tag, _ in libs:
    same = all(torch.equal(a, b) for a, b in zip(outs[tag], outs[t0]))
    print(f"{tag:28s} {best[tag] * 1e3:8.1f} us  {4 * R * V / best[tag] / 1e9:5.2f} TB/s  bitwise_equal_to_{t0}={same}",
          flush=True)
