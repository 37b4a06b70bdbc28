"""The lm_head softcap + statistics pass alone at the 4B training shape (9984 x 265408 bf16 logits, in place), for
rocprofv3 counter passes: python tools/softcap_prof.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spatialvla_amd import kernels as K

R, V = 9984, 265408
dev = "cuda"
torch.manual_seed(0)
logits = torch.empty(R, V, dtype=torch.bfloat16, device=dev)
logits.view(-1)[:].copy_((torch.randn(R * V // 64, device=dev) * 8).repeat_interleave(64).to(torch.bfloat16))
stats = torch.empty(R, (V + 127) // 128, 3, device=dev)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
K.softcap_ce_rows(logits, V, stats, 30.0)
e0.record()
for _ in range(reps):
    K.softcap_ce_rows(logits, V, stats, 30.0)
e1.record()
e1.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"softcap_rows {ms * 1e3:.1f} us  {2 * R * V * 2 / ms / 1e9:.2f} TB/s (read + write of the logits)")
