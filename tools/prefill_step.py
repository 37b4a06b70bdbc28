"""The B=1 prefill + first token of predict_action (configs[1]) replayed N times, for kernel traces:
python tools/prefill_step.py [N]"""
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402
from spatialvla_amd import presets  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
cfgd = presets.spatialvla_4b()
model = bench.build_model(cfgd, dev)
model.eval()
b = bench.make_batch(cfgd, 1, 4321, dev)
P = int((b["token_type_ids"][0] == 0).sum())
inputs = {"input_ids": b["input_ids"][:, :P], "pixel_values": b["pixel_values"], "intrinsic": b["intrinsic"]}
with torch.no_grad():
    for _ in range(3):
        model.predict_action(inputs, max_new_tokens=1, eos_token_id=-1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        model.predict_action(inputs, max_new_tokens=1, eos_token_id=-1)
    torch.cuda.synchronize()
print(f"prefill + first token: {(time.perf_counter() - t0) / n * 1e3:.2f} ms", flush=True)
