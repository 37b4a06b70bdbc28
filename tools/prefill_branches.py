"""Which branch of the B=1 prefill graph is critical: predict_action (prefill + first token) with the Zoe depth
forward, and with predict_depth replaced by a cached depth map (the Gemma2 prefill then waits only for SigLIP).
python tools/prefill_branches.py"""
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402
from spatialvla_amd import presets  # noqa: E402


def timed(model, inputs, n=20):
    with torch.no_grad():
        for _ in range(3):
            model.predict_action(inputs, max_new_tokens=1, eos_token_id=-1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            model.predict_action(inputs, max_new_tokens=1, eos_token_id=-1)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


dev = torch.device("cuda:0")
cfgd = presets.spatialvla_4b()
model = bench.build_model(cfgd, dev)
model.eval()
b = bench.make_batch(cfgd, 1, 4321, dev)
P = int((b["token_type_ids"][0] == 0).sum())
inputs = {"input_ids": b["input_ids"][:, :P], "pixel_values": b["pixel_values"], "intrinsic": b["intrinsic"]}
full = timed(model, inputs)
with torch.no_grad():
    depth = model.predict_depth(b["pixel_values"]).clone()
orig = model.predict_depth
model.predict_depth = lambda pv, _d=depth: _d
if hasattr(model, "clear_decode_cache"):
    model.clear_decode_cache()
nozoe = timed(model, inputs)
model.predict_depth = orig
print(f"prefill + first token: with Zoe {full:.2f} ms, Zoe skipped (cached depth) {nozoe:.2f} ms", flush=True)
