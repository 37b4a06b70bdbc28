"""Diagnostic (not a bench line): wall cost of the frozen ZoeDepth forward inside the training step.  Times the bench
step as is, then with predict_depth replaced by a cached depth map (the Zoe forward skipped), same box and batches.
python tools/zoe_cost.py [steps]"""
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402
from spatialvla_amd import presets  # noqa: E402
from spatialvla_amd.engine import TrainEngine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
cfgd = presets.spatialvla_4b()
model = bench.build_model(cfgd, dev)
eng = TrainEngine(model, lr=2e-5, total_steps=100, defer_host_checks=True)
batches = [bench.make_batch(cfgd, 32, 1234 + s, dev) for s in range(steps + 2)]


def run(tag):
    for s in range(2):
        eng.train_step(batches[s])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        eng.train_step(batches[2 + s])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(f"{tag}: {ms:.2f} ms/step", flush=True)
    return ms


a = run("with Zoe")
with torch.no_grad():
    depth = model.predict_depth(batches[0]["pixel_values"]).clone()
model.predict_depth = lambda pv, _d=depth: _d
b = run("Zoe skipped (cached depth)")
del model.predict_depth
c = run("with Zoe again")
print(f"Zoe wall cost ~ {(a + c) / 2 - b:.2f} ms/step")
