"""The frozen ZoeDepth forward of the training step alone (predict_depth at B=32 on the product path), for traces:
python tools/zoe_step.py [iters]  -- prints the mean wall time per forward."""
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402
from spatialvla_amd import presets  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda:0")
cfgd = presets.spatialvla_4b()
model = bench.build_model(cfgd, dev)
pv = bench.make_batch(cfgd, 32, 1234, dev)["pixel_values"]
with torch.no_grad():
    for _ in range(2):
        model.predict_depth(pv)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        model.predict_depth(pv)
    torch.cuda.synchronize()
print(f"predict_depth B=32: {(time.perf_counter() - t0) / n * 1e3:.2f} ms", flush=True)
