"""Which Python lines of the training step still launch ATen (at::native) kernels, and how long do they take?
One bench.py step (SpatialVLA-4B, B=32) under torch.profiler with stacks: for every CPU op whose own device kernels
are at::native ones, the device time summed over the step, grouped by the innermost spatialvla_amd / bench frames.
python tools/aten_sources.py [batch]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

from bench import build_model, make_batch


def main():
    from spatialvla_amd import presets
    from spatialvla_amd.engine import TrainEngine
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = torch.device("cuda:0")
    cfgd = json.loads(json.dumps(presets.spatialvla_4b()))
    model = build_model(cfgd, dev)
    eng = TrainEngine(model, lr=2e-5, weight_decay=0.0, max_grad_norm=1.0, warmup_ratio=0.005, total_steps=10)
    batches = [make_batch(cfgd, B, 1234 + s, dev) for s in range(3)]
    for b in batches[:2]:
        eng.train_step(b)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        eng.train_step(batches[2])
        torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages(group_by_stack_n=6):
        t = getattr(e, "self_device_time_total", None)
        if t is None:
            t = e.self_cuda_time_total
        if t <= 0 or not e.key.startswith("aten::"):
            continue
        frames = [f for f in (e.stack or []) if "spatialvla_amd" in f or "bench.py" in f][:3]
        rows.append((t, e.count, e.key, " <- ".join(frames)))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    print(f"ATen device time in one step: {tot / 1e3:.3f} ms over {sum(r[1] for r in rows)} ops")
    for t, n, name, where in rows[:45]:
        print(f"{t / 1e3:8.3f} ms  n={n:4d}  {name:28s} {where}")


if __name__ == "__main__":
    main()
