"""Diagnostic: TrainEngine losses / masters with and without gradient checkpointing (tiny model), under the current
SVLA_WGRAD_STREAM / SVLA_WGRAD_DEFER settings.  python tools/ckpt_diag.py"""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests")]
import harness as H  # noqa: E402
from spatialvla_amd import presets  # noqa: E402
from spatialvla_amd.engine import TrainEngine  # noqa: E402

cfgd = H.cfg_dict("tiny")
cuda = torch.device("cuda:0")
b = H.batch_tensors(presets.synthetic_batch(cfgd, batch=2, seed=6), cuda)
depth = torch.rand(2, 1, 224, 224, generator=torch.Generator().manual_seed(4)).mul(3).add(0.5).to(cuda)
res = {}
for ck in (False, True):
    model = H.build_hip_model(cfgd, "cuda:0")
    model.train()
    model.vision_zoe_model.eval()
    if ck:
        model.language_model._set_gradient_checkpointing()
    model.predict_depth = lambda pv, _d=depth: _d
    eng = TrainEngine(model, lr=1e-3, warmup_ratio=0.0, total_steps=10, max_grad_norm=1.0, bucket_bytes=1 << 16)
    out = []
    for s in range(1):
        loss = eng.train_step(b)
        torch.cuda.synchronize()
        out.append((float(loss), eng.flat_grad.float().norm().item(), float(eng.gnorm)))
    names = {id(p): n for n, p in model.named_parameters()}
    res[ck] = (out, eng.flat_grad.clone(), [(names[id(p)], o, p.numel()) for p, o in zip(eng.params, eng.offsets)])
    print(ck, out, flush=True)
g0, g1 = res[False][1], res[True][1]
d = (g0.float() - g1.float()).abs()
print("grad diff max", d.max().item(), "n diff", int((d > 0).sum()))
bad = []
for n, o, k in res[False][2]:
    a, c = g0[o:o + k].float(), g1[o:o + k].float()
    if not torch.equal(a, c):
        bad.append((n, a.norm().item(), c.norm().item()))
print(len(bad), "params differ")
for x in bad[:40]:
    print(x)
