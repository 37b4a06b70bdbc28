"""A/B one Gemma2DecoderLayer fwd+bwd (bench.py's gemma2_block workload) with and without ResidualSlot fusion,
interleaved on one box.  usage: python tools/block_ab.py [reps]
  python tools/block_ab.py flag norm_pair|attn_ds [reps]: the same A/B toggling one switch instead (the norm-pair
  fusion, or the stored-dS attention backward)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import SpatialVLAConfig, presets
from spatialvla_amd import functional as Fn
from spatialvla_amd.modeling_gemma2 import Gemma2DecoderLayer, KVMask

dev = "cuda"
cfg = SpatialVLAConfig(**presets.spatialvla_4b(False)).text_config
with torch.device(dev):
    layer = Gemma2DecoderLayer(cfg, 1).to(torch.bfloat16)
with torch.no_grad():
    for p in layer.parameters():
        if p.dim() >= 2:
            p.normal_(0, 0.02)
# flat parameter / gradient buffers in the engine's layout (TrainEngine: q|k|v adjacent, dW written in place)
from spatialvla_amd.engine import _group_params
ps = _group_params(layer)
offs, n = [], 0
for p in ps:
    offs.append(n); n += (p.numel() + 63) // 64 * 64
flat_p = torch.zeros(n, dtype=torch.bfloat16, device=dev)
flat_g = torch.zeros(n, dtype=torch.bfloat16, device=dev)
with torch.no_grad():
    for p, o in zip(ps, offs):
        v = flat_p[o:o + p.numel()].view_as(p); v.copy_(p.data); p.data = v
        p._svla_grad = flat_g[o:o + p.numel()].view_as(p); p._svla_accum = False
B, L = 32, 312
tt = torch.zeros(B, L, dtype=torch.long, device=dev); tt[:, L - 13:] = 1
mask = KVMask.build(torch.ones(B, L, dtype=torch.long, device=dev), tt, True, B, L, dev)
pos = torch.arange(1, L + 1, device=dev).unsqueeze(0).expand(B, L)
rope = layer.self_attn.rotary_emb.tables(pos, torch.bfloat16)
g = torch.Generator(device=dev).manual_seed(5)
x = torch.randn(B, L, cfg.hidden_size, device=dev, generator=g).to(torch.bfloat16).requires_grad_(True)
gy = torch.randn(B, L, cfg.hidden_size, device=dev, generator=g).to(torch.bfloat16)
Slot = Fn.ResidualSlot
if os.environ.get("SVLA_BLOCK_FP8"):  # BASELINE configs[4]: fp8 projections (forward + dgrad)
    layer.set_fp8_projections(True)


def run(use_slot, iters=10):
    Fn.ResidualSlot = Slot if use_slot else (lambda: None)
    s = torch.cuda.current_stream()
    out = []
    for it in range(iters + 2):
        for p in layer.parameters():
            p.grad = None
        x.grad = None
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(s)
        y = layer(x, mask, rope)
        e1.record(s)
        y.backward(gy)
        e2.record(s)
        e2.synchronize()
        if it >= 2:
            out.append((e0.elapsed_time(e1), e0.elapsed_time(e2)))
    return np.mean(out, 0), x.grad.clone()


if len(sys.argv) > 2 and sys.argv[1] == "flag":
    from spatialvla_amd import modeling_gemma2 as MG
    from spatialvla_amd import kernels as Kn
    sw = {"norm_pair": MG.FUSED_NORM_PAIR, "attn_ds": Kn.ATTN_DS, "wgrad_stream": Fn.WGRAD_STREAM, "wgrad_defer": Fn.WGRAD_DEFER,
          "side_cap": Fn.SIDE_CU_RESERVE}[sys.argv[2]]
    gs, ws = {}, {}
    for r in range(int(sys.argv[3]) if len(sys.argv) > 3 else 5):
        for mode in (0, 1):
            # side_cap: 0 vs SVLA_SIDE_CU_RESERVE_AB CUs reserved for the main stream
            sw[0] = (int(os.environ.get("SVLA_SIDE_CU_RESERVE_AB", "32")) * mode) if sys.argv[2] == "side_cap" \
                else bool(mode)
            (f, t), gx = run(True)
            gs[mode] = gx
            ws[mode] = flat_g.clone()
            print(f"{sys.argv[2]}={mode} fwd {f:.3f} ms  fwd+bwd {t:.3f} ms", flush=True)
    print("x.grad bitwise equal:", torch.equal(gs[0], gs[1]), " weight grads bitwise equal:", torch.equal(ws[0], ws[1]))
    sys.exit(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
if len(sys.argv) > 2:  # profile mode: one configuration only (for rocprofv3 --kernel-trace)
    (f, t), _ = run(sys.argv[2] == "1", iters=int(sys.argv[3]) if len(sys.argv) > 3 else 10)
    print(f"slot={sys.argv[2]} fwd {f:.3f} ms  fwd+bwd {t:.3f} ms", flush=True)
    sys.exit(0)
gs = {}
for r in range(reps):
    for mode in (0, 1):
        (f, t), gx = run(bool(mode))
        gs[mode] = gx
        print(f"slot={mode} fwd {f:.3f} ms  fwd+bwd {t:.3f} ms", flush=True)
print("x.grad bitwise equal:", torch.equal(gs[0], gs[1]))
