"""Per-module timing of the frozen ZoeDepth forward at B=32 (CUDA events around every module call),
with the memory format of each module's first input.  Diagnostic for the Zoe HIP path."""
import os, sys, time, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from transformers import ZoeDepthForDepthEstimation, CONFIG_MAPPING
from spatialvla_amd import presets
from spatialvla_amd.modeling_spatialvla import process_zoe

B = int(os.environ.get("ZB", "32"))
cfg = CONFIG_MAPPING["zoedepth"](**{k: v for k, v in presets._zoe_large().items() if k != "model_type"})
with torch.device("cuda"):
    zoe = ZoeDepthForDepthEstimation(cfg).to(torch.bfloat16).eval()
if os.environ.get("ZFAST", "1") == "1":  # the product's fast paths (spatialvla_amd/zoe_fast.py)
    from spatialvla_amd import zoe_fast
    zoe_fast.install(zoe)
pix = torch.rand(B, 3, 224, 224, device="cuda").to(torch.bfloat16)
stats = collections.OrderedDict()
ev = {}


def pre(mod, args):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    ev[id(mod)] = e


def post(mod, args, out):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    torch.cuda.synchronize()
    ms = ev[id(mod)].elapsed_time(e)
    x = args[0] if args and isinstance(args[0], torch.Tensor) else None
    desc = ""
    if x is not None:
        cl = x.is_contiguous(memory_format=torch.channels_last) if x.dim() == 4 else False
        desc = f"{tuple(x.shape)} {'CL' if cl and not x.is_contiguous() else ('C' if x.is_contiguous() else 'strided')}"
    k = mod._svla_name
    t, n, d = stats.get(k, (0.0, 0, desc))
    stats[k] = (t + ms, n + 1, d)


for name, m in zoe.named_modules():
    m._svla_name = f"{name} [{type(m).__name__}]"
    depth = name.count(".")
    if name and (depth <= 3 or "neck" in name or "head" in name):
        m.register_forward_pre_hook(pre)
        m.register_forward_hook(post)


@torch.no_grad()
def run():
    zpv, ph, pw = process_zoe(pix)
    return zoe(pixel_values=zpv).predicted_depth


run()
stats.clear()
run()
for k, (t, n, d) in stats.items():
    if t > 0.3:
        print(f"{t:9.3f} ms  n={n:3d}  {k:90s} {d}")
