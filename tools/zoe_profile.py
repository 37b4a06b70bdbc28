"""Profile the frozen ZoeDepth forward (BEiT-L/16 @384 + DPT neck + metric bins) at B=32 on one GPU:
torch.profiler op table with input shapes, and the wall time of predict_depth."""
import os, sys, time
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
    zoe_fast.install(zoe, convs=os.environ.get("ZCONV", "1") == "1")
pix = torch.rand(B, 3, 224, 224, device="cuda").to(torch.bfloat16)


@torch.no_grad()
def run():
    zpv, ph, pw = process_zoe(pix)
    d = zoe(pixel_values=zpv).predicted_depth
    return d


for _ in range(2):
    run()
torch.cuda.synchronize()
t0 = time.time()
for _ in range(3):
    run()
torch.cuda.synchronize()
print(f"zoe forward B={B} convs={os.environ.get('ZCONV', '1')}: {(time.time() - t0) / 3 * 1e3:.1f} ms", flush=True)
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU], record_shapes=True) as prof:
    run()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=40,
                                                         max_shapes_column_width=90))
