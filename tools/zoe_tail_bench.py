"""Time the fused Zoe metric tail (svla_zoe_metric_tail) against the stock transformers tail at B=32, 384x384."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from transformers import ZoeDepthForDepthEstimation, CONFIG_MAPPING
from spatialvla_amd import presets, kernels as Kn

cfg = CONFIG_MAPPING["zoedepth"](**{k: v for k, v in presets._zoe_large().items() if k != "model_type"})
zoe = ZoeDepthForDepthEstimation(cfg).cuda().to(torch.bfloat16).eval()
clb = zoe.metric_head.conditional_log_binomial
B, H, W, h, w = 32, 384, 384, 192, 192
cl = torch.channels_last
feat = torch.rand(B, 32, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
rel = torch.rand(B, H, W, device="cuda").mul(3).to(torch.bfloat16)
emb = torch.randn(B, 128, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
ctr = torch.rand(B, 64, h, w, device="cuda").mul(10).to(torch.bfloat16).contiguous(memory_format=cl)
F = torch.nn.functional


def stock():
    rc = F.interpolate(rel.unsqueeze(1), size=(H, W), mode="bilinear", align_corners=True)
    last = torch.cat([feat, rc], dim=1)
    be = F.interpolate(emb, (H, W), mode="bilinear", align_corners=True)
    x = clb(last, be)
    bc = F.interpolate(ctr, x.shape[-2:], mode="bilinear", align_corners=True)
    return torch.sum(x * bc, dim=1, keepdim=True)


fused = lambda: Kn.zoe_metric_tail(clb, feat, rel, emb, ctr)  # noqa: E731
with torch.no_grad():
    for name, fn in (("fused", fused), ("stock", stock), ("fused", fused)):
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5): out = fn()
        e1.record(); e1.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) / 5:.3f} ms", flush=True)
    r, f = stock(), fused()
    print("rel err", ((r - f).norm() / r.norm()).item())
