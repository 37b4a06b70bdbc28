"""Which blend order of svla_upsample_bilinear_nhwc matches torch's NHWC bilinear kernel bitwise (one build per
UPS_MODE under build/var)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from spatialvla_amd import kernels as K, _lib as L

torch.manual_seed(13)
cases = [((2, 256, 24, 24), dict(scale_factor=2, align_corners=True)), ((2, 128, 96, 96), dict(scale_factor=2, align_corners=True)),
         ((2, 32, 12, 20), dict(size=(24, 31), align_corners=False))]
for m in [int(v) for v in os.environ.get("UPS_MODES", "0").split(",")]:
    L._lib = L.load(os.path.abspath(f"build/var/libsvla_ups{m}.so"))
    res = []
    for shp, kw in cases:
        x = torch.randn(*shp, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        ref = F.interpolate(x, mode="bilinear", **kw)
        out = K.upsample_bilinear_cl(x, **kw)
        res.append(f"{(out != ref).sum().item()}/{ref.numel()} maxdiff {(out.float() - ref.float()).abs().max().item():.3g}")
    print(m, " | ".join(res), flush=True)
