import sys, torch, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transformers import ZoeDepthForDepthEstimation, CONFIG_MAPPING
from spatialvla_amd import zoe_fast, presets
cfg = CONFIG_MAPPING['zoedepth'](**{k: v for k, v in presets._zoe_large().items() if k != 'model_type'})
z = ZoeDepthForDepthEstimation(cfg).cuda().to(torch.bfloat16).eval()
zoe_fast.install(z)
orig = zoe_fast._beit_layer_forward
layer = [m for m in z.modules() if type(m).__name__ == 'BeitLayer'][0]
def spy(self, hidden_states, attention_mask=None, interpolate_pos_encoding=False, resolution=None, **kw):
    print("cuda", hidden_states.is_cuda, hidden_states.dtype, "mask", attention_mask is None, "training", self.training,
          "grad", torch.is_grad_enabled(), "hd", self.attention.head_dim, "stock", getattr(self, "_svla_stock", False), flush=True)
    return orig(self, hidden_states, attention_mask=attention_mask, interpolate_pos_encoding=interpolate_pos_encoding,
                resolution=resolution, **kw)
import types
layer.forward = types.MethodType(spy, layer)
with torch.no_grad():
    z(pixel_values=torch.randn(1, 3, 384, 384, device="cuda").to(torch.bfloat16))
