"""Container-only loader for the read-only reference at /root/reference.

TEST INFRASTRUCTURE ONLY. Nothing in the product package (`spatialvla_amd/`)
imports this file; it exists so `oracle/gen_golden.py` can run the reference's
own eager arithmetic and write golden vectors under `tests/golden/`.

The reference pins transformers 4.47 / torch 2.5 (reference requirements.txt:20);
this image has transformers 5.15 / torch 2.10 and no torchvision.  Importing
`model.modeling_gemma2` therefore raises an ordinary ImportError.  The shim below
patches only *names* (no reference file is modified, no reference source is
copied), exactly as SURVEY.md §8(c) lists:

1. `transformers.cache_utils.HybridCache`   -> an empty Cache subclass (name only;
   we always call with use_cache=False, so it is never constructed).
2. `transformers.modeling_utils.PretrainedConfig` -> `transformers.PretrainedConfig`.
3. `torchvision.transforms.functional.normalize` -> per-channel (t-mean)/std in the
   tensor's dtype, identical to torchvision for constant 3-channel mean/std.
4. After import: `Gemma2ForCausalLM._tied_weights_keys = None` (v5 expects a dict).
5. Per config: rope_theta, pad_token_id=0, eager attention on every sub-config
   (`configure_eager`).
"""
import os
import sys
import types

REFERENCE_ROOT = "/root/reference"


def reference_available() -> bool:
    return os.path.isdir(os.path.join(REFERENCE_ROOT, "model"))


def install():
    import torch
    import transformers
    import transformers.cache_utils as cu
    import transformers.modeling_utils as mu

    if not hasattr(cu, "HybridCache"):
        class HybridCache(cu.Cache):  # name-only stand-in, never instantiated
            pass
        cu.HybridCache = HybridCache
    mu.PretrainedConfig = transformers.PretrainedConfig

    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tvt = types.ModuleType("torchvision.transforms")
        tvf = types.ModuleType("torchvision.transforms.functional")

        def normalize(t, mean, std):
            m = torch.tensor(mean, dtype=t.dtype, device=t.device).view(-1, 1, 1)
            s = torch.tensor(std, dtype=t.dtype, device=t.device).view(-1, 1, 1)
            return (t - m) / s

        tvf.normalize = normalize
        tv.transforms = tvt
        tvt.functional = tvf
        sys.modules.update({"torchvision": tv, "torchvision.transforms": tvt,
                            "torchvision.transforms.functional": tvf})
    if REFERENCE_ROOT not in sys.path:
        sys.path.insert(0, REFERENCE_ROOT)

    from model.modeling_gemma2 import Gemma2ForCausalLM  # noqa: E402
    Gemma2ForCausalLM._tied_weights_keys = None
    import model.modeling_spatialvla as msv  # noqa: E402
    import model.configuration_spatialvla as csv  # noqa: E402
    return msv, csv


def configure_eager(cfg):
    """Apply shim item 5 to a reference SpatialVLAConfig."""
    cfg.text_config.rope_theta = 10000.0
    cfg.pad_token_id = 0
    for sub in (cfg.text_config, cfg.vision_config):
        sub._attn_implementation = "eager"
    if getattr(cfg, "vision_zoe_config", None) is not None:
        try:
            cfg.vision_zoe_config._attn_implementation = "eager"
            cfg.vision_zoe_config.backbone_config._attn_implementation = "eager"
        except Exception:
            pass
    return cfg
