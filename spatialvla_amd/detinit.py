"""Portable deterministic initialisation of a state dict by parameter name.

Each tensor is drawn from its own numpy PCG64 stream seeded by (seed, crc32(name)), so any
subset of a model (one decoder layer, the lm_head) can be regenerated bit-identically on any
host without materialising the rest.  Used for golden fixtures and for
the random-init weights of the benchmark.

Scale rules (keep activations O(1) through a random model):
* Gemma2 RMSNorm weights (zero-centred, `(1 + w)`, modeling_gemma2.py:64,73): N(0, 0.1)
* other 1-D `weight` (LayerNorm / BatchNorm): 1 + N(0, 0.1)
* 1-D biases and other vectors: N(0, 0.02)
* >=2-D tensors: N(0, 1/sqrt(fan_in)), fan_in = prod(shape[1:])
"""
import zlib

import numpy as np
import torch

_GEMMA_RMS = ("input_layernorm", "post_attention_layernorm", "pre_feedforward_layernorm",
              "post_feedforward_layernorm")


def _is_gemma_rms(name: str) -> bool:
    if any(k in name for k in _GEMMA_RMS):
        return True
    return name.endswith("language_model.model.norm.weight") or name == "model.norm.weight" or name == "norm.weight"


def canonical_name(name: str) -> str:
    """transformers-4.47 SigLIP keys carry a `vision_model.` infix that v5 drops; hash the v5 form so
    both spellings of a parameter draw the same values."""
    return name.replace("vision_tower.vision_model.", "vision_tower.")


def det_tensor(name: str, shape, seed: int = 0, scale: float = None) -> torch.Tensor:
    name = canonical_name(name)
    rng = np.random.default_rng([seed & 0xFFFFFFFF, zlib.crc32(name.encode())])
    x = rng.standard_normal(size=tuple(shape), dtype=np.float32)
    shape = tuple(shape)
    if scale is not None:
        x *= scale
    elif len(shape) >= 2:
        x *= 1.0 / np.sqrt(float(np.prod(shape[1:])))
    elif name.endswith("weight") and _is_gemma_rms(name):
        x *= 0.1
    elif name.endswith("weight"):
        x = 1.0 + 0.1 * x
    else:
        x *= 0.02
    return torch.from_numpy(x)


@torch.no_grad()
def deterministic_init_(module: torch.nn.Module, seed: int = 0, prefix: str = "", skip=()) -> None:
    """Overwrite every floating parameter of `module` in place (buffers untouched)."""
    for name, p in module.named_parameters():
        full = prefix + name
        if any(s in full for s in skip) or not p.is_floating_point():
            continue
        p.copy_(det_tensor(full, p.shape, seed).to(p.dtype))
