"""Portable deterministic initialisation of a state dict by parameter name.

Two generators share the scale rules below:
* det_tensor / deterministic_init_: numpy PCG64 normals (small fixtures; ~20 ns per element on one core).
* hash_tensor / hash_init_: a counter-based splitmix64 hash -> uniform values of the same standard deviation,
  written with int64 torch ops only, so CPU and GPU produce bit-identical tensors and a 4B-parameter model is
  initialised on the GPU in well under a second (the 4B golden fixture, tests/golden/full4b.safetensors).

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


# ---------------------------------------------------------------------------------------- counter-based hash init
def _i64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


_SM1, _SM2, _SM3 = _i64(0x9E3779B97F4A7C15), _i64(0xBF58476D1CE4E5B9), _i64(0x94D049BB133111EB)


def _srl(z: torch.Tensor, s: int) -> torch.Tensor:
    """logical shift right of an int64 tensor (torch's >> is arithmetic)"""
    return (z >> s) & ((1 << (64 - s)) - 1)


def _std_of(name: str, shape):
    """(std, offset) of the det_tensor scale rules."""
    if len(shape) >= 2:
        return 1.0 / np.sqrt(float(np.prod(shape[1:]))), 0.0
    if name.endswith("weight") and _is_gemma_rms(name):
        return 0.1, 0.0
    if name.endswith("weight"):
        return 0.1, 1.0
    return 0.02, 0.0


def hash_tensor(name: str, shape, seed: int = 0, device="cpu", dtype=torch.bfloat16, chunk: int = 1 << 26):
    """Element i of tensor `name`: z = splitmix64(key + (i+1) * golden), u = top 24 bits of z,
    x = offset + (u * 2^-23 - 1) * (std * sqrt(3))  (uniform, variance std^2; every fp32 step is exact except the
    final scale multiply and offset add, which round identically on any IEEE device), then cast to `dtype` (RNE)."""
    name = canonical_name(name)
    shape = tuple(shape)
    std, off = _std_of(name, shape)
    scale = float(np.float32(std * np.sqrt(3.0)))
    key = _i64(((seed & 0xFFFFFFFF) << 32) | zlib.crc32(name.encode()))
    n = int(np.prod(shape)) if shape else 1
    out = torch.empty(n, dtype=dtype, device=device)
    for s0 in range(0, n, chunk):
        m = min(chunk, n - s0)
        z = torch.arange(s0 + 1, s0 + m + 1, dtype=torch.int64, device=device)
        z.mul_(_SM1).add_(key)
        z = (z ^ _srl(z, 30)).mul_(_SM2)
        z = (z ^ _srl(z, 27)).mul_(_SM3)
        z = z ^ _srl(z, 31)
        u = _srl(z, 40).to(torch.float32)
        x = u.mul_(2.0 ** -23).sub_(1.0).mul_(scale)
        if off:
            x.add_(off)
        out[s0:s0 + m] = x.to(dtype)
    return out.view(shape)


@torch.no_grad()
def hash_init_(module: torch.nn.Module, seed: int = 0, prefix: str = "", skip=()) -> None:
    """hash_tensor for every floating parameter of `module`, generated on the parameter's own device."""
    for name, p in module.named_parameters():
        full = prefix + name
        if any(s in full for s in skip) or not p.is_floating_point():
            continue
        p.copy_(hash_tensor(full, p.shape, seed, device=p.device, dtype=p.dtype))
