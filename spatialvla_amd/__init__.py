"""spatialvla_amd — MI355X-native (gfx950) SpatialVLA-4B hot path.

Drop-in for the reference's model surface (model/__init__.py:16-30): `SpatialVLAConfig`,
`SpatialVLAForConditionalGeneration`, `SpatialVLAPreTrainedModel`, `Gemma2ForCausalLM`,
`SpatialVLAProcessor`, `SpatialActionTokenizer`, `ActionTokenizer`.
Compute runs on libsvla.so (hand-written HIP/CDNA4 kernels behind the C-ABI in include/svla.h);
`spatialvla_amd.engine` holds the data-parallel training step (flat buffers, fused AdamW, RCCL).
"""
from .configuration_spatialvla import SpatialVLAConfig

__all__ = ["SpatialVLAConfig", "SpatialVLAForConditionalGeneration", "SpatialVLAPreTrainedModel",
           "Gemma2ForCausalLM", "SpatialVLAProcessor", "SpatialActionTokenizer", "ActionTokenizer"]


def __getattr__(name):
    if name in ("SpatialVLAForConditionalGeneration", "SpatialVLAPreTrainedModel"):
        from . import modeling_spatialvla as m
        return getattr(m, name)
    if name == "SpatialVLAProcessor":
        from .processing_spatialvla import SpatialVLAProcessor
        return SpatialVLAProcessor
    if name in ("SpatialActionTokenizer", "ActionTokenizer"):
        from . import action_tokenizer as at
        return getattr(at, name)
    if name == "Gemma2ForCausalLM":
        from .modeling_gemma2 import Gemma2ForCausalLM
        return Gemma2ForCausalLM
    raise AttributeError(name)
