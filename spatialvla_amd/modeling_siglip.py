"""SigLIP vision tower (So400m/14 @224) on the libsvla HIP kernels.

Replaces the transformers SigLIP module the reference instantiates with
`AutoModel.from_config(config.vision_config)` (model/modeling_spatialvla.py:166, called at :310).
Parameter names follow the transformers 4.47 `SiglipVisionModel` the reference pins
(requirements.txt:20): vision_model.{embeddings.{patch_embedding,position_embedding},
encoder.layers.{i}.{layer_norm1,self_attn.{q,k,v,out}_proj,layer_norm2,mlp.{fc1,fc2}}, post_layernorm}.
"""
import torch
from torch import nn

from . import functional as Fn


class SiglipVisionEmbeddings(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.embed_dim = config.hidden_size
        self.image_size = config.image_size
        self.patch_size = config.patch_size
        self.patch_embedding = nn.Conv2d(config.num_channels, self.embed_dim, kernel_size=self.patch_size,
                                         stride=self.patch_size, padding="valid")
        self.num_patches = (self.image_size // self.patch_size) ** 2
        self.num_positions = self.num_patches
        self.position_embedding = nn.Embedding(self.num_positions, self.embed_dim)

    def forward(self, pixel_values):
        """pixel_values [B,3,S,S] bf16, already SigLIP-normalised -> [B*np, H]."""
        if pixel_values.shape[-1] != self.image_size or pixel_values.shape[-2] != self.image_size:
            raise ValueError("interpolate_pos_encoding is not supported on the HIP path")
        return Fn.PatchEmbedFn.apply(pixel_values, self.patch_embedding.weight, self.patch_embedding.bias,
                                     self.position_embedding.weight, self.patch_size)


class SiglipAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.embed_dim = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.head_dim = self.embed_dim // self.num_heads
        if self.head_dim * self.num_heads != self.embed_dim:
            raise ValueError("embed_dim must be divisible by num_heads")
        self.scale = self.head_dim ** -0.5
        self.dropout = config.attention_dropout
        self.k_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.v_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.q_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.out_proj = nn.Linear(self.embed_dim, self.embed_dim)

    def forward_residual(self, x2d, res2d, B, Lq, slot=None):
        cfg = Fn.SiglipAttnCfg(B, Lq, self.num_heads, self.head_dim, self.scale)
        return Fn.SiglipAttentionFn.apply(x2d, res2d, self.q_proj.weight, self.q_proj.bias, self.k_proj.weight,
                                          self.k_proj.bias, self.v_proj.weight, self.v_proj.bias,
                                          self.out_proj.weight, self.out_proj.bias, cfg, slot)


class SiglipMLP(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        if config.hidden_act not in ("gelu_pytorch_tanh", "gelu_tanh"):
            raise ValueError(f"SiglipMLP: activation {config.hidden_act!r} not supported")
        self.fc1 = nn.Linear(config.hidden_size, config.intermediate_size)
        self.fc2 = nn.Linear(config.intermediate_size, config.hidden_size)

    def forward_residual(self, x2d, res2d, slot=None):
        return Fn.SiglipMLPFn.apply(x2d, res2d, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, slot)


class SiglipEncoderLayer(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.embed_dim = config.hidden_size
        self.layer_norm1 = nn.LayerNorm(self.embed_dim, eps=config.layer_norm_eps)
        self.self_attn = SiglipAttention(config)
        self.layer_norm2 = nn.LayerNorm(self.embed_dim, eps=config.layer_norm_eps)
        self.mlp = SiglipMLP(config)

    def forward(self, h2d, B, Lq):
        s1, s2 = Fn.ResidualSlot(), Fn.ResidualSlot()  # see Fn.ResidualSlot
        x = Fn.LayerNormFn.apply(h2d, self.layer_norm1.weight, self.layer_norm1.bias, self.layer_norm1.eps, s1)
        h2d = self.self_attn.forward_residual(x, h2d, B, Lq, s1)
        x = Fn.LayerNormFn.apply(h2d, self.layer_norm2.weight, self.layer_norm2.bias, self.layer_norm2.eps, s2)
        return self.mlp.forward_residual(x, h2d, s2)


class SiglipEncoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.layers = nn.ModuleList([SiglipEncoderLayer(config) for _ in range(config.num_hidden_layers)])


class SiglipVisionTransformer(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.embeddings = SiglipVisionEmbeddings(config)
        self.encoder = SiglipEncoder(config)
        self.post_layernorm = nn.LayerNorm(config.hidden_size, eps=config.layer_norm_eps)
        if getattr(config, "vision_use_head", False):
            raise ValueError("vision_use_head=True is not part of SpatialVLA (PaliGemma uses the patch tokens)")

    def forward(self, pixel_values):
        B = pixel_values.shape[0]
        h = self.embeddings(pixel_values)
        Lq = self.embeddings.num_patches
        hook = getattr(self, "_svla_layer_grad_hook", None)  # DP: gradients of layers >= i written (engine.py)
        pwait = getattr(self, "_svla_param_wait", None)      # ZeRO-1: parameters of layer i all-gathered
        for i, layer in enumerate(self.encoder.layers):
            if hook is not None and h.requires_grad:
                h.register_hook(lambda g, i=i: hook(i))
            if pwait is not None:
                pwait(("siglip", i))
            h = layer(h, B, Lq)
        h = Fn.LayerNormFn.apply(h, self.post_layernorm.weight, self.post_layernorm.bias, self.post_layernorm.eps, None)
        return h.view(B, Lq, -1)


class SiglipVisionModel(nn.Module):
    """Key prefix `vision_model.` as in transformers 4.47 SiglipVisionModel."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.vision_model = SiglipVisionTransformer(config)

    def forward(self, pixel_values):
        return self.vision_model(pixel_values)
