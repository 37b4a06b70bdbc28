"""Gemma2 decoder (text side of SpatialVLA) on the libsvla HIP kernels.

Module tree, attribute names and therefore state-dict keys are those of the reference
(model/modeling_gemma2.py: Gemma2RMSNorm :60, Gemma2MLP :80, Gemma2RotaryEmbedding :95,
Gemma2Attention :325, Gemma2DecoderLayer :436, Gemma2Model :647, Gemma2ForCausalLM :887), so
reference checkpoints load unchanged.  Compute goes through `spatialvla_amd.functional` only.

The reference's attention plug-in point GEMMA2_ATTENTION_FUNCTION (:317-322) is kept: every key
("eager", "sdpa", "flash_attention_2", "flex_attention") maps to the one HIP implementation with the
reference *eager* semantics (prefix-LM mask).  Inside the model the fused
path (QKV GEMM -> attention with RoPE on load -> O GEMM) is used; the plug-in is for callers that
hand in already-rotated q/k/v as the reference does.
"""
import math
import os
import warnings
from dataclasses import dataclass
from typing import Optional

import torch
import torch.utils.checkpoint
from torch import nn

from . import functional as Fn
from . import kernels as Kn


@dataclass
class KVMask:
    """The reference's additive [B,1,L,L] mask (modeling_spatialvla.py:258-306), as per-key classes:
    0 = visible to every query, 1 = visible to queries at or after the key, 2 = never visible."""
    kv_class: torch.Tensor  # uint8 [B, L]

    @staticmethod
    def build(attention_mask: Optional[torch.Tensor], token_type_ids: Optional[torch.Tensor], is_training: bool,
              B: int, L: int, device) -> "KVMask":
        if is_training:
            if attention_mask is None:
                cls = torch.ones(B, L, dtype=torch.uint8, device=device)  # plain causal
            else:
                valid = attention_mask != 0
                cls = torch.where(valid, 1, 2).to(torch.uint8)
                # :304-305 — columns with token_type 0 are unmasked for every row (incl. padded ones, Q2)
                cls = torch.where(token_type_ids == 0, 0, cls).to(torch.uint8)
        else:
            # :294 — inference prefill: bidirectional inside the sequence, padded keys masked
            if attention_mask is None:
                cls = torch.zeros(B, L, dtype=torch.uint8, device=device)
            else:
                cls = torch.where(attention_mask != 0, 0, 2).to(torch.uint8)
        return KVMask(cls.contiguous())


class Gemma2KVCache:
    """Key/value cache of greedy decoding: the reference's HybridCache (transformers cache_utils, built at
    modeling_gemma2.py:712-720, updated at :387-395) for sequences shorter than the sliding window (4096) —
    there every layer, sliding or global, keeps all keys, and the window is applied as a mask by the kernel.

    Layout in HBM: key_cache / value_cache [layers, B, capacity, Hkv*D] bf16 (one row per token, heads
    back to back, rotated keys); kv_class [B, capacity] uint8 per-key classes (KVMask: prompt keys 0 or 2,
    generated keys 1)."""

    def __init__(self, config, batch_size: int, capacity: int, device, dtype=torch.bfloat16):
        kd = config.num_key_value_heads * config.head_dim
        self.config = config
        self.key_cache = torch.empty(config.num_hidden_layers, batch_size, capacity, kd, dtype=dtype, device=device)
        self.value_cache = torch.empty_like(self.key_cache)
        self.kv_class = torch.full((batch_size, capacity), 2, dtype=torch.uint8, device=device)
        self.seen_tokens = 0

    @property
    def capacity(self) -> int:
        return self.key_cache.shape[2]

    def get_seq_length(self, layer_idx: int = 0) -> int:
        return self.seen_tokens

    def append_classes(self, cls: torch.Tensor):
        """Classes of the next cls.shape[1] tokens (called once per forward, before the layers)."""
        n = cls.shape[1]
        if self.seen_tokens + n > self.capacity:
            raise ValueError(f"KV cache full: {self.seen_tokens} + {n} tokens > capacity {self.capacity}")
        self.kv_class[:, self.seen_tokens:self.seen_tokens + n] = cls


class Gemma2RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.zeros(dim))

    def forward(self, x, slot=None, mx=None):
        shp = x.shape
        return Fn.RMSNormFn.apply(x.reshape(-1, shp[-1]), self.weight, self.eps, slot, mx).view(shp)

    def add_forward(self, residual, y, slot=None, mx_grad=None):
        """residual + self(y) (decoder-layer residual branches); mx_grad: an MXSlot for the MX copy of y's gradient."""
        shp = y.shape
        return Fn.AddRMSNormFn.apply(residual.reshape(-1, shp[-1]), y.reshape(-1, shp[-1]), self.weight,
                                     self.eps, slot, mx_grad).view(shp)

    def extra_repr(self):
        return f"{tuple(self.weight.shape)}, eps={self.eps}"


class Gemma2MLP(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.hidden_size = config.hidden_size
        self.intermediate_size = config.intermediate_size
        self.gate_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.up_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.down_proj = nn.Linear(self.intermediate_size, self.hidden_size, bias=False)
        act = getattr(config, "hidden_activation", None) or getattr(config, "hidden_act", "gelu_pytorch_tanh")
        if act not in ("gelu_pytorch_tanh", "gelu_tanh"):
            raise ValueError(f"Gemma2MLP: activation {act!r} not supported (kernel implements gelu_pytorch_tanh)")

    def forward(self, x, mx_in=None, mx_dout=None):
        shp = x.shape
        out = Fn.GemmaMLPFn.apply(x.reshape(-1, shp[-1]), self.gate_proj.weight, self.up_proj.weight,
                                  self.down_proj.weight, getattr(self, "_svla_fp8", None), mx_in, mx_dout)
        return out.view(*shp[:-1], self.hidden_size)


class Gemma2RotaryEmbedding(nn.Module):
    def __init__(self, dim, max_position_embeddings=2048, base=10000, device=None):
        super().__init__()
        self.dim = dim
        self.max_position_embeddings = max_position_embeddings
        self.base = base
        inv_freq = 1.0 / (self.base ** (torch.arange(0, self.dim, 2, dtype=torch.int64).float() / self.dim))
        self.register_buffer("inv_freq", tensor=inv_freq, persistent=False)

    @torch.no_grad()
    def tables(self, position_ids: torch.Tensor, dtype) -> tuple:
        """cos/sin in the activation dtype (reference :106-120 rounds them): [L, dim/2] when the batch
        shares its positions (a [L] / [1, L] tensor or a stride-0 expand of one), else [B*L, dim/2], one row per
        token (b, t) at row b*L + t -- the per-sequence positions the reference's generate derives for padded
        prompts (modeling_gemma2.py:1039-1042).  The kernels read table row m % rows for token row m.  No host sync
        (usable inside a graph capture)."""
        if position_ids.dim() == 2:
            if position_ids.shape[0] == 1 or position_ids.stride(0) == 0:
                position_ids = position_ids[0]
            else:
                position_ids = position_ids.reshape(-1)
        freqs = position_ids.float()[:, None] * self.inv_freq.float().to(position_ids.device)[None, :]
        return freqs.cos().to(dtype).contiguous(), freqs.sin().to(dtype).contiguous()


def _plugin(module, query, key, value, mask, **kw):
    """GEMMA2_ATTENTION_FUNCTION entry: reference signature (modeling_gemma2.py:169-195, 403-405)."""
    kv_class = mask.kv_class if isinstance(mask, KVMask) else None
    if mask is not None and not isinstance(mask, KVMask):
        raise ValueError("HIP attention takes a KVMask (per-key classes), not a dense additive mask")
    out = Fn.hip_attention(query, key, value, module.scaling, module.attn_logit_softcapping or 0.0, kv_class,
                           module.sliding_window or 0)
    return out, None


GEMMA2_ATTENTION_FUNCTION = {"flash_attention_2": _plugin, "flex_attention": _plugin, "eager": _plugin,
                             "sdpa": _plugin}


class Gemma2Attention(nn.Module):
    def __init__(self, config, layer_idx: Optional[int] = None):
        super().__init__()
        self.config = config
        self.layer_idx = layer_idx
        self.attention_dropout = config.attention_dropout
        self.hidden_size = config.hidden_size
        self.num_heads = config.num_attention_heads
        self.head_dim = config.head_dim
        self.num_key_value_heads = config.num_key_value_heads
        self.num_key_value_groups = self.num_heads // self.num_key_value_heads
        self.max_position_embeddings = config.max_position_embeddings
        self.rope_theta = _rope_theta(config)
        self.is_causal = True
        self.scaling = config.query_pre_attn_scalar ** -0.5
        self.sliding_window = config.sliding_window if not bool(layer_idx % 2) else None
        self.attn_logit_softcapping = config.attn_logit_softcapping
        bias = getattr(config, "attention_bias", False)
        if bias:
            raise ValueError("attention_bias=True is not part of the Gemma2 hot path")
        self.q_proj = nn.Linear(self.hidden_size, self.num_heads * self.head_dim, bias=False)
        self.k_proj = nn.Linear(self.hidden_size, self.num_key_value_heads * self.head_dim, bias=False)
        self.v_proj = nn.Linear(self.hidden_size, self.num_key_value_heads * self.head_dim, bias=False)
        self.o_proj = nn.Linear(self.num_heads * self.head_dim, self.hidden_size, bias=False)
        self.rotary_emb = Gemma2RotaryEmbedding(self.head_dim, self.max_position_embeddings, self.rope_theta)

    def attn_cfg(self, B: int, Lq: int) -> "Fn.GemmaAttnCfg":
        return Fn.GemmaAttnCfg(B, Lq, self.num_heads, self.num_key_value_heads, self.head_dim, self.scaling,
                               float(self.attn_logit_softcapping or 0.0), int(self.sliding_window or 0))

    def forward(self, hidden_states, attention_mask: KVMask, rope: tuple, cache: Optional[Gemma2KVCache] = None,
                attn_sink: Optional[list] = None, mx_in=None, mx_dout=None):
        B, Lq, H = hidden_states.shape
        cfg = self.attn_cfg(B, Lq)
        cos, sin = rope
        if cache is not None:
            i = self.layer_idx
            out = Fn.gemma_attention_cached(hidden_states.reshape(B * Lq, H), self.q_proj.weight, self.k_proj.weight,
                                            self.v_proj.weight, self.o_proj.weight, cos, sin, cache.key_cache[i],
                                            cache.value_cache[i], cache.kv_class, cache.seen_tokens, cfg)
            return out.view(B, Lq, H)
        if cos.shape[0] != Lq and torch.is_grad_enabled() and (
                hidden_states.requires_grad or any(w.requires_grad for w in (self.q_proj.weight, self.k_proj.weight,
                                                                             self.v_proj.weight, self.o_proj.weight))):
            # autograd.Function.forward runs with grad mode off, so this is checked here, where the caller's grad
            # mode is visible: the attention backward applies the RoPE transpose with table row = position in the
            # sequence, which per-sequence tables ([B*L] rows, padded prompts) would not match
            raise NotImplementedError("per-sequence position_ids are an inference path (the reference's training "
                                      "positions are shared: modeling_spatialvla.py:367-372); run under no_grad")
        capture = {} if attn_sink is not None else None
        out = Fn.GemmaAttentionFn.apply(hidden_states.reshape(B * Lq, H), self.q_proj.weight, self.k_proj.weight,
                                        self.v_proj.weight, self.o_proj.weight, cos, sin, attention_mask.kv_class,
                                        cfg, getattr(self, "_svla_fp8", None), capture, mx_in, mx_dout)
        if attn_sink is not None:
            attn_sink.append(Fn.gemma_attention_weights(capture["qkv"], attention_mask.kv_class, cfg))
        return out.view(B, Lq, H)


def _rope_theta(config):
    th = getattr(config, "rope_theta", None)
    if th is None:
        rp = getattr(config, "rope_parameters", None) or {}
        th = rp.get("rope_theta", 10000.0)
    return float(th)


# training forward: the post-attention + pre-feedforward norm pair as one launch (Fn.AddRMSNorm2Fn); False = the two
# separate Functions (A/B and bitwise tests)
FUSED_NORM_PAIR = [os.environ.get("SVLA_FUSED_NORM_PAIR", "1") != "0"]


class Gemma2DecoderLayer(nn.Module):
    def __init__(self, config, layer_idx: int):
        super().__init__()
        self.hidden_size = config.hidden_size
        self.config = config
        self.is_sliding = not bool(layer_idx % 2)
        self.self_attn = Gemma2Attention(config=config, layer_idx=layer_idx)
        self.mlp = Gemma2MLP(config)
        self.input_layernorm = Gemma2RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.post_attention_layernorm = Gemma2RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.pre_feedforward_layernorm = Gemma2RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.post_feedforward_layernorm = Gemma2RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        self.sliding_window = config.sliding_window

    def set_fp8_projections(self, enabled: bool):
        """BASELINE configs[4]: run the forward q|k|v, o, gate|up and down projections of this layer on the fp8
        MFMA GEMM (row-wise e4m3 activations and weights, fp32 accumulation); the backward stays bf16.  Training
        and the uncached forward only -- the KV-cached decode keeps the bf16 GEMV path."""
        f8 = Fn.FP8Weights() if enabled else None
        self.self_attn._svla_fp8 = f8
        self.mlp._svla_fp8 = f8

    def forward(self, hidden_states, attention_mask: KVMask, rope: tuple, cache: Optional[Gemma2KVCache] = None,
                attn_sink: Optional[list] = None):
        # reference :475-496 (sandwich norms + residuals)
        # each residual-stream tensor has two consumers (pre-norm, residual add): a ResidualSlot sums their
        # gradients inside the pre-norm's backward kernel instead of an autograd add
        s1, s2 = Fn.ResidualSlot(), Fn.ResidualSlot()
        # fp8 projections (configs[4]): the norms also emit the MX e4m3 copies of q|k|v's and gate|up's inputs
        f8 = getattr(self.self_attn, "_svla_fp8", None) if cache is None else None
        # (and the backward norms those of the o and down dgrad inputs)
        mx_a, mx_m = Fn.mx_slot_for(f8, "qkv"), Fn.mx_slot_for(f8, "gate_up")
        mx_da, mx_dm = Fn.mx_slot_for(f8, "o"), Fn.mx_slot_for(f8, "down")
        x = self.input_layernorm(hidden_states, s1, mx_a)
        a = self.self_attn(x, attention_mask, rope, cache, attn_sink, mx_a, mx_da)
        pa, pf = self.post_attention_layernorm, self.pre_feedforward_layernorm
        if FUSED_NORM_PAIR[0]:
            # post-attention norm + residual and the pre-feedforward norm in one launch (AddRMSNorm2Fn); h's
            # residual-branch gradient arrives through s2 (post_feedforward's add parks it there)
            shp = a.shape
            h, x = Fn.AddRMSNorm2Fn.apply(hidden_states.reshape(-1, shp[-1]), a.reshape(-1, shp[-1]), pa.weight,
                                          pf.weight, pa.eps, pf.eps, s1, s2, mx_m, mx_da)
            h, x = h.view(shp), x.view(shp)
        else:
            h = pa.add_forward(hidden_states, a, s1, mx_da)
            x = pf(h, s2, mx_m)
        m = self.mlp(x, mx_m, mx_dm)
        return self.post_feedforward_layernorm.add_forward(h, m, s2, mx_dm)


class Gemma2Model(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.padding_idx = config.pad_token_id
        self.vocab_size = config.vocab_size
        self.embed_tokens = nn.Embedding(config.vocab_size, config.hidden_size, self.padding_idx)
        self.layers = nn.ModuleList([Gemma2DecoderLayer(config, i) for i in range(config.num_hidden_layers)])
        self.norm = Gemma2RMSNorm(config.hidden_size, eps=config.rms_norm_eps)
        # reference :669 / :752-762: the training forward re-runs each decoder layer in the backward when set
        # (Gemma2ForCausalLM._set_gradient_checkpointing)
        self.gradient_checkpointing = False

    def get_input_embeddings(self):
        return self.embed_tokens

    def set_input_embeddings(self, value):
        self.embed_tokens = value

    def forward(self, hidden_states, attention_mask: KVMask, position_ids, output_hidden_states=False,
                cache: Optional[Gemma2KVCache] = None, attn_sink: Optional[list] = None):
        """hidden_states: inputs_embeds already multiplied by the bf16 normalizer (fused in the merge
        kernel, reference :741-742).  With a cache, attention_mask holds the classes of the new tokens only
        (they are appended to the cache's classes) and the cache advances by the new tokens."""
        if cache is not None:
            if torch.is_grad_enabled() and hidden_states.requires_grad:
                raise ValueError("the KV cache is an inference path: run it under torch.no_grad()")
            cache.append_classes(attention_mask.kv_class)
        rope = self.layers[0].self_attn.rotary_emb.tables(position_ids, hidden_states.dtype)
        if attn_sink is not None and cache is not None:
            raise NotImplementedError("output_attentions with a KV cache: run the uncached forward")
        if cache is not None and not output_hidden_states:
            return self._forward_cached(hidden_states, attention_mask, rope, cache), None
        all_h = () if output_hidden_states else None
        hook = getattr(self, "_svla_layer_grad_hook", None)
        pwait = getattr(self, "_svla_param_wait", None)  # ZeRO-1: parameters of layer i all-gathered (engine.py)
        for i, layer in enumerate(self.layers[: self.config.num_hidden_layers]):
            if output_hidden_states:
                all_h += (hidden_states,)
            if hook is not None and hidden_states.requires_grad:
                # fires once d(layer input) is complete, i.e. after every weight grad of layers >= i
                hidden_states.register_hook(lambda g, i=i: hook(i))
            if pwait is not None:
                pwait(("gemma", i))
            if (self.gradient_checkpointing and self.training and cache is None and attn_sink is None
                    and torch.is_grad_enabled()):
                # reference :752-762: the layer's activations are dropped after the forward and the layer re-runs in
                # the backward (non-reentrant torch.utils.checkpoint: the saved tensors of the HIP autograd Functions
                # are recomputed, bitwise, since every kernel is deterministic)
                hidden_states = torch.utils.checkpoint.checkpoint(layer, hidden_states, attention_mask, rope,
                                                                  use_reentrant=False)
            else:
                hidden_states = layer(hidden_states, attention_mask, rope, cache, attn_sink)
        if cache is not None:
            cache.seen_tokens += hidden_states.shape[1]
        if pwait is not None:
            pwait("head")
        hidden_states = self.norm(hidden_states)
        if output_hidden_states:
            all_h += (hidden_states,)
        return hidden_states, all_h


    def _forward_cached(self, hidden, attention_mask, rope, cache):
        """Inference layer loop (prefill into / decode from the cache): each residual add is fused with the norm
        that consumes its result -- post_attention + pre_feedforward, post_feedforward + the next layer's
        input_layernorm (or the final norm) -- bitwise the reference order (:475-496, :777), two norm launches per
        layer instead of four."""
        layers = self.layers[: self.config.num_hidden_layers]
        pwait = getattr(self, "_svla_param_wait", None)
        if pwait is not None:
            for i in range(len(layers)):
                pwait(("gemma", i))
            pwait("head")
        shp = hidden.shape
        H = shp[-1]
        res = hidden.reshape(-1, H).contiguous()
        if (Fn.DECODE_NORM_FUSED[0] and cache.seen_tokens > 0 and res.shape[0] <= 8
                and H <= Kn.GEMV_NORM_MAX_K and H % 8 == 0
                and all(getattr(l.mlp, "_svla_fp8", None) is None for l in layers)):
            return self._decode_fused(res, shp, rope, cache)
        x = layers[0].input_layernorm(res)
        for i, layer in enumerate(layers):
            a = layer.self_attn(x.view(shp), attention_mask, rope, cache).reshape(-1, H)
            pa, pf = layer.post_attention_layernorm, layer.pre_feedforward_layernorm
            h, x = torch.empty_like(res), torch.empty_like(res)
            Kn.add_rmsnorm2_fwd(res, a, pa.weight, pf.weight, pa.eps, pf.eps, h, x)
            m = layer.mlp(x).reshape(-1, H)
            nxt = layers[i + 1].input_layernorm if i + 1 < len(layers) else self.norm
            po = layer.post_feedforward_layernorm
            res, x = torch.empty_like(res), torch.empty_like(res)
            Kn.add_rmsnorm2_fwd(h, m, po.weight, nxt.weight, po.eps, nxt.eps, res, x)
        cache.seen_tokens += shp[1]
        return x.view(shp)


    def _decode_fused(self, res, shp, rope, cache):
        """A decode step (<= 8 new tokens) with every norm pair between sublayers inside the next projection's GEMV
        (svla_gemv_rmsnorm2): post_feedforward + the next input_layernorm in the q|k|v GEMV, post_attention +
        pre_feedforward in the gate|up GEMV -- the outputs of _forward_cached's unfused loop, two launches fewer per
        layer (modeling_gemma2.py:475-496, :777)."""
        layers = self.layers[: self.config.num_hidden_layers]
        B, Lq = shp[0], shp[1]
        cos, sin = rope
        x = layers[0].input_layernorm(res)
        h = m = None
        for i, layer in enumerate(layers):
            at, mlp = layer.self_attn, layer.mlp
            pre = None
            if i > 0:
                po = layers[i - 1].post_feedforward_layernorm
                res = torch.empty_like(h)
                pre = (h, m, po.weight, layer.input_layernorm.weight, po.eps, layer.input_layernorm.eps, res)
            fuse_o = Fn.DECODE_O_FUSED[0] and Fn.DECODE_MLP_PERSIST[0]  # o projection inside the MLP's launch
            a = Fn.gemma_attention_cached(x if i == 0 else None, at.q_proj.weight, at.k_proj.weight, at.v_proj.weight,
                                          at.o_proj.weight, cos, sin, cache.key_cache[i], cache.value_cache[i],
                                          cache.kv_class, cache.seen_tokens, at.attn_cfg(B, Lq), pre=pre,
                                          skip_o=fuse_o)
            pa, pf = layer.post_attention_layernorm, layer.pre_feedforward_layernorm
            h = torch.empty_like(res)
            m = Fn.gemma_mlp_decode(res, None if fuse_o else a, pa.weight, pf.weight, pa.eps, pf.eps, h,
                                    mlp.gate_proj.weight, mlp.up_proj.weight, mlp.down_proj.weight,
                                    o=(a, at.o_proj.weight) if fuse_o else None)
        po = layers[-1].post_feedforward_layernorm
        res, x = torch.empty_like(h), torch.empty_like(h)
        Kn.add_rmsnorm2_fwd(h, m, po.weight, self.norm.weight, po.eps, self.norm.eps, res, x)
        cache.seen_tokens += shp[1]
        return x.view(shp)


class Gemma2ForCausalLM(nn.Module):
    _tied_weights_keys = None

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.model = Gemma2Model(config)
        self.vocab_size = config.vocab_size
        self.lm_head = nn.Linear(config.hidden_size, config.vocab_size, bias=False)

    def get_input_embeddings(self):
        return self.model.embed_tokens

    def set_input_embeddings(self, value):
        self.model.embed_tokens = value

    def get_output_embeddings(self):
        return self.lm_head

    def set_output_embeddings(self, new_embeddings):
        self.lm_head = new_embeddings

    def get_decoder(self):
        return self.model

    def set_decoder(self, decoder):
        self.model = decoder

    def _set_gradient_checkpointing(self, enable: bool = True, gradient_checkpointing_func=None):
        """The reference training script's call (train/spatialvla_pretrain.py:333-334 -> transformers'
        _set_gradient_checkpointing, which flips `gradient_checkpointing` on the modules that have it); the decoder
        then re-runs each layer in the backward (modeling_gemma2.py:752-762, here Gemma2Model.forward with
        torch.utils.checkpoint, non-reentrant whatever gradient_checkpointing_func says: the layer hooks of the ZeRO-1
        exchange and the side-stream weight gradients need the non-reentrant engine).  Activation memory of the 26
        layers drops to their inputs; one more forward per step."""
        for m in self.modules():
            if hasattr(m, "gradient_checkpointing"):
                m.gradient_checkpointing = bool(enable)
                m._gradient_checkpointing_func = gradient_checkpointing_func

    def prepare_inputs_for_generation(self, input_ids, past_key_values=None, attention_mask=None, inputs_embeds=None,
                                      cache_position=None, position_ids=None, use_cache=True, num_logits_to_keep=None,
                                      **kwargs):
        """Reference :1015-1091 for the KV cache here (Gemma2KVCache): input_ids sliced to the tokens not yet in the
        cache, per-sequence positions attention_mask.cumsum - 1 (pads 1) for those tokens, inputs_embeds only at
        the first step.  The 2-D attention_mask is passed through: SpatialVLAForConditionalGeneration.forward builds
        the per-key classes from it (the reference builds the 4-D HybridCache mask here instead, :1057-1077)."""
        if past_key_values is not None:
            if inputs_embeds is not None:
                input_ids = input_ids[:, -cache_position.shape[0]:]
            elif input_ids.shape[1] != cache_position.shape[0]:
                input_ids = input_ids[:, cache_position]
        if attention_mask is not None and position_ids is None:
            position_ids = attention_mask.long().cumsum(-1) - 1
            position_ids.masked_fill_(attention_mask == 0, 1)
            if past_key_values is not None:
                position_ids = position_ids[:, -input_ids.shape[1]:].clone(memory_format=torch.contiguous_format)
        if inputs_embeds is not None and int(cache_position[0]) == 0:
            model_inputs = {"inputs_embeds": inputs_embeds, "input_ids": None}
        else:
            model_inputs = {"input_ids": input_ids.clone(memory_format=torch.contiguous_format), "inputs_embeds": None}
        if num_logits_to_keep is not None:
            model_inputs["num_logits_to_keep"] = num_logits_to_keep
        model_inputs.update({"position_ids": position_ids, "cache_position": cache_position,
                             "past_key_values": past_key_values, "use_cache": use_cache,
                             "attention_mask": attention_mask})
        return model_inputs

    def head(self, hidden_states, target, stash):
        """lm_head + softcap (reference :993-997) fused with the shifted CE; returns (logits2d, loss)."""
        pwait = getattr(self, "_svla_param_wait", None)
        if pwait is not None:
            pwait("head")
        cap = float(self.config.final_logit_softcapping or 0.0)
        if cap <= 0:
            raise ValueError("final_logit_softcapping must be set for the fused softcap/CE head")
        return Fn.LMHeadCEFn.apply(hidden_states.reshape(-1, hidden_states.shape[-1]), self.lm_head.weight, target,
                                   cap, stash)
