"""SpatialVLAForConditionalGeneration on MI355X: the drop-in model class.

Mirrors the reference's public surface (model/modeling_spatialvla.py:162-526): constructor
signature, sub-module attribute names (= state-dict keys), `forward(...)`
arguments and the `SpatialVLACausalLMOutputWithPast` return, `get_image_features`,
`backproject_patch`, `predict_action`, `from_pretrained` (spatial-embedding tail copy :524-525).

Hot-path compute runs on libsvla (HIP, gfx950) through `spatialvla_amd.functional`:
SigLIP, Ego3D, projector, embedding merge, 26 Gemma2 layers, softcapped lm_head + CE.
The frozen ZoeDepth estimator runs under no_grad with its BEiT layers, every convolution, the DPT resizes and the
metric-head tail on libsvla (zoe_fast); its preprocessing (reflect pad + bicubic, process_zoe) and the attractor /
seed-regressor modules are the remaining stock PyTorch-ROCm ops.
"""
import os
import warnings
from dataclasses import dataclass
from typing import List, Optional, Tuple, Union

import torch
import torch.nn.functional as F
from torch import nn
from transformers import GenerationMixin, PreTrainedModel
from transformers.utils import ModelOutput

from . import functional as Fn
from . import zoe_fast

# the Zoe depth + Ego3D encoding of the training forward on the side stream beside SigLIP (SVLA_ZOE_STREAM=0: serial)
ZOE_STREAM = [os.environ.get("SVLA_ZOE_STREAM", "1") != "0"]
# ... also inside the captured B=1 prefill graph (two branches of the graph): prefill + first token 15.3 -> 12.6 ms,
# configs[1] (prompt -> 4 tokens) 20.9 -> 18.2 ms (profiles/r8y_prefill_zoe_branch_ab.txt)
ZOE_STREAM_CAPTURE = [os.environ.get("SVLA_ZOE_STREAM_CAPTURE", "1") != "0"]
from . import kernels as K
from .configuration_spatialvla import SpatialVLAConfig
from .modeling_gemma2 import Gemma2ForCausalLM, Gemma2KVCache, KVMask
from .modeling_siglip import SiglipVisionModel

SIGLIP_MEAN, SIGLIP_STD = (0.5, 0.5, 0.5), (0.5, 0.5, 0.5)
ZOE_MEAN, ZOE_STD = (0.5, 0.5, 0.5), (0.5, 0.5, 0.5)


class Ego3DPositionEmbeddingMLP(nn.Module):
    """Reference :41-97.  Frequency encoding is done by the svla_ego3d_encode kernel (fused with the
    depth back-projection); the MLP head runs on HIP GEMM/LayerNorm/ReLU kernels and its last Linear
    adds the SigLIP features in its epilogue (:327-328)."""

    def __init__(self, in_channels=3, num_pos_feats=768, n_freqs=8, logscale=True):
        super().__init__()
        self.n_freqs = n_freqs
        self.freq_out_channels = in_channels * (2 * n_freqs + 1)
        if not logscale:
            raise ValueError("only logscale frequency bands are used by SpatialVLA")
        freq_bands = 2 ** torch.linspace(0, n_freqs - 1, n_freqs)
        center = torch.tensor([0.0, 0.0, 2.0]).repeat(in_channels // 3)
        self.register_buffer("freq_bands", freq_bands, persistent=False)
        self.register_buffer("center", center, persistent=False)
        self.position_embedding_head = nn.Sequential(
            nn.Linear(self.freq_out_channels, num_pos_feats),
            nn.LayerNorm(num_pos_feats),
            nn.ReLU(),
            nn.Linear(num_pos_feats, num_pos_feats),
        )
        for p in self.parameters():
            if p.dim() > 1:
                nn.init.xavier_uniform_(p, gain=0.01)

    def forward_residual(self, feat_padded, residual2d):
        """feat_padded [N, round8(F)] (zero tail) -> residual + head(feat)."""
        h0, ln, _, h3 = self.position_embedding_head
        x = Fn.LinearFn.apply(feat_padded, h0.weight, h0.bias, None, 1.0)
        x = Fn.LayerNormFn.apply(x, ln.weight, ln.bias, ln.eps, None)
        x = Fn.ReLUFn.apply(x)
        return Fn.LinearFn.apply(x, h3.weight, h3.bias, residual2d, 1.0)


_ZOE_CONSTS = {}


def _zoe_norm_consts(dtype, device):
    """Zoe mean/std as device tensors, made once per (dtype, device): no host->device copy per call, so the
    preprocessing can sit inside a captured HIP graph."""
    key = (dtype, str(device))
    if key not in _ZOE_CONSTS:
        _ZOE_CONSTS[key] = (torch.tensor(ZOE_MEAN, dtype=dtype, device=device).view(1, -1, 1, 1),
                            torch.tensor(ZOE_STD, dtype=dtype, device=device).view(1, -1, 1, 1))
    return _ZOE_CONSTS[key]


def process_zoe(pixel_values, pad_mode="reflect", output_size=(384, 512)):
    """Reference :99-110 (ZoeDepth preprocessing): reflect pad 31, bicubic to 384^2 (align_corners), normalise.  On
    the GPU (bf16) one libsvla kernel (svla_zoe_preprocess); other devices / dtypes run the stock ops."""
    ph, pw = 31, 31
    if pixel_values.is_cuda and pixel_values.dtype == torch.bfloat16 and pad_mode == "reflect":
        C = pixel_values.shape[1]  # mean / std as the bf16 values TF.normalize uses on a bf16 image
        return (K.zoe_preprocess(pixel_values.contiguous(), ph, (384, 384),
                                 [float(torch.tensor(v, dtype=torch.bfloat16)) for v in ZOE_MEAN[:C]],
                                 [float(torch.tensor(v, dtype=torch.bfloat16)) for v in ZOE_STD[:C]]), ph, pw)
    images = F.pad(pixel_values, (pw, pw, ph, ph), mode=pad_mode)
    images = F.interpolate(images, size=(384, 384), mode="bicubic", align_corners=True)
    mean, std = _zoe_norm_consts(images.dtype, images.device)
    images = (images - mean) / std
    return images, ph, pw


@dataclass
class SpatialVLACausalLMOutputWithPast(ModelOutput):
    loss: Optional[torch.FloatTensor] = None
    logits: torch.FloatTensor = None
    past_key_values: Optional[Union[List[torch.FloatTensor], object]] = None
    hidden_states: Optional[Tuple[torch.FloatTensor]] = None
    attentions: Optional[Tuple[torch.FloatTensor]] = None
    image_hidden_states: Optional[torch.FloatTensor] = None


class SpatialVLAMultiModalProjector(nn.Module):
    def __init__(self, config: SpatialVLAConfig):
        super().__init__()
        self.linear = nn.Linear(config.vision_config.hidden_size, config.vision_config.projection_dim, bias=True)


class SpatialVLAPreTrainedModel(PreTrainedModel):
    config_class = SpatialVLAConfig
    base_model_prefix = "model"
    # gradient_checkpointing_enable / the training script's language_model._set_gradient_checkpointing(): the Gemma2
    # decoder layers re-run in the backward (Gemma2ForCausalLM._set_gradient_checkpointing); the vision tower's flag is
    # recorded only, as in the reference (spatialvla_pretrain.py:331 sets an attribute its encoder never reads)
    supports_gradient_checkpointing = True
    _no_split_modules = ["SpatialVLAMultiModalProjector", "ZoeDepthForDepthEstimation", "Ego3DPositionEmbeddingMLP"]

    def _init_weights(self, module):
        std = getattr(self.config, "initializer_range", None) or self.config.text_config.initializer_range
        if isinstance(module, (nn.Linear, nn.Conv2d)):
            module.weight.data.normal_(mean=0.0, std=std)
            if module.bias is not None:
                module.bias.data.zero_()
        elif isinstance(module, nn.Embedding):
            module.weight.data.normal_(mean=0.0, std=std)
            if module.padding_idx is not None:
                module.weight.data[module.padding_idx].zero_()


class SpatialVLAForConditionalGeneration(SpatialVLAPreTrainedModel, GenerationMixin):
    def __init__(self, config: SpatialVLAConfig, vision_model=None, vision_zoe_model=None, projector_model=None,
                 language_model=None):
        super().__init__(config)
        self.vision_tower = vision_model or SiglipVisionModel(config.vision_config)
        self.multi_modal_projector = projector_model or SpatialVLAMultiModalProjector(config)
        self.vocab_size = config.text_config.vocab_size
        self.language_model = language_model or Gemma2ForCausalLM(config.text_config)
        if config.use_vision_zoe:
            from transformers import ZoeDepthForDepthEstimation  # frozen 3p module tree; compute patched by zoe_fast
            self.vision_zoe_model = vision_zoe_model or ZoeDepthForDepthEstimation(config.vision_zoe_config)
            zoe_fast.install(self.vision_zoe_model)
            self.position_embedding_3d = Ego3DPositionEmbeddingMLP(
                config.ego3d_patch_reso ** 2 * 3, num_pos_feats=config.vision_config.hidden_size,
                n_freqs=config.n_freqs)
            patch_size, reso, image_size = (config.vision_config.patch_size, config.ego3d_patch_reso,
                                            config.vision_config.image_size)
            y, x = torch.meshgrid(torch.arange(0, image_size, patch_size // reso),
                                  torch.arange(0, image_size, patch_size // reso), indexing="ij")
            y, x = y + patch_size / reso / 2, x + patch_size / reso / 2
            uv_h = torch.stack([x, y, torch.ones_like(x)], dim=0).reshape(3, -1)
            self.register_buffer("uv_h", uv_h, persistent=False)
        if config.use_spatial_token:
            self.spatial_embed_tokens = nn.Embedding(config.spatial_token_num, config.text_config.hidden_size)
        else:
            self.spatial_embed_tokens = None
        self.pad_token_id = config.pad_token_id if config.pad_token_id is not None else -1
        # predict_action replays each decode step from a captured HIP graph (SVLA_DECODE_GRAPHS=0: eager launches)
        self.decode_graphs = os.environ.get("SVLA_DECODE_GRAPHS", "1") != "0"
        # reference raises on an image-token count mismatch inside the same forward (:379-385), and so does this
        # forward by default (one host read of the count).  defer_checks = True (opt-in: TrainEngine(...,
        # defer_host_checks=True), bench.py) copies the count to pinned host memory behind an event instead and
        # raises at the next forward / check_deferred(), so a training step never waits on the GPU.
        self.strict_checks = True
        self.defer_checks = False
        self._deferred = []
        self.last_stash = {}
        self.post_init()

    # ------------------------------------------------------------------ deferred host checks
    @staticmethod
    def _pinned_i64(dev):
        return torch.zeros(1, dtype=torch.int64, pin_memory=dev.type == "cuda")  # torch's caching host allocator

    def _defer(self, value, check):
        """check(v) on the device scalar `value`: at once (the reference's synchronous raise, default), or, with
        defer_checks, after copying it to pinned host memory behind an event at the next check_deferred().
        CPU tensors are always checked at once."""
        if value.device.type != "cuda" or not self.defer_checks:
            check(int(value))
            return
        buf = self._pinned_i64(value.device)
        buf.copy_(value.reshape(1).to(torch.int64), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._deferred.append((buf, ev, check))

    def check_deferred(self):
        """Run the pending host checks (waits for their events: recorded one forward earlier, long complete)."""
        pend, self._deferred = self._deferred, []
        for buf, ev, check in pend:
            ev.synchronize()
            check(int(buf[0]))

    # ------------------------------------------------------------------ reference accessors
    def get_input_embeddings(self):
        return self.language_model.get_input_embeddings()

    def set_input_embeddings(self, value):
        self.language_model.set_input_embeddings(value)

    def get_output_embeddings(self):
        return self.language_model.get_output_embeddings()

    def set_output_embeddings(self, new_embeddings):
        self.language_model.set_output_embeddings(new_embeddings)

    def get_decoder(self):
        return self.language_model.get_decoder()

    def set_decoder(self, decoder):
        self.language_model.set_decoder(decoder)

    def tie_weights(self, *args, **kwargs):
        return None  # SpatialVLA unties lm_head (spatialvla_pretrain.py:321-325)

    def _set_gradient_checkpointing(self, enable: bool = True, gradient_checkpointing_func=None):
        """gradient_checkpointing_enable() lands here: the Gemma2 layers recompute in the backward (see
        Gemma2ForCausalLM._set_gradient_checkpointing); the vision tower's flag is recorded only."""
        self.language_model._set_gradient_checkpointing(enable, gradient_checkpointing_func)
        self.vision_tower.gradient_checkpointing = bool(enable)

    # ------------------------------------------------------------------ image path
    @torch.no_grad()
    def predict_depth(self, pixel_values):
        """Zoe depth at image resolution (reference :314-323), frozen; the estimator's layers on libsvla (zoe_fast)."""
        zoe_pv, ph, pw = process_zoe(pixel_values, pad_mode="reflect")
        pvh, pvw = pixel_values.shape[-2:]
        depth = self.vision_zoe_model(pixel_values=zoe_pv).predicted_depth
        if depth.is_cuda and depth.dtype == torch.bfloat16:  # resize + crop in one kernel (svla_zoe_depth_resize)
            return K.zoe_depth_resize(depth.contiguous(), ph, (pvh, pvw))
        depth = F.interpolate(depth.unsqueeze(1), size=(pvh + 2 * ph, pvw + 2 * pw), mode="bicubic",
                              align_corners=True)[..., ph:-ph, pw:-pw]
        return depth.contiguous()

    @torch.no_grad()
    def ego3d_features(self, intrinsic, depth, kinv=None):
        """backproject_patch (:195-223) + frequency_encoding (:74-91) in one kernel -> [B*np, round8(F)]."""
        cfg = self.config
        B = depth.shape[0]
        np_ = (cfg.vision_config.image_size // cfg.vision_config.patch_size) ** 2
        nfeat = self.position_embedding_3d.freq_out_channels
        dt = self.multi_modal_projector.linear.weight.dtype
        feat = torch.empty(B * np_, K.round_up(nfeat, 8), dtype=dt, device=depth.device)
        if kinv is None:
            kinv = K.inv3x3(intrinsic)
        K.ego3d_encode(depth.float().contiguous(), kinv, self.uv_h.float().contiguous(),
                       cfg.vision_config.patch_size, cfg.ego3d_patch_reso, cfg.n_freqs, feat)
        return feat

    def backproject_patch(self, K_: torch.Tensor, depth: torch.Tensor, patch_size=14, reso=2) -> torch.Tensor:
        """Reference :195-223 — returns xyz [B, np, 3*reso^2] (fp32), computed by the HIP kernel."""
        B = depth.shape[0]
        np_ = (depth.shape[-2] // patch_size) * (depth.shape[-1] // patch_size)
        nfeat = 3 * reso * reso * (2 * self.config.n_freqs + 1)
        feat = torch.empty(B * np_, K.round_up(nfeat, 8), dtype=torch.bfloat16, device=depth.device)
        xyz = torch.empty(B, np_, 3 * reso * reso, dtype=torch.float32, device=depth.device)
        K.ego3d_encode(depth.float().contiguous(), K.inv3x3(K_),
                       self.uv_h.float().contiguous(), patch_size, reso, self.config.n_freqs, feat, xyz)
        return xyz

    def _wait_all_params(self):
        """ZeRO-1: land every parameter all-gather still in flight (TrainEngine leaves them to the next forward's
        wait points, which a replayed inference graph does not contain)."""
        wait_all = getattr(self, "_svla_param_wait_all", None)
        if wait_all is not None:
            wait_all()

    def _wait_params(self):
        pwait = getattr(self, "_svla_param_wait", None)  # ZeRO-1: embeddings / projector / Ego3D all-gathered
        if pwait is not None:
            pwait("pre")

    def get_image_features(self, pixel_values: torch.FloatTensor, intrinsic: torch.FloatTensor, kinv=None,
                           depth=None):
        """Reference :308-333 -> [B, np, H_text].  depth: a precomputed Zoe depth (predict_action computes it outside
        its prefill graph); None = predict it here."""
        self._wait_params()
        dt = self.multi_modal_projector.linear.weight.dtype
        pv = pixel_values.to(dt).contiguous()
        sig_in = torch.empty_like(pv)
        K.affine(pv, 1.0 / SIGLIP_STD[0], -SIGLIP_MEAN[0], sig_in)  # TF.normalize (:309)
        B = pv.shape[0]
        enc = None
        capturing = pv.is_cuda and torch.cuda.is_current_stream_capturing()
        if self.config.use_vision_zoe and depth is None and ZOE_STREAM[0] and pv.is_cuda and \
                (not capturing or ZOE_STREAM_CAPTURE[0]) and \
                Fn.side_stream(pv.device) != torch.cuda.current_stream(pv.device):
            # the frozen Zoe estimator and the Ego3D encoding (no autograd) on the side stream, beside the SigLIP
            # tower: two independent networks, each filling the CUs the other's kernel tails leave idle (also inside
            # the captured B=1 prefill graph: a fork / join of two branches)
            main = torch.cuda.current_stream(pv.device)
            side = Fn.side_stream(pv.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                enc = self.ego3d_features(intrinsic, self.predict_depth(pixel_values.to(dt)), kinv)
            feats = self.vision_tower(sig_in)                       # [B, np, Hv]
            main.wait_stream(side)
            if not capturing:  # (a captured graph's pool keeps its buffers alive for every replay)
                enc.record_stream(main)  # allocated on the side stream, read (and saved for backward) on this one
        else:
            feats = self.vision_tower(sig_in)                       # [B, np, Hv]
        Hv = feats.shape[-1]
        sel = feats.reshape(-1, Hv)
        if self.config.use_vision_zoe:
            if enc is None:
                if depth is None:
                    depth = self.predict_depth(pixel_values.to(dt))
                enc = self.ego3d_features(intrinsic, depth, kinv)  # kinv: precomputed outside a graph capture
            sel = self.position_embedding_3d.forward_residual(enc, sel)
        lin = self.multi_modal_projector.linear
        img = Fn.LinearFn.apply(sel, lin.weight, lin.bias, None, 1.0 / (self.config.text_config.hidden_size ** 0.5))
        return img.view(B, -1, img.shape[-1])

    # ------------------------------------------------------------------ forward
    def _merge_inputs(self, input_ids, image_features):
        self._wait_params()
        cfg = self.config
        B, Lq = input_ids.shape
        dev = input_ids.device
        embed_w = self.get_input_embeddings().weight
        if embed_w.requires_grad and torch.is_grad_enabled():
            raise NotImplementedError("training embed_tokens is not supported: freeze it as the reference does "
                                      "(freeze_llm_embed, spatialvla_pretrain.py:341-342)")
        ids = input_ids.reshape(-1).contiguous()
        img_index = None
        if image_features is not None:
            img_mask = ids == cfg.image_token_index
            n_img = image_features.shape[0] * image_features.shape[1]
            if self.strict_checks:
                def check(n_tok, n_img=n_img):
                    if n_tok != n_img:
                        raise ValueError(
                            "Number of images does not match number of special image tokens in the input text. "
                            f"Got {n_tok} image tokens in the text but {n_img} tokens from image embeddings.")
                self._defer(img_mask.sum(), check)
            # image rows beyond the features (a mismatch, reported by a deferred check) read the text embedding
            # instead of past the end of the feature rows
            idx = torch.cumsum(img_mask.to(torch.int32), 0) - 1
            img_index = torch.where(img_mask & (idx < n_img), idx, -1).to(torch.int32)
        spatial_w, sort_rows, offsets, a0 = None, None, None, 0
        if cfg.use_spatial_token:
            spatial_w = self.spatial_embed_tokens.weight
            a0, na = int(cfg.action_token_begin_idx), spatial_w.shape[0]
            sel = (ids >= a0) & (ids < a0 + na)
            key = torch.where(sel, ids - a0, na)
            skey, order = torch.sort(key, stable=True)
            sort_rows = order.to(torch.int32)
            # CSR row offsets of each spatial-token id in the sorted order: a binary search instead of a
            # scatter_add histogram (every non-action token hits one bin: 0.11 ms of atomics at B=32)
            offsets = torch.searchsorted(skey, torch.arange(na + 1, dtype=skey.dtype, device=dev)).to(torch.int32)
        hidden = cfg.text_config.hidden_size
        normalizer = float(torch.tensor(hidden ** 0.5, dtype=embed_w.dtype))
        img2d = image_features.reshape(-1, image_features.shape[-1]) if image_features is not None else None
        out = Fn.EmbedMergeFn.apply(ids, img_index, img2d, spatial_w, embed_w, a0, normalizer, sort_rows, offsets)
        return out.view(B, Lq, hidden)

    def _merge_embeds(self, input_ids, inputs_embeds, image_features):
        """forward(inputs_embeds=...) (reference :361-387): the caller's embeddings instead of the table lookup, the
        spatial-token override (x * 0.0 + spatial row, quirk Q10) and the image-slot scatter keyed by input_ids, then
        the bf16 normalizer (modeling_gemma2.py:741-742).  Rare path: stock torch ops on the device, differentiable
        in inputs_embeds, the spatial table and the image features."""
        self._wait_params()
        cfg = self.config
        emb = inputs_embeds.to(self.multi_modal_projector.linear.weight.dtype).clone()
        if cfg.use_spatial_token and input_ids is not None:
            a0, na = int(cfg.action_token_begin_idx), int(cfg.spatial_token_num)
            sel = (input_ids >= a0) & (input_ids < a0 + na)
            emb[sel] = emb[sel] * 0.0 + self.spatial_embed_tokens.weight[input_ids[sel] - a0]
        if image_features is not None:
            m = (input_ids == cfg.image_token_index).unsqueeze(-1).expand_as(emb)
            if self.strict_checks:
                n_img = image_features.shape[0] * image_features.shape[1]

                def check(n_tok, n_img=n_img):
                    if n_tok != n_img:
                        raise ValueError(
                            "Number of images does not match number of special image tokens in the input text. "
                            f"Got {n_tok} image tokens in the text but {n_img} tokens from image embeddings.")
                self._defer((input_ids == cfg.image_token_index).sum(), check)
            emb = emb.masked_scatter(m, image_features.to(emb.dtype))
        normalizer = torch.tensor(cfg.text_config.hidden_size ** 0.5, dtype=emb.dtype, device=emb.device)
        return emb * normalizer

    def _label_rows(self, target):
        """Rows with a label, for the lm_head backward, without a host sync: the labelled rows first in order
        (stable sort of the validity flag) and their count copied to pinned memory behind an event recorded
        here -- the backward reads it after the whole forward, when the event has long completed."""
        valid = target >= 0
        order = torch.argsort((~valid).to(torch.int8), stable=True)
        if target.device.type != "cuda":
            return order, int(valid.sum()), None
        buf = self._pinned_i64(target.device)
        buf.copy_(valid.sum().reshape(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return order, buf, ev

    @staticmethod
    def _targets(labels, attention_mask, B, Lq, dev, pad_mask=None):
        """Shifted CE targets per row (reference :415-430): target[b,t] = labels[b,t+1] where
        attention_mask[b,t+1] != 0 and label != -100, else -1 (ignored); last position ignored."""
        t = torch.full((B, Lq), -1, dtype=torch.int64, device=dev)
        if labels is None:
            return t.reshape(-1)
        sl = labels[:, 1:].clone()
        if attention_mask is not None:
            sl = torch.where(attention_mask[:, 1:] != 0, sl, -100)
        sl = torch.where(sl == -100, -1, sl)
        t[:, :-1] = sl
        return t.reshape(-1).contiguous()

    def forward(
        self,
        input_ids: torch.LongTensor = None,
        pixel_values: torch.FloatTensor = None,
        actions: Optional[torch.FloatTensor] = None,
        intrinsic: Optional[torch.Tensor] = None,
        attention_mask: Optional[torch.Tensor] = None,
        position_ids: Optional[torch.LongTensor] = None,
        past_key_values=None,
        token_type_ids: Optional[torch.LongTensor] = None,
        cache_position: Optional[torch.LongTensor] = None,
        inputs_embeds: Optional[torch.FloatTensor] = None,
        labels: Optional[torch.LongTensor] = None,
        use_cache: Optional[bool] = None,
        output_attentions: Optional[bool] = None,
        output_hidden_states: Optional[bool] = None,
        return_dict: Optional[bool] = None,
        num_logits_to_keep: int = 0,
        kv_mask: Optional[KVMask] = None,
    ) -> Union[Tuple, SpatialVLACausalLMOutputWithPast]:
        self.check_deferred()
        cache = past_key_values
        if cache is not None and not isinstance(cache, Gemma2KVCache):
            raise ValueError("past_key_values must be a Gemma2KVCache (see new_cache())")
        return_dict = True if return_dict is None else return_dict
        is_training = token_type_ids is not None and labels is not None  # reference :359
        if input_ids is None:
            if inputs_embeds is None:
                raise ValueError("forward needs input_ids (and optionally inputs_embeds)")
            if pixel_values is not None or self.config.use_spatial_token:
                # the reference reads input_ids for the image slots and the spatial tokens (:363-365, :376)
                raise ValueError("inputs_embeds without input_ids: the image and spatial-token merges need the ids")
        B, Lq = (input_ids if input_ids is not None else inputs_embeds).shape[:2]
        dev = (input_ids if input_ids is not None else inputs_embeds).device
        if cache is None and use_cache and not torch.is_grad_enabled():
            cache = self.new_cache(B, Lq + 256)

        image_features = None
        if pixel_values is not None:
            image_features = self.get_image_features(pixel_values, intrinsic)

        if labels is not None and input_ids is not None:  # reference :390-395 (BC path), sync-free
            has_pad = (labels == self.pad_token_id).any()
            labels = torch.where(has_pad & (input_ids == self.pad_token_id), -100, labels)

        if inputs_embeds is not None:
            hidden = self._merge_embeds(input_ids, inputs_embeds, image_features)
        else:
            hidden = self._merge_inputs(input_ids, image_features)
        past = cache.seen_tokens if cache is not None else 0
        if position_ids is None:
            start = past if cache_position is None else int(cache_position[0])
            position_ids = (torch.arange(start, start + Lq, device=dev) + 1)[None]  # 1-indexed (:372, :473-474)
        if kv_mask is not None:
            mask = kv_mask
        elif past == 0:
            mask = KVMask.build(attention_mask, token_type_ids, is_training, B, Lq, dev)
        else:
            # decode step: new tokens see the prompt and every earlier token (HybridCache path, :387-395);
            # attention_mask (if given) spans past + new tokens as in HF generate
            cls = torch.ones(B, Lq, dtype=torch.uint8, device=dev)
            if attention_mask is not None:
                cls = torch.where(attention_mask[:, -Lq:].to(dev) != 0, 1, 2).to(torch.uint8)
            mask = KVMask(cls.contiguous())
        attn_sink = [] if output_attentions else None
        h, all_h = self.language_model.model(hidden, mask, position_ids, output_hidden_states=bool(output_hidden_states),
                                             cache=cache, attn_sink=attn_sink)

        target = self._targets(labels, attention_mask, B, Lq, dev)
        stash = {}
        if labels is not None and torch.is_grad_enabled():
            stash["row_plan"] = self._label_rows(target)
        logits2d, loss = self.language_model.head(h, target, stash)
        self.last_stash = stash
        logits = logits2d.view(B, Lq, -1)
        if num_logits_to_keep:
            logits = logits[:, -num_logits_to_keep:]
        if labels is None:
            loss = None
        if not return_dict:
            out = (logits,)
            return (loss,) + out if loss is not None else out
        return SpatialVLACausalLMOutputWithPast(loss=loss, logits=logits, past_key_values=cache, hidden_states=all_h,
                                                attentions=tuple(attn_sink) if attn_sink is not None else None,
                                                image_hidden_states=image_features)

    def action_argmax(self):
        """argmax over V of the last forward's logits [B*L] (int64), computed in the lm_head epilogue
        (train/monkey_patch.py:267 uses logits[..., :-1, :].argmax(-1))."""
        return self.last_stash.get("argmax")

    def action_token_ranges(self, action_tokenizer=None):
        """Inclusive token-id bounds (translation lo, hi, rotation lo, hi, gripper lo, hi) of the spatial action
        tokens: from `action_tokenizer` (or self.action_tokenizer, as train/monkey_patch.py:270-297 reads them) when
        given, else the canonical 4096 / 4096 / 2 split of the spatial_token_num tokens at action_token_begin_idx
        (scripts/action_config.json)."""
        at = action_tokenizer if action_tokenizer is not None else getattr(self, "action_tokenizer", None)
        if at is not None:
            return tuple(int(v) for t in (at.translation_tokenizer, at.rotation_tokenizer, at.gripper_tokenizer)
                         for v in (t.token_start_idx, t.token_end_idx))
        a0, n = int(self.config.action_token_begin_idx), int(self.config.spatial_token_num)
        if n != 8194:
            raise ValueError("action_token_ranges: pass the action tokenizer (non-canonical spatial_token_num)")
        return (a0, a0 + 4095, a0 + 4096, a0 + 8191, a0 + 8192, a0 + 8193)

    def action_metrics(self, labels: torch.Tensor, actions: Optional[torch.Tensor] = None, action_tokenizer=None,
                       argmax: Optional[torch.Tensor] = None):
        """The per-step metrics of the reference's compute_loss (train/monkey_patch.py:267-324) for the last
        training forward: accuracy, translation_accuracy, rotation_accuracy, gripper_accuracy as device fp32
        scalars, from the argmax the lm_head epilogue already produced (no [B, L, V] argmax pass, no host sync);
        with `actions` and an action tokenizer also l1_loss, decoded on the host as the reference does (:308-311)."""
        B, Lq = labels.shape
        am = argmax if argmax is not None else self.action_argmax()
        if am is None:
            raise ValueError("action_metrics: no argmax of a previous forward (run a training forward first)")
        am = am.view(B, -1)
        ranges = self.action_token_ranges(action_tokenizer)
        _counts, acc = K.action_accuracy(am, labels.contiguous(), ranges)
        out = {"accuracy": acc[0], "translation_accuracy": acc[1], "rotation_accuracy": acc[2],
               "gripper_accuracy": acc[3]}
        at = action_tokenizer if action_tokenizer is not None else getattr(self, "action_tokenizer", None)
        if actions is not None and at is not None:
            sl = labels[:, 1:]
            mask = (sl >= ranges[0]) & (sl <= ranges[5])
            pred_ids = am[:, :Lq - 1][mask].cpu().numpy().reshape(-1, 3)
            gt = actions.reshape(-1, 7).to(device="cpu", dtype=torch.float32)
            out["l1_loss"] = F.l1_loss(torch.tensor(at.decode_token_ids_to_actions(pred_ids)), gt)
        return out

    # ------------------------------------------------------------------ inference
    def new_cache(self, batch_size: int, capacity: int) -> Gemma2KVCache:
        """An empty KV cache for `capacity` tokens per sequence (prompt + generated)."""
        w = self.language_model.lm_head.weight
        return Gemma2KVCache(self.config.text_config, batch_size, capacity, w.device, w.dtype)

    def _prompt_classes(self, am, B, P, dev):
        if am is None:
            return torch.zeros(B, P, dtype=torch.uint8, device=dev)
        return torch.where(am.to(dev) != 0, 0, 2).to(torch.uint8).contiguous()

    def _next_token(self, h, finished, eos):
        """Greedy pick from the last position's logits (softcapped lm_head, argmax in its epilogue); sequences
        that already emitted eos get pad, as HF generate does for finished sequences."""
        B = h.shape[0]
        stash = {}
        tgt = torch.full((B,), -1, dtype=torch.int64, device=h.device)
        self.language_model.head(h[:, -1:].contiguous(), tgt, stash)
        nxt = stash["argmax"].view(B, 1)
        if eos is not None:
            nxt = torch.where(finished, torch.full_like(nxt, max(self.pad_token_id, 0)), nxt)
            finished = finished | (nxt == eos)
        return nxt, finished

    def _predict_inputs(self, model_inputs):
        dev = self.language_model.lm_head.weight.device
        ids = model_inputs["input_ids"].to(dev)
        pv = model_inputs.get("pixel_values")
        pv = pv.to(dev, torch.bfloat16) if pv is not None else None
        intr = model_inputs.get("intrinsic")
        intr = intr.to(dev, torch.bfloat16) if intr is not None else None
        return ids, pv, intr, model_inputs.get("attention_mask"), dev

    DECODE_STATES_MAX = 2      # decode states (KV cache + captured graphs) kept per model, least recently used out
    DECODE_CAPACITY_STEP = 64  # cache capacities are bucketed: prompts of nearby lengths share one state
    EOS_CHECK_EVERY = 8        # predict_action reads the device's finished flags once per this many decode steps

    def enable_fp8_projections(self, enabled: bool = True):
        """BASELINE configs[4]: the Gemma2 q|k|v, o, gate|up and down forward projections on the fp8 (OCP e4m3,
        row-scaled) MFMA GEMM, the attention and every backward GEMM unchanged (bf16).  Tolerances: tests/
        test_fp8_gpu.py; the captured prefill/decode graphs are dropped (the prefill changes)."""
        for layer in self.language_model.model.layers:
            layer.set_fp8_projections(enabled)
        self.clear_decode_cache()

    def clear_decode_cache(self):
        """Drop every persistent decode state (KV caches, captured prefill/decode graphs and their memory pool).
        The graphs hold raw pointers to the weights they were captured with, so anything that rebinds parameter
        storage (TrainEngine's flat buffers, load_state_dict with assign, .to()) must call this."""
        self.__dict__["_svla_decode_states"] = {}

    @staticmethod
    def _prompt_positions(valid: torch.Tensor) -> torch.Tensor:
        """Per-sequence positions of a (possibly padded) prompt, as the reference's generate derives them:
        attention_mask.cumsum(-1) - 1, pads set to 1 (modeling_gemma2.py:1039-1042), then + 1
        (modeling_spatialvla.py:473-474).  valid: bool [B, L]."""
        pos = valid.to(torch.int64).cumsum(-1) - 1
        return pos.masked_fill(~valid, 1) + 1

    def _decode_state(self, B: int, capacity: int, dev):
        """Persistent decode state per (batch, bucketed capacity): the KV cache, the static token buffer the captured
        graphs read, the graphs themselves keyed by cache position (one private memory pool shared by all of a
        state's graphs), and one side stream for their eager warm-ups.  Reused across predict_action calls, so a
        control loop replays the same graphs every call; at most DECODE_STATES_MAX states are kept (LRU)."""
        from collections import OrderedDict
        states = self.__dict__.get("_svla_decode_states")
        if not isinstance(states, OrderedDict):
            states = self.__dict__["_svla_decode_states"] = OrderedDict()
        cap = -(-capacity // self.DECODE_CAPACITY_STEP) * self.DECODE_CAPACITY_STEP
        key = (B, cap, str(dev))
        st = states.get(key)
        # the graphs hold raw pointers: to the weights (rebound by TrainEngine) and, with fp8 projections, to the
        # e4m3 weight copies, which the next eager forward after an optimizer step (WEIGHT_EPOCH) frees and rebuilds
        fp8 = any(getattr(l.mlp, "_svla_fp8", None) is not None for l in self.language_model.model.layers)
        wptr = (self.language_model.lm_head.weight.data_ptr(), Fn.WEIGHT_EPOCH[0] if fp8 else -1)
        if st is not None and st["wptr"] != wptr:  # weights were rebound since capture: the graphs are stale
            states.pop(key)
            st = None
        if st is None:
            while len(states) >= self.DECODE_STATES_MAX:
                states.popitem(last=False)
            st = {"cache": self.new_cache(B, cap), "graphs": {}, "prefill": {}, "wptr": wptr,
                  "tok": torch.zeros(B, 1, dtype=torch.int64, device=dev),
                  # greedy bookkeeping read / written inside the step graphs: finished rows, eos / pad ids (-1 = no
                  # eos), every generated token at its cache position
                  "fin": torch.zeros(B, 1, dtype=torch.bool, device=dev),
                  "eos": torch.full((1, 1), -1, dtype=torch.int64, device=dev),
                  "pad": torch.zeros(1, 1, dtype=torch.int64, device=dev),
                  "toks": torch.zeros(B, cap + 1, dtype=torch.int64, device=dev),
                  "npad": torch.zeros(B, 1, dtype=torch.int64, device=dev),  # pads in each prompt (static input)
                  "cls": KVMask(torch.ones(B, 1, dtype=torch.uint8, device=dev)),
                  "pool": torch.cuda.graph_pool_handle() if dev.type == "cuda" else None,
                  "side": torch.cuda.Stream(device=dev) if dev.type == "cuda" else None}
            states[key] = st
        states.move_to_end(key)
        return st

    def _prefill_body(self, st, x):
        """Vision tower + Ego3D/Zoe + Gemma2 prefill over the prompt (filling the cache) + the first greedy token."""
        ids, cache = x["ids"], st["cache"]
        feats = (self.get_image_features(x["pv"], x["intr"], x["kinv"], x.get("depth")) if x["pv"] is not None
                 else None)
        pos = self._prompt_positions(x["cls"] != 2)  # per-sequence positions of a padded batch (1..P unpadded)
        strict, self.strict_checks = self.strict_checks, False  # checked on the host by predict_action
        try:
            hidden = self._merge_inputs(ids, feats)
        finally:
            self.strict_checks = strict
        h, _ = self.language_model.model(hidden, KVMask(x["cls"]), pos, cache=cache)
        stash = {}
        tgt = torch.full((ids.shape[0],), -1, dtype=torch.int64, device=ids.device)
        self.language_model.head(h[:, -1:].contiguous(), tgt, stash)
        return stash["argmax"]

    def _prefill_graph(self, st, x):
        """The prefill as one HIP graph per (prompt length, with/without image): ~2000 launches (SigLIP, the frozen
        Zoe forward, 26 Gemma2 layers) whose host cost at B=1 rivals their GPU time.  Inputs are copied into the
        graph's static buffers; shapes, the cache and the positions are baked in."""
        cache = st["cache"]
        key = (x["ids"].shape[1], x["pv"] is not None)
        if key in st["prefill"] and st["prefill"][key] is None:
            return self._prefill_body(st, x)
        g = st["prefill"].get(key)
        if g is None:
            static = {k: (v.clone() if v is not None else None) for k, v in x.items()}
            side = st["side"]
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # eager warm-up: lazy kernel attributes, GEMM workspaces, Zoe caches
                self._prefill_body(st, static)
            cache.seen_tokens = 0
            torch.cuda.current_stream().wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            try:
                # captured on the warm-up stream, where the eager warm-up ran (lazy kernel attributes, weight caches)
                with torch.cuda.graph(graph, pool=st["pool"], stream=side):
                    out = self._prefill_body(st, static)
            except RuntimeError as e:  # an op of the prefill cannot be captured: run this shape eagerly from now on
                cache.seen_tokens = 0
                torch.cuda.synchronize()
                st["prefill"][key] = None
                import traceback
                where = [f"{fr.filename.split('/')[-1]}:{fr.lineno} {fr.name}" for fr in traceback.extract_tb(e.__traceback__)]
                warnings.warn(f"prefill graph capture failed at {' <- '.join(reversed(where[-6:]))}: "
                              f"{str(e).splitlines()[0]}; prefill runs eagerly")
                return self._prefill_body(st, x)
            cache.seen_tokens = 0
            g = st["prefill"][key] = (graph, static, out)
        graph, static, out = g
        for k, v in x.items():
            if v is not None:
                static[k].copy_(v)
        graph.replay()
        return out

    def _decode_body(self, st, p0):
        """One decode step at cache position p0: the token in st["tok"] -> argmax of its logits [B]."""
        tok, cache = st["tok"], st["cache"]
        # 1-indexed (:372, :473-474); a sequence with n pads in its prompt is n positions behind its cache row
        pos = (p0 + 1) - st["npad"]
        h, _ = self.language_model.model(self._merge_inputs(tok, None), st["cls"], pos, cache=cache)
        stash = {}
        tgt = torch.full((tok.shape[0],), -1, dtype=torch.int64, device=tok.device)
        self.language_model.head(h[:, -1:].contiguous(), tgt, stash)
        return stash["argmax"]

    def _greedy_bookkeep(self, st, p0, am):
        """The greedy loop's per-token update on the device (so a run of steps needs no host round trip): rows that
        already emitted eos get pad, newly finished rows are marked, the token is fed to the next step and kept at
        its cache position p0 + 1 (reference generate: unfinished_sequences / pad_token_id handling)."""
        nxt = torch.where(st["fin"], st["pad"], am.view(-1, 1))
        st["fin"].logical_or_(nxt == st["eos"])
        st["tok"].copy_(nxt)
        st["toks"][:, p0 + 1:p0 + 2].copy_(nxt)

    def _decode_step_graph(self, st, p0):
        """The decode step as a HIP graph (torch.cuda.CUDAGraph on ROCm), captured once per cache position: a
        B=1 step is ~300 small launches whose host-side cost exceeds their GPU time, and a graph replays them
        as one submission.  Positions, cache rows and sequence lengths are baked into each graph."""
        cache = st["cache"]
        g = st["graphs"].get(p0)
        if g is None:
            side = st["side"]
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # eager warm-up (lazy kernel attributes); rewrites row p0 identically
                saved = (st["tok"].clone(), st["fin"].clone())
                self._greedy_bookkeep(st, p0, self._decode_body(st, p0))
                st["tok"].copy_(saved[0])
                st["fin"].copy_(saved[1])
            cache.seen_tokens = p0
            torch.cuda.current_stream().wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, pool=st["pool"], stream=side):  # on the warm-up stream, as the prefill
                out = self._decode_body(st, p0)
                self._greedy_bookkeep(st, p0, out)
            cache.seen_tokens = p0
            g = st["graphs"][p0] = (graph, out)
        g[0].replay()
        cache.seen_tokens = p0 + 1
        return g[1]

    @torch.no_grad()
    def predict_action(self, model_inputs, max_new_tokens: int = 256, eos_token_id: Optional[int] = None):
        """Greedy decode with a KV cache (reference :484-492 -> generate(max_new_tokens=256, do_sample=False)
        with HybridCache).  Prefill: the prompt (image features merged, positions 1..P) attends bidirectionally
        (:294) and fills the cache; decode: one token per step at position P+i+1 (:473-474), no pixel values
        after step 0 (:475-476), attending to the prompt and every earlier generated token.  Stops when every
        sequence has emitted eos or after max_new_tokens."""
        self._wait_all_params()
        ids, pv, intr, am, dev = self._predict_inputs(model_inputs)
        eos = eos_token_id if eos_token_id is not None else self.config.text_config.eos_token_id
        B, P = ids.shape
        graphs = self.decode_graphs and dev.type == "cuda"
        st = self._decode_state(B, P + max_new_tokens, dev)
        cache = st["cache"]
        cache.seen_tokens = 0
        cls = self._prompt_classes(am, B, P, dev)
        st["npad"].copy_((cls == 2).sum(-1, keepdim=True))
        if pv is not None and self.strict_checks:  # reference :379-385, checked before any graph replay
            vc = self.config.vision_config
            n_img = B * (vc.image_size // vc.patch_size) ** 2
            n_tok = int((model_inputs["input_ids"] == self.config.image_token_index).sum())
            if n_tok != n_img:
                raise ValueError("Number of images does not match number of special image tokens in the input text. "
                                 f"Got {n_tok} image tokens in the text but {n_img} tokens from image embeddings.")
        # inv(K) (reference :221): the closed-form HIP inverse, captured into the prefill graph with the rest
        kinv = None
        # the frozen Zoe forward is captured with the rest of the prefill: every convolution of it runs on libsvla
        # (zoe_fast), no vendor library creates handles lazily under the capture
        prefill = {"ids": ids, "pv": pv, "intr": intr, "cls": cls, "kinv": kinv}
        first = self._prefill_graph(st, prefill) if graphs else self._prefill_body(st, prefill)
        cache.seen_tokens = P
        # the per-token update runs on the device (_greedy_bookkeep); the host reads the finished flags only every
        # EOS_CHECK_EVERY steps and cuts the output where the last row finished -- the tokens and the length are the
        # step-by-step loop's
        st["eos"].fill_(-1 if eos is None else int(eos))
        st["pad"].fill_(max(self.pad_token_id, 0))
        nxt = first.view(B, 1)
        st["fin"].copy_(nxt == st["eos"])
        st["tok"].copy_(nxt)
        st["toks"][:, P:P + 1].copy_(nxt)
        steps = 0
        while steps < max_new_tokens - 1:
            if eos is not None and steps % self.EOS_CHECK_EVERY == 0 and bool(st["fin"].all()):
                break
            p0 = cache.seen_tokens
            if graphs:
                self._decode_step_graph(st, p0)
            else:
                self._greedy_bookkeep(st, p0, self._decode_body(st, p0))
                cache.seen_tokens = p0 + 1
            steps += 1
        toks = st["toks"][:, P:P + steps + 1].clone()
        K.check_decode_mlp_timeouts("predict_action")
        if eos is not None:  # the step-by-step loop's length: up to the token where the last row finished
            hit = toks == eos
            if bool(hit.any(1).all()):
                n = toks.shape[1]
                first_eos = torch.where(hit, torch.arange(n, device=dev), n).min(1).values
                toks = toks[:, :int(first_eos.max()) + 1]
        return toks

    # ------------------------------------------------------------------ HF generate() surface
    def prepare_inputs_for_generation(self, input_ids, past_key_values=None, inputs_embeds=None, cache_position=None,
                                      position_ids=None, pixel_values=None, intrinsic=None, attention_mask=None,
                                      token_type_ids=None, use_cache=True, num_logits_to_keep=None, labels=None,
                                      **kwargs):
        """Reference :445-482: the language model's hook (slicing to the uncached tokens, per-sequence positions),
        positions + 1 (PaliGemma positions are 1-indexed), pixel values only at the first step, intrinsic passed
        through.  The prefill's bidirectional prefix mask (:478-480) is built by forward() from the 2-D mask."""
        model_inputs = self.language_model.prepare_inputs_for_generation(
            input_ids, past_key_values=past_key_values, inputs_embeds=inputs_embeds, attention_mask=attention_mask,
            position_ids=position_ids, cache_position=cache_position, use_cache=use_cache,
            num_logits_to_keep=num_logits_to_keep, **kwargs)
        if model_inputs.get("position_ids") is not None:
            model_inputs["position_ids"] += 1
        if int(cache_position[0]) == 0:
            model_inputs["pixel_values"] = pixel_values
        model_inputs["token_type_ids"] = token_type_ids if int(cache_position[0]) == 0 and labels is not None else None
        model_inputs["intrinsic"] = intrinsic
        return model_inputs

    @torch.no_grad()
    def generate(self, input_ids=None, pixel_values=None, intrinsic=None, attention_mask=None,
                 max_new_tokens: Optional[int] = None, do_sample: Optional[bool] = None, eos_token_id=None,
                 pad_token_id=None, generation_config=None, **kwargs):
        """Greedy `generate` as the reference's predict_action calls it (:491, HF generate with do_sample=False over a
        HybridCache): the loop runs prepare_inputs_for_generation -> forward(past_key_values=Gemma2KVCache) per step
        and returns prompt + new tokens; finished sequences get pad_token_id, the loop stops once every sequence
        emitted eos.  Every step is eager here; predict_action is the graph-replayed fast path with the same tokens."""
        # HF precedence: explicit arguments override the generation_config, which overrides the defaults
        if generation_config is not None:
            if max_new_tokens is None:
                max_new_tokens = getattr(generation_config, "max_new_tokens", None)
            if do_sample is None:
                do_sample = getattr(generation_config, "do_sample", None)
            eos_token_id = getattr(generation_config, "eos_token_id", None) if eos_token_id is None else eos_token_id
            pad_token_id = getattr(generation_config, "pad_token_id", None) if pad_token_id is None else pad_token_id
        max_new_tokens = 256 if max_new_tokens is None else int(max_new_tokens)
        do_sample = bool(do_sample)
        if do_sample or int(kwargs.pop("num_beams", 1)) != 1:
            raise NotImplementedError("generate: greedy decoding only (the reference calls do_sample=False)")
        kwargs.pop("token_type_ids", None)
        for k in ("output_attentions", "output_hidden_states", "return_dict_in_generate", "use_cache"):
            kwargs.pop(k, None)
        if kwargs:
            raise TypeError(f"generate: unsupported arguments {sorted(kwargs)}")
        self._wait_all_params()
        eos = eos_token_id if eos_token_id is not None else self.config.text_config.eos_token_id
        if isinstance(eos, (list, tuple)):
            eos = eos[0] if eos else None
        pad = pad_token_id if pad_token_id is not None else max(self.pad_token_id, 0)
        dev = self.language_model.lm_head.weight.device
        ids = input_ids.to(dev)
        B, P = ids.shape
        am = (attention_mask.to(dev) if attention_mask is not None
              else torch.ones(B, P, dtype=torch.int64, device=dev))
        pv = pixel_values.to(dev, torch.bfloat16) if pixel_values is not None else None
        intr = intrinsic.to(dev, torch.bfloat16) if intrinsic is not None else None
        cache = self.new_cache(B, P + max_new_tokens)
        cache_position = torch.arange(P, device=dev)
        finished = torch.zeros(B, dtype=torch.bool, device=dev)
        for _ in range(max_new_tokens):
            mi = self.prepare_inputs_for_generation(ids, past_key_values=cache, cache_position=cache_position,
                                                    pixel_values=pv, intrinsic=intr, attention_mask=am)
            mi.pop("cache_position")
            self(**mi, return_dict=True)
            nxt = self.action_argmax().view(B, -1)[:, -1]
            if eos is not None:
                nxt = torch.where(finished, torch.full_like(nxt, pad), nxt)
                finished = finished | (nxt == eos)
            ids = torch.cat([ids, nxt[:, None]], 1)
            am = torch.cat([am, torch.ones(B, 1, dtype=am.dtype, device=dev)], 1)
            cache_position = cache_position[-1:] + 1
            if eos is not None and bool(finished.all()):
                break
        K.check_decode_mlp_timeouts("generate")
        return ids

    @torch.no_grad()
    def predict_action_uncached(self, model_inputs, max_new_tokens: int = 256, eos_token_id: Optional[int] = None):
        """The same greedy decode as full re-forwards over prompt + generated tokens (no cache): prompt keys
        class 0, generated keys class 1.  Kept as the parity reference of the cached path."""
        self._wait_all_params()
        ids, pv, intr, am, dev = self._predict_inputs(model_inputs)
        eos = eos_token_id if eos_token_id is not None else self.config.text_config.eos_token_id
        B, P = ids.shape
        feats = self.get_image_features(pv, intr) if pv is not None else None
        finished = torch.zeros(B, 1, dtype=torch.bool, device=dev)
        out = []
        cur = ids
        for _ in range(max_new_tokens):
            if eos is not None and out and bool(finished.all()):
                break
            Lc = cur.shape[1]
            cls = torch.ones(B, Lc, dtype=torch.uint8, device=dev)
            cls[:, :P] = self._prompt_classes(am, B, P, dev)
            pos = self._prompt_positions(cls != 2)  # generated tokens: the attention mask extended by ones
            h, _ = self.language_model.model(self._merge_inputs(cur, feats), KVMask(cls.contiguous()), pos)
            nxt, finished = self._next_token(h, finished, eos)
            out.append(nxt)
            cur = torch.cat([cur, nxt], 1)
        return torch.cat(out, 1)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, *model_args, **kwargs):
        model = super().from_pretrained(pretrained_model_name_or_path, *model_args, **kwargs)
        if model.config.use_spatial_token:  # reference :524-525
            model.language_model.model.embed_tokens.weight.data[-model.config.spatial_token_num:] = \
                model.spatial_embed_tokens.weight.data
        return model
