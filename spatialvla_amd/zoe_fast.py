"""Fast paths for the frozen ZoeDepth estimator (transformers ZoeDepth/BEiT [3p], called by the reference at
model/modeling_spatialvla.py:314-323), installed per instance by `install(zoe)`.  All are bitwise identical to the
stock modules except the BEiT layers and the metric tail, which keep the modules' bf16 rounding points but sum in
another order (tolerances in tests/test_model_gpu.py):

* BEiT relative position bias (transformers beit BeitRelativePositionBias.forward): the reference path
  re-interpolates the bias table and rebuilds the [577, 577] index on the host for every layer and every
  forward.  The estimator is frozen, so the gathered [heads, 577, 577] bias is cached per layer, keyed on the
  arguments and the table's storage/version (a reload or in-place update recomputes it).
* Conditional log-binomial head (ZoeDepthConditionalLogBinomialSoftmax.forward): the channel concat of the
  contiguous main feature with the channels-last interpolated bin embedding runs as a mixed-layout copy
  (~10 ms at B=32, 384x384).  Concatenating after one explicit NCHW copy gives the same tensor.
* DPT neck resizes (ZoeDepthFeatureFusionLayer's interpolate(scale_factor=2, align_corners=True) and the relative
  head's nn.Upsample) on channels-last bf16 maps: svla_upsample_bilinear_nhwc (csrc/zoe.hip), torch's NHWC bilinear
  arithmetic at 8 channels per thread instead of one element (the stock kernel moved ~0.5 TB/s).
* BEiT layers (BeitLayer.forward) in inference: LayerNorm, the q|k|v / o / fc1 / fc2 GEMMs with fused bias, exact
  GELU and layer-scale + residual epilogues, and the head_dim-64 attention with the additive relative position
  bias, all on libsvla (functional.beit_layer); the bias is copied once per layer into [heads, L, round8(L)] rows.
* DPT readout projections (ZoeDepthReassembleStage.readout_projects[i] = Linear(2H, H) + exact GELU): one libsvla
  GEMM with the BIAS_GELU_ERF epilogue (bf16(gelu_erf(bf16(acc + b))), the eager module's rounding points) instead
  of the stock Linear (hipBLASLt) + elementwise GELU.
* Metric head tail (ZoeDepthMetricDepthEstimationHead.forward after the last attractor): on the GPU the
  relative-depth concat, both bilinear upsamplings, the 1x1-conv MLP, the log-binomial softmax over the bins
  and the bin-centre expectation run as one HIP kernel (svla_zoe_metric_tail, csrc/zoe.hip) with the eager
  path's bf16 rounding points; the seed regressor, projectors and attractors stay stock modules.
"""
import types

import torch


def _cached_rel_pos_bias(orig_forward):
    def forward(self, window_size, interpolate_pos_encoding: bool = False, dim_size=None):
        t = self.relative_position_bias_table
        key = (tuple(window_size), bool(interpolate_pos_encoding), dim_size, t.data_ptr(), t._version, t.dtype,
               t.device, torch.is_grad_enabled())
        hit = getattr(self, "_svla_bias_cache", None)
        if hit is not None and hit[0] == key:
            return hit[1]
        out = orig_forward(window_size, interpolate_pos_encoding=interpolate_pos_encoding, dim_size=dim_size)
        if not torch.is_grad_enabled():
            self._svla_bias_cache = (key, out)
        return out
    return forward


def _logbinomial_forward(self, main_feature, condition_feature):
    if condition_feature.dim() == 4 and not condition_feature.is_contiguous():
        condition_feature = condition_feature.contiguous()
    if main_feature.dim() == 4 and not main_feature.is_contiguous():
        main_feature = main_feature.contiguous()
    return type(self).forward(self, main_feature, condition_feature)


def _metric_head_forward(self, outconv_activation, bottleneck, feature_blocks, relative_depth):
    """ZoeDepthMetricDepthEstimationHead.forward (transformers zoedepth [3p]) with the fused tail."""
    clb = self.conditional_log_binomial
    if (not outconv_activation.is_cuda or clb.mlp[0].out_channels != 80 or clb.log_binomial_transform.k != 64
            or outconv_activation.dtype != torch.bfloat16):
        # the kernel is built for the nyu-kitti head (64 bins, 80 hidden channels, bf16); other configs
        # (e.g. the tiny test estimator) keep the stock tail
        return type(self).forward(self, outconv_activation, bottleneck, feature_blocks, relative_depth)
    x = self.conv2(bottleneck)
    _, seed_bin_centers = self.seed_bin_regressor(x)
    if self.bin_centers_type in ["normed", "hybrid2"]:
        prev_bin = (seed_bin_centers - self.min_depth) / (self.max_depth - self.min_depth)
    else:
        prev_bin = seed_bin_centers
    prev_bin_embedding = self.seed_projector(x)
    for projector, attractor, feature in zip(self.projectors, self.attractors, feature_blocks):
        bin_embedding = projector(feature)
        bin, bin_centers = attractor(bin_embedding, prev_bin, prev_bin_embedding, interpolate=True)
        prev_bin = bin.clone()
        prev_bin_embedding = bin_embedding.clone()
    from . import kernels as K
    return K.zoe_metric_tail(self.conditional_log_binomial, outconv_activation, relative_depth, bin_embedding,
                             bin_centers), None


def _interp(x, size=None, scale_factor=None, mode="bilinear", align_corners=None):
    """nn.functional.interpolate for the DPT neck: channels-last bf16 maps go through the HIP resize kernel
    (svla_upsample_bilinear_nhwc, torch's NHWC bilinear arithmetic, 8 channels per thread); anything else
    keeps the stock op."""
    if (mode == "bilinear" and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous()):
        from . import kernels as K
        return K.upsample_bilinear_cl(x, size=size, scale_factor=scale_factor, align_corners=bool(align_corners))
    return torch.nn.functional.interpolate(x, size=size, scale_factor=scale_factor, mode=mode,
                                           align_corners=align_corners)


def _fusion_forward(self, hidden_state, residual=None):
    """ZoeDepthFeatureFusionLayer.forward (transformers zoedepth / dpt [3p]) with the resize on the HIP kernel."""
    if residual is not None:
        if hidden_state.shape != residual.shape:
            residual = _interp(residual, size=(hidden_state.shape[2], hidden_state.shape[3]), mode="bilinear",
                               align_corners=False)
        hidden_state = hidden_state + self.residual_layer1(residual)
    hidden_state = self.residual_layer2(hidden_state)
    hidden_state = _interp(hidden_state, scale_factor=2, mode="bilinear", align_corners=self.align_corners)
    return self.projection(hidden_state)


def _upsample_forward(self, x):
    """nn.Upsample(scale_factor, mode="bilinear", align_corners) of the relative-depth head."""
    if self.size is None and self.recompute_scale_factor is None:
        return _interp(x, scale_factor=self.scale_factor, mode=self.mode, align_corners=self.align_corners)
    return type(self).forward(self, x)


def _padded_bias(layer, rpb):
    """[1, heads, L, L] relative position bias -> [heads, L, round8(L)] rows for svla_attn_fwd, cached per layer
    against the (cached) bias tensor."""
    key = (rpb.data_ptr(), rpb._version, tuple(rpb.shape))
    hit = getattr(layer, "_svla_bias", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    h, L = rpb.shape[1], rpb.shape[-1]
    out = torch.zeros(h, L, (L + 7) // 8 * 8, dtype=torch.bfloat16, device=rpb.device)
    out[:, :, :L] = rpb[0]
    layer._svla_bias = (key, out)
    return out


def _beit_layer_forward(self, hidden_states, attention_mask=None, interpolate_pos_encoding=False, resolution=None,
                        **kwargs):
    """BeitLayer.forward (transformers beit [3p]) on the HIP kernels (functional.beit_layer) for the frozen
    estimator's inference: bf16 on the GPU, head_dim 64, no extra attention mask; anything else keeps the stock
    module."""
    at = self.attention
    if (not hidden_states.is_cuda or hidden_states.dtype != torch.bfloat16 or attention_mask is not None
            or self.training or torch.is_grad_enabled() or at.head_dim != 64
            or getattr(self, "_svla_stock", False)):
        return type(self).forward(self, hidden_states, attention_mask=attention_mask,
                                  interpolate_pos_encoding=interpolate_pos_encoding, resolution=resolution, **kwargs)
    bias = None
    if self.relative_position_bias is not None:
        height, width = resolution
        window_size = (height // self.patch_size, width // self.patch_size)
        rpb = self.relative_position_bias(window_size, interpolate_pos_encoding, dim_size=hidden_states.shape[1])
        bias = _padded_bias(self, rpb.to(torch.bfloat16))
    from . import functional as Fn
    return Fn.beit_layer(self, hidden_states, bias)


def _readout_forward(self, x):
    """nn.Sequential(Linear(2H, H), GELU(erf)) of ZoeDepthReassembleStage (transformers zoedepth [3p]) as one GEMM
    with the fused bias + exact-GELU epilogue; other inputs (grad mode, fp32, CPU) keep the stock modules."""
    lin = self[0]
    if (not x.is_cuda or x.dtype != torch.bfloat16 or torch.is_grad_enabled() or lin.bias is None
            or lin.weight.dtype != torch.bfloat16 or x.shape[-1] % 8 or lin.out_features % 8):
        return torch.nn.Sequential.forward(self, x)
    from . import _lib as L
    from . import kernels as K
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    out = torch.empty(x2.shape[0], lin.out_features, dtype=x.dtype, device=x.device)
    K.linear_fwd(x2, [lin.weight], out, kind=L.EPI_BIAS_GELU_ERF, bias=lin.bias)
    return out.view(*shp[:-1], lin.out_features)


def _is_exact_gelu(m) -> bool:
    if isinstance(m, torch.nn.GELU):
        return m.approximate == "none"
    name = type(m).__name__
    return name == "GELUActivation" and getattr(m, "act", None) in (torch.nn.functional.gelu,)


def install(zoe: torch.nn.Module, tail: bool = True, beit: bool = True, readout: bool = True) -> torch.nn.Module:
    """Patch the instances inside `zoe` (idempotent).  tail=False / beit=False / readout=False keep the stock
    metric-head tail / BEiT layers / readout projections (the other paths are bitwise identical to the stock
    modules)."""
    for m in zoe.modules():
        name = type(m).__name__
        if name == "ZoeDepthReassembleStage" and readout and hasattr(m, "readout_projects"):
            for seq in m.readout_projects:
                if (not getattr(seq, "_svla_fast", False) and len(seq) == 2 and isinstance(seq[0], torch.nn.Linear)
                        and _is_exact_gelu(seq[1])):
                    seq.forward = types.MethodType(_readout_forward, seq)
                    seq._svla_fast = True
        if name == "BeitRelativePositionBias" and not getattr(m, "_svla_fast", False):
            m.forward = types.MethodType(_cached_rel_pos_bias(m.forward), m)
            m._svla_fast = True
        elif name == "ZoeDepthConditionalLogBinomialSoftmax" and not getattr(m, "_svla_fast", False):
            m.forward = types.MethodType(_logbinomial_forward, m)
            m._svla_fast = True
        elif name == "ZoeDepthFeatureFusionLayer" and not getattr(m, "_svla_fast", False):
            m.forward = types.MethodType(_fusion_forward, m)
            m._svla_fast = True
        elif (isinstance(m, torch.nn.Upsample) and m.mode == "bilinear" and not getattr(m, "_svla_fast", False)):
            m.forward = types.MethodType(_upsample_forward, m)
            m._svla_fast = True
        elif name == "BeitLayer" and beit and not getattr(m, "_svla_fast", False):
            m.forward = types.MethodType(_beit_layer_forward, m)
            m._svla_fast = True
        elif name == "ZoeDepthMetricDepthEstimationHead" and tail and not getattr(m, "_svla_fast", False):
            m.forward = types.MethodType(_metric_head_forward, m)
            m._svla_fast = True
    return zoe
