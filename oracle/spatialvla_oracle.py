"""CPU restatement ("port") of the reference's eager SpatialVLA forward/backward.

TEST INFRASTRUCTURE ONLY — this is the parity oracle and the `cpu_baseline` of bench.py.  It is
never imported by the product package (`spatialvla_amd/`), and nothing here is a product path.

It restates, op for op and with the same bf16 rounding points, the reference eager path:
  * SigLIP vision tower: transformers 4.47 siglip (3p, requirements.txt:20) — embeddings (conv
    patchify + position embedding), encoder layers (pre-LN, eager attention with fp32 softmax cast
    back to bf16, GELU-tanh MLP), post LayerNorm; called at model/modeling_spatialvla.py:310.
  * Ego3D: backproject_patch (modeling_spatialvla.py:195-223) + frequency_encoding (:74-91) + MLP (:59-64, :93-97).
  * projector + /sqrt(H) (:124-128, :331-332); embedding merge (:361-387).
  * prefix-LM mask (:258-306), Gemma2 layers (model/modeling_gemma2.py:60-506), normalizer (:741-742),
    lm_head + softcap (:993-997), shifted masked CE (modeling_spatialvla.py:415-430).
  * ZoeDepth itself is the transformers module (3p), run frozen under no_grad as in the reference.
  * the per-step action metrics of the patched Trainer.compute_loss (train/monkey_patch.py:267-324).
Pinned by tests/test_cpu.py (and tests/test_action_tokenizer.py) against tests/golden/*, which
oracle/gen_golden.py, gen_action_golden.py and gen_metrics_golden.py produced by running the reference's own code.
"""
import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

BF16 = torch.bfloat16


def _lin(x, w, b=None):
    return F.linear(x, w, b)


def gelu_tanh(x):
    return F.gelu(x, approximate="tanh")


# ---------------------------------------------------------------------------------------- SigLIP
def siglip(P: Dict[str, torch.Tensor], vc: dict, pix, prefix="vision_tower."):
    p = lambda n: P[prefix + n]  # noqa: E731
    B = pix.shape[0]
    x = F.conv2d(pix, p("embeddings.patch_embedding.weight"), p("embeddings.patch_embedding.bias"),
                 stride=vc["patch_size"])
    h = x.flatten(2).transpose(1, 2)
    h = h + p("embeddings.position_embedding.weight")[None]
    H, nh = vc["hidden_size"], vc["num_attention_heads"]
    D = H // nh
    eps = vc.get("layer_norm_eps", 1e-6)
    for i in range(vc["num_hidden_layers"]):
        q_ = lambda n: p(f"encoder.layers.{i}.{n}")  # noqa: E731
        r = h
        x = F.layer_norm(h, (H,), q_("layer_norm1.weight"), q_("layer_norm1.bias"), eps)
        q = _lin(x, q_("self_attn.q_proj.weight"), q_("self_attn.q_proj.bias")).view(B, -1, nh, D).transpose(1, 2)
        k = _lin(x, q_("self_attn.k_proj.weight"), q_("self_attn.k_proj.bias")).view(B, -1, nh, D).transpose(1, 2)
        v = _lin(x, q_("self_attn.v_proj.weight"), q_("self_attn.v_proj.bias")).view(B, -1, nh, D).transpose(1, 2)
        a = torch.matmul(q, k.transpose(-1, -2)) * (D ** -0.5)
        a = F.softmax(a, dim=-1, dtype=torch.float32).to(q.dtype)
        o = torch.matmul(a, v).transpose(1, 2).reshape(B, -1, H)
        o = _lin(o, q_("self_attn.out_proj.weight"), q_("self_attn.out_proj.bias"))
        h = r + o
        r = h
        x = F.layer_norm(h, (H,), q_("layer_norm2.weight"), q_("layer_norm2.bias"), eps)
        x = _lin(gelu_tanh(_lin(x, q_("mlp.fc1.weight"), q_("mlp.fc1.bias"))), q_("mlp.fc2.weight"), q_("mlp.fc2.bias"))
        h = r + x
    return F.layer_norm(h, (H,), p("post_layernorm.weight"), p("post_layernorm.bias"), eps)


# ---------------------------------------------------------------------------------------- Ego3D
def uv_h_buffer(image_size, patch_size, reso, dtype):
    y, x = torch.meshgrid(torch.arange(0, image_size, patch_size // reso),
                          torch.arange(0, image_size, patch_size // reso), indexing="ij")
    y, x = y + patch_size / reso / 2, x + patch_size / reso / 2
    return torch.stack([x, y, torch.ones_like(x)], 0).reshape(3, -1).to(dtype)  # bf16-quantised (Q7)


def backproject(K, depth, uv_h, patch_size=14, reso=2):
    b, c, h, w = depth.shape
    hp, wp = h // patch_size, w // patch_size
    pd = F.interpolate(depth, size=(hp * reso, wp * reso), mode="area").reshape(b, c, -1)
    pc = (torch.linalg.inv(K.float()) @ uv_h.float()) * pd
    return pc.reshape(b, 3, hp, reso, wp, reso).permute(0, 2, 4, 3, 5, 1).reshape(b, hp * wp, -1)


def freq_encode(xyz, n_freqs, dtype):
    freq = (2 ** torch.linspace(0, n_freqs - 1, n_freqs)).to(dtype).to(xyz.device)
    center = torch.tensor([0.0, 0.0, 2.0]).repeat(xyz.shape[-1] // 3).to(dtype).to(xyz.device)
    xn = ((xyz - center) / 2.0).to(freq.dtype)
    xf = xn.unsqueeze(-1) * freq
    return torch.cat([xn.unsqueeze(-1), torch.sin(xf), torch.cos(xf)], -1).reshape(*xyz.shape[:2], -1)


def ego3d_mlp(P, enc, prefix="position_embedding_3d.position_embedding_head."):
    x = _lin(enc, P[prefix + "0.weight"], P[prefix + "0.bias"])
    x = F.layer_norm(x, (x.shape[-1],), P[prefix + "1.weight"], P[prefix + "1.bias"], 1e-5)
    x = F.relu(x)
    return _lin(x, P[prefix + "3.weight"], P[prefix + "3.bias"])


def zoe_depth(zoe_model, pixel_values):
    ph = pw = 31
    im = F.pad(pixel_values, (pw, pw, ph, ph), mode="reflect")
    im = F.interpolate(im, size=(384, 384), mode="bicubic", align_corners=True)
    im = (im - 0.5) / 0.5
    with torch.no_grad():
        d = zoe_model(pixel_values=im).predicted_depth
        h, w = pixel_values.shape[-2:]
        d = F.interpolate(d.unsqueeze(1), size=(h + 2 * ph, w + 2 * pw), mode="bicubic",
                          align_corners=True)[..., ph:-ph, pw:-pw]
    return d


# ---------------------------------------------------------------------------------------- Gemma2
def rms(x, w, eps):
    o = x.float()
    o = o * torch.rsqrt(o.pow(2).mean(-1, keepdim=True) + eps)
    return (o * (1.0 + w.float())).type_as(x)


def rope_tables(pos, dim, dtype, theta=10000.0):
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.int64, device=pos.device).float() / dim))
    # the inv_freq buffer is cast with the model (`model.to(bf16)` / DeepSpeed bf16), so the reference
    # runs RoPE on bf16-quantised frequencies, upcast at modeling_gemma2.py:109 (quirk Q11)
    inv = inv.to(dtype).float()
    f = (inv[None, :, None].float() @ pos[:, None, :].float()).transpose(1, 2)
    e = torch.cat((f, f), -1)
    return e.cos().to(dtype), e.sin().to(dtype)


def rot_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), -1)


def prefix_mask(attn_mask, tt, is_training, L, dtype):
    """_update_causal_mask (modeling_spatialvla.py:258-306), eager branch."""
    mn = torch.finfo(dtype).min
    dev = attn_mask.device
    cm = torch.full((L, L), mn, dtype=dtype, device=dev)
    if is_training:
        cm = torch.triu(cm, 1)
    else:
        cm[:, :L] = 0.0
    cm = cm * (torch.arange(L, device=dev) > torch.arange(L, device=dev).reshape(-1, 1))
    B = attn_mask.shape[0]
    cm = cm[None, None].expand(B, 1, -1, -1).clone()
    pm = (cm + attn_mask[:, None, None, :].to(dtype)) == 0
    cm = cm.masked_fill(pm, mn)
    if is_training:
        cm = cm.masked_fill(tt[:, None, None, :] == 0, 0)
    return cm


def gemma_layer(P, tc, i, h, mask, cos, sin, prefix="language_model.model.", attn_sink=None):
    p = lambda n: P[f"{prefix}layers.{i}.{n}"]  # noqa: E731
    eps = tc["rms_norm_eps"]
    B, L, H = h.shape
    nh, nkv, D = tc["num_attention_heads"], tc["num_key_value_heads"], tc["head_dim"]
    if i % 2 == 0 and mask is not None:  # sliding layers (:461-473)
        sw = torch.tril(torch.ones_like(mask, dtype=torch.bool), diagonal=-tc["sliding_window"])
        mask = torch.where(sw, torch.finfo(h.dtype).min, mask)
    r = h
    x = rms(h, p("input_layernorm.weight"), eps)
    q = _lin(x, p("self_attn.q_proj.weight")).view(B, L, nh, D).transpose(1, 2)
    k = _lin(x, p("self_attn.k_proj.weight")).view(B, L, nkv, D).transpose(1, 2)
    v = _lin(x, p("self_attn.v_proj.weight")).view(B, L, nkv, D).transpose(1, 2)
    c, s = cos.unsqueeze(1), sin.unsqueeze(1)
    q = q * c + rot_half(q) * s
    k = k * c + rot_half(k) * s
    rep = nh // nkv
    k = k[:, :, None].expand(B, nkv, rep, L, D).reshape(B, nh, L, D)
    v = v[:, :, None].expand(B, nkv, rep, L, D).reshape(B, nh, L, D)
    a = torch.matmul(q, k.transpose(2, 3)) * (tc["query_pre_attn_scalar"] ** -0.5)
    cap = tc["attn_logit_softcapping"]
    a = torch.tanh(a / cap) * cap
    a = a + mask[:, :, :, :L]
    a = F.softmax(a, dim=-1, dtype=torch.float32).to(q.dtype)
    if attn_sink is not None:  # output_attentions (:193-195 returns attn_weights)
        attn_sink.append(a)
    o = torch.matmul(a, v).transpose(1, 2).reshape(B, L, -1)
    o = _lin(o, p("self_attn.o_proj.weight"))
    h = r + rms(o, p("post_attention_layernorm.weight"), eps)
    r = h
    x = rms(h, p("pre_feedforward_layernorm.weight"), eps)
    x = _lin(gelu_tanh(_lin(x, p("mlp.gate_proj.weight"))) * _lin(x, p("mlp.up_proj.weight")),
             p("mlp.down_proj.weight"))
    return r + rms(x, p("post_feedforward_layernorm.weight"), eps)


# ---------------------------------------------------------------------------------------- full model
def forward(P: Dict[str, torch.Tensor], cfg: dict, batch: Dict[str, torch.Tensor], zoe_model=None,
            is_training: Optional[bool] = None, depth: Optional[torch.Tensor] = None, cap: Optional[dict] = None,
            mask4d: Optional[torch.Tensor] = None, attn_sink: Optional[list] = None):
    """Returns (loss or None, logits bf16 [B, L, V]).  `P` maps reference parameter names -> tensors
    (vision keys without the 4.47 `vision_model.` infix, as transformers 5 names them).  mask4d: an explicit
    additive [B, 1, L, L] mask, passed through as the reference passes a 4-D attention_mask
    (modeling_spatialvla.py:288-289, modeling_gemma2.py:863-865)."""
    vc, tc = cfg["vision_config"], cfg["text_config"]
    dt = BF16
    ids = batch["input_ids"]
    labels = batch.get("labels")
    tt = batch.get("token_type_ids")
    am = batch.get("attention_mask")
    if is_training is None:
        is_training = tt is not None and labels is not None
    B, L = ids.shape
    pv = batch["pixel_values"].to(dt)
    # image features (:308-333)
    feats = siglip(P, vc, (pv - 0.5) / 0.5)
    if cfg.get("use_vision_zoe", True):
        if depth is None:
            depth = zoe_depth(zoe_model, pv)
        uv = uv_h_buffer(vc["image_size"], vc["patch_size"], cfg["ego3d_patch_reso"], dt).to(ids.device)
        with torch.no_grad():
            xyz = backproject(batch["intrinsic"].to(dt), depth, uv, vc["patch_size"], cfg["ego3d_patch_reso"])
            enc = freq_encode(xyz, cfg["n_freqs"], dt)
        feats = feats + ego3d_mlp(P, enc)
        if cap is not None:
            cap["depth"], cap["xyz"] = depth, xyz
    img = _lin(feats, P["multi_modal_projector.linear.weight"], P["multi_modal_projector.linear.bias"])
    img = img / (tc["hidden_size"] ** 0.5)
    if cap is not None:
        cap["image_features"] = img
    # embedding merge (:361-387)
    emb = P["language_model.model.embed_tokens.weight"][ids].clone()
    if cfg.get("use_spatial_token"):
        a0, na = cfg["action_token_begin_idx"], cfg["spatial_token_num"]
        sel = (ids >= a0) & (ids < a0 + na)
        emb[sel] = emb[sel] * 0.0 + P["spatial_embed_tokens.weight"][ids[sel] - a0]
    m = (ids == cfg["image_token_index"]).unsqueeze(-1).expand_as(emb)
    emb = emb.masked_scatter(m, img.to(emb.dtype))
    if labels is not None and (labels == 0).any():
        labels = torch.where(ids == 0, -100, labels)
    if am is None:
        am = torch.ones_like(ids)
    mask = mask4d if mask4d is not None else prefix_mask(am, tt if tt is not None else torch.zeros_like(ids),
                                                         is_training, L, dt)
    pos = batch.get("position_ids")  # given: used as is (:367-372); generate passes per-sequence ones
    if pos is None:
        pos = (torch.arange(L, device=ids.device) + 1)[None]
    cos, sin = rope_tables(pos, tc["head_dim"], dt, tc.get("rope_theta", 10000.0))
    h = emb * torch.tensor(tc["hidden_size"] ** 0.5, dtype=dt)
    for i in range(tc["num_hidden_layers"]):
        h = gemma_layer(P, tc, i, h, mask, cos, sin, attn_sink=attn_sink)
    h = rms(h, P["language_model.model.norm.weight"], tc["rms_norm_eps"])
    logits = _lin(h, P["language_model.lm_head.weight"])
    fc = tc["final_logit_softcapping"]
    logits = torch.tanh(logits / fc) * fc
    loss = None
    if labels is not None:
        lf = logits.float()
        sl, sy = lf[..., :-1, :], labels[..., 1:]
        keep = am[:, -sl.shape[1]:] != 0
        loss = F.cross_entropy(sl[keep].reshape(-1, lf.shape[-1]), sy[keep].reshape(-1))
    return loss, logits


def decode_mask(prompt_len: int, L: int, B: int, dtype=BF16):
    """The attention a greedy decode sees, restated without a cache: prompt rows attend to the whole prompt
    (inference prefill mask, modeling_spatialvla.py:291-296 with is_training False), generated token t attends to
    the prompt and every generated token <= t (HybridCache decode steps, modeling_gemma2.py:387-395, 868-873).
    Prompt rows never see generated keys, so their K/V equal the cached prefill's."""
    mn = torch.finfo(dtype).min
    m = torch.full((L, L), mn, dtype=dtype)
    m[:, :prompt_len] = 0.0
    i = torch.arange(L)
    gen = (i[:, None] >= prompt_len) & (i[None, :] >= prompt_len) & (i[None, :] <= i[:, None])
    m = torch.where(gen, torch.zeros((), dtype=dtype), m)
    return m[None, None].expand(B, 1, L, L).contiguous()


@torch.no_grad()
def greedy_decode(P, cfg, batch, zoe_model=None, n_new: int = 4, depth=None):
    """predict_action / generate(do_sample=False) (modeling_spatialvla.py:484-492) restated as full re-forwards:
    positions 1..L (:367-372, :473-474), image features merged every step (same values the cached path reuses),
    next token = argmax of the last position's softcapped bf16 logits.  Returns (tokens [B, n], top-1 minus
    top-2 logit margin [B, n])."""
    ids = batch["input_ids"]
    B, Pl = ids.shape
    am = batch.get("attention_mask")
    toks, margins = [], []
    cur = ids
    for _ in range(n_new):
        Lc = cur.shape[1]
        b = {"input_ids": cur, "pixel_values": batch["pixel_values"], "intrinsic": batch["intrinsic"]}
        mask = decode_mask(Pl, Lc, B).to(cur.device)
        if am is not None:  # padded prompts (generate): per-sequence positions, padded key columns masked
            am_c = torch.cat([am, torch.ones(B, Lc - Pl, dtype=am.dtype, device=am.device)], 1)
            pos = am_c.long().cumsum(-1) - 1                                      # modeling_gemma2.py:1039-1042
            b["position_ids"] = pos.masked_fill(am_c == 0, 1) + 1                 # modeling_spatialvla.py:473-474
            mask = mask.masked_fill((am_c == 0)[:, None, None, :], torch.finfo(mask.dtype).min)
        _, logits = forward(P, cfg, b, zoe_model, is_training=False, depth=depth, mask4d=mask)
        last = logits[:, -1].float()
        top2 = last.topk(2, -1).values
        nxt = last.argmax(-1, keepdim=True)
        toks.append(nxt)
        margins.append((top2[:, 0] - top2[:, 1])[:, None])
        cur = torch.cat([cur, nxt], 1)
    return torch.cat(toks, 1), torch.cat(margins, 1)


def params_from_model_state(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Rename product state-dict keys (4.47 `vision_tower.vision_model.` infix) to the oracle's names."""
    return {k.replace("vision_tower.vision_model.", "vision_tower."): v for k, v in sd.items()}


def build_params(cfg: dict, seed: int, dtype=BF16, requires_grad=True, zoe_model_names=(), init="normal"):
    """Deterministic parameters by name (spatialvla_amd.detinit rules) for every hot-path tensor; init "normal"
    (det_tensor, the tiny fixtures) or "hash" (hash_tensor, the 4B fixtures)."""
    from spatialvla_amd.detinit import det_tensor, hash_tensor
    shapes = param_shapes(cfg)
    P = {}
    for n, shp in shapes.items():
        t = det_tensor(n, shp, seed).to(dtype) if init == "normal" else hash_tensor(n, shp, seed, dtype=dtype)
        if requires_grad and n != "language_model.model.embed_tokens.weight":
            t.requires_grad_(True)
        P[n] = t
    return P


def param_shapes(cfg: dict) -> Dict[str, tuple]:
    vc, tc = cfg["vision_config"], cfg["text_config"]
    H, I, C, p = vc["hidden_size"], vc["intermediate_size"], 3, vc["patch_size"]
    np_ = (vc["image_size"] // p) ** 2
    s = {"vision_tower.embeddings.patch_embedding.weight": (H, C, p, p),
         "vision_tower.embeddings.patch_embedding.bias": (H,),
         "vision_tower.embeddings.position_embedding.weight": (np_, H)}
    for i in range(vc["num_hidden_layers"]):
        b = f"vision_tower.encoder.layers.{i}."
        for n in ("layer_norm1", "layer_norm2"):
            s[b + n + ".weight"] = (H,)
            s[b + n + ".bias"] = (H,)
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            s[b + f"self_attn.{n}.weight"] = (H, H)
            s[b + f"self_attn.{n}.bias"] = (H,)
        s[b + "mlp.fc1.weight"] = (I, H)
        s[b + "mlp.fc1.bias"] = (I,)
        s[b + "mlp.fc2.weight"] = (H, I)
        s[b + "mlp.fc2.bias"] = (H,)
    s["vision_tower.post_layernorm.weight"] = (H,)
    s["vision_tower.post_layernorm.bias"] = (H,)
    Ht = tc["hidden_size"]
    s["multi_modal_projector.linear.weight"] = (Ht, H)
    s["multi_modal_projector.linear.bias"] = (Ht,)
    if cfg.get("use_vision_zoe", True):
        nf = cfg["ego3d_patch_reso"] ** 2 * 3 * (2 * cfg["n_freqs"] + 1)
        e = "position_embedding_3d.position_embedding_head."
        s[e + "0.weight"] = (H, nf)
        s[e + "0.bias"] = (H,)
        s[e + "1.weight"] = (H,)
        s[e + "1.bias"] = (H,)
        s[e + "3.weight"] = (H, H)
        s[e + "3.bias"] = (H,)
    if cfg.get("use_spatial_token"):
        s["spatial_embed_tokens.weight"] = (cfg["spatial_token_num"], Ht)
    V = tc["vocab_size"]
    s["language_model.model.embed_tokens.weight"] = (V, Ht)
    nh, nkv, D, It = tc["num_attention_heads"], tc["num_key_value_heads"], tc["head_dim"], tc["intermediate_size"]
    for i in range(tc["num_hidden_layers"]):
        b = f"language_model.model.layers.{i}."
        s[b + "self_attn.q_proj.weight"] = (nh * D, Ht)
        s[b + "self_attn.k_proj.weight"] = (nkv * D, Ht)
        s[b + "self_attn.v_proj.weight"] = (nkv * D, Ht)
        s[b + "self_attn.o_proj.weight"] = (Ht, nh * D)
        s[b + "mlp.gate_proj.weight"] = (It, Ht)
        s[b + "mlp.up_proj.weight"] = (It, Ht)
        s[b + "mlp.down_proj.weight"] = (Ht, It)
        for n in ("input_layernorm", "post_attention_layernorm", "pre_feedforward_layernorm",
                  "post_feedforward_layernorm"):
            s[b + n + ".weight"] = (Ht,)
    s["language_model.model.norm.weight"] = (Ht,)
    s["language_model.lm_head.weight"] = (V, Ht)
    return s


def build_params_random(cfg: dict, seed: int, dtype=BF16):
    """Fast random parameters (torch CPU generator) for timing the oracle as the CPU baseline —
    same shapes and scale rules as build_params, not bit-identical to it."""
    g = torch.Generator().manual_seed(seed)
    P = {}
    for n, shp in param_shapes(cfg).items():
        if len(shp) >= 2:
            fan = 1
            for d in shp[1:]:
                fan *= d
            t = (torch.randn(shp, generator=g, dtype=torch.float32) / math.sqrt(fan)).to(dtype)
        elif n.endswith("weight") and ("layernorm" in n and n.startswith("language_model") or n.endswith("model.norm.weight")):
            t = torch.zeros(shp, dtype=dtype)
        elif n.endswith("weight"):
            t = torch.ones(shp, dtype=dtype)
        else:
            t = torch.zeros(shp, dtype=dtype)
        if n != "language_model.model.embed_tokens.weight":
            t.requires_grad_(True)
        P[n] = t
    return P


# ---------------------------------------------------------------------------------------- action metrics
def action_metrics(pred: torch.Tensor, labels: torch.Tensor, ranges, actions=None, decode=None) -> Dict[str, float]:
    """train/monkey_patch.py:267-324: pred [B, >= L-1] argmax ids of logits[:, :-1], labels [B, L]; ranges = (trans lo,
    hi, rot lo, hi, grip lo, hi) inclusive token ids.  Accuracies as float32 divisions; with `actions` [B, n, 7] and
    `decode` (SpatialActionTokenizer.decode_token_ids_to_actions), the L1 loss of the decoded predictions."""
    t_lo, t_hi, r_lo, r_hi, g_lo, g_hi = (int(v) for v in ranges)
    L = labels.shape[1]
    shift_pred = pred[:, :L - 1]
    shift_labels = labels[:, 1:]
    mask = (shift_labels >= t_lo) & (shift_labels <= g_hi)                                     # :270-272
    gt, pr = shift_labels[mask], shift_pred[mask]
    ok = gt == pr
    out = {"accuracy": float(ok.sum().float() / mask.sum().float())}                          # :275
    for name, lo, hi in (("translation", t_lo, t_hi), ("rotation", r_lo, r_hi), ("gripper", g_lo, g_hi)):
        m = (gt >= lo) & (gt <= hi)                                                             # :282, :288, :294
        out[name + "_accuracy"] = float((gt[m] == pr[m]).sum().float() / m.sum().float())       # :304-306
    if actions is not None and decode is not None:                                              # :308-311
        gt_a = actions.reshape(-1, 7).to(device="cpu", dtype=torch.float32)
        pa = decode(pr.cpu().numpy().reshape(-1, 3))
        out["l1_loss"] = float(F.l1_loss(torch.tensor(pa), gt_a))
    return out
