"""Generate golden vectors by running the REFERENCE's own eager code (container only).

TEST INFRASTRUCTURE ONLY — never imported by the product package, never shipped as a
product path.  Requires /root/reference (absent on the GPU box); the fixtures it writes
under tests/golden/ are what travels.

Run:  python oracle/gen_golden.py            (writes tests/golden/*.safetensors + *.json)

What is pinned (SURVEY.md §8(c) "Golden-vector plan"):
* tiny_train  — BASELINE configs[0] tiny model, deterministic weights (spatialvla_amd.detinit,
  regenerated from names, so weights are not committed), synthetic OXE batch B=2:
  training-mode forward (prefix-LM mask, reference modeling_spatialvla.py:293,304-305),
  loss, logits, image features, depth, every trainable gradient, action argmax.
* tiny_prefill — same weights/inputs, inference mask (fully bidirectional prefix,
  modeling_spatialvla.py:294), logits only.
* tiny_ragged — right-padded ragged batch (collator monkey_patch.py:21-41) to pin Q2
  (padded key columns un-masked in training).
* layer4b_* — one Gemma2 decoder layer and one SigLIP encoder layer at SpatialVLA-4B
  widths (B=1, L=312 / 256): outputs and input-grads in full, param-grad norms.
* full4b — the whole SpatialVLA-4B model (SigLIP-So400m + ZoeDepth BEiT-L + Ego3D + Gemma2-2B, V=265347) with
  counter-hash weights (spatialvla_amd.detinit.hash_init_: bit-identical on CPU and GPU, so 8 GB of weights
  never travel), one training forward+backward at B=1, L=312: loss, per-row argmax / top-2 margin / lse, the
  logits of the 13 labelled rows over the action-token range, logits of all rows at 256 fixed columns, Zoe depth,
  xyz, image features, every trainable gradient's norm and a linear sketch of it (a hash-signed +-1 sum of the
  rows of a matrix, a 1-D gradient in full).
* decode_tiny / decode4b — greedy decode (predict_action, modeling_spatialvla.py:484-492) by the reference model
  itself, restated without a cache (the HybridCache constructor does not run under transformers 5): each step
  re-forwards prompt + generated tokens with the 4-D mask the cached path sees (prompt bidirectional,
  :291-296; generated tokens causal, modeling_gemma2.py:387-395), next token = argmax of the last row.
"""
import json
import os
import sys

import numpy as np
import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from spatialvla_amd import presets  # noqa: E402
from spatialvla_amd.detinit import deterministic_init_, det_tensor, hash_init_  # noqa: E402
import ref_shim  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
SEED = 1234


def build_reference_model(cfgdict, init="normal"):
    msv, csv = ref_shim.install()
    cfg = csv.SpatialVLAConfig(**json.loads(json.dumps(cfgdict)))
    ref_shim.configure_eager(cfg)
    torch.manual_seed(0)
    model = msv.SpatialVLAForConditionalGeneration(cfg)
    model = model.to(torch.bfloat16)
    if init == "normal":
        deterministic_init_(model, seed=SEED)
    else:
        hash_init_(model, seed=SEED)
    model.train()
    if cfg.use_vision_zoe:
        model.vision_zoe_model.eval()
        for p in model.vision_zoe_model.parameters():
            p.requires_grad_(False)
    model.language_model.model.embed_tokens.weight.requires_grad_(False)  # spatialvla_pretrain.py:342
    return model, cfg


def batch_tensors(b):
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    t["pixel_values"] = t["pixel_values"].to(torch.bfloat16)   # SURVEY Q8 (DeepSpeed bf16 input cast)
    t["intrinsic"] = t["intrinsic"].to(torch.bfloat16)
    return t


def run_train(model, t):
    cap = {}
    if model.config.use_vision_zoe:
        orig_bp = model.backproject_patch

        def bp(K, depth, patch_size=14, reso=2):
            cap["depth"] = depth.detach().clone()
            out = orig_bp(K, depth, patch_size=patch_size, reso=reso)
            cap["xyz"] = out.detach().clone()
            return out
        model.backproject_patch = bp
    orig_gif = model.get_image_features

    def gif(pv, k):
        out = orig_gif(pv, k)
        cap["image_features"] = out.detach().clone()
        return out
    model.get_image_features = gif
    model.zero_grad(set_to_none=True)
    out = model(input_ids=t["input_ids"], pixel_values=t["pixel_values"], intrinsic=t["intrinsic"],
                attention_mask=t["attention_mask"], token_type_ids=t["token_type_ids"], labels=t["labels"],
                use_cache=False, return_dict=True)
    out.loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    model.get_image_features = orig_gif
    if "depth" in cap:
        model.backproject_patch = orig_bp
    return out, cap, grads


def gen_tiny(ragged=False):
    cfgd = presets.tiny()
    model, cfg = build_reference_model(cfgd)
    b = presets.synthetic_batch(cfgd, batch=2 if not ragged else 3, seed=7 if not ragged else 11, ragged=ragged)
    t = batch_tensors(b)
    out, cap, grads = run_train(model, t)
    logits = out.logits.detach()
    shift_argmax = logits[:, :-1].float().argmax(-1)
    top2 = logits[:, :-1].float().topk(2, dim=-1).values
    d = {f"in.{k}": v.contiguous() for k, v in t.items()}
    d.update({"out.loss": out.loss.detach().float().reshape(1), "out.logits": logits.contiguous(),
              "out.argmax": shift_argmax.contiguous(), "out.top2_margin": (top2[..., 0] - top2[..., 1]).contiguous(),
              "out.image_features": cap["image_features"].contiguous()})
    if "depth" in cap:
        d["out.depth"] = cap["depth"].contiguous()
        d["out.xyz"] = cap["xyz"].contiguous()
    for n, g in grads.items():
        if ragged:  # summaries only (keeps the fixture small)
            d[f"gradnorm.{n}"] = g.float().norm().reshape(1)
        else:
            d[f"grad.{n}"] = g.contiguous()
    if ragged:
        d.pop("out.image_features", None)
        d.pop("out.xyz", None)
    name = "tiny_ragged" if ragged else "tiny_train"
    save_file(d, os.path.join(OUT, f"{name}.safetensors"))
    print(name, "loss", out.loss.item(), "n_grads", len(grads),
          "bytes", os.path.getsize(os.path.join(OUT, f"{name}.safetensors")))

    if not ragged:
        with torch.no_grad():
            o2 = model(input_ids=t["input_ids"], pixel_values=t["pixel_values"], intrinsic=t["intrinsic"],
                       attention_mask=t["attention_mask"], use_cache=False, return_dict=True)
        save_file({"out.logits": o2.logits.contiguous()}, os.path.join(OUT, "tiny_prefill.safetensors"))
        print("tiny_prefill saved")
    return cfgd


def gen_layer4b():
    """One Gemma2 decoder layer + one SigLIP encoder layer at 4B widths, via reference classes."""
    msv, csv = ref_shim.install()
    from model.modeling_gemma2 import Gemma2DecoderLayer
    cfgd = presets.spatialvla_4b(use_vision_zoe=False)
    cfg = csv.SpatialVLAConfig(**json.loads(json.dumps(cfgd)))
    ref_shim.configure_eager(cfg)
    tc = cfg.text_config
    res = {}
    # ---- Gemma2 layer 1 (global layer) and 0 (sliding layer) at B=1, L=312, prefix 299 ----
    L, P = 312, 299
    pos = (torch.arange(L) + 1)[None]
    h = det_tensor("gemma.in", (1, L, tc.hidden_size), SEED, scale=1.0).to(torch.bfloat16).requires_grad_(True)
    gout = det_tensor("gemma.gout", (1, L, tc.hidden_size), SEED, scale=1.0).to(torch.bfloat16)
    # training prefix-LM mask, reference _update_causal_mask :291-305 with token_type = (i >= P)
    mn = torch.finfo(torch.bfloat16).min
    m = torch.full((L, L), mn, dtype=torch.bfloat16).triu(1)
    m[:, :P] = 0
    mask = m[None, None]
    for li in (0, 1):
        layer = Gemma2DecoderLayer(tc, layer_idx=li).to(torch.bfloat16)
        deterministic_init_(layer, seed=SEED, prefix=f"language_model.model.layers.{li}.")
        layer.train()
        h.grad = None
        y = layer(h, attention_mask=mask, position_ids=pos, use_cache=False)[0]
        (y.float() * gout.float()).sum().backward()
        if li == 1:
            res[f"gemma{li}.out"] = y.detach().contiguous()
            res[f"gemma{li}.dx"] = h.grad.detach().clone().contiguous()
        else:
            res[f"gemma{li}.out_rows"] = y.detach()[0, ::13].contiguous()
            res[f"gemma{li}.dx_rows"] = h.grad.detach()[0, ::13].contiguous()
            res[f"gemma{li}.out_norm"] = y.float().norm().reshape(1)
            res[f"gemma{li}.dx_norm"] = h.grad.float().norm().reshape(1)
        for n, p in layer.named_parameters():
            res[f"gemma{li}.gradnorm.{n}"] = p.grad.float().norm().reshape(1)
            res[f"gemma{li}.gradrow0.{n}"] = p.grad.reshape(p.grad.shape[0], -1)[0, :64].contiguous()
    res["gemma.in"] = h.detach().contiguous()
    # ---- SigLIP encoder layer at 1152 width, 256 tokens ----
    from transformers.models.siglip.modeling_siglip import SiglipEncoderLayer
    vc = cfg.vision_config
    vc._attn_implementation = "eager"
    sl = SiglipEncoderLayer(vc).to(torch.bfloat16)
    deterministic_init_(sl, seed=SEED, prefix="vision_tower.vision_model.encoder.layers.0.")
    sl.train()
    x = det_tensor("siglip.in", (1, 256, vc.hidden_size), SEED, scale=1.0).to(torch.bfloat16).requires_grad_(True)
    go = det_tensor("siglip.gout", (1, 256, vc.hidden_size), SEED, scale=1.0).to(torch.bfloat16)
    y = sl(x, attention_mask=None)
    y = y[0] if isinstance(y, tuple) else y
    (y.float() * go.float()).sum().backward()
    res["siglip.in"] = x.detach().contiguous()
    res["siglip.out"] = y.detach().contiguous()
    res["siglip.dx"] = x.grad.detach().contiguous()
    for n, p in sl.named_parameters():
        res[f"siglip.gradnorm.{n}"] = p.grad.float().norm().reshape(1)
    save_file(res, os.path.join(OUT, "layer4b.safetensors"))
    print("layer4b bytes", os.path.getsize(os.path.join(OUT, "layer4b.safetensors")))


def sketch(name, g):
    from spatialvla_amd.detinit import hash_tensor
    g = g.float()
    if g.dim() < 2:
        return g
    r = hash_tensor(name + "#sketch", (g.shape[0],), 0, device=g.device, dtype=torch.float32).sign()
    return r @ g.reshape(g.shape[0], -1)


def decode_mask(prompt_len, L, B):
    """additive [B,1,L,L]: prompt rows see the prompt (inference prefill, modeling_spatialvla.py:291-296),
    generated row t sees the prompt and generated tokens <= t (cached decode, modeling_gemma2.py:387-395)."""
    mn = torch.finfo(torch.bfloat16).min
    m = torch.full((L, L), mn, dtype=torch.bfloat16)
    m[:, :prompt_len] = 0.0
    i = torch.arange(L)
    gen = (i[:, None] >= prompt_len) & (i[None, :] >= prompt_len) & (i[None, :] <= i[:, None])
    m = torch.where(gen, torch.zeros((), dtype=torch.bfloat16), m)
    return m[None, None].expand(B, 1, L, L).contiguous()


@torch.no_grad()
def ref_greedy(model, ids, pv, intr, n_new, depth_cap=None):
    """Greedy decode through the reference forward (4-D mask passthrough, :288-289), no cache."""
    B, P = ids.shape
    cur, toks, margins = ids, [], []
    for step in range(n_new):
        Lc = cur.shape[1]
        out = model(input_ids=cur, pixel_values=pv, intrinsic=intr, attention_mask=decode_mask(P, Lc, B),
                    use_cache=False, return_dict=True)
        last = out.logits[:, -1].float()
        top2 = last.topk(2, -1).values
        nxt = last.argmax(-1, keepdim=True)
        toks.append(nxt)
        margins.append((top2[:, 0] - top2[:, 1])[:, None])
        cur = torch.cat([cur, nxt], 1)
        print(f"  decode step {step}: tokens {nxt.view(-1).tolist()} margins {margins[-1].view(-1).tolist()}",
              flush=True)
    return torch.cat(toks, 1), torch.cat(margins, 1)


def gen_decode_tiny():
    cfgd = presets.tiny()
    model, cfg = build_reference_model(cfgd)
    model.eval()
    b = presets.synthetic_batch(cfgd, batch=2, seed=7)
    t = batch_tensors(b)
    P = int((t["token_type_ids"][0] == 0).sum())
    ids = t["input_ids"][:, :P]
    cap = {}
    orig_bp = model.backproject_patch

    def bp(K, depth, patch_size=14, reso=2):
        cap.setdefault("depth", depth.detach().clone())
        return orig_bp(K, depth, patch_size=patch_size, reso=reso)
    model.backproject_patch = bp
    toks, margins = ref_greedy(model, ids, t["pixel_values"], t["intrinsic"], 6)
    save_file({"in.input_ids": ids.contiguous(), "in.pixel_values": t["pixel_values"].contiguous(),
               "in.intrinsic": t["intrinsic"].contiguous(), "out.depth": cap["depth"].contiguous(),
               "out.tokens": toks.contiguous(), "out.margins": margins.contiguous()},
              os.path.join(OUT, "decode_tiny.safetensors"))
    print("decode_tiny tokens", toks.tolist())


def padded_decode_mask(am, n_new):
    """additive [B,1,L,L] of a padded greedy decode: the inference prefill mask (bidirectional, padded key columns
    masked: modeling_spatialvla.py:291-305 with is_training False) for prompt rows; generated row t sees the valid
    prompt keys and generated tokens <= t (HybridCache decode, modeling_gemma2.py:387-395)."""
    B, P = am.shape
    L = P + n_new
    m = decode_mask(P, L, B).clone()
    mn = torch.finfo(torch.bfloat16).min
    pad_cols = torch.cat([am == 0, torch.zeros(B, n_new, dtype=torch.bool)], 1)  # [B, L]
    return torch.where(pad_cols[:, None, None, :], torch.full((), mn, dtype=torch.bfloat16), m)


@torch.no_grad()
def ref_greedy_padded(model, ids, am, pv, intr, n_new):
    """Greedy decode of a left-padded batch through the reference forward, no cache: per-sequence positions as
    prepare_inputs_for_generation derives them (attention_mask.cumsum(-1) - 1, pads 1, modeling_gemma2.py:1039-1042;
    + 1, modeling_spatialvla.py:473-474), the generate-time attention mask extended by ones."""
    B, P = ids.shape
    cur, toks, margins = ids, [], []
    for step in range(n_new):
        Lc = cur.shape[1]
        am_c = torch.cat([am, torch.ones(B, Lc - P, dtype=am.dtype)], 1)
        pos = am_c.long().cumsum(-1) - 1
        pos.masked_fill_(am_c == 0, 1)
        pos = pos + 1
        mask = padded_decode_mask(am, Lc - P)
        out = model(input_ids=cur, pixel_values=pv, intrinsic=intr, attention_mask=mask, position_ids=pos,
                    use_cache=False, return_dict=True)
        last = out.logits[:, -1].float()
        top2 = last.topk(2, -1).values
        nxt = last.argmax(-1, keepdim=True)
        toks.append(nxt)
        margins.append((top2[:, 0] - top2[:, 1])[:, None])
        cur = torch.cat([cur, nxt], 1)
        print(f"  padded decode step {step}: tokens {nxt.view(-1).tolist()} margins {margins[-1].view(-1).tolist()}",
              flush=True)
    return torch.cat(toks, 1), torch.cat(margins, 1)


def gen_decode_padded():
    """decode_padded: B=3 prompts of different lengths, left-padded (pad id 0, attention_mask 0), greedy 6 tokens."""
    cfgd = presets.tiny()
    model, cfg = build_reference_model(cfgd)
    model.eval()
    b = presets.synthetic_batch(cfgd, batch=3, seed=21)
    t = batch_tensors(b)
    P = int((t["token_type_ids"][0] == 0).sum())
    ids = t["input_ids"][:, :P].clone()
    am = torch.ones_like(ids)
    n_img = int((ids[0] == cfg.image_token_index).sum())
    for row, drop in ((0, 5), (2, 2)):  # shorter prompts: drop text tokens after the image block, pad on the left
        keep = torch.cat([ids[row, :n_img + 1], ids[row, n_img + 1 + drop:]])
        ids[row] = torch.cat([torch.zeros(drop, dtype=ids.dtype), keep])
        am[row, :drop] = 0
    cap = {}
    orig_bp = model.backproject_patch

    def bp(K, depth, patch_size=14, reso=2):
        cap.setdefault("depth", depth.detach().clone())
        return orig_bp(K, depth, patch_size=patch_size, reso=reso)
    model.backproject_patch = bp
    toks, margins = ref_greedy_padded(model, ids, am, t["pixel_values"], t["intrinsic"], 6)
    save_file({"in.input_ids": ids.contiguous(), "in.attention_mask": am.contiguous(),
               "in.pixel_values": t["pixel_values"].contiguous(), "in.intrinsic": t["intrinsic"].contiguous(),
               "out.depth": cap["depth"].contiguous(), "out.tokens": toks.contiguous(),
               "out.margins": margins.contiguous()}, os.path.join(OUT, "decode_padded.safetensors"))
    print("decode_padded tokens", toks.tolist())


def gen_full4b():
    """The whole 4B model, hash-initialised, B=1 training step + greedy decode of 4 tokens."""
    import time
    cfgd = presets.spatialvla_4b()
    t0 = time.time()
    model, cfg = build_reference_model(cfgd, init="hash")
    print(f"4B reference model built + hash-initialised in {time.time() - t0:.0f}s", flush=True)
    b = presets.synthetic_batch(cfgd, batch=1, seed=4242)
    t = batch_tensors(b)
    t0 = time.time()
    out, cap, grads = run_train(model, t)
    print(f"4B train fwd+bwd {time.time() - t0:.0f}s loss {out.loss.item():.6f}", flush=True)
    logits = out.logits.detach()                 # [1, L, V] bf16 (softcapped)
    lf = logits[0, :-1].float()                  # shifted rows
    top2 = lf.topk(2, -1).values
    lse = torch.logsumexp(lf, -1)
    labels = t["labels"][0, 1:]
    rows = torch.nonzero(labels != -100).view(-1)
    a0, na = cfg.action_token_begin_idx, cfg.spatial_token_num
    g = torch.Generator().manual_seed(5)
    cols = torch.randperm(logits.shape[-1], generator=g)[:256].sort().values
    d = {f"in.{k}": v.contiguous() for k, v in t.items()}
    d.update({"out.loss": out.loss.detach().float().reshape(1),
              "out.argmax": lf.argmax(-1).contiguous(), "out.top2_margin": (top2[:, 0] - top2[:, 1]).contiguous(),
              "out.lse": lse.contiguous(), "out.label_rows": rows.contiguous(),
              "out.action_logits": logits[0, rows, a0:a0 + na].contiguous(),
              "out.cols": cols.contiguous(), "out.col_logits": logits[0][:, cols].contiguous(),
              "out.image_features": cap["image_features"].contiguous(),
              "out.depth": cap["depth"].float().contiguous(), "out.xyz": cap["xyz"].float().contiguous()})
    for n, gr in grads.items():
        d[f"gradnorm.{n}"] = gr.float().norm().reshape(1)
        # a linear sketch of the whole gradient: a +-1 combination of the rows of a matrix (signs from the counter
        # hash, so the GPU test regenerates them), a 1-D gradient in full.  Plain column sums are a poor sketch:
        # softmax / norm backward make many gradients' row sums cancel to rounding noise.
        d[f"gradsum.{n}"] = sketch(n, gr).contiguous()
    del grads, out
    model.zero_grad(set_to_none=True)
    model.eval()
    P = int((t["token_type_ids"][0] == 0).sum())
    ids = t["input_ids"][:, :P]
    t0 = time.time()
    toks, margins = ref_greedy(model, ids, t["pixel_values"], t["intrinsic"], 4)
    print(f"4B greedy decode {time.time() - t0:.0f}s tokens {toks.tolist()}", flush=True)
    d["decode.tokens"] = toks.contiguous()
    d["decode.margins"] = margins.contiguous()
    save_file(d, os.path.join(OUT, "full4b.safetensors"))
    print("full4b bytes", os.path.getsize(os.path.join(OUT, "full4b.safetensors")))


if __name__ == "__main__":
    if not ref_shim.reference_available():
        print("reference not present; nothing to do")
        sys.exit(0)
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(os.cpu_count())
    which = sys.argv[1:] or ["tiny", "ragged", "layer4b", "decode_tiny", "full4b"]
    if "tiny" in which:
        gen_tiny(False)
    if "ragged" in which:
        gen_tiny(True)
    if "layer4b" in which:
        gen_layer4b()
    if "decode_tiny" in which:
        gen_decode_tiny()
    if "decode_padded" in which:
        gen_decode_padded()
    if "full4b" in which:
        gen_full4b()
