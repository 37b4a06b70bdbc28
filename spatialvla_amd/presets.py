"""Canonical configurations and synthetic OXE-shaped batches (SURVEY.md §8 "Canonical shapes").

* `spatialvla_4b()`  — SpatialVLA-4B: PaliGemma2-3B-pt-224 backbone (SigLIP-So400m/14 + Gemma2-2B)
  + ZoeDepth (BEiT-L/16 @384) + Ego3D (reso 2, 8 freqs) + 8194 spatial action tokens, V = 265347.
  Shapes from reference train/spatialvla_pretrain.py:249-319 and scripts/action_config.json:2-15.
* `tiny()` — BASELINE.json configs[0]: the same layer kinds and per-head widths
  (SigLIP head_dim 72, Gemma2 head_dim 256, GQA 2:1) with 2 layers each, so the HIP
  kernels run at their real inner dimensions while the CPU oracle finishes in seconds.
* `synthetic_batch()` — a batch laid out like data/dataset.py:145-153 after the collator
  train/monkey_patch.py:21-41: 256 x <image>, bos, prompt, "\\n", 3*chunk action ids, eos.
"""
import math

import numpy as np

# Gemma / PaliGemma token ids (<image> = 257152, action begin = 257153)
BOS_ID = 2
EOS_ID = 1
NEWLINE_ID = 108
PAD_ID = 0

# scripts/intrinsics.json:3 (640x480 camera), scaled to 224x224 as processing_spatialvla.py:91-95
_K_640 = ((623.588, 0.0, 319.501), (0.0, 623.588, 239.545), (0.0, 0.0, 1.0))


def intrinsic_224():
    sx, sy = 224.0 / 640.0, 224.0 / 480.0
    k = np.array(_K_640, dtype=np.float64)
    k[0] *= sx
    k[1] *= sy
    return k.astype(np.float32)


def _zoe_large():
    # ZoeDepth nyu-kitti: BEiT-L/16 @384 backbone (transformers ZoeDepthConfig defaults)
    return {"model_type": "zoedepth"}


def _zoe_tiny():
    return {
        "model_type": "zoedepth",
        "backbone_config": {
            "model_type": "beit", "hidden_size": 32, "num_hidden_layers": 4, "num_attention_heads": 2,
            "intermediate_size": 64, "image_size": 384, "patch_size": 16, "out_indices": [1, 2, 3, 4],
            "use_relative_position_bias": True, "reshape_hidden_states": False, "layer_scale_init_value": 0.1,
        },
        "neck_hidden_sizes": [16, 32, 64, 128], "fusion_hidden_size": 32, "bottleneck_features": 32,
        "bin_embedding_dim": 16,
    }


def spatialvla_4b(use_vision_zoe=True):
    text_vocab = 257152          # Gemma 256000 + 1024 <loc> + 128 <seg>
    image_token = text_vocab     # <image>
    action_begin = image_token + 1
    n_action = 8194              # scripts/action_config.json:14
    vocab = action_begin + n_action  # 265347
    return dict(
        vision_config=dict(model_type="siglip_vision_model", hidden_size=1152, intermediate_size=4304,
                           num_hidden_layers=27, num_attention_heads=16, patch_size=14, image_size=224,
                           layer_norm_eps=1e-6, hidden_act="gelu_pytorch_tanh", vision_use_head=False,
                           projection_dim=2304),
        text_config=dict(model_type="gemma2", hidden_size=2304, intermediate_size=9216, num_hidden_layers=26,
                         num_attention_heads=8, num_key_value_heads=4, head_dim=256, query_pre_attn_scalar=256,
                         attn_logit_softcapping=50.0, final_logit_softcapping=30.0, sliding_window=4096,
                         rms_norm_eps=1e-6, rope_theta=10000.0, hidden_activation="gelu_pytorch_tanh",
                         vocab_size=vocab, pad_token_id=0, bos_token_id=BOS_ID, eos_token_id=EOS_ID,
                         tie_word_embeddings=False, max_position_embeddings=8192),
        vision_zoe_config=_zoe_large() if use_vision_zoe else None,
        image_token_index=image_token, vocab_size=vocab, projection_dim=2304, hidden_size=2304,
        action_token_begin_idx=action_begin, spatial_token_num=n_action, use_spatial_token=True,
        ego3d_patch_reso=2, n_freqs=8, use_vision_zoe=use_vision_zoe, pad_token_id=0,
    )


def tiny(use_vision_zoe=True):
    text_vocab = 512
    image_token = text_vocab
    action_begin = image_token + 1
    n_action = 64
    vocab = action_begin + n_action  # 577: odd, exercises the lm_head vocab tail
    return dict(
        vision_config=dict(model_type="siglip_vision_model", hidden_size=144, intermediate_size=288,
                           num_hidden_layers=2, num_attention_heads=2, patch_size=14, image_size=224,
                           layer_norm_eps=1e-6, hidden_act="gelu_pytorch_tanh", vision_use_head=False,
                           projection_dim=256),
        text_config=dict(model_type="gemma2", hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                         num_attention_heads=2, num_key_value_heads=1, head_dim=256, query_pre_attn_scalar=256,
                         attn_logit_softcapping=50.0, final_logit_softcapping=30.0, sliding_window=4096,
                         rms_norm_eps=1e-6, rope_theta=10000.0, hidden_activation="gelu_pytorch_tanh",
                         vocab_size=vocab, pad_token_id=0, bos_token_id=BOS_ID, eos_token_id=EOS_ID,
                         tie_word_embeddings=False, max_position_embeddings=8192),
        vision_zoe_config=_zoe_tiny() if use_vision_zoe else None,
        image_token_index=image_token, vocab_size=vocab, projection_dim=256, hidden_size=256,
        action_token_begin_idx=action_begin, spatial_token_num=n_action, use_spatial_token=True,
        ego3d_patch_reso=2, n_freqs=8, use_vision_zoe=use_vision_zoe, pad_token_id=0,
    )


def synthetic_batch(cfg: dict, batch: int, seed: int, prompt_len: int = 41, chunk: int = 4,
                    pad_to: int = 0, ragged: bool = False):
    """Synthetic OXE-shaped training batch (numpy; SURVEY.md §8(d) "Synthetic inputs").

    input_ids = 256 x <image> | bos | prompt | "\\n" | 3*chunk action ids | eos, token_type 1 on the
    suffix (actions + eos), labels = ids on the suffix else -100 (processing_spatialvla.py:189-191),
    attention_mask = ids != pad (monkey_patch.py:33).  With `ragged`, prompt lengths vary per row and
    rows are right-padded with pad id 0 / label -100 / token_type 0 exactly as the collator does.
    """
    rng = np.random.default_rng(seed)
    vc = cfg["vision_config"]
    n_img = (vc["image_size"] // vc["patch_size"]) ** 2
    text_vocab = cfg["image_token_index"]
    a0, na = cfg["action_token_begin_idx"], cfg["spatial_token_num"]
    rows = []
    for b in range(batch):
        pl = prompt_len if not ragged else int(rng.integers(max(1, prompt_len // 2), prompt_len + 1))
        prompt = rng.integers(3, text_vocab, size=pl)
        acts = rng.integers(a0, a0 + na, size=3 * chunk)
        prefix = np.concatenate([np.full(n_img, cfg["image_token_index"]), [BOS_ID], prompt, [NEWLINE_ID]])
        suffix = np.concatenate([acts, [EOS_ID]])
        rows.append((prefix, suffix))
    L = max(len(p) + len(s) for p, s in rows)
    L = max(L, pad_to)
    ids = np.full((batch, L), PAD_ID, dtype=np.int64)
    tt = np.zeros((batch, L), dtype=np.int64)
    labels = np.full((batch, L), -100, dtype=np.int64)
    for b, (p, s) in enumerate(rows):
        n = len(p) + len(s)
        ids[b, :n] = np.concatenate([p, s])
        tt[b, len(p):n] = 1
        labels[b, len(p):n] = s
    attn = (ids != PAD_ID).astype(np.int64)
    hw = vc["image_size"]
    pixel_values = rng.random((batch, 3, hw, hw), dtype=np.float32)
    k = np.broadcast_to(intrinsic_224(), (batch, 3, 3)).copy()
    return dict(input_ids=ids, token_type_ids=tt, labels=labels, attention_mask=attn,
                pixel_values=pixel_values, intrinsic=k)


def num_image_tokens(cfg: dict) -> int:
    vc = cfg["vision_config"]
    return (vc["image_size"] // vc["patch_size"]) ** 2


def gemma_normalizer_bf16(hidden: int) -> float:
    """tensor(hidden**0.5, dtype=bf16) as a python float (modeling_gemma2.py:741)."""
    import torch
    return float(torch.tensor(math.sqrt(hidden), dtype=torch.bfloat16))
