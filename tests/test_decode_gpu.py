"""KV-cached greedy decode: the decode attention kernel against an fp32 eager reference and
against the prefill flash kernel, and the cached predict_action / forward(past_key_values=...) against full
re-forwards on the same weights (reference generate path: model/modeling_spatialvla.py:440-492)."""
import os

import pytest
import torch
from safetensors.torch import load_file

import harness as H
from test_kernels_gpu import _r, _ref_attn

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.mark.parametrize("D,Hq,Hkv,Lk,Lq,window,cap", [
    (256, 8, 4, 300, 1, 0, 50.0),     # Gemma2-2B widths, one new token after a 299-token prompt
    (256, 8, 4, 303, 4, 0, 50.0),     # four new tokens at once (causal among themselves)
    (256, 2, 1, 560, 1, 0, 50.0),
    (256, 8, 2, 1000, 2, 0, 50.0),    # GQA group of 4
    (128, 2, 2, 77, 1, 16, 0.0),      # sliding window masks the far keys
    (64, 2, 1, 129, 3, 0, 0.0),
    (256, 8, 4, 4500, 1, 4096, 50.0),  # past the Gemma2 sliding window
])
def test_attn_decode_kernel(cuda, D, Hq, Hkv, Lk, Lq, window, cap):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(11)
    B, cap_rows = 2, Lk + 7
    kd = Hkv * D
    kc = _r(B, cap_rows, kd)
    vc = _r(B, cap_rows, kd)
    qfull = _r(B, Lk, Hq * D)
    P = Lk - Lq - 5 if Lk - Lq - 5 > 0 else 0
    cls = torch.full((B, cap_rows), 2, dtype=torch.uint8, device=cuda)
    cls[:, :P] = 0
    cls[:, P:Lk] = 1
    cls[1, 3] = 2  # a padded prompt key
    q = qfull[:, Lk - Lq:].reshape(B * Lq, Hq * D).contiguous()
    out = torch.empty(B * Lq, Hq * D, dtype=BF, device=cuda)
    Kn.attn_decode(q, Lq, kc, vc, Lk, Hq, Hkv, D, 1 / 16, cap, cls, window, out)
    ref = _ref_attn(qfull.view(B, Lk, Hq, D), kc[:, :Lk].view(B, Lk, Hkv, D), vc[:, :Lk].view(B, Lk, Hkv, D),
                    1 / 16, cap, cls[:, :Lk], window)[:, Lk - Lq:]
    assert H.rel_l2(out.view(B, Lq, Hq, D), ref) < 1e-2
    if D == 256 and Lk <= 8192:
        # the same rows from the prefill flash kernel (what the uncached re-forward computes)
        qkv = torch.cat([qfull.view(B * Lk, -1), kc[:, :Lk].reshape(B * Lk, kd), vc[:, :Lk].reshape(B * Lk, kd)], 1)
        cls_l = cls[:, :Lk].contiguous()  # held: attn_args keeps only its pointer
        a = Kn.attn_args(B, Lk, Hq, Hkv, D, qkv[:, :Hq * D], qkv.stride(0), qkv[:, Hq * D:Hq * D + kd],
                         qkv.stride(0), qkv[:, Hq * D + kd:], qkv.stride(0), 1 / 16, cap, cls_l, window)
        full = torch.empty(B * Lk, Hq * D, dtype=BF, device=cuda)
        Kn.attn_fwd(a, full, torch.empty(B, Hq, Lk, device=cuda))
        rows = full.view(B, Lk, Hq * D)[:, Lk - Lq:].float()
        assert H.rel_l2(out.view(B, Lq, Hq * D), rows) < 5e-3


def test_attn_decode_rejects_bad_args(cuda):
    from spatialvla_amd import kernels as Kn
    kc = _r(1, 64, 256)
    q = _r(1, 3 * 256)  # Hq=3, Hkv=1: group 3 unsupported
    with pytest.raises(RuntimeError):
        Kn.attn_decode(q, 1, kc, kc, 10, 3, 1, 256, 1 / 16, 50.0, None, 0, torch.empty_like(q))


def _tiny_model(cuda):
    g = load_file(os.path.join(os.path.dirname(__file__), "golden", "tiny_train.safetensors"))
    model = H.build_hip_model(H.cfg_dict("tiny"), "cuda:0")
    model.predict_depth = lambda p: g["out.depth"].to(cuda)
    return model, g


def test_predict_action_cached_equals_uncached(cuda):
    """Greedy tokens of the KV-cached decode equal those of full re-forwards over prompt + generated tokens."""
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"][:, :-13]  # prompt only (prefix)
    inputs = {"input_ids": ids, "pixel_values": g["in.pixel_values"], "intrinsic": g["in.intrinsic"]}
    cached = model.predict_action(inputs, max_new_tokens=8, eos_token_id=-1)
    full = model.predict_action_uncached(inputs, max_new_tokens=8, eos_token_id=-1)
    assert cached.shape == (2, 8)
    assert torch.equal(cached, full), (cached, full)


def test_predict_action_eos_pads_finished(cuda):
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"][:, :-13]
    inputs = {"input_ids": ids, "pixel_values": g["in.pixel_values"], "intrinsic": g["in.intrinsic"]}
    free = model.predict_action(inputs, max_new_tokens=4, eos_token_id=-1)
    eos = int(free[0, 1])  # make sequence 0 finish at its second token
    out = model.predict_action(inputs, max_new_tokens=4, eos_token_id=eos)
    ref = model.predict_action_uncached(inputs, max_new_tokens=4, eos_token_id=eos)
    assert torch.equal(out, ref)
    assert out[0, 1] == eos and bool((out[0, 2:] == max(model.pad_token_id, 0)).all())


def test_forward_past_key_values_matches_reforward(cuda):
    """forward(use_cache=True) then forward(past_key_values=cache) on two more tokens gives the logits of a full
    forward whose appended tokens see the prompt and earlier tokens only (the HybridCache decode semantics)."""
    from spatialvla_amd.modeling_gemma2 import Gemma2KVCache, KVMask
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"].to(cuda)
    B, L = ids.shape
    P = L - 13
    pv, intr = g["in.pixel_values"].to(cuda), g["in.intrinsic"].to(cuda)
    with torch.no_grad():
        o1 = model(input_ids=ids[:, :P], pixel_values=pv, intrinsic=intr, use_cache=True)
        cache = o1.past_key_values
        assert isinstance(cache, Gemma2KVCache) and cache.get_seq_length() == P
        o2 = model(input_ids=ids[:, P:P + 1], past_key_values=cache)
        o3 = model(input_ids=ids[:, P + 1:P + 3], past_key_values=cache)
        assert cache.get_seq_length() == P + 3
        cls = torch.ones(B, P + 3, dtype=torch.uint8, device=cuda)
        cls[:, :P] = 0
        ref = model(input_ids=ids[:, :P + 3], pixel_values=pv, intrinsic=intr, kv_mask=KVMask(cls)).logits
    assert H.rel_l2(o1.logits, ref[:, :P]) < H.LOGITS_TOL  # prompt rows never see the appended tokens
    assert H.rel_l2(o2.logits, ref[:, P:P + 1]) < H.LOGITS_TOL
    assert H.rel_l2(o3.logits, ref[:, P + 1:P + 3]) < H.LOGITS_TOL
    assert torch.equal(o3.logits.float().argmax(-1), ref[:, P + 1:P + 3].float().argmax(-1))
