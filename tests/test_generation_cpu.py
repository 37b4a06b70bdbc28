"""Host-side surface of the drop-in model that needs no kernel launch (CPU):
  * prepare_inputs_for_generation (reference model/modeling_spatialvla.py:445-482 over modeling_gemma2.py:1015-1091):
    slicing to the uncached tokens, per-sequence positions from the attention mask + 1, pixel values only at the
    first step, intrinsic passed through;
  * the gradient-checkpointing calls of the reference training script (train/spatialvla_pretrain.py:331-334) and
    gradient_checkpointing_enable() set the flag the decoder's recompute path reads (tests/test_model_gpu.py
    test_gradient_checkpointing_recomputes_bitwise runs it);
  * a grad-enabled attention forward with per-sequence RoPE tables (padded prompts) is refused up front: the
    attention backward's RoPE transpose reads table row = position in the sequence."""
import pytest
import torch

import harness as H


@pytest.fixture(scope="module")
def tiny_model():
    from spatialvla_amd import SpatialVLAConfig
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    return SpatialVLAForConditionalGeneration(SpatialVLAConfig(**H.cfg_dict("tiny"))).to(torch.bfloat16)


def _reference_positions(am):
    """modeling_gemma2.py:1039-1040, then modeling_spatialvla.py:473-474."""
    pos = am.long().cumsum(-1) - 1
    pos.masked_fill_(am == 0, 1)
    return pos + 1


def test_prepare_inputs_for_generation_steps(tiny_model):
    m = tiny_model
    B, P = 2, 7
    ids = torch.randint(3, 400, (B, P))
    am = torch.ones(B, P, dtype=torch.int64)
    am[1, :2] = 0  # left padding of the second prompt
    pv, intr = torch.rand(B, 3, 224, 224), torch.eye(3).expand(B, 3, 3)
    cache = m.new_cache(B, P + 4)
    # prefill step
    mi = m.prepare_inputs_for_generation(ids, past_key_values=cache, cache_position=torch.arange(P),
                                         pixel_values=pv, intrinsic=intr, attention_mask=am)
    assert torch.equal(mi["input_ids"], ids) and mi["inputs_embeds"] is None
    assert torch.equal(mi["position_ids"], _reference_positions(am))
    assert mi["pixel_values"] is pv and mi["intrinsic"] is intr and mi["past_key_values"] is cache
    assert mi["attention_mask"] is am and mi["use_cache"]
    # first decode step: only the new token, its position, no pixels
    ids2 = torch.cat([ids, torch.tensor([[11], [12]])], 1)
    am2 = torch.cat([am, torch.ones(B, 1, dtype=torch.int64)], 1)
    cache.seen_tokens = P
    mi = m.prepare_inputs_for_generation(ids2, past_key_values=cache, cache_position=torch.tensor([P]),
                                         pixel_values=pv, intrinsic=intr, attention_mask=am2)
    assert torch.equal(mi["input_ids"], ids2[:, P:])
    assert torch.equal(mi["position_ids"], _reference_positions(am2)[:, -1:])
    assert mi["position_ids"].tolist() == [[P + 1], [P - 1]]
    assert "pixel_values" not in mi or mi["pixel_values"] is None


def test_generate_rejects_sampling(tiny_model):
    with pytest.raises(NotImplementedError):
        tiny_model.generate(torch.ones(1, 3, dtype=torch.int64), do_sample=True)


def test_gradient_checkpointing_surface_accepted(tiny_model):
    m = tiny_model
    m.vision_tower.gradient_checkpointing = True           # train/spatialvla_pretrain.py:329
    m.language_model._set_gradient_checkpointing()           # :331-332
    assert m.language_model.model.gradient_checkpointing is True
    m.gradient_checkpointing_enable()
    assert m.language_model.model.gradient_checkpointing is True
    m.gradient_checkpointing_disable()
    assert m.language_model.model.gradient_checkpointing is False


def test_training_forward_with_per_sequence_positions_refused(tiny_model):
    from spatialvla_amd.modeling_gemma2 import KVMask
    att = tiny_model.language_model.model.layers[0].self_attn
    B, L, H = 2, 5, tiny_model.config.text_config.hidden_size
    x = torch.zeros(B, L, H, dtype=torch.bfloat16, requires_grad=True)
    pos = torch.tensor([[1, 2, 3, 4, 5], [1, 1, 1, 2, 3]])  # a padded second prompt: its own positions
    rope = att.rotary_emb.tables(pos, torch.bfloat16)
    assert rope[0].shape[0] == B * L
    with pytest.raises(NotImplementedError, match="per-sequence position_ids"):
        att(x, KVMask(torch.zeros(B, L, dtype=torch.uint8)), rope)
