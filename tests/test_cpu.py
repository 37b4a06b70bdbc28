"""CPU suite: the oracle pinned against the reference's golden vectors, the C-ABI surface, host logic."""
import ctypes
import json
import os
import re

import pytest
import torch

import harness as H

GOLD = os.path.join(os.path.dirname(__file__), "golden")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    from safetensors.torch import load_file
    return load_file(os.path.join(GOLD, name))


# ------------------------------------------------------------------------------ oracle vs reference goldens
@pytest.fixture(scope="module")
def tiny_oracle():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    cfgd = H.cfg_dict("tiny")
    P, zoe = H.build_oracle(cfgd)
    return cfgd, P, zoe


def test_oracle_matches_reference_tiny_train_bitexact(tiny_oracle):
    cfgd, P, zoe = tiny_oracle
    g = _load("tiny_train.safetensors")
    batch = {k[3:]: v for k, v in g.items() if k.startswith("in.")}
    loss, logits, grads, cap = H.run_oracle(P, zoe, cfgd, batch)
    assert torch.equal(cap["depth"], g["out.depth"])
    assert torch.equal(cap["image_features"], g["out.image_features"])
    assert torch.equal(logits.to(torch.bfloat16), g["out.logits"])
    assert float(loss) == float(g["out.loss"][0])
    for k, v in g.items():
        if k.startswith("grad."):
            assert torch.equal(grads[k[5:]].to(torch.bfloat16), v), k


def test_oracle_matches_reference_prefill(tiny_oracle):
    import spatialvla_oracle as O
    cfgd, P, zoe = tiny_oracle
    g, gp = _load("tiny_train.safetensors"), _load("tiny_prefill.safetensors")
    b = {k[3:]: v for k, v in g.items() if k.startswith("in.")}
    b.pop("labels")
    b.pop("token_type_ids")
    with torch.no_grad():
        _, logits = O.forward(P, cfgd, b, zoe, depth=g["out.depth"])
    assert torch.equal(logits, gp["out.logits"])


def test_oracle_matches_reference_ragged(tiny_oracle):
    cfgd, P, zoe = tiny_oracle
    g = _load("tiny_ragged.safetensors")
    b = {k[3:]: v for k, v in g.items() if k.startswith("in.")}
    assert (b["attention_mask"] == 0).any(), "fixture must contain padding"
    loss, logits, grads, _ = H.run_oracle(P, zoe, cfgd, b)
    assert float(loss) == float(g["out.loss"][0])
    assert torch.equal(logits.to(torch.bfloat16), g["out.logits"])
    for k, v in g.items():
        if k.startswith("gradnorm."):
            assert abs(grads[k[9:]].norm().item() - v.item()) <= 1e-6 * max(1.0, v.item()), k


def test_oracle_greedy_decode_matches_reference(tiny_oracle):
    """The oracle's uncached greedy decode (prompt bidirectional, generated tokens causal) reproduces the tokens
    and margins the reference model produced (oracle/gen_golden.py gen_decode_tiny)."""
    import spatialvla_oracle as O
    cfgd, P, zoe = tiny_oracle
    g = _load("decode_tiny.safetensors")
    b = {k[3:]: v for k, v in g.items() if k.startswith("in.")}
    toks, margins = O.greedy_decode(P, cfgd, b, zoe, n_new=g["out.tokens"].shape[1], depth=g["out.depth"])
    assert torch.equal(toks, g["out.tokens"])
    assert torch.equal(margins, g["out.margins"])


def test_oracle_padded_greedy_decode_matches_reference(tiny_oracle):
    """Left-padded prompts of different lengths: per-sequence positions (attention_mask.cumsum) and masked pad keys
    reproduce the reference model's greedy tokens and margins bit for bit (oracle/gen_golden.py gen_decode_padded)."""
    import spatialvla_oracle as O
    cfgd, P, zoe = tiny_oracle
    g = _load("decode_padded.safetensors")
    b = {k[3:]: v for k, v in g.items() if k.startswith("in.")}
    toks, margins = O.greedy_decode(P, cfgd, b, zoe, n_new=g["out.tokens"].shape[1], depth=g["out.depth"])
    assert torch.equal(toks, g["out.tokens"])
    assert torch.equal(margins, g["out.margins"])


def test_hash_init_bitwise_reproducible():
    """spatialvla_amd.detinit.hash_tensor: the counter-hash init of the 4B fixture -- independent of chunking and
    a pure function of (name, shape, seed); the GPU test repeats the check on the device."""
    from spatialvla_amd.detinit import hash_tensor
    a = hash_tensor("language_model.model.layers.3.mlp.up_proj.weight", (96, 40), 1234)
    b = hash_tensor("language_model.model.layers.3.mlp.up_proj.weight", (96, 40), 1234, chunk=7)
    assert torch.equal(a, b)
    c = hash_tensor("vision_tower.vision_model.encoder.layers.0.layer_norm1.weight", (1152,), 1234)
    d = hash_tensor("vision_tower.encoder.layers.0.layer_norm1.weight", (1152,), 1234)  # canonical name
    assert torch.equal(c, d) and abs(float(c.float().mean()) - 1.0) < 0.02
    e = hash_tensor("language_model.model.layers.3.mlp.up_proj.weight", (96, 40), 1235)
    assert not torch.equal(a, e)
    x = hash_tensor("w", (4096, 512), 0, dtype=torch.float32)
    assert abs(float(x.std()) * 512 ** 0.5 - 1.0) < 0.01


def test_oracle_gemma_layer_4b_matches_reference():
    import spatialvla_oracle as O
    from spatialvla_amd import presets
    from spatialvla_amd.detinit import det_tensor
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = _load("layer4b.safetensors")
    cfgd = json.loads(json.dumps(presets.spatialvla_4b(use_vision_zoe=False)))
    tc = cfgd["text_config"]
    shapes = O.param_shapes(cfgd)
    P = {}
    for n, s in shapes.items():
        if n.startswith("language_model.model.layers.1."):
            P[n] = det_tensor(n, s, H.SEED).to(torch.bfloat16).requires_grad_(True)
    L, Pf = 312, 299
    h = g["gemma.in"].clone().requires_grad_(True)
    am = torch.ones(1, L, dtype=torch.long)
    tt = torch.zeros(1, L, dtype=torch.long)
    tt[:, Pf:] = 1
    mask = O.prefix_mask(am, tt, True, L, torch.bfloat16)
    cos, sin = O.rope_tables((torch.arange(L) + 1)[None], 256, torch.bfloat16)
    y = O.gemma_layer(P, tc, 1, h, mask, cos, sin)
    gout = det_tensor("gemma.gout", (1, L, 2304), H.SEED, scale=1.0).to(torch.bfloat16)
    (y.float() * gout.float()).sum().backward()
    assert torch.equal(y.detach(), g["gemma1.out"])
    assert torch.equal(h.grad, g["gemma1.dx"])


# ------------------------------------------------------------------------------ C-ABI surface
def test_header_symbols_exported_by_library():
    """libsvla.so loads (no GPU needed) and exports every entry point declared in include/svla.h."""
    from spatialvla_amd import _lib
    hdr = open(os.path.join(REPO, "include", "svla.h")).read()
    names = set(re.findall(r"^\s*(?:const char\*|int|size_t|void)\s+(svla_\w+)\s*\(", hdr, re.M))
    assert len(names) >= 20
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert names == set(_lib.SIGNATURES), "python binding must cover exactly the header"
    # the binding's argument count equals the prototype's (a wrong count only fails at the first GPU call)
    body = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    for m in re.finditer(r"(?:const char\*|int|size_t|void)\s+(svla_\w+)\s*\(([^)]*)\)\s*;", body):
        params = [p for p in m.group(2).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(_lib.SIGNATURES[m.group(1)][1]), (m.group(1), len(params))
    _lib.load()
    assert b"gfx950" in _lib.lib().svla_version()


def test_product_never_imports_oracle():
    pkg = os.path.join(REPO, "spatialvla_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "spatialvla_oracle" not in src and "ref_shim" not in src and "/root/reference" not in src, f


# ------------------------------------------------------------------------------ host logic
@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("ragged", [False, True])
def test_kvmask_matches_reference_additive_mask(training, ragged):
    import spatialvla_oracle as O
    from spatialvla_amd import presets
    from spatialvla_amd.modeling_gemma2 import KVMask
    cfgd = H.cfg_dict("tiny")
    b = presets.synthetic_batch(cfgd, batch=3, seed=5, ragged=ragged)
    am, tt = torch.from_numpy(b["attention_mask"]), torch.from_numpy(b["token_type_ids"])
    B, L = am.shape
    dense = O.prefix_mask(am, tt, training, L, torch.bfloat16)[:, 0]
    visible_ref = dense == 0
    cls = KVMask.build(am, tt, training, B, L, "cpu").kv_class.long()
    i = torch.arange(L)[:, None]
    j = torch.arange(L)[None, :]
    visible = (cls[:, None, :] == 0) | ((cls[:, None, :] == 1) & (j <= i))
    assert torch.equal(visible, visible_ref)


@pytest.mark.parametrize("training,ragged", [(True, False), (True, True), (False, True)])
def test_plugin_mask_classes_from_additive_mask(training, ragged):
    """The GEMMA2_ATTENTION_FUNCTION adapter recovers per-key classes from the reference's dense mask."""
    import spatialvla_oracle as O
    from spatialvla_amd import presets
    from spatialvla_amd.functional import kv_class_from_additive_mask
    from spatialvla_amd.modeling_gemma2 import KVMask
    cfgd = H.cfg_dict("tiny")
    b = presets.synthetic_batch(cfgd, batch=3, seed=7, ragged=ragged)
    am, tt = torch.from_numpy(b["attention_mask"]), torch.from_numpy(b["token_type_ids"])
    B, L = am.shape
    dense = O.prefix_mask(am, tt, training, L, torch.bfloat16)
    got = kv_class_from_additive_mask(dense, B, L, L, "cpu")
    vis = dense[:, 0] == 0
    i = torch.arange(L)
    rebuilt = (got[:, None, :] == 0) | ((got[:, None, :] == 1) & (i[None, :] <= i[:, None]))
    assert torch.equal(rebuilt, vis)
    if not ragged:
        assert torch.equal(got, KVMask.build(am, tt, training, B, L, "cpu").kv_class)
    bad = dense.clone()
    bad[0, 0, 3, 1] = torch.finfo(torch.bfloat16).min   # one masked cell in an otherwise visible column
    with pytest.raises(ValueError):
        kv_class_from_additive_mask(bad, B, L, L, "cpu")


def test_ce_targets_match_reference_shift():
    from spatialvla_amd import presets
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration as M
    cfgd = H.cfg_dict("tiny")
    b = presets.synthetic_batch(cfgd, batch=3, seed=9, ragged=True)
    labels, am = torch.from_numpy(b["labels"]), torch.from_numpy(b["attention_mask"])
    B, L = labels.shape
    t = M._targets(labels, am, B, L, "cpu").view(B, L)
    sl, keep = labels[:, 1:], am[:, 1:] != 0
    ref = torch.where(keep & (sl != -100), sl, -1)
    assert torch.equal(t[:, :-1], ref) and (t[:, -1] == -1).all()


def test_synthetic_batch_layout_4b():
    from spatialvla_amd import presets
    cfgd = presets.spatialvla_4b()
    b = presets.synthetic_batch(cfgd, batch=2, seed=0)
    assert b["input_ids"].shape == (2, 312)
    assert (b["input_ids"][:, :256] == cfgd["image_token_index"]).all()
    assert (b["token_type_ids"].sum(1) == 13).all()
    assert cfgd["vocab_size"] == 265347 and cfgd["action_token_begin_idx"] == 257153
    a0 = cfgd["action_token_begin_idx"]
    acts = b["input_ids"][:, 299:311]
    assert ((acts >= a0) & (acts < a0 + 8194)).all()


def test_model_state_dict_keys_match_reference_weight_abi():
    """State-dict keys are the weight ABI; compare with the reference's trainable set."""
    from spatialvla_amd import SpatialVLAConfig
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    g = _load("tiny_train.safetensors")
    m = SpatialVLAForConditionalGeneration(SpatialVLAConfig(**H.cfg_dict("tiny")))
    mine = {k.replace("vision_tower.vision_model.", "vision_tower.") for k, _ in m.named_parameters()}
    ref = {k[5:] for k in g if k.startswith("grad.")}
    assert ref <= mine
    extra = {k for k in mine - ref if not k.startswith("vision_zoe_model.")}
    assert extra == {"language_model.model.embed_tokens.weight"}  # frozen in the reference


def test_from_pretrained_roundtrip_reference_layout(tmp_path):
    """save_pretrained -> from_pretrained on a checkpoint in the reference's key layout (the transformers
    SiglipVisionModel / Gemma2ForCausalLM names of tests/golden/tiny_train.safetensors): every tensor comes back
    bitwise, and the last spatial_token_num rows of embed_tokens are overwritten by spatial_embed_tokens as the
    reference's from_pretrained does (model/modeling_spatialvla.py:524-525)."""
    from safetensors.torch import load_file
    from spatialvla_amd import SpatialVLAConfig
    from spatialvla_amd.detinit import deterministic_init_
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    cfg = SpatialVLAConfig(**H.cfg_dict("tiny"))
    m = SpatialVLAForConditionalGeneration(cfg).to(torch.bfloat16)
    deterministic_init_(m, seed=5)
    n = cfg.spatial_token_num
    with torch.no_grad():  # make the tail copy observable: stored tail != spatial_embed_tokens
        m.language_model.model.embed_tokens.weight[-n:] = 0.25
    m.save_pretrained(tmp_path, safe_serialization=True)
    files = sorted(tmp_path.glob("*.safetensors"))
    assert files
    saved = {}
    for f in files:
        saved.update(load_file(str(f)))
    ref_keys = {k[5:] for k in _load("tiny_train.safetensors") if k.startswith("grad.")}
    on_disk = {k.replace("vision_tower.vision_model.", "vision_tower.") for k in saved}
    assert ref_keys <= on_disk  # the checkpoint carries the reference's names
    m2 = SpatialVLAForConditionalGeneration.from_pretrained(tmp_path, torch_dtype=torch.bfloat16)
    sd1, sd2 = m.state_dict(), m2.state_dict()
    assert set(sd1) == set(sd2)
    emb = "language_model.model.embed_tokens.weight"
    for k, v in sd1.items():
        if k in (emb, "language_model.lm_head.weight"):
            continue
        assert torch.equal(sd2[k], v), k
    e1, e2 = sd1[emb], sd2[emb]
    assert torch.equal(e2[:-n], e1[:-n])
    assert torch.equal(e2[-n:], sd2["spatial_embed_tokens.weight"])
    assert not torch.equal(e2[-n:], e1[-n:])


def test_product_fails_loudly_without_gpu():
    from spatialvla_amd import SpatialVLAConfig
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    from spatialvla_amd import presets
    cfgd = H.cfg_dict("tiny")
    m = SpatialVLAForConditionalGeneration(SpatialVLAConfig(**cfgd)).to(torch.bfloat16)
    b = H.batch_tensors(presets.synthetic_batch(cfgd, batch=1, seed=0), "cpu")
    with pytest.raises(Exception):
        m(**b)


def test_kv_cache_layout_and_capacity():
    """Gemma2KVCache (HybridCache stand-in): per-layer [B, capacity, Hkv*D] rows, classes appended per forward,
    overflow raises (host logic only; the kernels are in tests/test_decode_gpu.py)."""
    from spatialvla_amd import SpatialVLAConfig
    from spatialvla_amd.modeling_gemma2 import Gemma2KVCache
    cfg = SpatialVLAConfig(**H.cfg_dict("tiny")).text_config
    c = Gemma2KVCache(cfg, batch_size=2, capacity=10, device="cpu")
    kd = cfg.num_key_value_heads * cfg.head_dim
    assert c.key_cache.shape == (cfg.num_hidden_layers, 2, 10, kd) and c.value_cache.shape == c.key_cache.shape
    assert c.get_seq_length() == 0 and c.capacity == 10
    c.append_classes(torch.zeros(2, 7, dtype=torch.uint8))
    c.seen_tokens = 7
    c.append_classes(torch.ones(2, 3, dtype=torch.uint8))
    assert c.kv_class[:, :7].eq(0).all() and c.kv_class[:, 7:].eq(1).all()
    c.seen_tokens = 10
    with pytest.raises(ValueError):
        c.append_classes(torch.ones(2, 1, dtype=torch.uint8))


def test_softcap_reciprocal_multiply_exact_on_bf16():
    """The GEMM/GEMV softcap epilogues divide by the cap as a multiply by RN(1/cap) (svla_common.h softcap_bf16):
    exact at bf16 for every finite bf16 input at caps 30 and 50 (exhaustive)."""
    import runpy
    runpy.run_path(os.path.join(REPO, "tools", "check_softcap_recip.py"))


def test_beit_mask_none_under_graph_capture(monkeypatch):
    """zoe_fast makes the BEiT encoder's no-padding mask `None` in every mode: transformers materialises an
    all-visible additive mask while a HIP graph is capturing (masking_utils.is_tracing), which would route every
    BeitLayer of the captured prefill to the stock path."""
    from transformers import BeitConfig
    from transformers.models.beit import modeling_beit as mb
    from spatialvla_amd import zoe_fast
    zoe_fast._patch_beit_mask()
    cfg = BeitConfig(hidden_size=32, num_hidden_layers=1, num_attention_heads=2, intermediate_size=64)
    cfg._attn_implementation = "eager"  # as the estimator runs (its BeitLayer adds the mask to the scores)
    emb = torch.zeros(2, 5, 32)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)
    assert mb.create_bidirectional_mask._svla_orig(config=cfg, inputs_embeds=emb, attention_mask=None) is not None
    assert mb.create_bidirectional_mask(config=cfg, inputs_embeds=emb, attention_mask=None) is None
    pad = torch.ones(2, 5, dtype=torch.long)
    pad[1, 3:] = 0
    m = mb.create_bidirectional_mask(config=cfg, inputs_embeds=emb, attention_mask=pad)
    assert m is not None
