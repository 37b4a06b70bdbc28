"""Spatial action tokenizer / decode_actions / intrinsics scaling vs golden vectors produced by the reference
itself (oracle/gen_action_golden.py: reference model/action_tokenizer.py and
SpatialVLAProcessor.decode_actions on uniform and Gaussian bin policies).  CPU only; exact equality for
token ids, float64 exact for decoded actions."""
import os

import numpy as np
import pytest

from spatialvla_amd import action_tokenizer as AT

GOLD = os.path.join(os.path.dirname(__file__), "golden", "action_tokenizer.npz")
NUM_BINS = {"translation": {"theta_bins": 16, "phi_bins": 32, "r_bins": 8},
            "rotation": {"roll_bins": 16, "pitch_bins": 16, "yaw_bins": 16}, "gripper": 2, "total": 8194}
BASE = 257153


class FakeTokenizer:
    def __init__(self, base=BASE):
        self.vocab, self.base = {}, base

    def add_tokens(self, toks, special_tokens=False):
        for t in toks:
            self.vocab.setdefault(t, self.base + len(self.vocab))

    def convert_tokens_to_ids(self, t):
        return self.vocab[t]


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _policy(g, name):
    pol = {}
    for kind, axes in AT.RANGE_BINS.items():
        pol[kind] = {a: g[f"{name}/policy/{kind}/{a}"] for a in axes}
    return pol


@pytest.mark.parametrize("name", ["uniform", "gs_bridge", "gs_fractal"])
def test_encode_decode_matches_reference(gold, name):
    tok = FakeTokenizer()
    sat = AT.SpatialActionTokenizer(tok, NUM_BINS, bin_policy=_policy(gold, name), use_spherical=True)
    assert sat.vocab_size == 8194 and sat.action_token_begin_idx == int(gold[f"{name}/begin"]) == BASE
    ids = sat.token_ids(gold["actions"])
    np.testing.assert_array_equal(ids, gold[f"{name}/ids"])
    np.testing.assert_array_equal(sat.decode_token_ids_to_actions(gold[f"{name}/ids"]), gold[f"{name}/decoded"])
    np.testing.assert_array_equal(sat.decode_token_ids_to_actions(gold[f"{name}/all_ids"]),
                                  gold[f"{name}/all_decoded"])


def test_uniform_policy_recomputed(gold):
    pol = AT.bin_policy_from(NUM_BINS, None)
    for kind, axes in AT.RANGE_BINS.items():
        for a in axes:
            np.testing.assert_array_equal(np.asarray(pol[kind][a]), gold[f"uniform/policy/{kind}/{a}"])


def test_gaussian_policy_is_equal_probability():
    from scipy.stats import norm
    gs = {k: {"mu": 0.1 * i, "sigma": 0.3 + 0.05 * i}
          for i, k in enumerate(["theta", "phi", "r", "roll", "pitch", "yaw"])}
    pol = AT.bin_policy_from(NUM_BINS, gs)
    for kind, axes in AT.RANGE_BINS.items():
        for a, (lo, hi) in axes.items():
            e = np.asarray(pol[kind][a])
            g = gs[a.split("_")[0]]
            p = norm.cdf(e, loc=g["mu"], scale=g["sigma"])
            assert e[0] >= lo - 1e-12 and e[-1] <= hi + 1e-12 and np.all(np.diff(e) > 0)
            np.testing.assert_allclose(np.diff(p), np.diff(p).mean(), rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("name", ["uniform", "gs_bridge"])
def test_decode_actions_matches_reference(gold, name):
    tok = FakeTokenizer()
    sat = AT.SpatialActionTokenizer(tok, NUM_BINS, bin_policy=_policy(gold, name))
    stats = {"bridge": {"action": {"q01": list(gold[f"{name}/q01"]), "q99": list(gold[f"{name}/q99"]),
                                   "mask": list(gold[f"{name}/mask"])}}}
    res = AT.decode_actions(gold[f"{name}/gen_ids"], sat, stats, "bridge", action_chunk_size=4, eos_token_id=1)
    np.testing.assert_array_equal(res["actions"], gold[f"{name}/gen_actions"])


def test_intrinsics_scaling(gold):
    keys = [k.split("/", 1)[1] for k in gold if k.startswith("intrinsics_raw/")]
    assert keys
    cfg = {k: {"intrinsic": gold[f"intrinsics_raw/{k}"].tolist(), "height": int(gold[f"intrinsics_hw/{k}"][0]),
               "width": int(gold[f"intrinsics_hw/{k}"][1])} for k in keys}
    got = AT.scale_intrinsics(cfg, 224, 224)
    for k in keys:
        np.testing.assert_array_equal(got[k], gold[f"intrinsics/{k}"])


def test_prompt_layout_matches_synthetic_batch():
    from spatialvla_amd import presets
    out = AT.prompt_token_layout(list(range(100, 141)), image_token_id=257152, image_seq_len=256, bos_id=2,
                                 newline_ids=[108], suffix_ids=list(range(257153, 257165)), eos_id=1)
    assert out["input_ids"].shape == (312,)
    assert out["token_type_ids"].sum() == 13 and (out["labels"] != -100).sum() == 13
    assert out["input_ids"][256] == 2 and out["input_ids"][-1] == 1


def test_gripper_threshold_and_clip():
    tok = FakeTokenizer()
    sat = AT.SpatialActionTokenizer(tok, NUM_BINS)
    a = np.array([[0, 0, 0, 0, 0, 0, 0.5], [0, 0, 0, 0, 0, 0, 0.4999], [5, 5, 5, 5, 5, 5, 5]])
    ids = sat.token_ids(a)
    assert ids[0, 2] == BASE + 8193 and ids[1, 2] == BASE + 8192
    dec = sat.decode_token_ids_to_actions(ids)
    assert np.all(np.abs(dec[:, :6]) <= 1.0)
