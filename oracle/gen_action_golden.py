"""Golden vectors for the spatial action tokenizer and decode_actions, produced by the REFERENCE itself.

TEST INFRASTRUCTURE ONLY (container-side; needs /root/reference).  Runs the reference's
model/action_tokenizer.py SpatialActionTokenizer (uniform bins and the Gaussian bin policies of
scripts/gs_bridge.json / gs_fractal.json) and SpatialVLAProcessor.decode_actions
(processing_spatialvla.py:221-253, called unbound on a minimal stand-in object), with a minimal fake
text tokenizer (the only part of a tokenizer these use: add_tokens + convert_tokens_to_ids).
Writes tests/golden/action_tokenizer.npz.  The reference module is imported, never copied.

    python oracle/gen_action_golden.py
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "action_tokenizer.npz")
BASE_VOCAB = 257153  # PaliGemma2 vocabulary incl. <image> (SURVEY.md §8 canonical shapes)


class FakeTokenizer:
    """add_tokens / convert_tokens_to_ids over a base vocabulary of BASE_VOCAB ids."""

    def __init__(self, base=BASE_VOCAB):
        self.vocab = {}
        self.base = base
        self.vocab_size = base
        self.eos_token = "<eos>"

    def add_tokens(self, toks, special_tokens=False):
        n = 0
        for t in toks:
            if t not in self.vocab:
                self.vocab[t] = self.base + len(self.vocab)
                n += 1
        return n

    def convert_tokens_to_ids(self, t):
        return self.vocab[t]

    def __len__(self):
        return self.base + len(self.vocab)


def _import_reference():
    sys.path.insert(0, REF)
    import transformers.processing_utils as pu
    import transformers.models.paligemma.processing_paligemma as pp
    # names removed in transformers 5 that processing_spatialvla imports but decode_actions never uses
    for mod, name in ((pu, "_validate_images_text_input_order"), (pp, "make_batched_images"),
                      (pp, "build_string_from_input"), (pp, "_is_str_or_image")):
        if not hasattr(mod, name):
            setattr(mod, name, lambda *a, **k: None)
    from model import action_tokenizer as at
    from model import processing_spatialvla as ps
    return at, ps


def main():
    at, ps = _import_reference()
    cfg = json.load(open(os.path.join(REF, "scripts", "action_config.json")))
    num_bins = cfg["num_bins"]
    rng = np.random.default_rng(2024)
    out = {}
    policies = {"uniform": None}
    for name in ("gs_bridge", "gs_fractal"):
        policies[name] = json.load(open(os.path.join(REF, "scripts", name + ".json")))
    # actions: uniform in the cube, Gaussian-ish, exact bin edges / boundaries, out-of-range values
    a = np.concatenate([
        rng.uniform(-1, 1, (512, 7)),
        np.clip(rng.normal(0, 0.3, (512, 7)), -1.5, 1.5),
        np.array([[0, 0, 0, 0, 0, 0, 0.5], [1, 1, 1, 1, 1, 1, 1], [-1, -1, -1, -1, -1, -1, -1],
                  [2, -3, 0.5, 4, -4, 0.0, 0.49], [0, 0, 1e-9, -1e-9, 1e-9, 0, 0.5000001]]),
    ])
    out["actions"] = a
    for pname, gs in policies.items():
        tok = FakeTokenizer()
        sat = at.SpatialActionTokenizer(tok, num_bins=num_bins, gs_params=gs, use_spherical=cfg["use_spherical"],
                                        min_sigma=0.0)
        strs = sat(a)
        ids = np.vectorize(tok.convert_tokens_to_ids)(strs).astype(np.int64)
        out[f"{pname}/ids"] = ids
        out[f"{pname}/decoded"] = sat.decode_token_ids_to_actions(ids)
        # every token id of the vocabulary (and out-of-range ids, which are clipped) decoded
        all_ids = np.stack([np.arange(BASE_VOCAB - 5, BASE_VOCAB + sat.vocab_size + 5)] * 3, axis=1)
        all_ids[:, 1] = np.clip(all_ids[:, 1] + 4096, 0, None)
        all_ids[:, 2] = BASE_VOCAB + 8192 + (np.arange(all_ids.shape[0]) % 4) - 1
        out[f"{pname}/all_ids"] = all_ids
        out[f"{pname}/all_decoded"] = sat.decode_token_ids_to_actions(all_ids)
        for axis_kind, axes in sat.bin_policy.items():
            for axis, edges in axes.items():
                out[f"{pname}/policy/{axis_kind}/{axis}"] = np.asarray(edges, dtype=np.float64)
        out[f"{pname}/begin"] = np.array(sat.action_token_begin_idx)
        # decode_actions (un-normalisation with q01/q99 + mask) through the reference processor method
        stats = {"bridge": {"action": {"q01": list(rng.uniform(-0.05, -0.01, 7)),
                                       "q99": list(rng.uniform(0.01, 0.05, 7)),
                                       "mask": [True] * 6 + [False]}}}
        stub = types.SimpleNamespace(action_tokenizer=sat, statistics=stats, action_chunk_size=4,
                                     tokenizer=types.SimpleNamespace(eos_token=tok.eos_token))
        gen = ids[:4].reshape(1, -1)
        gen = np.concatenate([gen, np.full((1, 3), 1, dtype=np.int64)], axis=1)  # trailing eos-like ids
        import torch
        res = ps.SpatialVLAProcessor.decode_actions(stub, torch.from_numpy(gen), unnorm_key="bridge")
        out[f"{pname}/gen_ids"] = gen
        out[f"{pname}/gen_actions"] = np.asarray(res["actions"])
        out[f"{pname}/q01"] = np.array(stats["bridge"]["action"]["q01"])
        out[f"{pname}/q99"] = np.array(stats["bridge"]["action"]["q99"])
        out[f"{pname}/mask"] = np.array(stats["bridge"]["action"]["mask"])
    # intrinsics scaling (processing_spatialvla.py:87-95) for every dataset in scripts/intrinsics.json
    intr = json.load(open(os.path.join(REF, "scripts", "intrinsics.json")))
    import torch
    for k, v in intr.items():
        K = torch.tensor(v["intrinsic"]).float()
        K[:2] *= torch.tensor([224 / v["width"], 224 / v["height"]])[:, None]
        out[f"intrinsics/{k}"] = K.numpy()
        out[f"intrinsics_raw/{k}"] = np.array(v["intrinsic"], dtype=np.float64)
        out[f"intrinsics_hw/{k}"] = np.array([v["height"], v["width"]])
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays")


if __name__ == "__main__":
    main()
