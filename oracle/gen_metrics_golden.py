"""Golden vectors for the per-step action metrics, produced by the REFERENCE itself.

TEST INFRASTRUCTURE ONLY (container-side; needs /root/reference).  Runs the reference's patched
Trainer.compute_loss (train/monkey_patch.py:222-326) unbound, on a stand-in trainer/model whose forward returns
prepared logits: the argmax over V of the shifted logits, the action-token masks of the SpatialActionTokenizer id
ranges, the overall / translation / rotation / gripper accuracies and the L1 loss of the decoded actions
(:267-324).  The tokenizer is a minimal fake (add_tokens / convert_tokens_to_ids over the PaliGemma2 base
vocabulary).  Writes tests/golden/action_metrics.npz: inputs (argmax ids, labels, actions) and the logged values.
The reference module is imported, never copied.

    python oracle/gen_metrics_golden.py
"""
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "action_metrics.npz")
sys.path.insert(0, HERE)
from gen_action_golden import BASE_VOCAB, FakeTokenizer, _import_reference  # noqa: E402


def main():
    at, _ps = _import_reference()
    sys.path.insert(0, REF)
    import train.monkey_patch as mp
    cfg = json.load(open(os.path.join(REF, "scripts", "action_config.json")))
    tok = FakeTokenizer()
    sat = at.SpatialActionTokenizer(tok, num_bins=cfg["num_bins"], gs_params=None, use_spherical=cfg["use_spherical"])
    V = BASE_VOCAB + sat.vocab_size
    rng = np.random.default_rng(77)
    out = {}
    for case, (B, L, p_ok) in enumerate([(3, 40, 0.6), (2, 33, 0.0), (4, 29, 1.0), (5, 50, 0.3)]):
        n_act = 12  # chunk of 4 steps x 3 tokens, then eos
        actions = rng.uniform(-1, 1, (B, 4, 7))
        ids = np.stack([np.vectorize(tok.convert_tokens_to_ids)(sat(actions[b])).reshape(-1) for b in range(B)])
        labels = np.full((B, L), -100, dtype=np.int64)
        labels[:, L - n_act - 1:L - 1] = ids
        labels[:, L - 1] = 1  # eos label: outside the action range
        # predictions at position t for label t+1: p_ok of the action rows correct, the rest a random id that is an
        # action token of another class, an action token of the same class, or a text token
        pred = rng.integers(0, BASE_VOCAB, (B, L)).astype(np.int64)
        for b in range(B):
            for t in range(L - 1):
                gt = labels[b, t + 1]
                if gt >= BASE_VOCAB and rng.uniform() < p_ok:
                    pred[b, t] = gt
                elif gt >= BASE_VOCAB:
                    pred[b, t] = rng.choice([rng.integers(BASE_VOCAB, V), gt + 1 if gt + 1 < V else gt - 1,
                                             rng.integers(0, BASE_VOCAB)])
        logits = torch.zeros(B, L, V)
        logits.scatter_(2, torch.from_numpy(pred)[..., None], 1.0)
        logged = {}
        trainer = types.SimpleNamespace(
            label_smoother=None, compute_loss_func=None, model_accepts_loss_kwargs=False,
            args=types.SimpleNamespace(past_index=-1, average_tokens_across_devices=False),
            log=lambda d: logged.update(d))
        inputs = {"labels": torch.from_numpy(labels), "actions": torch.from_numpy(actions).to(torch.bfloat16)}

        class ModelStub:  # the reference model's role in compute_loss: outputs + .action_tokenizer
            action_tokenizer = sat

            def __call__(self, **kw):
                return {"loss": torch.tensor(0.0), "logits": logits}
        model_call = ModelStub()
        mp.compute_loss(trainer, model_call, inputs)
        out[f"c{case}/pred"] = pred
        out[f"c{case}/labels"] = labels
        out[f"c{case}/actions"] = actions.astype(np.float32)
        out[f"c{case}/actions_bf16"] = inputs["actions"].float().numpy()
        for k in ("accuracy", "translation_accuracy", "rotation_accuracy", "gripper_accuracy", "l1_loss"):
            out[f"c{case}/{k}"] = np.array(logged[k], dtype=np.float64)
        print(case, {k: round(v, 6) for k, v in logged.items()})
    out["begin"] = np.array(sat.action_token_begin_idx)
    out["ranges"] = np.array([sat.translation_tokenizer.token_start_idx, sat.translation_tokenizer.token_end_idx,
                              sat.rotation_tokenizer.token_start_idx, sat.rotation_tokenizer.token_end_idx,
                              sat.gripper_tokenizer.token_start_idx, sat.gripper_tokenizer.token_end_idx])
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays")


if __name__ == "__main__":
    main()
