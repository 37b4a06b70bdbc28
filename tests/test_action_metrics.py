"""Per-step action metrics (BASELINE a17: train/monkey_patch.py:267-324) against golden values the reference's own
compute_loss logged (oracle/gen_metrics_golden.py).  CPU: the oracle restatement, exact.  GPU: the
svla_action_accuracy kernel (integer counts, float32 divisions), exact, and the model's action_metrics() on the
lm_head epilogue's argmax after a training forward."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden", "action_metrics.npz")
NAMES = ("accuracy", "translation_accuracy", "rotation_accuracy", "gripper_accuracy")
NUM_BINS = {"translation": {"theta_bins": 16, "phi_bins": 32, "r_bins": 8},
            "rotation": {"roll_bins": 16, "pitch_bins": 16, "yaw_bins": 16}, "gripper": 2, "total": 8194}


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _cases(g):
    return sorted({k.split("/")[0] for k in g if k.startswith("c")})


def _tokenizer():
    from test_action_tokenizer import FakeTokenizer
    from spatialvla_amd.action_tokenizer import SpatialActionTokenizer
    return SpatialActionTokenizer(FakeTokenizer(), NUM_BINS)


def test_oracle_action_metrics_match_reference(gold):
    import spatialvla_oracle as O
    sat = _tokenizer()
    assert tuple(gold["ranges"]) == (sat.translation_tokenizer.token_start_idx, sat.translation_tokenizer.token_end_idx,
                                     sat.rotation_tokenizer.token_start_idx, sat.rotation_tokenizer.token_end_idx,
                                     sat.gripper_tokenizer.token_start_idx, sat.gripper_tokenizer.token_end_idx)
    for c in _cases(gold):
        got = O.action_metrics(torch.from_numpy(gold[f"{c}/pred"]), torch.from_numpy(gold[f"{c}/labels"]),
                               gold["ranges"], actions=torch.from_numpy(gold[f"{c}/actions_bf16"]),
                               decode=sat.decode_token_ids_to_actions)
        for k in NAMES + ("l1_loss",):
            assert got[k] == float(gold[f"{c}/{k}"]), (c, k, got[k], float(gold[f"{c}/{k}"]))


def test_model_action_token_ranges_canonical():
    from spatialvla_amd import SpatialVLAConfig, presets
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    cfg = SpatialVLAConfig(**presets.tiny())
    m = SpatialVLAForConditionalGeneration.__new__(SpatialVLAForConditionalGeneration)
    torch.nn.Module.__init__(m)
    m.config = cfg
    cfg.action_token_begin_idx, cfg.spatial_token_num = 257153, 8194
    sat = _tokenizer()
    assert m.action_token_ranges() == m.action_token_ranges(sat)


@pytest.mark.gpu
def test_action_accuracy_kernel_matches_reference(gold, cuda):
    from spatialvla_amd import kernels as K
    for c in _cases(gold):
        pred = torch.from_numpy(gold[f"{c}/pred"]).to(cuda)
        labels = torch.from_numpy(gold[f"{c}/labels"]).to(cuda)
        counts, acc = K.action_accuracy(pred, labels, gold["ranges"])
        torch.cuda.synchronize()
        for i, k in enumerate(NAMES):
            assert float(acc[i]) == float(gold[f"{c}/{k}"]), (c, k, float(acc[i]), float(gold[f"{c}/{k}"]))
        cnt = counts.cpu().tolist()
        assert cnt[0] == cnt[2] + cnt[4] + cnt[6] and cnt[1] == cnt[3] + cnt[5] + cnt[7]


@pytest.mark.gpu
def test_model_action_metrics_after_training_forward(gold, cuda):
    """tiny model, one training forward: action_metrics() from the epilogue argmax == the oracle restatement on the
    argmax of the returned logits (identical wherever the argmax is; here compared on the HIP argmax itself)."""
    import harness as H
    import spatialvla_oracle as O
    from spatialvla_amd import presets
    cfgd = H.cfg_dict("tiny")
    model = H.build_hip_model(cfgd, cuda)
    b = H.batch_tensors(presets.synthetic_batch(cfgd, batch=3, seed=5), cuda)
    model.predict_depth = lambda pv: torch.rand(pv.shape[0], 1, 224, 224, device=cuda) * 3 + 0.5
    out = model(**b, return_dict=True)
    a0 = cfgd["action_token_begin_idx"]
    n = cfgd["spatial_token_num"]
    ranges = (a0, a0 + n // 2 - 2, a0 + n // 2 - 1, a0 + n - 3, a0 + n - 2, a0 + n - 1)
    class _At:  # token ranges only (the tiny config's action vocabulary is not the canonical 8194)
        def __init__(self, lo, hi):
            self.token_start_idx, self.token_end_idx = lo, hi
    at = type("AT", (), {})()
    at.translation_tokenizer, at.rotation_tokenizer, at.gripper_tokenizer = (
        _At(ranges[0], ranges[1]), _At(ranges[2], ranges[3]), _At(ranges[4], ranges[5]))
    got = model.action_metrics(b["labels"], action_tokenizer=at)
    am = model.action_argmax().view(3, -1).cpu()
    top2 = out.logits.float().topk(2, -1).values.cpu()
    strict = top2[..., 0] > top2[..., 1]  # the epilogue argmax is of the same bf16 logits: equal wherever no tie
    assert torch.equal(am[strict], out.logits.float().argmax(-1).cpu()[strict])
    ref = O.action_metrics(am, b["labels"].cpu(), ranges)
    for k in NAMES:
        g, r = float(got[k]), ref[k]
        assert (np.isnan(g) and np.isnan(r)) or g == r, (k, g, r)
