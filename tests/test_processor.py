"""SpatialVLAProcessor (the AutoProcessor half of the drop-in) against golden outputs of the reference's own
SpatialVLAProcessor (oracle/gen_processor_golden.py): prompt layout, token ids, token types, labels, pixel values,
scaled intrinsics and decode_actions, exactly.  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

import processor_fixtures as PF

GOLD = os.path.join(os.path.dirname(__file__), "golden", "processor.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


def _proc(gold):
    from spatialvla_amd import SpatialVLAProcessor
    return SpatialVLAProcessor(PF.build_image_processor(), PF.build_tokenizer(),
                               statistics=json.loads(str(gold["statistics"])),
                               intrinsic_config=json.loads(str(gold["intrinsic_config"])),
                               action_config=json.loads(str(gold["action_config"])), action_chunk_size=4)


def _cases(gold):
    from PIL import Image
    imgs = [Image.fromarray(a) for a in gold["images"]]
    return {
        "train": dict(images=imgs[0], text="What action should the robot take to pick the cup?",
                      unnorm_key="bridge_orig/1.0.0", suffix_actions=gold["suffix_actions"], return_tensors="pt"),
        "infer_batch": dict(images=imgs[:2], text=["pick up the cup", "open the drawer"], unnorm_key="nope",
                            return_tensors="pt"),
        "image_token_in_prompt": dict(images=[imgs[2]], text=["<image>stack the blocks"], unnorm_key="default",
                                      return_tensors="pt"),
        "text_suffix": dict(images=imgs[1], text="move", suffix="left", unnorm_key="bridge_orig/1.0.0",
                            return_tensors="pt"),
    }


def test_processor_call_matches_reference(gold):
    proc = _proc(gold)
    assert proc.image_token_id == int(gold["image_token_id"])
    assert proc.action_tokenizer.action_token_begin_idx == int(gold["action_begin"])
    for name, kw in _cases(gold).items():
        bf = proc(**kw)
        keys = {k.split("/", 1)[1] for k in gold if k.startswith(name + "/")}
        assert set(bf.keys()) == keys, (name, set(bf.keys()), keys)
        for k in keys:
            got = bf[k].numpy() if hasattr(bf[k], "numpy") else np.asarray(bf[k])
            np.testing.assert_array_equal(got, gold[f"{name}/{k}"], err_msg=f"{name}/{k}")


def test_processor_layout_is_the_training_batch_layout(gold):
    proc = _proc(gold)
    bf = proc(**_cases(gold)["train"])
    ids, tt, lab = bf["input_ids"][0], bf["token_type_ids"][0], bf["labels"][0]
    n_img = int((ids == proc.image_token_id).sum())
    assert n_img == 256 and int(ids[256]) == proc.tokenizer.bos_token_id
    assert int(tt.sum()) == 13 and int(ids[-1]) == proc.tokenizer.eos_token_id      # 12 action tokens + eos
    a0 = proc.action_tokenizer.action_token_begin_idx
    assert bool(((ids[-13:-1] >= a0) & (ids[-13:-1] < a0 + 8194)).all())
    assert torch.equal(lab[tt == 1], ids[tt == 1]) and bool((lab[tt == 0] == -100).all())


def test_decode_actions_matches_reference(gold):
    proc = _proc(gold)
    res = proc.decode_actions(torch.from_numpy(gold["decode/gen"]), unnorm_key="bridge_orig/1.0.0")
    np.testing.assert_array_equal(res["actions"], gold["decode/actions"])
    np.testing.assert_array_equal(res["action_ids"], gold["decode/action_ids"])


def test_processor_save_load_roundtrip(gold, tmp_path):
    from spatialvla_amd import SpatialVLAProcessor
    proc = _proc(gold)
    proc.save_pretrained(str(tmp_path))
    back = SpatialVLAProcessor.from_pretrained(str(tmp_path))
    kw = _cases(gold)["train"]
    a, b = proc(**kw), back(**kw)
    for k in a:
        assert torch.equal(torch.as_tensor(a[k]), torch.as_tensor(b[k])), k
    assert back.action_chunk_size == 4 and back.statistics == proc.statistics


def test_package_exports_reference_names():
    import spatialvla_amd as S
    for n in ("SpatialVLAConfig", "SpatialVLAForConditionalGeneration", "SpatialVLAPreTrainedModel",
              "Gemma2ForCausalLM", "SpatialVLAProcessor", "SpatialActionTokenizer", "ActionTokenizer"):
        assert getattr(S, n) is not None and n in S.__all__
