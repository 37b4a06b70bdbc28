"""Golden vectors for SpatialVLAProcessor (__call__ and decode_actions), produced by the REFERENCE itself.

TEST INFRASTRUCTURE ONLY (container-side; needs /root/reference).  Imports the reference's
model/processing_spatialvla.py and runs SpatialVLAProcessor on a small Gemma tokenizer and the SigLIP image
processor (tests/processor_fixtures.py).  transformers 5 removed four PaliGemma helpers the reference imports; they
are restated here from transformers 4.47 (the reference's pin, requirements.txt:20), with the 4.47
PaliGemmaProcessorKwargs defaults:
  _validate_images_text_input_order -> swap (text, images) given in that order; make_batched_images -> flatten a
  list of lists; build_string_from_input -> image tokens * n + bos + prompt + "\\n"; _is_str_or_image.
Writes tests/golden/processor.npz.  The reference module is imported, never copied.

    python oracle/gen_processor_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden", "processor.npz")
sys.path.insert(0, os.path.join(REPO, "tests"))
import processor_fixtures as PF  # noqa: E402


def _shim():
    import transformers.processing_utils as pu
    import transformers.models.paligemma.processing_paligemma as pp
    from transformers.image_utils import is_valid_image

    def is_str_or_image(elem):
        return isinstance(elem, str) or is_valid_image(elem)

    def validate_order(images, text):
        def texty(x):
            return isinstance(x, str) or (isinstance(x, list) and x and all(isinstance(t, str) for t in x))
        if texty(images) and text is not None and not texty(text):
            return text, images
        return images, text

    def make_batched_images(images):
        if isinstance(images, (list, tuple)) and images and isinstance(images[0], (list, tuple)):
            return [img for sub in images for img in sub]
        return list(images) if isinstance(images, (list, tuple)) else [images]

    def build_string_from_input(prompt, bos_token, image_seq_len, image_token, num_images):
        return f"{image_token * image_seq_len * num_images}{bos_token}{prompt}\n"

    pu._validate_images_text_input_order = validate_order
    pp.make_batched_images = make_batched_images
    pp.build_string_from_input = build_string_from_input
    pp._is_str_or_image = is_str_or_image
    pp.PaliGemmaProcessorKwargs._defaults = {"text_kwargs": {"padding": False},
                                             "images_kwargs": {"data_format": "channels_first"}}
    sys.path.insert(0, REF)
    from model import processing_spatialvla as ps
    return ps


def main():
    ps = _shim()
    intr = json.load(open(os.path.join(REF, "scripts", "intrinsics.json")))
    acfg = json.load(open(os.path.join(REF, "scripts", "action_config.json")))
    rng = np.random.default_rng(11)
    stats = {"bridge_orig/1.0.0": {"action": {"q01": list(rng.uniform(-0.05, -0.01, 7)),
                                              "q99": list(rng.uniform(0.01, 0.05, 7)),
                                              "mask": [True] * 6 + [False]}}}
    proc = ps.SpatialVLAProcessor(PF.build_image_processor(), PF.build_tokenizer(), statistics=stats,
                                  intrinsic_config=intr, action_config=acfg, action_chunk_size=4)
    out = {"intrinsic_config": np.array(json.dumps(intr)), "action_config": np.array(json.dumps(acfg)),
           "statistics": np.array(json.dumps(stats))}
    imgs = PF.images(3, seed=5)
    acts = rng.uniform(-1, 1, (4, 7))
    cases = {
        "train": dict(images=imgs[0], text="What action should the robot take to pick the cup?",
                      unnorm_key="bridge_orig/1.0.0", suffix_actions=acts, return_tensors="pt"),
        "infer_batch": dict(images=imgs[:2], text=["pick up the cup", "open the drawer"], unnorm_key="nope",
                            return_tensors="pt"),
        "image_token_in_prompt": dict(images=[imgs[2]], text=["<image>stack the blocks"], unnorm_key="default",
                                      return_tensors="pt"),
        "text_suffix": dict(images=imgs[1], text="move", suffix="left", unnorm_key="bridge_orig/1.0.0",
                            return_tensors="pt"),
    }
    for name, kw in cases.items():
        bf = proc(**kw)
        for k, v in bf.items():
            out[f"{name}/{k}"] = np.asarray(v.numpy() if hasattr(v, "numpy") else v)
        print(name, {k: tuple(np.asarray(v).shape) for k, v in bf.items()})
    out["suffix_actions"] = acts
    gen = np.concatenate([out["train/input_ids"][:, -13:-1], np.array([[1]])], axis=1)
    res = proc.decode_actions(__import__("torch").from_numpy(gen), unnorm_key="bridge_orig/1.0.0")
    out["decode/gen"] = gen
    out["decode/actions"] = res["actions"]
    out["decode/action_ids"] = res["action_ids"]
    out["image_token_id"] = np.array(proc.image_token_id)
    out["action_begin"] = np.array(proc.action_tokenizer.action_token_begin_idx)
    out["images"] = np.stack([np.asarray(im) for im in imgs])
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays")


if __name__ == "__main__":
    main()
