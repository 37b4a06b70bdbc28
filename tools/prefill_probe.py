"""Time and trace predict_action(max_new_tokens=1) (vision + Zoe + Gemma2 prefill + first token) at B=1."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bench import build_model, make_batch
    from spatialvla_amd import presets
    dev = torch.device("cuda:0")
    cfgd = json.loads(json.dumps(presets.spatialvla_4b()))
    model = build_model(cfgd, dev).eval()
    b = make_batch(cfgd, 1, 4321, dev)
    P = int((b["token_type_ids"][0] == 0).sum())
    inputs = {"input_ids": b["input_ids"][:, :P], "pixel_values": b["pixel_values"], "intrinsic": b["intrinsic"]}
    with torch.no_grad():
        for _ in range(3):
            model.predict_action(inputs, max_new_tokens=1, eos_token_id=-1)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        parts = {}
        for name, fn in (("depth", lambda: model.predict_depth(inputs["pixel_values"])),
                         ("image_features", lambda: model.get_image_features(inputs["pixel_values"],
                                                                             inputs["intrinsic"])),
                         ("predict_1", lambda: model.predict_action(inputs, max_new_tokens=1, eos_token_id=-1))):
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            parts[name] = round(sorted(ts)[2], 2)
    print(json.dumps({"prefill_parts_ms": parts}), flush=True)


if __name__ == "__main__":
    main()
