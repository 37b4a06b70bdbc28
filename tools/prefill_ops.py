"""Diagnostic: the ATen ops (outside libsvla) that the 4B predict_action prefill dispatches, then a graph-captured
predict_action.  Used to find stock ops that call a vendor library under a HIP graph capture."""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from spatialvla_amd import presets  # noqa: E402

BLAS = ("mm", "addmm", "bmm", "baddbmm", "_scaled_mm", "addmv", "mv", "matmul", "linear", "dot", "_addmm_activation")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()
        self.where = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        self.ops[name] += 1
        if name in BLAS + ("_local_scalar_dense",):
            self.where.setdefault(name, []).append("".join(traceback.format_stack(limit=10)[:-1]))
        return func(*args, **(kwargs or {}))


def main():
    dev = torch.device("cuda", 0)
    cfgd = presets.spatialvla_4b()
    model = bench.build_model(cfgd, dev)
    b = bench.make_batch(cfgd, 1, 4321, dev)
    P = int((b["token_type_ids"][0] == 0).sum())
    inputs = {"input_ids": b["input_ids"][:, :P], "pixel_values": b["pixel_values"], "intrinsic": b["intrinsic"]}
    model.eval()
    model.decode_graphs = False
    with torch.no_grad():
        model.predict_action(inputs, max_new_tokens=2, eos_token_id=-1)
        log = Log()
        with log:
            model.predict_action(inputs, max_new_tokens=2, eos_token_id=-1)
    torch.cuda.synchronize()
    print("ATen ops in eager predict_action:", dict(log.ops.most_common()), flush=True)
    for k, v in log.where.items():
        for i, w in enumerate(v[:6]):
            print(f"--- {k} #{i}:\n{w}", flush=True)
    model.decode_graphs = True
    orig = model._prefill_body

    class Print(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            shapes = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)][:3]
            print("capture op", func.__name__, shapes, flush=True)
            return func(*args, **(kwargs or {}))

    def body(st, x):
        if torch.cuda.is_current_stream_capturing():
            with Print():
                return orig(st, x)
        return orig(st, x)
    model._prefill_body = body
    with torch.no_grad():
        out = model.predict_action(inputs, max_new_tokens=4, eos_token_id=-1)
    torch.cuda.synchronize()
    print("graph predict_action ok", out.tolist() if hasattr(out, "tolist") else out, flush=True)


if __name__ == "__main__":
    main()
