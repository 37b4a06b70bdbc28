"""Which op of the B=1 prefill (predict_action, eager) still launches a vendor GEMM (Cijk_* = hipBLASLt)?  Prints the
torch ops whose CUDA kernels are Cijk_*, with shapes and the Python stack."""
import json, os, sys
os.environ["SVLA_DECODE_GRAPHS"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import profile, ProfilerActivity


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
        model.predict_action(inputs, max_new_tokens=2, eos_token_id=-1)
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
            model.predict_action(inputs, max_new_tokens=2, eos_token_id=-1)
            torch.cuda.synchronize()
    seen = 0
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and "Cijk" in ev.name:
            seen += 1
    print("Cijk kernels:", seen)
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        if ev.name in ("aten::addmm", "aten::mm", "aten::matmul", "aten::linear", "aten::bmm", "aten::baddbmm",
                       "aten::convolution", "aten::_convolution"):
            stack = [s for s in (ev.stack or []) if "site-packages" not in s][:4]
            print(ev.name, ev.input_shapes[:3], " | ", " <- ".join(stack) or (ev.stack or [])[:3])


main()
