"""Inference latency of SpatialVLA-4B greedy decode on one MI355X (BASELINE configs[1]: 1 image + prompt ->
action tokens, bf16), KV-cached (predict_action) beside the uncached re-forward (predict_action_uncached).

Prints one JSON line: prefill ms (SigLIP + Ego3D/Zoe + 299-token Gemma2 prefill + first token), ms per cached
decode token, and that step's weight-streaming roofline — a decode step at B=1 reads every Gemma2 weight and
the lm_head once (algorithmic bytes = their bf16 size), so achieved GB/s = bytes / step time against 8 TB/s.
Synthetic OXE-shaped prompt, random-init weights.
"""
import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timed(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        ev[0].record()
        out = fn()
        ev[1].record()
        torch.cuda.synchronize()
        times.append(ev[0].elapsed_time(ev[1]))
    times.sort()
    return times[len(times) // 2], out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--new-tokens", type=int, default=4)
    ap.add_argument("--long", type=int, default=36, help="extra tokens for the per-token slope")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-uncached", action="store_true")
    args = ap.parse_args()
    from bench import build_model, make_batch
    from spatialvla_amd import presets
    dev = torch.device("cuda:0")
    cfgd = json.loads(json.dumps(presets.spatialvla_4b()))
    model = build_model(cfgd, dev).eval()
    b = make_batch(cfgd, args.batch, 4321, dev)
    P = int((b["token_type_ids"][0] == 0).sum())  # prompt = image tokens + bos + prompt ids + "\n"
    inputs = {"input_ids": b["input_ids"][:, :P], "pixel_values": b["pixel_values"], "intrinsic": b["intrinsic"]}

    n_new, n_long = args.new_tokens, args.new_tokens + args.long
    pa = lambda n: model.predict_action(inputs, max_new_tokens=n, eos_token_id=-1)  # noqa: E731
    with torch.no_grad():
        pa(n_long)  # warm-up: kernel loads, hipBLASLt plans, and the decode-step graphs of every position
        t1, _ = timed(lambda: pa(1), args.reps)
        tn, toks = timed(lambda: pa(n_new), args.reps)
        tl, _ = timed(lambda: pa(n_long), max(3, args.reps // 2))
        per_tok = (tl - t1) / (n_long - 1)
        graphs_on = model.decode_graphs
        model.decode_graphs = False
        toks_eager = pa(n_new)
        model.decode_graphs = graphs_on
        res_unc = None
        if not args.no_uncached:
            tu, toks_u = timed(lambda: model.predict_action_uncached(inputs, max_new_tokens=n_new, eos_token_id=-1),
                               max(2, args.reps // 2))
            res_unc = {"ms": round(tu, 2), "tokens_equal": bool(torch.equal(toks, toks_u))}
    lm = model.language_model
    wbytes = sum(p.numel() * p.element_size() for p in lm.model.layers.parameters())
    wbytes += lm.lm_head.weight.numel() * lm.lm_head.weight.element_size()
    wbytes += lm.model.norm.weight.numel() * lm.model.norm.weight.element_size()
    gbs = wbytes / (per_tok * 1e-3) / 1e9
    graphs = bool(model.decode_graphs)
    print(json.dumps({
        "metric": "SpatialVLA-4B greedy decode latency (BASELINE configs[1])", "unit": "ms", "batch": args.batch,
        "prompt_tokens": P, "new_tokens": n_new, "ms_total": round(tn, 2), "ms_prefill_plus_first": round(t1, 2),
        "ms_per_decode_token": round(per_tok, 3), "tokens_per_s_decode": round(1000.0 * args.batch / per_tok, 1),
        "uncached": res_unc, "decode_graphs": graphs, "graph_tokens_equal_eager": bool(torch.equal(toks, toks_eager)),
        "decode_roofline": {"bound": "hbm", "algorithmic_bytes_per_token_step": wbytes, "achieved": round(gbs, 1),
                            "peak": 8000.0, "unit": "GB/s", "frac": round(gbs / 8000.0, 4)},
        "dtype": "bf16", "data": "synthetic OXE-shaped prompt, random-init weights"}), flush=True)


if __name__ == "__main__":
    main()
