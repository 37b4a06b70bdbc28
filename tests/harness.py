"""Shared parity harness: the HIP model (spatialvla_amd) vs the CPU oracle (oracle/spatialvla_oracle.py)
on the same deterministic weights and the same synthetic OXE-shaped batch.

Tolerances: logits rel-L2 <= 1e-2; per-tensor grad rel-L2 <= 3e-2 (bf16 end-to-end; typical
values are ~1e-2); action argmax identical wherever the oracle's top-1/top-2 margin exceeds 0.05 (bf16 logits
quantise at 1/32 near |30|), and reported separately on the labelled (action-token) rows.
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

SEED = 1234
LOGITS_TOL = 1e-2
GRAD_TOL = 3e-2
MARGIN = 0.05


def rel_l2(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def cfg_dict(name="tiny"):
    from spatialvla_amd import presets
    return json.loads(json.dumps(getattr(presets, name)()))


def build_hip_model(cfgd, device="cuda:0", seed=SEED):
    from spatialvla_amd import SpatialVLAConfig
    from spatialvla_amd.detinit import deterministic_init_
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    cfg = SpatialVLAConfig(**cfgd)
    if cfg.vision_zoe_config is not None:
        cfg.vision_zoe_config._attn_implementation = "eager"
        cfg.vision_zoe_config.backbone_config._attn_implementation = "eager"
    m = SpatialVLAForConditionalGeneration(cfg).to(torch.bfloat16)
    deterministic_init_(m, seed=seed)
    m.language_model.model.embed_tokens.weight.requires_grad_(False)
    if cfg.use_vision_zoe:
        m.vision_zoe_model.eval()
        for p in m.vision_zoe_model.parameters():
            p.requires_grad_(False)
    return m.to(device)


def build_oracle(cfgd, seed=SEED):
    import spatialvla_oracle as O
    from spatialvla_amd.detinit import deterministic_init_
    P = O.build_params(cfgd, seed)
    zoe = None
    if cfgd.get("use_vision_zoe", True):
        from transformers import ZoeDepthConfig, ZoeDepthForDepthEstimation
        zc = ZoeDepthConfig(**cfgd["vision_zoe_config"])
        zc._attn_implementation = "eager"
        zc.backbone_config._attn_implementation = "eager"
        zoe = ZoeDepthForDepthEstimation(zc).to(torch.bfloat16).eval()
        deterministic_init_(zoe, seed=seed, prefix="vision_zoe_model.")
    return P, zoe


def batch_tensors(b, device):
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    t["pixel_values"] = t["pixel_values"].to(torch.bfloat16)
    t["intrinsic"] = t["intrinsic"].to(torch.bfloat16)
    return {k: v.to(device) for k, v in t.items()}


def run_hip(model, batch, depth=None):
    """Training forward + backward on the HIP model; returns (loss, logits[B,L,V], grads by oracle name)."""
    if depth is not None:
        model.predict_depth = lambda pv, _d=depth: _d.to(pv.device)
    model.zero_grad(set_to_none=True)
    out = model(**{k: v for k, v in batch.items()}, return_dict=True)
    out.loss.backward()
    torch.cuda.synchronize()
    grads = {}
    for n, p in model.named_parameters():
        # under a TrainEngine the kernels write dW into the flat gradient buffer (p._svla_grad), not p.grad
        g = p.grad if p.grad is not None else (getattr(p, "_svla_grad", None) if p.requires_grad else None)
        if g is not None:
            grads[n.replace("vision_tower.vision_model.", "vision_tower.")] = g.detach().float().cpu()
    return out.loss.detach().float().cpu(), out.logits.detach().float().cpu(), grads, model.action_argmax()


def run_oracle(P, zoe, cfgd, batch_cpu, depth=None):
    import spatialvla_oracle as O
    for t in P.values():
        t.grad = None
    cap = {}
    loss, logits = O.forward(P, cfgd, batch_cpu, zoe, depth=depth, cap=cap)
    loss.backward()
    grads = {n: t.grad.float() for n, t in P.items() if t.grad is not None}
    return loss.detach().float(), logits.detach().float(), grads, cap


def compare(loss_h, logits_h, grads_h, argmax_h, loss_r, logits_r, grads_r, labels=None):
    B, L, V = logits_r.shape
    res = {"loss_hip": float(loss_h), "loss_ref": float(loss_r), "logits_rel": rel_l2(logits_h, logits_r)}
    rels = {}
    for n, g in grads_r.items():
        if n not in grads_h:
            continue
        if n.endswith("self_attn.k_proj.bias"):
            # d loss / d k_bias is analytically 0 (softmax is invariant to a per-row shift q.b); both sides
            # hold rounding noise only: require the same noise scale instead of a relative error
            rels[n] = 0.0 if grads_h[n].norm() <= 3 * g.float().norm() + 1e-3 else float("inf")
        else:
            rels[n] = rel_l2(grads_h[n], g)
    missing = sorted(set(grads_r) - set(grads_h))
    res["grad_rel"] = rels
    res["grad_rel_max"] = max(rels.values()) if rels else 0.0
    res["grads_missing"] = missing
    ref_top2 = logits_r[:, :-1].topk(2, -1).values
    margin = ref_top2[..., 0] - ref_top2[..., 1]
    ref_am = logits_r[:, :-1].argmax(-1)
    hip_am = argmax_h.view(B, L)[:, :-1].cpu()
    agree = hip_am == ref_am
    conf = margin > MARGIN
    res["argmax_agree"] = float(agree.float().mean())
    res["argmax_agree_confident"] = float(agree[conf].float().mean()) if conf.any() else 1.0
    if labels is not None:  # the action rows: positions whose next token is a label (the CE / accuracy rows)
        act = labels[:, 1:].cpu() != -100
        res["argmax_agree_action_rows"] = float(agree[act].float().mean()) if act.any() else 1.0
        res["argmax_agree_action_rows_confident"] = float(agree[act & conf].float().mean()) if (act & conf).any() else 1.0
    return res


def greedy_tokens_agree(got: torch.Tensor, ref: torch.Tensor, margins: torch.Tensor, tol: float = MARGIN):
    """Greedy tokens vs the reference's: per sequence, every step must match until the first step whose
    reference top-1/top-2 margin is <= tol (a near-tie that fp rounding may legitimately flip, after which the
    sequences diverge).  Returns (#steps compared, #steps matched)."""
    got, ref, margins = got.cpu(), ref.cpu(), margins.float().cpu()
    n_cmp = n_ok = 0
    for b in range(ref.shape[0]):
        for s in range(ref.shape[1]):
            n_cmp += 1
            if int(got[b, s]) == int(ref[b, s]):
                n_ok += 1
                continue
            assert float(margins[b, s]) <= tol, (b, s, int(got[b, s]), int(ref[b, s]), float(margins[b, s]))
            break
    return n_cmp, n_ok


def tiny_parity_run(device="cuda:0", batch=2, seed=7, ragged=False):
    """End-to-end tiny-config parity: HIP model on `device` vs CPU oracle, same weights and batch.
    The oracle's depth map is fed to both sides so the frozen 3p depth estimator's GPU/CPU numerics
    do not mask hot-path differences (depth parity is tested separately)."""
    from spatialvla_amd import presets
    cfgd = cfg_dict("tiny")
    b = presets.synthetic_batch(cfgd, batch=batch, seed=seed, ragged=ragged)
    bc = batch_tensors(b, "cpu")
    P, zoe = build_oracle(cfgd)
    loss_r, logits_r, grads_r, cap = run_oracle(P, zoe, cfgd, bc)
    model = build_hip_model(cfgd, device)
    bd = {k: v.to(device) for k, v in bc.items()}
    loss_h, logits_h, grads_h, am = run_hip(model, bd, depth=cap["depth"])
    return compare(loss_h, logits_h, grads_h, am, loss_r, logits_r, grads_r, labels=bc["labels"])
