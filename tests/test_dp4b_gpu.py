"""BASELINE configs[3]'s code path at the 4B workload: the ZeRO-1 exchange of TrainEngine (scripts/zero1.json:2-10)
with the real SpatialVLA-4B bucket layout (~25 buckets of 256 MB, lm_head larger than one bucket) and the per-layer
gradient hooks at full depth (26 Gemma2 + 27 SigLIP layers), 2 ranks over gloo, both on cuda:0 (the GPU box has one
card; the 8-GPU RCCL run is the driver's), against one process training on the concatenated batch.

Each rank trains on one episode of a 2-episode synthetic OXE batch for 2 steps; the single process on both episodes.
Compared on sampled tensors (whole parameters, lm_head a row block), gathered from the ranks' owned ZeRO chunks:
  * loss: the label-count-weighted mean of the rank losses equals the single-process loss (5e-3 relative), step 2
    included -- so the all-gathered parameters of step 1 are the single process's;
  * grad norm (after the reduce-scatter, clip input): 2e-2 relative;
  * step 1 (identical weights on every process), the exchange: each rank's owned chunks after the bf16 AVG
    reduce-scatter equal the fp32 mean of the two ranks' local gradients (captured as each bucket enters the
    reduce-scatter) within one bf16 rounding of the addends' magnitude, elementwise;
  * step 1, the model: that mean vs the single process's gradient, rel-L2 <= GRAD_TOL (3e-2, every tensor) on the
    scale of the addends, max(||g_single||, ||(|g_0| + |g_1|) / 2||) -- a
    gradient summed over two halves that cancel (the last SigLIP q bias) carries the halves' bf16 rounding.  The
    per-rank GEMMs see M = 312 instead of 624 rows (other tile / stream-K schedules, other fp32 partial-sum orders);
  * step 2, bounded by a measured noise floor: AdamW's first update is lr * g / |g| elementwise, so every element
    whose step-1 gradient is at bf16 noise level moves by +-lr on one side and -+lr on the other (update rel-L2
    ~0.1, r4 measurement) and the step-2 gradients are those of different weights.  The floor is the same quantity
    between two single-process runs that differ only in GEMM blocking (SVLA gemm variant 2: no stream-K, no tail
    split, so other fp32 partial-sum orders); the DP step-2 gradient (on the addends' scale, as step 1) must stay
    within 2 * floor + 0.02 of the single process's;
  * the fp32 masters after 2 AdamW steps: every element within 2 * steps * lr of the single process's (AdamW moves an
    element by at most lr per step), and the ranks' bf16 parameters bitwise identical.
The measured numbers go to gpurun_out/parity/dp4b.json."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import harness as H

pytestmark = pytest.mark.gpu

STEPS = 2
WORLD = 2
LR = 1e-4
# (parameter name, first row, rows) -- rows None = the whole tensor
SAMPLES = [
    ("language_model.model.layers.0.self_attn.q_proj.weight", 0, None),
    ("language_model.model.layers.0.self_attn.v_proj.weight", 0, None),
    ("language_model.model.layers.12.mlp.down_proj.weight", 0, None),
    ("language_model.model.layers.25.mlp.gate_proj.weight", 0, None),
    ("language_model.model.layers.25.self_attn.o_proj.weight", 0, None),
    ("language_model.model.layers.3.post_feedforward_layernorm.weight", 0, None),
    ("language_model.model.norm.weight", 0, None),
    ("language_model.lm_head.weight", 257153, 4096),   # the first 4096 action-token rows
    ("language_model.lm_head.weight", 1000, 2048),
    ("spatial_embed_tokens.weight", 0, None),
    ("multi_modal_projector.linear.weight", 0, None),
    ("vision_tower.vision_model.encoder.layers.5.mlp.fc1.weight", 0, None),
    ("vision_tower.vision_model.encoder.layers.26.self_attn.q_proj.bias", 0, None),
    ("vision_tower.vision_model.embeddings.patch_embedding.weight", 0, None),
    ("position_embedding_3d.position_embedding_head.0.weight", 0, None),
]


def _grad_tol(name):
    """GRAD_TOL for every sampled tensor at step 1 (measured r4: max 2.5e-2, spatial_embed_tokens; the q/k-projection
    exception of test_full4b_gpu.py is not needed here: layer 0 q_proj 1.8e-2)."""
    return H.GRAD_TOL


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(device):
    from spatialvla_amd import SpatialVLAConfig, presets
    from spatialvla_amd.detinit import hash_init_
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    cfg = SpatialVLAConfig(**json.loads(json.dumps(presets.spatialvla_4b())))
    cfg.vision_zoe_config._attn_implementation = "eager"
    cfg.vision_zoe_config.backbone_config._attn_implementation = "eager"
    with torch.device(device):
        m = SpatialVLAForConditionalGeneration(cfg)
    m = m.to(torch.bfloat16)
    hash_init_(m, seed=H.SEED)
    m.language_model.model.embed_tokens.weight.requires_grad_(False)
    m.vision_zoe_model.eval()
    for p in m.vision_zoe_model.parameters():
        p.requires_grad_(False)
    m.train()
    m.vision_zoe_model.eval()
    return m


def _batches(device):
    from spatialvla_amd import presets
    cfgd = H.cfg_dict("spatialvla_4b")
    return [H.batch_tensors(presets.synthetic_batch(cfgd, batch=WORLD, seed=300 + s), device) for s in range(STEPS)]


def _owned_samples(eng, names):
    """{(name, row0): (flat element indices relative to the slice, averaged grad, fp32 master, digest of the whole
    bf16 slice, slice length)} for the parts of each sampled slice inside this rank's owned ZeRO chunks."""
    import hashlib
    ex = eng.exchange
    pidx = {id(p): i for i, p in enumerate(eng.params)}
    out = {}
    for name, r0, nr in SAMPLES:
        p = names[name]
        i = pidx[id(p)]
        row = p.numel() // p.shape[0] if p.dim() > 1 else 1
        lo = eng.offsets[i] + r0 * row
        hi = lo + (nr * row if nr is not None else p.numel() - r0 * row)
        idx, g, m = [], [], []
        digest = hashlib.sha1(eng.flat_param[lo:hi].view(torch.int16).cpu().numpy().tobytes()).hexdigest()
        for b in range(len(eng.buckets)):
            o, c = ex.owned(b)
            a, e = max(lo, o), min(hi, o + c)
            if a >= e:
                continue
            so = eng.shard_offsets[b] + (a - o)
            idx.append(np.arange(a - lo, e - lo))
            g.append(eng.flat_grad[a:e].float().cpu().numpy())
            m.append(eng.master[so:so + (e - a)].cpu().numpy())
        cat = (lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.float32))  # noqa: E731
        out[(name, r0)] = (np.concatenate(idx) if idx else np.zeros(0, np.int64), cat(g), cat(m), digest, hi - lo)
    return out


def _slices(eng, names):
    pidx = {id(p): i for i, p in enumerate(eng.params)}
    out = {}
    for name, r0, nr in SAMPLES:
        p = names[name]
        row = p.numel() // p.shape[0] if p.dim() > 1 else 1
        lo = eng.offsets[pidx[id(p)]] + r0 * row
        out[(name, r0)] = (lo, lo + (nr * row if nr is not None else p.numel() - r0 * row))
    return out


def _capture_local(eng, names):
    """Wrap the exchange's reduce-scatter so that each bucket's local (pre-exchange) gradient of the sampled slices is
    copied out as the bucket enters the collective.  Returns the {(name, row0): fp32 array} being filled."""
    ex = eng.exchange
    sl = _slices(eng, names)
    local = {k: np.full(hi - lo, np.nan, np.float32) for k, (lo, hi) in sl.items()}
    orig = ex._reduce_scatter

    def rs(b):
        s, e = ex.buckets[b]
        for k, (lo, hi) in sl.items():
            a, z = max(lo, s), min(hi, e)
            if a < z:
                local[k][a - lo:z - lo] = ex.fg[a:z].float().cpu().numpy()
        orig(b)

    ex._reduce_scatter = rs
    return local, orig


def _train(rank, world, device):
    from spatialvla_amd.engine import TrainEngine
    model = _model(device)
    names = dict(model.named_parameters())
    per = WORLD // world
    depth = torch.rand(WORLD, 1, 224, 224, generator=torch.Generator().manual_seed(11)).mul(3).add(0.5).to(device)
    model.predict_depth = lambda pv, _d=depth[rank * per:(rank + 1) * per]: _d
    init = {}
    for name, r0, nr in SAMPLES:
        t = names[name].detach()
        t = t.reshape(t.shape[0], -1)[r0:(r0 + nr if nr is not None else None)] if t.dim() > 1 else t
        init[(name, r0)] = t.float().cpu().numpy().ravel().copy()
    eng = TrainEngine(model, lr=LR, warmup_ratio=0.0, total_steps=100, max_grad_norm=1.0)
    losses, gnorms, samples, locals_ = [], [], [], []
    local, orig = _capture_local(eng, names) if world > 1 else (None, None)
    for s, b in enumerate(_batches(device)):
        part = {k: v[rank * per:(rank + 1) * per] for k, v in b.items()}
        losses.append(float(eng.train_step(part).item()))
        gnorms.append(float(eng.gnorm.item()))
        if world == 1:
            local = {k: eng.flat_grad[lo:hi].float().cpu().numpy() for k, (lo, hi) in _slices(eng, names).items()}
        assert all(not np.isnan(v).any() for v in local.values()), "a sampled slice was never reduce-scattered"
        locals_.append({k: v.copy() for k, v in local.items()})
        for v in local.values():
            v.fill(np.nan)  # the next step's reduce-scatter must fill every sampled element again
        eng.sync_params()
        torch.cuda.synchronize()
        samples.append(_owned_samples(eng, names))
    if world > 1:
        eng.exchange._reduce_scatter = orig
    return {"losses": losses, "gnorms": gnorms, "samples": samples, "local": locals_, "init": init,
            "nbuckets": len(eng.buckets), "hooked": len(eng.exchange.ready_end)}


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _train(rank, world, "cuda:0")))
    except Exception as e:  # surface the failure instead of a queue timeout
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _assemble(parts, key):
    n = parts[0][key][4]
    g, m = (np.full(n, np.nan, np.float32) for _ in range(2))
    cover = np.zeros(n, np.int64)
    for r in parts:
        idx, gg, mm, _, _ = r[key]
        g[idx], m[idx] = gg, mm
        cover[idx] += 1
    return g, m, cover


@pytest.mark.timeout(1100)
def test_dp2_zero1_4b_equals_single_process(cuda):
    torch.cuda.empty_cache()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=900) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
    for r, v in res:
        assert isinstance(v, dict), (r, v)
    assert all(p.exitcode == 0 for p in procs)
    ranks = [v for _, v in res]
    single = _train(0, 1, "cuda:0")
    from spatialvla_amd import kernels as Kn
    v0 = Kn.gemm_variant
    Kn.gemm_variant = 2  # the noise floor: the same single-process training with other GEMM blockings
    try:
        alt = _train(0, 1, "cuda:0")
    finally:
        Kn.gemm_variant = v0
    assert ranks[0]["nbuckets"] > 16 and ranks[0]["hooked"] >= 26 + 27  # the real 4B layout, every layer hooked
    report = {"losses_dp": [r["losses"] for r in ranks], "losses_single": single["losses"],
              "gnorm_dp": ranks[0]["gnorms"], "gnorm_single": single["gnorms"], "tensors": {}}
    for s in range(STEPS):
        mean = float(np.mean([r["losses"][s] for r in ranks]))  # 13 labelled tokens per episode: equal weights
        assert abs(mean - single["losses"][s]) <= 5e-3 * abs(single["losses"][s]), (s, mean, single["losses"][s])
        for r in ranks:
            assert r["gnorms"][s] == ranks[0]["gnorms"][s]
        assert ranks[0]["gnorms"][s] == pytest.approx(single["gnorms"][s], rel=2e-2)
    bound = 2 * STEPS * LR * 1.05
    for name, r0, _ in SAMPLES:
        key = (name, r0)
        rec = {}
        for s in range(STEPS):
            g, m, cover = _assemble([r["samples"][s] for r in ranks], key)
            assert (cover == 1).all(), (key, "owned chunks must tile every parameter exactly once")
            idx1, g1, m1, _, _ = single["samples"][s][key]
            assert np.array_equal(idx1, np.arange(len(g1)))
            l0, l1 = (r["local"][s][key] for r in ranks)
            mean = 0.5 * (l0 + l1)
            mag = 0.5 * (np.abs(l0) + np.abs(l1))
            scale = max(float(np.linalg.norm(g1)), float(np.linalg.norm(mag)), 1e-30)
            ga = alt["samples"][s][key][1]
            if s == 0:
                rec["exchange_excess"] = float(np.max(np.abs(g - mean) - 2.0 ** -8 * mag))  # <= 0: within bound
                rec["grad_rel"] = float(np.linalg.norm(mean - g1) / scale)
                rec["grad_rel_plain"] = float(np.linalg.norm(mean - g1) / max(float(np.linalg.norm(g1)), 1e-30))
                rec["grad_tol"] = _grad_tol(name)
                rec["floor_step1"] = float(np.linalg.norm(ga - g1) / scale)
            else:
                rec["grad_rel_step2"] = float(np.linalg.norm(mean - g1) / scale)
                rec["grad_rel_step2_plain"] = float(np.linalg.norm(g - g1) / max(float(np.linalg.norm(g1)), 1e-30))
                rec["floor_step2"] = float(np.linalg.norm(ga - g1) / scale)
            if s == STEPS - 1:
                p0 = single["init"][key]
                d1 = m1 - p0
                rec["update_rel"] = float(np.linalg.norm((m - p0) - d1) / max(float(np.linalg.norm(d1)), 1e-30))
                rec["master_maxdiff"] = float(np.abs(m - m1).max())
                rec["ranks_bitwise"] = len({r["samples"][s][key][3] for r in ranks}) == 1
        report["tensors"][f"{name}[{r0}:]"] = rec
    d = os.environ.get("SVLA_PARITY_DIR", os.path.join(H.REPO, "gpurun_out", "parity"))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "dp4b.json"), "w") as f:
        json.dump(report, f, indent=1)
    print("dp4b:", json.dumps({k: v for k, v in report.items() if k != "tensors"}),
          {k: (round(v["grad_rel"], 5), round(v["floor_step1"], 5), round(v["grad_rel_step2"], 5),
               round(v["floor_step2"], 5)) for k, v in report["tensors"].items()})
    for k, v in report["tensors"].items():
        assert v["exchange_excess"] <= 0.0, (k, v)
        # step 1: GRAD_TOL, or twice the same-process noise floor where the GEMM blockings alone move a tensor more
        # (the short-M split-K dispatch: per-rank SigLIP GEMMs of 256 rows split k unlike the 512-row single process;
        # SigLIP layer 26 q bias measured 4.3e-2 against a 3.8e-2 floor)
        assert v["grad_rel"] <= max(v["grad_tol"], 2.0 * v["floor_step1"]), (k, v)
        assert v["grad_rel_step2"] <= 2.0 * v["floor_step2"] + 0.02, (k, v)
        assert v["master_maxdiff"] <= bound, (k, v, bound)
        assert v["ranks_bitwise"], k  # the ranks' bf16 parameters after the all-gather: bitwise identical
