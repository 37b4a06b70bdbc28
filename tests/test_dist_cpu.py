"""World-size-2 gloo tests (CPU) of the data-parallel exchange (spatialvla_amd.engine: ZeRO-1 reduce-scatter of
the flat gradient buffer, sharded optimizer state, all-gather of the parameters; scripts/zero1.json).

The tiny SpatialVLA model is built on the CPU (modules only: its forward needs the HIP kernels, exercised by the
GPU test tests/test_dp_gpu.py).  Each rank writes its own synthetic gradients into the flat buffer, the layer
hooks fire in backward order as the autograd hooks would, and the optimizer math is a torch stand-in injected
into the engine (the HIP AdamW has its own GPU test).  Checked: every rank ends with the parameters a single
process computes from the mean gradient (= the gradient of the concatenated batch for a mean loss), buckets go
out before finish_reduce(), and the sharded optimizer state covers the flat buffer exactly once."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class TorchOptKernels:
    """fp32 torch statement of svla_sumsq_bf16 / svla_clip_scale / svla_adamw (include/svla.h) for the CPU tests."""

    @staticmethod
    def sumsq(x, out):
        out.copy_(x.float().pow(2).sum().reshape(1))

    @staticmethod
    def clip_scale(sumsq, max_norm, clip, norm_out):
        nrm = sumsq.sqrt()
        norm_out.copy_(nrm)
        clip.copy_(torch.clamp(max_norm / (nrm + 1e-6), max=1.0))

    @staticmethod
    def adamw(master, param, grad, m, v, lr, b1, b2, eps, wd, step, clip):
        g = grad.float() * clip
        m.mul_(b1).add_((1 - b1) * g)
        v.mul_(b2).add_((1 - b2) * g * g)
        bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
        master.sub_(lr * ((m / bc1) / ((v / bc2).sqrt() + eps) + wd * master))
        param.copy_(master.to(torch.bfloat16))


def _tiny_model():
    sys.path.insert(0, REPO)
    from spatialvla_amd import SpatialVLAConfig, presets
    from spatialvla_amd.detinit import deterministic_init_
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    cfg = SpatialVLAConfig(**presets.tiny())
    model = SpatialVLAForConditionalGeneration(cfg).to(torch.bfloat16)
    deterministic_init_(model, seed=3)
    model.language_model.model.embed_tokens.weight.requires_grad_(False)
    if cfg.use_vision_zoe:
        for p in model.vision_zoe_model.parameters():
            p.requires_grad_(False)
    return model


def _fake_backward(engine, grads):
    """Write grads (flat, in the flat layout) and fire the layer hooks in backward order, as autograd does."""
    ex = engine.exchange
    model = engine.model
    nl = len(model.language_model.model.layers)
    ns = len(model.vision_tower.vision_model.encoder.layers)
    engine.flat_grad.copy_(grads)
    launched = []
    for i in reversed(range(nl)):
        ex.on_grads_ready(("gemma", i))
        launched.append(len(ex._rs))
    for i in reversed(range(ns)):
        ex.on_grads_ready(("siglip", i))
        launched.append(len(ex._rs))
    return launched


def _rank_grads(n, step, rank):
    g = torch.Generator().manual_seed(1000 * step + 17 * rank + 1)
    return (torch.randn(n, generator=g) * 0.05).to(torch.bfloat16)


def _worker(rank, world, port, bucket_bytes, steps, q, reduce_only=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spatialvla_amd.engine import TrainEngine
        model = _tiny_model()
        eng = TrainEngine(model, lr=1e-3, warmup_ratio=0.0, total_steps=100, bucket_bytes=bucket_bytes,
                          max_grad_norm=0.5, kernels=TorchOptKernels)
        n = eng.numel
        if reduce_only:  # the averaged gradient chunks this rank owns after the bf16 AVG reduce-scatter
            _fake_backward(eng, _rank_grads(n, 0, rank))
            eng.exchange.finish_reduce()
            own = [(o, eng.flat_grad[o:o + c].float().numpy().copy()) for o, c in
                   (eng.exchange.owned(b) for b in range(len(eng.buckets)))]
            q.put((rank, own, eng.buckets, n))
            return
        early = []
        for step in range(steps):
            grads = _rank_grads(n, step, rank)
            early.append(_fake_backward(eng, grads))
            eng.exchange.finish_reduce()
            eng.optimizer_step()
            eng.sync_params()
        full = eng.full_master()
        # numpy, pickled by value: a shared-memory tensor would vanish with this process
        q.put((rank, eng.flat_param.float().numpy().copy(), full.numpy().copy(), early, eng.buckets, n,
               eng.shard_numel, float(eng.gnorm.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bucket_bytes", [(2, 1 << 14), (2, 1 << 30), (8, 1 << 14)])
def test_zero1_exchange_gloo(world, bucket_bytes):
    """world 2 against the single process bit for bit in the gradient (one bf16 rounding of a 2-term sum is the fp32
    mean rounded); world 8 (the configs[3] rank count) within the AdamW bound: the 8-term bf16 ring sum rounds at
    every hop, which can flip the sign of a noise-level element's normalised update."""
    steps = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_bytes, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference on the mean gradient; the flat layout differs (bucket padding depends on the
    # world size), so compare per parameter
    from spatialvla_amd.engine import TrainEngine
    model1 = _tiny_model()
    eng1 = TrainEngine(model1, lr=1e-3, warmup_ratio=0.0, total_steps=100, bucket_bytes=bucket_bytes,
                       max_grad_norm=0.5, kernels=TorchOptKernels)
    n2 = res[0][5]
    assert n2 >= eng1.numel
    for step in range(steps):
        gs = [_rank_grads(n2, step, r) for r in range(world)]
        mean2 = torch.stack([g.float() for g in gs]).mean(0)
        g1 = torch.zeros(eng1.numel, dtype=torch.bfloat16)
        for p1, o1, o2 in zip(eng1.params, eng1.offsets, _offsets_world(eng1, world, bucket_bytes)):
            g1[o1:o1 + p1.numel()] = mean2[o2:o2 + p1.numel()].to(torch.bfloat16)
        eng1.flat_grad.copy_(g1)
        eng1.optimizer_step()
    offs2 = _offsets_world(eng1, world, bucket_bytes)
    for rank, flat_param, full_master, early, buckets, n, shard_numel, gnorm in res:
        flat_param, full_master = torch.from_numpy(flat_param), torch.from_numpy(full_master)
        assert n == n2
        assert sum(e - s for s, e in buckets) == n and shard_numel * world == n
        assert buckets[0][0] == 0 and all(a[1] == b[0] for a, b in zip(buckets, buckets[1:]))
        if bucket_bytes < (1 << 20):
            assert len(buckets) > 3 and early[0][-1] > 0 and early[0][-1] < len(buckets)  # some went out early
        assert gnorm == pytest.approx(float(eng1.gnorm.item()), rel=1e-2)
        for p1, o1, o2 in zip(eng1.params, eng1.offsets, offs2):
            k = p1.numel()
            ref = eng1.flat_param[o1:o1 + k].float()
            got = flat_param[o2:o2 + k]
            assert torch.allclose(got, ref, atol=2e-2, rtol=0), (rank, o1)       # bf16 params, every rank
            mref = eng1.master[o1:o1 + k]
            if world == 2:
                assert torch.allclose(full_master[o2:o2 + k], mref, atol=1e-4, rtol=1e-3), (rank, o1)
            else:  # AdamW moves an element by at most lr per step
                assert (full_master[o2:o2 + k] - mref).abs().max() <= 2 * steps * 1e-3 * 1.01, (rank, o1)
    # every rank holds identical parameters after the all-gather
    for r in res[1:]:
        assert (res[0][1] == r[1]).all()


def test_zero1_bf16_avg_bound_world8():
    """configs[3]'s exchange at its rank count (8, gloo on the CPU): buckets padded to multiples of 8 x 64 elements,
    the owned chunks tile the flat buffer exactly once, and the bf16 AVG reduce-scatter stays inside the bound of
    DESIGN.md §6 -- per element |avg - mean| <= (N-1)/N * u * sum_i |g_i| + u * |avg| (u = 2^-8, one rounding per
    ring hop and one for the division), measured rms well below the 5e-3 estimate there."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 1 << 14, 1, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    buckets, n = res[0][2], res[0][3]
    assert len(buckets) > 3 and all((e - s) % (world * 64) == 0 for s, e in buckets)
    gs = torch.stack([_rank_grads(n, 0, r).float() for r in range(world)])
    mean, asum = gs.mean(0), gs.abs().sum(0)
    got = torch.full((n,), float("nan"))
    cover = torch.zeros(n, dtype=torch.int64)
    for _, own, _, _ in res:
        for o, v in own:
            got[o:o + len(v)] = torch.from_numpy(v)
            cover[o:o + len(v)] += 1
    assert (cover == 1).all()
    u = 2.0 ** -8
    err = (got - mean).abs()
    bound = (world - 1) / world * u * asum + u * got.abs() + 1e-12
    assert (err <= bound).all(), float((err / bound).max())
    rms_rel = float(err.norm() / mean.norm())
    print(f"world-8 bf16 AVG: rms rel error {rms_rel:.3e}, max err/bound {float((err / bound).max()):.3f}")
    assert rms_rel < 5e-3, rms_rel


def _offsets_world(eng1, world, bucket_bytes):
    """Parameter offsets of the flat layout a `world`-rank engine builds (same algorithm as TrainEngine)."""
    cap = max(1, bucket_bytes // 2)
    quant = world * eng1.ALIGN
    offs, n, bstart = [], 0, 0
    for i, p in enumerate(eng1.params):
        offs.append(n)
        n += (p.numel() + eng1.ALIGN - 1) // eng1.ALIGN * eng1.ALIGN
        if n - bstart >= cap or i + 1 == len(eng1.params):
            n = (n + quant - 1) // quant * quant
            bstart = n
    return offs


def test_lr_schedule_matches_hf_linear_warmup():
    """lr of optimizer step k == get_linear_schedule_with_warmup's LambdaLR lr at step k (HF Trainer order:
    optimizer.step() then scheduler.step()), finetune_full.sh:74-77."""
    from transformers import get_linear_schedule_with_warmup
    from spatialvla_amd.engine import TrainEngine
    e = TrainEngine.__new__(TrainEngine)
    e.lr, e.warmup_steps, e.total_steps = 2e-5, 5, 40
    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=2e-5)
    sch = get_linear_schedule_with_warmup(opt, 5, 40)
    for k in range(1, 41):
        assert e.lr_at(k - 1) == pytest.approx(opt.param_groups[0]["lr"], abs=1e-12), k
        opt.step()
        sch.step()
