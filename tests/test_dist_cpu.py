"""World-size-2 gloo tests (CPU) of the data-parallel gradient exchange (spatialvla_amd.engine.GradExchange):
bucketing at parameter boundaries, layer-triggered overlapped launches, averaging == mean of ranks'
gradients (i.e. the single-process gradient of the concatenated global batch for a mean loss)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, bucket_bytes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spatialvla_amd.engine import GradExchange
        offs, n = [], 0
        for s in sizes:
            offs.append(n)
            n += (s + 63) // 64 * 64
        g = torch.Generator().manual_seed(100 + rank)
        flat = torch.randn(n, generator=g).to(torch.bfloat16)
        local = flat.clone()
        ex = GradExchange(flat, offs, bucket_bytes=bucket_bytes)
        # pretend 3 "layers" own consecutive thirds of the params: trigger in backward order
        k = len(sizes)
        ex.layer_ready = [k - 1, (2 * k) // 3 - 1, k // 3 - 1]
        ex.on_layer_grad(2)
        ex.on_layer_grad(1)
        launched_early = len(ex._launched)
        ex.finish()
        gathered = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        ref = torch.stack([t.float() for t in gathered]).mean(0)
        err = (flat.float() - ref).abs().max().item()
        q.put((rank, err, launched_early, ex.buckets, n))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes", [1 << 10, 1 << 30])
def test_grad_exchange_world2_gloo(bucket_bytes):
    sizes = [300, 1000, 64, 4096, 7, 513, 2048, 999, 128]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, bucket_bytes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, early, buckets, n in res:
        assert err <= 1e-2, (rank, err)  # bf16 rounding of the averaged values
        assert buckets[0][0] == 0 and buckets[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(buckets, buckets[1:]))
        if bucket_bytes < (1 << 20):
            assert len(buckets) > 3 and early > 0  # some buckets went out before finish()


def test_lr_schedule_linear_warmup_decay():
    from spatialvla_amd.engine import TrainEngine
    e = TrainEngine.__new__(TrainEngine)
    e.lr, e.warmup_steps, e.total_steps = 2e-5, 5, 1000
    assert e.lr_at(1) == pytest.approx(2e-5 / 5)
    assert e.lr_at(5) == pytest.approx(2e-5)
    assert e.lr_at(1000) == 0.0
    assert e.lr_at(500) == pytest.approx(2e-5 * 500 / 995)
