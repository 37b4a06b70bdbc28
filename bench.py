"""SpatialVLA-4B training-step benchmark on MI355X (BASELINE.json metric).

python bench.py --gpus N --steps K --warmup W        (N>1: launched by torch.distributed.run, one rank/GPU)

One step = forward + backward + DP gradient all-reduce (RCCL) + grad clip + AdamW over one synthetic
OXE-shaped batch of B=32 episodes per GPU (BASELINE configs[2]/[3]): 224x224 image + 56-token text
(256 <image> + bos + 41 prompt + "\\n" + 12 action tokens + eos = 312 tokens).  Weights are random
(no checkpoint offline); inputs are pre-staged in HBM before timing.  Prints ONE JSON line (rank 0).

Extra objects:
  roofline     — the dominant kernel (the Gemma2 gate/up GeGLU GEMM, M=B*312, N=2*9216, K=2304): every
                 launch of it inside the timed steps is bracketed by HIP events on its launch stream;
                 algorithmic FLOPs per launch / mean launch time vs the bf16 dense MFMA peak (2.5 PFLOP/s).
  gemma2_block — the north-star target: one Gemma2 decoder layer fwd+bwd at B=32 timed in isolation (untimed
                 region), algorithmic FLOPs / time vs the same peak (target frac >= 0.40).
  cpu_baseline — the CPU oracle (oracle/spatialvla_oracle.py, the reference eager restatement) fwd+bwd
                 at B=1 on this host's cores, rank 0 / N=1 only.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_BF16_TFLOPS = 2500.0          # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0           # MI355X dense fp8 (MX-scaled e4m3) MFMA
GFLOP_PER_EPISODE = 6136.1         # fwd+bwd algorithmic FLOPs per episode at L=312


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--config", default="spatialvla_4b", choices=["spatialvla_4b", "tiny"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-decode", action="store_true", help="skip the B=1 decode-latency leg")
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-fp8-leg", action="store_true", help="skip the configs[4] fp8 leg of the N=1 line")
    ap.add_argument("--backend", default=os.environ.get("SVLA_BENCH_BACKEND", "nccl"), choices=["nccl", "gloo"],
                    help="N>1 process-group backend: nccl (= RCCL, one rank per GPU; the scaling runs) or gloo (tests)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on cuda:0 (tests of the N>1 path on a one-GPU box, with --backend gloo)")
    ap.add_argument("--fp8", action="store_true",
                    help="BASELINE configs[4]: Gemma2 q|k|v, o, gate|up, down forward projections on the fp8 MFMA GEMM")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(cfgd, device):
    from spatialvla_amd import SpatialVLAConfig
    from spatialvla_amd.engine import random_init_
    from spatialvla_amd.modeling_spatialvla import SpatialVLAForConditionalGeneration
    cfg = SpatialVLAConfig(**cfgd)
    with torch.device(device):
        model = SpatialVLAForConditionalGeneration(cfg)
    model = model.to(torch.bfloat16)
    random_init_(model, seed=0)
    model.language_model.model.embed_tokens.weight.requires_grad_(False)   # spatialvla_pretrain.py:342
    if cfg.use_vision_zoe:                                                 # :349-350
        model.vision_zoe_model.eval()
        for p in model.vision_zoe_model.parameters():
            p.requires_grad_(False)
    model.train()
    if cfg.use_vision_zoe:
        model.vision_zoe_model.eval()
    return model


def make_batch(cfgd, B, seed, device):
    from spatialvla_amd import presets
    b = presets.synthetic_batch(cfgd, batch=B, seed=seed)
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    t["pixel_values"] = t["pixel_values"].to(torch.bfloat16)
    t["intrinsic"] = t["intrinsic"].to(torch.bfloat16)
    return {k: v.to(device, non_blocking=True) for k, v in t.items()}


def pmc_traffic():
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes of the same build
    (profiles/<tag>_pmc_fetch.json + <tag>_pmc_write.json, written by tools/r1_measure.sh: FETCH_SIZE doubled
    per the gfx950 note of MI355X_MICROARCH.md, WRITE_SIZE as read); None when absent."""
    import glob
    tags = sorted(os.path.basename(f)[: -len("_pmc_fetch.json")]
                  for f in glob.glob(os.path.join(REPO, "profiles", "*_pmc_fetch.json")))
    for tag in reversed(tags):
        try:
            f = json.load(open(os.path.join(REPO, "profiles", f"{tag}_pmc_fetch.json")))
            w = json.load(open(os.path.join(REPO, "profiles", f"{tag}_pmc_write.json")))
            return {"bytes": round(f["hbm_read_bytes_per_launch"] + w["hbm_write_bytes_per_launch"]),
                    "read": round(f["hbm_read_bytes_per_launch"]), "write": round(w["hbm_write_bytes_per_launch"]),
                    "source": f"profiles/{tag}_pmc_fetch.json + {tag}_pmc_write.json"}
        except (OSError, KeyError, ValueError):
            continue
    return None


def dominant_kernel_roofline(records, fp8=False):
    """Roofline of the Gemma2 gate/up GEMM with the fused GeGLU epilogue (the largest kernel of the step):
    its launches inside the timed region, each bracketed by HIP events on the stream it was launched on.
    fp8 (configs[4]): the e4m3 MFMA kernel against the dense fp8 peak."""
    ms = [e0.elapsed_time(e1) for (e0, e1, *_s) in records]
    M, N, K = records[0][2:]
    avg = float(np.mean(ms))
    flops = 2.0 * M * N * K                          # algorithmic: M x (2I) x H multiply-adds
    ach = flops / (avg * 1e-3) / 1e12
    ob = 1 if fp8 else 2                             # operand bytes per element
    bytes_alg = ob * (M * K + N * K) + 2.0 * 3 * M * (N // 2)   # x, Wg, Wu read; h, g, u written (bf16)
    if fp8:
        bytes_alg += (M * K + N * K) / 32                # one E8M0 block scale per 32 operand elements
    peak = PEAK_FP8_TFLOPS if fp8 else PEAK_BF16_TFLOPS
    kern = ("svla gemm4mx_kernel (256x256 tile, 4 waves x 128x128, v_mfma_scale_f32_32x32x64_f8f6f4 e4m3, OCP MX "
            "E8M0 block scales per 32 k)"
            if fp8 else "svla gemm4_kernel_00g (256x256 tile, 4 waves x 128x128, AGPR C^T accumulators, gate/up B "
                        "fragments paired per output block, GeGLU stored straight from the accumulators)")
    return {"kernel": kern + " EPI_GEGLU (Gemma2 gate/up, M=%d N=%d K=%d)" % (M, N, K),
            "bound": "mfma", "achieved": round(ach, 1), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "traffic": None if fp8 else pmc_traffic(), "avg_launch_ms": round(avg, 4),
            "launches_timed": len(ms), "algorithmic_flops_per_launch": flops,
            "algorithmic_bytes_per_launch": bytes_alg}


def fp8_leg(model, engine, batches, args):
    """BASELINE configs[4] beside the bf16 line (N=1, after the timed region, same model and batches): the training
    step with the Gemma2 q|k|v, o, gate|up and down projections on the fp8 (e4m3, OCP MX block-scaled) MFMA GEMM, forward and
    dgrad, weight copies re-quantised after every optimizer step; timed like the main line (barrier-free: one rank).
    roofline: the fp8 gate/up GeGLU launches inside the timed steps vs the dense fp8 peak (5 PFLOP/s)."""
    from spatialvla_amd import functional as Fn
    from spatialvla_amd import kernels as K
    model.enable_fp8_projections(True)
    try:
        n = len(batches)
        for s in range(min(2, args.warmup)):
            engine.train_step(batches[s % n])
        torch.cuda.synchronize()
        ev = K.launch_timer["geglu_fp8"] = []
        ev_bf = K.launch_timer["geglu"] = []  # gate|up left on bf16 (SVLA_FP8_SITES without gate_up)
        t0 = time.perf_counter()
        for s in range(args.steps):
            loss = engine.train_step(batches[s % n])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        K.launch_timer.pop("geglu_fp8")
        K.launch_timer.pop("geglu")
    finally:
        model.enable_fp8_projections(False)
    B = args.batch
    return {"what": "BASELINE configs[4] at N=1: fwd+bwd+AdamW with fp8 Gemma2 projections (fwd + dgrad), B=%d" % B,
            "value": round(B * args.steps / dt, 3), "unit": "episodes/s", "ms_per_step": round(dt / args.steps * 1e3, 2),
            "steps": args.steps, "final_loss": round(float(loss.item()), 4),
            "fp8_sites": sorted(Fn.FP8_SITES[0]),
            "roofline": dominant_kernel_roofline(ev, fp8=True) if ev else dominant_kernel_roofline(ev_bf)}


def gemma2_block_roofline(model, B, L, device, iters=20):
    """The north-star target: one Gemma2DecoderLayer fwd+bwd at B episodes x L tokens (sandwich norms, QKV+RoPE,
    prefix-LM GQA attention with softcap, o_proj, GeGLU MLP; every dW written), timed in isolation with HIP
    events on the stream the kernels run on.  Algorithmic FLOPs = 3 x fwd matmul FLOPs (SURVEY §8a a14:
    1283.9 GFLOP/episode over 26 layers)."""
    from spatialvla_amd.modeling_gemma2 import KVMask
    lm = model.language_model.model
    layer = lm.layers[1]
    cfg = lm.config
    tt = torch.zeros(B, L, dtype=torch.long, device=device)
    tt[:, L - 13:] = 1
    mask = KVMask.build(torch.ones(B, L, dtype=torch.long, device=device), tt, True, B, L, device)
    pos = torch.arange(1, L + 1, device=device).unsqueeze(0).expand(B, L)
    rope = layer.self_attn.rotary_emb.tables(pos, torch.bfloat16)
    g = torch.Generator(device=device).manual_seed(5)
    x = torch.randn(B, L, cfg.hidden_size, device=device, generator=g).to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(B, L, cfg.hidden_size, device=device, generator=g).to(torch.bfloat16)
    H, I, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    hq, hkv = cfg.num_attention_heads, cfg.num_key_value_heads
    mac_tok = H * (hq + 2 * hkv) * D + hq * D * H + 3 * H * I + 2 * hq * L * D
    flops = 3 * 2.0 * mac_tok * B * L
    stream = torch.cuda.current_stream()
    # iterations run back to back (the host queues them ahead of the GPU, as in the training step this layer sits
    # in) between two events; fwd from events around each forward.  A GPU-side spin ahead of each iteration (tried in
    # round 4) lowered the clock the layer then ran at: 5.5 ms against 5.0-5.1 ms back to back on the same box.
    def one(ev=None):
        x.grad = None
        if ev is not None:
            ev[0].record(stream)
        y = layer(x, mask, rope)
        if ev is not None:
            ev[1].record(stream)
        y.backward(gy)
    for _ in range(3):
        one()
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(iters)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for it in range(iters):
        one(evs[it])
    e1.record(stream)
    e1.synchronize()
    fwd_ms = [a.elapsed_time(b) for a, b in evs]
    tot_ms = [e0.elapsed_time(e1) / iters]
    ms = float(np.median(tot_ms))
    ach = flops / (ms * 1e-3) / 1e12
    return {"what": f"Gemma2DecoderLayer fwd+bwd, B={B} x L={L} (M={B * L} token rows)", "bound": "mfma",
            "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
            "ms_fwd_bwd": round(ms, 3), "ms_fwd": round(float(np.median(fwd_ms)), 3), "iters": iters,
            "algorithmic_flops": flops, "target_frac": 0.40}


def decode_latency(model, cfgd, device, n_new=4, n_long=40):
    """BASELINE configs[1] beside the training line (after the timed region, same weights): B=1 greedy decode
    through predict_action -- prefill (vision + Zoe + Gemma2 over the 299-token prompt + first token) and the
    KV-cached decode steps, both replayed from HIP graphs -- timed with HIP events, median of 5."""
    b = make_batch(cfgd, 1, 4321, device)
    P = int((b["token_type_ids"][0] == 0).sum())
    inputs = {"input_ids": b["input_ids"][:, :P], "pixel_values": b["pixel_values"], "intrinsic": b["intrinsic"]}
    model.eval()

    def med(n):
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            model.predict_action(inputs, max_new_tokens=n, eos_token_id=-1)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return sorted(ts)[2]

    with torch.no_grad():
        model.predict_action(inputs, max_new_tokens=n_long, eos_token_id=-1)  # captures every graph once
        t1, tn, tl = med(1), med(n_new), med(n_long)
    per_tok = (tl - t1) / (n_long - 1)
    lm = model.language_model
    wbytes = sum(p.numel() * p.element_size() for p in lm.model.layers.parameters()) + \
        lm.lm_head.weight.numel() * lm.lm_head.weight.element_size()
    return {"what": "B=1 predict_action: 1 image + 299-token prompt -> 4 tokens (BASELINE configs[1])",
            "ms_total": round(tn, 2), "ms_prefill_plus_first": round(t1, 2), "ms_per_decode_token": round(per_tok, 3),
            "decode_roofline": {"bound": "hbm", "achieved": round(wbytes / (per_tok * 1e-3) / 1e9, 1),
                                "peak": 8000.0, "unit": "GB/s", "algorithmic_bytes_per_token": wbytes}}


def _usable_cpus():
    """CPUs this process may actually run on: the affinity mask, capped by a cgroup CPU quota if one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                n = min(n, max(1, int(int(quota) // int(period))))
        except (OSError, ValueError):
            pass
    return n


def _cpu_isa():
    try:
        flags = next(l for l in open("/proc/cpuinfo") if l.startswith("flags")).split()
    except (OSError, StopIteration):
        return "unknown"
    tags = [f for f in ("amx_bf16", "avx512_bf16", "avx512f", "avx2") if f in flags]
    return "+".join(tags) or "baseline x86-64"


def cpu_baseline(cfgd, iters, batches=(1, 2)):
    """Reference eager restatement (oracle, test infrastructure) fwd+bwd on the host cores, per BASELINE.md §3:
    every usable core, bf16, B=1 and B=2, 1 warm-up + `iters` timed iterations each, median."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import spatialvla_oracle as O
    from spatialvla_amd import presets
    threads = _usable_cpus()
    torch.set_num_threads(threads)
    t_build = time.perf_counter()
    P = O.build_params_random(cfgd, seed=0)
    zoe = None
    if cfgd.get("use_vision_zoe", True):
        from transformers import ZoeDepthConfig, ZoeDepthForDepthEstimation
        zoe = ZoeDepthForDepthEstimation(ZoeDepthConfig(**cfgd["vision_zoe_config"])).to(torch.bfloat16).eval()
    log(f"[cpu_baseline] oracle built in {time.perf_counter() - t_build:.1f}s, {threads} threads "
        f"(os.cpu_count() {os.cpu_count()})")
    per_b = {}
    for B in batches:
        b = presets.synthetic_batch(cfgd, batch=B, seed=99)
        t = {k: torch.from_numpy(v) for k, v in b.items()}
        t["pixel_values"] = t["pixel_values"].to(torch.bfloat16)
        t["intrinsic"] = t["intrinsic"].to(torch.bfloat16)
        times = []
        for i in range(iters + 1):
            for v in P.values():
                v.grad = None
            t0 = time.perf_counter()
            loss, _ = O.forward(P, cfgd, t, zoe)
            loss.backward()
            dt = time.perf_counter() - t0
            log(f"[cpu_baseline] B={B} iter {i}: {dt:.2f}s")
            if i > 0:
                times.append(dt)
        per_b[B] = float(np.median(times))
    eps = {B: B / t for B, t in per_b.items()}
    best = max(eps, key=eps.get)
    return {"value": round(eps[best], 4), "unit": "episodes/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "isa": _cpu_isa(),
            "sample": "oracle fwd+bwd (bf16, torch CPU), 1 warm-up + %d timed iters per batch, median: %s; value = B=%d"
                      % (iters, ", ".join(f"B={B} {per_b[B]:.2f}s/step = {eps[B]:.4f} ep/s" for B in batches), best)}


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: run this script under torch.distributed.run with one rank
    per GPU as a child process (nothing here has touched the GPU yet) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] spawning {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.share_device and args.backend == "nccl":
        sys.exit("bench.py: --share-device needs --backend gloo (RCCL refuses two ranks on one GPU)")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    from spatialvla_amd import presets
    from spatialvla_amd.engine import TrainEngine
    cfgd = json.loads(json.dumps(getattr(presets, args.config)()))
    B = args.batch
    t0 = time.perf_counter()
    model = build_model(cfgd, device)
    if args.fp8:
        model.enable_fp8_projections(True)
    n_train = sum(p.numel() for p in model.parameters() if p.requires_grad)
    total = args.warmup + args.steps
    # SVLA_OPT_OVERLAP=1: AdamW of step k beside step k+1's forward (TrainEngine overlap_optimizer); measured no
    # faster at N=1 (216.3 vs 216.8 ms, profiles/r5w_step_ab_opt_overlap.txt), so the serial step is the default
    engine = TrainEngine(model, lr=2e-5, weight_decay=0.0, max_grad_norm=1.0, warmup_ratio=0.005,
                         total_steps=max(total, 10), defer_host_checks=True,
                         overlap_optimizer=os.environ.get("SVLA_OPT_OVERLAP", "0") != "0")
    log(f"[bench] rank {rank}/{world}: model built in {time.perf_counter() - t0:.1f}s, trainable {n_train / 1e9:.3f}B, "
        f"flat buffers {engine.numel / 1e9:.3f}B elems, buckets {len(engine.buckets)}")
    batches = [make_batch(cfgd, B, args.seed + 1000 * rank + s, device) for s in range(total)]
    torch.cuda.synchronize()
    losses = []
    for s in range(args.warmup):
        ts = time.perf_counter()
        losses.append(engine.train_step(batches[s]))
        torch.cuda.synchronize()
        log(f"[bench] warmup step {s}: {time.perf_counter() - ts:.3f}s loss {losses[-1].item():.4f}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    from spatialvla_amd import kernels as K
    tkey = "geglu_fp8" if args.fp8 else "geglu"
    geglu_events = K.launch_timer[tkey] = []
    t_start = time.perf_counter()
    for s in range(args.steps):
        if s == args.steps - 1 and os.environ.get("SVLA_GEMM_LOG"):  # tools/ab_trace.py: GEMM call sequence
            K.gemm_log = []
        losses.append(engine.train_step(batches[args.warmup + s]))
    if K.gemm_log is not None:
        json.dump(K.gemm_log, open(os.environ["SVLA_GEMM_LOG"], "w"))
        K.gemm_log = None
    torch.cuda.synchronize()
    K.launch_timer.pop(tkey)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t_start
    # the slowest rank's clock: every rank's seconds gathered (the JSON line carries them), value from the MAX
    per_rank = [dt]
    if world > 1:
        dts = [torch.zeros(1, dtype=torch.float64, device=device) for _ in range(world)]
        dist.all_gather(dts, torch.tensor([dt], dtype=torch.float64, device=device))
        per_rank = [float(t.item()) for t in dts]
    dt = max(per_rank)
    final_loss = float(losses[-1].item())
    ms_step = dt / args.steps * 1e3
    eps = world * B * args.steps / dt
    result = {
        "metric": "episodes/sec fwd+bwd SpatialVLA-4B, 224px+56tok batch, 1/2/4/8 MI355X",
        "value": round(eps, 3), "unit": "episodes/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 2), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp8-e4m3 fwd projections / bf16" if args.fp8 else "bf16",
        "data": "synthetic OXE-shaped batches (random ids/pixels), random-init weights",
        "config": {"workload": ("SpatialVLA-4B fwd+bwd+AdamW, fp8 Gemma2 projections (BASELINE configs[4])" if args.fp8
                                else "SpatialVLA-4B fwd+bwd+AdamW (BASELINE configs[2]/[3])"), "model": args.config,
                   "global_batch": world * B, "per_gpu_batch": B, "seq_len": 312, "parallelism": f"dp{world}",
                   "trainable_params": n_train},
        "mfu_model_flops": round(eps * GFLOP_PER_EPISODE / 1e3 / (world * PEAK_BF16_TFLOPS), 4),
        "final_loss": round(final_loss, 4),
    }
    if world > 1:
        result["per_rank_seconds"] = [round(t, 6) for t in per_rank]
        result["timed_seconds_max"] = round(dt, 6)
        result["backend"] = args.backend
    if world == 1 and not args.fp8 and not args.no_fp8_leg and args.config == "spatialvla_4b":
        result["fp8"] = fp8_leg(model, engine, batches, args)
    if rank == 0:
        result["roofline"] = dominant_kernel_roofline(geglu_events, fp8=args.fp8)
        if args.config == "spatialvla_4b":
            result["gemma2_block"] = gemma2_block_roofline(model, B, 312, device)
        if world == 1 and not args.no_cpu_baseline and not args.fp8:
            del batches, engine
            torch.cuda.empty_cache()
            result["cpu_baseline"] = cpu_baseline(cfgd, args.cpu_iters)
        if world == 1 and args.config == "spatialvla_4b" and not args.no_decode and not args.fp8:
            result["decode"] = decode_latency(model, cfgd, device)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
