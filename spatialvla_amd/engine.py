"""Data-parallel training step for SpatialVLA on MI355X (replaces the reference's HF Trainer + DeepSpeed
ZeRO-1 path: train/spatialvla_pretrain.py:383-399, scripts/zero1.json, train/dist_utils.py:29-99).

Design (one process per GPU, torch.distributed over RCCL/xGMI):
  * All trainable parameters live in ONE flat bf16 buffer (params are views), their gradients in one flat bf16
    buffer: the HIP autograd Functions write dW straight into those views (`param._svla_grad`), so there is no
    per-parameter grad allocation and no autograd accumulation.
  * The flat order is the reverse of the forward order (lm_head, final norm, Gemma2 layers 25..0, spatial
    embeddings, projector, SigLIP post-LN and layers 26..0, patch embedding, Ego3D MLP), so the buffer fills from
    the front during backward.  It is cut into buckets (~256 MB) at parameter boundaries.
  * ZeRO stage 1 (scripts/zero1.json:2-10, "stage": 1, reduce_scatter, overlap_comm, allgather): every bucket is
    padded to a multiple of world x 64 elements and split into `world` equal chunks; rank r owns chunk r of every
    bucket -- its fp32 master weights and AdamW moments (the sharded optimizer state) hold just those chunks.
      - backward: as soon as the layers of a bucket have written their gradients (layer hooks on the Gemma2 and
        SigLIP layer inputs), the bucket is reduce-scattered (AVG) on RCCL's stream, overlapping the rest of the
        backward; `finish_reduce()` launches the rest and waits.
      - step: grad-norm clip (max_grad_norm, Trainer default 1.0) over the owned chunks + one scalar all-reduce,
        then AdamW (betas 0.9/0.999, eps 1e-8, zero1.json:23-34) on the owned chunks only, then every bucket is
        all-gathered back into the flat bf16 parameter buffer (async).
      - forward: each layer waits for the all-gather of its bucket just before it runs (parameter wait points),
        so the gathers overlap the optimizer of later buckets and the forward of earlier layers.
    Volume per GPU per step: reduce-scatter + all-gather of the 3.07 B bf16 parameters, 2 x (N-1)/N x 6.14 GB --
    the same bytes as an all-reduce -- while AdamW touches 1/N of the parameters (28 B/param -> 86 GB / N).
  * world == 1: no collectives, one AdamW launch over the whole flat buffer.
  * LR schedule: linear warmup (warmup_ratio) then linear decay, as finetune_full.sh:74-77 with the HF Trainer's
    get_linear_schedule_with_warmup.
"""
import math
from typing import Dict, List

import re

import torch
import torch.distributed as dist

from . import functional as Fn
from . import kernels as K

BF16 = torch.bfloat16


def _group_params(gmod) -> List[torch.nn.Parameter]:
    """gmod's parameters in registration order, except that the q, k, v projection weights of an attention
    module sit back to back (q|k|v) ahead of their biases: the flat buffer then holds the fused q|k|v weight as
    one [3H, H] matrix, so the forward and dgrad GEMMs see one unsegmented operand and the three weight
    gradients one output (SigLIP registers k, v, q with biases in between)."""
    named = list(gmod.named_parameters())
    pmap = dict(named)
    out, done = [], set()
    for n, p in named:
        m = re.match(r"(.*self_attn\.)[qkv]_proj\.(weight|bias)$", n)
        if m is None:
            out.append(p)
            continue
        pre = m.group(1)
        if pre in done:
            continue
        done.add(pre)
        for suf in ("q_proj.weight", "k_proj.weight", "v_proj.weight", "q_proj.bias", "k_proj.bias", "v_proj.bias"):
            if pre + suf in pmap:
                out.append(pmap[pre + suf])
    return out


# Parameter wait points of the forward (ZeRO all-gather), in execution order: "pre" (start of forward:
# embeddings, projector, Ego3D, spatial tokens), ("siglip", i), ("gemma", i), "head" (final norm + lm_head).
def _param_groups(model):
    """[(wait point, module)] in backward-completion order (the flat buffer order)."""
    lm = model.language_model
    nl = len(lm.model.layers)
    groups = [("head", lm.lm_head), ("head", lm.model.norm)]
    groups += [(("gemma", i), lm.model.layers[i]) for i in reversed(range(nl))]
    if getattr(model, "spatial_embed_tokens", None) is not None:
        groups.append(("pre", model.spatial_embed_tokens))
    groups.append(("pre", model.multi_modal_projector))
    vt = model.vision_tower.vision_model
    ns = len(vt.encoder.layers)
    groups.append(("pre", vt.post_layernorm))
    groups += [(("siglip", i), vt.encoder.layers[i]) for i in reversed(range(ns))]
    groups.append(("pre", vt.embeddings))
    if getattr(model, "position_embedding_3d", None) is not None:
        # not ordered by a data dependency against the SigLIP layer hooks: kept after every hooked group
        groups.append(("pre", model.position_embedding_3d))
    return groups


def _wait_rank(point, n_siglip):
    if point == "pre":
        return 0
    if point == "head":
        return 10 ** 6
    kind, i = point
    return 1 + i if kind == "siglip" else 1 + n_siglip + i


class ZeroExchange:
    """ZeRO-1 collectives over the flat gradient / parameter buffers (see the module docstring).  `buckets` are
    (start, end) element ranges, each a multiple of world x 64 long; rank r owns [start + r*c, start + (r+1)*c),
    c = (end - start) / world, of every bucket."""

    def __init__(self, flat_param, flat_grad, buckets, process_group=None):
        self.fp, self.fg = flat_param, flat_grad
        self.buckets = buckets
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world > 1 else 0
        self.chunk = [(e - s) // self.world for s, e in buckets]
        self._rs = {}        # bucket -> pending reduce-scatter work
        self._ag = {}        # bucket -> pending all-gather work
        self.ready_end: Dict[object, int] = {}  # grad hook point -> flat index below which every grad is written
        self.wait_buckets: Dict[object, List[int]] = {}  # parameter wait point -> buckets to wait for

    def owned(self, b):
        """(flat start, length) of this rank's chunk of bucket b."""
        s, _ = self.buckets[b]
        c = self.chunk[b]
        return s + self.rank * c, c

    # ---------------------------------------------------------------- backward: reduce-scatter
    def on_grads_ready(self, point):
        end = self.ready_end.get(point)
        if end is None or self.world == 1:
            return
        Fn.join_side_work()  # weight gradients still running on the side stream (functional._SideWork)
        for b, (s, e) in enumerate(self.buckets):
            if e <= end and b not in self._rs:
                self._reduce_scatter(b)

    def _reduce_scatter(self, b):
        """In place: the output is this rank's chunk of the input bucket (NCCL's in-place form).  The same call on
        every backend -- RCCL on the GPUs, gloo in the CPU tests -- so the tests run the code path of the 8-GPU
        run.  AVG on bf16: RCCL rounds to bf16 at every ring hop (DESIGN.md §6 states the bound)."""
        s, e = self.buckets[b]
        o, c = self.owned(b)
        self._rs[b] = dist.reduce_scatter_tensor(self.fg[o:o + c], self.fg[s:e], op=dist.ReduceOp.AVG,
                                                 group=self.pg, async_op=True)

    def finish_reduce(self):
        """Launch the buckets no hook covered and wait for every reduce-scatter (stream-ordered on nccl)."""
        if self.world == 1:
            return
        for b in range(len(self.buckets)):
            if b not in self._rs:
                self._reduce_scatter(b)
        for w in self._rs.values():
            w.wait()
        self._rs.clear()

    # ---------------------------------------------------------------- step: all-gather
    def all_gather(self, b):
        """In place: the input is this rank's chunk of the output bucket.  Left in flight; the forward's parameter
        wait points (or land_before_update) complete it."""
        if self.world == 1:
            return
        s, e = self.buckets[b]
        o, c = self.owned(b)
        self._ag[b] = dist.all_gather_into_tensor(self.fp[s:e], self.fp[o:o + c], group=self.pg, async_op=True)

    def _land(self, b):
        self._ag.pop(b).wait()

    def land(self, b):
        """Complete bucket b's all-gather if one is in flight (before AdamW rewrites its send buffer)."""
        if b in self._ag:
            self._land(b)

    def wait_params(self, point):
        for b in self.wait_buckets.get(point, ()):
            if b in self._ag:
                self._land(b)

    def wait_all_params(self):
        for b in list(self._ag):
            self._land(b)


class TrainEngine:
    ALIGN = 64  # elements; keeps every view 128-B aligned (kernel loads are 16 B)

    def __init__(self, model, lr: float = 2e-5, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 max_grad_norm: float = 1.0, warmup_ratio: float = 0.005, total_steps: int = 1000,
                 process_group=None, bucket_bytes: int = 256 << 20, overlap: bool = True, kernels=None,
                 defer_host_checks: bool = False, overlap_optimizer: bool = False):
        """kernels: the optimizer kernel module (sumsq / clip_scale / adamw); the libsvla wrappers unless a test
        injects a stand-in to exercise the exchange logic without a GPU.
        defer_host_checks: opt-in; the model's image-token count check (reference modeling_spatialvla.py:379-385)
        is then raised from the next forward instead of the current one, so no step waits on a host read.
        overlap_optimizer: opt-in; AdamW runs bucket by bucket on its own stream in the order the next forward needs
        the parameters, and that forward waits per layer for its own bucket (the ZeRO-1 parameter wait points), so
        the HBM-bound update overlaps the compute-bound forward.  The parameters, master weights and moments are then
        final only once the next forward's wait points, `synchronize()`, `sync_params()` or `full_master()` ran:
        code that reads them directly after `train_step` must call `synchronize()` first."""
        self.model = model
        self._opt_events: Dict[int, object] = {}  # bucket -> event after its side-stream AdamW (overlap_optimizer)
        if defer_host_checks and hasattr(model, "defer_checks"):
            model.defer_checks = True
        self.K = kernels if kernels is not None else K
        if hasattr(model, "clear_decode_cache"):  # captured decode graphs point at the storage rebound below
            model.clear_decode_cache()
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.warmup_steps = int(math.ceil(warmup_ratio * total_steps))
        self.total_steps = total_steps
        self.step_count = 0
        dev = next(model.parameters()).device
        self.device = dev
        world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.world = world
        self.overlap_opt = bool(overlap_optimizer) and dev.type == "cuda"
        # its own stream: the forward's side stream (functional.side_stream) carries the frozen Zoe estimator, which
        # must not queue behind the optimizer
        self._opt_stream = torch.cuda.Stream(dev) if self.overlap_opt else None

        # ---- flat layout: parameters in backward order, buckets cut at parameter boundaries and padded to a
        # multiple of world * ALIGN elements (the ZeRO chunks of every rank are equal and aligned)
        seen, entries = set(), []   # (param, wait point, group index)
        groups = _param_groups(model)
        for gi, (point, gmod) in enumerate(groups):
            for p in _group_params(gmod):
                if p.requires_grad and id(p) not in seen:
                    seen.add(id(p))
                    entries.append((p, point, gi))
        for p in model.parameters():  # anything not covered above (kept last, waited at the start of forward)
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                entries.append((p, "pre", len(groups)))
        cap = max(1, bucket_bytes // 2)
        quant = world * self.ALIGN
        offs, buckets, n, bstart = [], [], 0, 0
        for i, (p, _, _) in enumerate(entries):
            offs.append(n)
            n += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
            if n - bstart >= cap or i + 1 == len(entries):
                n = (n + quant - 1) // quant * quant
                buckets.append((bstart, n))
                bstart = n
        self.params = [e[0] for e in entries]
        self.offsets = offs
        vision = set()
        for mod in (getattr(model, "vision_tower", None), getattr(model, "multi_modal_projector", None),
                    getattr(model, "position_embedding_3d", None)):
            if mod is not None:
                vision.update(id(p) for p in mod.parameters())
        self.vision_slices = [(o, p.numel()) for p, o in zip(self.params, offs) if id(p) in vision]
        self.numel = n
        self.buckets = buckets
        self.flat_param = torch.zeros(n, dtype=BF16, device=dev)
        self.flat_grad = torch.zeros(n, dtype=BF16, device=dev)
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                view = self.flat_param[o:o + p.numel()].view_as(p)
                view.copy_(p.data.to(BF16))
                p.data = view
                p._svla_grad = self.flat_grad[o:o + p.numel()].view_as(p)
                p._svla_accum = False
                Fn.register_flat_param(p)
        self.exchange = ZeroExchange(self.flat_param, self.flat_grad, buckets, process_group)
        ex = self.exchange
        # ---- sharded optimizer state: fp32 master / m / v of the owned chunk of every bucket, back to back
        self.shard_offsets, sn = [], 0
        for b in range(len(buckets)):
            self.shard_offsets.append(sn)
            sn += ex.owned(b)[1]
        self.shard_numel = sn
        self.master = torch.empty(sn, dtype=torch.float32, device=dev)
        self.m = torch.zeros(sn, dtype=torch.float32, device=dev)
        self.v = torch.zeros(sn, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for b in range(len(buckets)):
                o, c = ex.owned(b)
                so = self.shard_offsets[b]
                self.master[so:so + c].copy_(self.flat_param[o:o + c].float())
        self.sumsq_parts = torch.zeros(len(buckets), dtype=torch.float32, device=dev)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.clip = torch.ones(1, dtype=torch.float32, device=dev)
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=dev)

        # ---- hook points: gradient readiness (backward) and parameter waits (forward)
        ends: Dict[int, int] = {}
        for (p, point, gi), o in zip(entries, offs):
            ends[gi] = o + p.numel()
        hookable = {}
        for gi, (point, gmod) in enumerate(groups):
            if isinstance(point, tuple) and gi in ends:
                # the input grad of layer i is complete => every group before it in the flat order is written
                hookable[point] = max(v for g, v in ends.items() if g <= gi)
        ex.ready_end = hookable
        ns = len(model.vision_tower.vision_model.encoder.layers)
        first_wait = {}
        for (p, point, gi), o in zip(entries, offs):
            for b, (s, e) in enumerate(buckets):
                if s <= o < e:
                    r = _wait_rank(point, ns)
                    if b not in first_wait or r < first_wait[b][0]:
                        first_wait[b] = (r, point)
        for b, (r, point) in first_wait.items():
            ex.wait_buckets.setdefault(point, []).append(b)
        self.gather_order = sorted(first_wait, key=lambda b: first_wait[b][0])
        self.opt_order = self.gather_order + [b for b in range(len(buckets)) if b not in first_wait]
        if world > 1 or self.overlap_opt:
            lm = model.language_model.model
            vt = model.vision_tower.vision_model
            if overlap and world > 1:
                lm._svla_layer_grad_hook = lambda i: ex.on_grads_ready(("gemma", i))
                vt._svla_layer_grad_hook = lambda i: ex.on_grads_ready(("siglip", i))
            for mod in (model, model.language_model, lm, vt):  # wait points: "pre", ("siglip", i), ("gemma", i), "head"
                mod._svla_param_wait = self._param_wait
            # inference entry points (predict_action) replay captured graphs that contain no wait points
            model._svla_param_wait_all = self.sync_params

    # ------------------------------------------------------------------ optimizer
    def lr_at(self, step: int) -> float:
        """transformers get_linear_schedule_with_warmup's lr_lambda at scheduler step `step` (0-based): the HF
        Trainer's optimizer step k runs at lr_lambda(k - 1) (LambdaLR steps after the optimizer), so the first
        update of a warmup run has lr 0."""
        if step < self.warmup_steps:
            return self.lr * step / max(1, self.warmup_steps)
        return self.lr * max(0.0, (self.total_steps - step) / max(1, self.total_steps - self.warmup_steps))

    def _param_wait(self, point):
        """Forward wait point: the buckets whose first user is `point` -- their side-stream AdamW
        (overlap_optimizer) and their all-gather (N > 1)."""
        if self._opt_events:
            cur = torch.cuda.current_stream(self.device)
            for b in self.exchange.wait_buckets.get(point, ()):
                ev = self._opt_events.pop(b, None)
                if ev is not None:
                    cur.wait_event(ev)
        self.exchange.wait_params(point)

    def synchronize(self):
        """Make the current stream wait for every side-stream AdamW still in flight (overlap_optimizer)."""
        if self._opt_events:
            torch.cuda.current_stream(self.device).wait_stream(self._opt_stream)
            self._opt_events.clear()

    def optimizer_step(self):
        """clip + AdamW on the owned chunks, then the parameter all-gathers (left in flight: the next forward's
        layers wait for their own bucket).  overlap_optimizer: AdamW and the gathers go to the side stream, bucket
        by bucket in the next forward's order, each followed by an event its wait point waits for."""
        self.step_count += 1
        lr = self.lr_at(self.step_count - 1)
        ex = self.exchange
        Kx = self.K
        if self.world == 1:
            Kx.sumsq(self.flat_grad, self.sumsq)
        else:
            for b in range(len(self.buckets)):
                o, c = ex.owned(b)
                Kx.sumsq(self.flat_grad[o:o + c], self.sumsq_parts[b:b + 1])
            torch.sum(self.sumsq_parts, 0, keepdim=True, out=self.sumsq)
            dist.all_reduce(self.sumsq, op=dist.ReduceOp.SUM, group=ex.pg)
        Kx.clip_scale(self.sumsq, self.max_grad_norm, self.clip, self.gnorm)
        Fn.WEIGHT_EPOCH[0] += 1  # AdamW below rewrites the bf16 weights behind torch's version counters
        if self.overlap_opt:
            main = torch.cuda.current_stream(self.device)
            side = self._opt_stream
            side.wait_stream(main)  # the clip scale and every gradient are final
            with torch.cuda.stream(side):
                for b in self.opt_order:
                    ex.land(b)
                    o, c = ex.owned(b)
                    so = self.shard_offsets[b]
                    Kx.adamw(self.master[so:so + c], self.flat_param[o:o + c], self.flat_grad[o:o + c],
                             self.m[so:so + c], self.v[so:so + c], lr, self.betas[0], self.betas[1], self.eps,
                             self.wd, self.step_count, self.clip)
                    ex.all_gather(b)
                    ev = torch.cuda.Event()
                    ev.record(side)
                    self._opt_events[b] = ev
            return
        if self.world == 1:
            Kx.adamw(self.master, self.flat_param, self.flat_grad, self.m, self.v, lr, self.betas[0], self.betas[1],
                    self.eps, self.wd, self.step_count, self.clip)
            return
        for b in self.gather_order:
            # a bucket no forward wait point landed (e.g. SigLIP's after a text-only batch) still has last step's
            # gather in flight, reading the chunk AdamW is about to rewrite
            ex.land(b)
            o, c = ex.owned(b)
            so = self.shard_offsets[b]
            Kx.adamw(self.master[so:so + c], self.flat_param[o:o + c], self.flat_grad[o:o + c], self.m[so:so + c],
                    self.v[so:so + c], lr, self.betas[0], self.betas[1], self.eps, self.wd, self.step_count, self.clip)
            ex.all_gather(b)

    def train_step(self, batch: Dict[str, torch.Tensor]):
        """forward + backward + ZeRO-1 exchange + clip + AdamW; returns the loss tensor (no host sync).
        A batch without pixel_values leaves the vision-side gradients unwritten: they are zeroed (an unused
        parameter's gradient is zero, as in the reference's DeepSpeed step), not left at the previous step's."""
        out = self.model(**batch, return_dict=True)
        self.synchronize()  # overlap_optimizer: every AdamW done before the backward rewrites the gradients
        out.loss.backward()
        if batch.get("pixel_values") is None:
            for o, n in self.vision_slices:
                self.flat_grad[o:o + n].zero_()
        self.exchange.finish_reduce()
        self.optimizer_step()
        return out.loss.detach()

    def sync_params(self):
        """Wait for every parameter update and all-gather still in flight (before evaluation or saving)."""
        self.synchronize()
        self.exchange.wait_all_params()

    def full_master(self) -> torch.Tensor:
        """The fp32 master weights in the flat layout (gathered across ranks; tests / checkpoints)."""
        self.synchronize()
        ex = self.exchange
        if self.world == 1:
            return self.master.clone()
        out = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        for b, (s, e) in enumerate(self.buckets):
            so, c = self.shard_offsets[b], ex.chunk[b]
            parts = [torch.empty(c, dtype=torch.float32, device=self.device) for _ in range(self.world)]
            dist.all_gather(parts, self.master[so:so + c].contiguous(), group=ex.pg)
            out[s:e].copy_(torch.cat(parts))
        return out


def random_init_(model, seed: int = 0, std: float = 0.02):
    """Fast on-device random init for benchmarking (weights of the right architecture, no checkpoint):
    N(0, std) matrices, LayerNorm weights 1 / biases 0, Gemma RMSNorm weights 0."""
    g = torch.Generator(device=next(model.parameters()).device)
    g.manual_seed(seed)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() >= 2:
                p.normal_(0.0, std, generator=g)
            elif "layernorm" in n and "language_model" in n or n.endswith("model.norm.weight"):
                p.zero_()
            elif n.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()
