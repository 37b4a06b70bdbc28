"""Data-parallel training step for SpatialVLA on MI355X (replaces the reference's HF Trainer + DeepSpeed
ZeRO path: train/spatialvla_pretrain.py:383-399, scripts/zero1.json, train/dist_utils.py:29-99).

Design (one process per GPU, torch.distributed over RCCL/xGMI):
  * All trainable parameters live in ONE flat bf16 buffer (params are views), their gradients in one
    flat bf16 buffer: the HIP autograd Functions write dW straight into those views
    (`param._svla_grad`), so there is no per-parameter grad allocation and no autograd accumulation.
  * The flat order is the reverse of the forward order (lm_head, final norm, layers 25..0, merge,
    projector, Ego3D, SigLIP), so buckets complete in backward order.  Buckets are all-reduced
    (average) as soon as their last layer's backward has produced its gradients (layer hooks), on
    RCCL's stream, overlapping the rest of the backward; the step waits once before the optimizer.
  * Gradient clipping (max_grad_norm, Trainer default 1.0) and AdamW (scripts/zero1.json:23-34:
    betas (0.9, 0.999), eps 1e-8) are two HIP kernels over the flat fp32 master / m / v buffers.
  * LR schedule: linear warmup (warmup_ratio) then linear decay, as finetune_full.sh:74-77.
"""
import math
from typing import Dict, List, Optional

import re

import torch
import torch.distributed as dist

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


def _forward_order(model) -> List[torch.nn.Parameter]:
    """Trainable parameters in backward-completion order (reverse of the forward pass)."""
    seen, order = set(), []
    lm = model.language_model
    groups = [lm.lm_head, lm.model.norm] + list(reversed(list(lm.model.layers)))
    if getattr(model, "spatial_embed_tokens", None) is not None:
        groups.append(model.spatial_embed_tokens)
    groups.append(model.multi_modal_projector)
    if getattr(model, "position_embedding_3d", None) is not None:
        groups.append(model.position_embedding_3d)
    vt = model.vision_tower.vision_model
    groups += [vt.post_layernorm] + list(reversed(list(vt.encoder.layers))) + [vt.embeddings]
    for gmod in groups:
        for p in _group_params(gmod):
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                order.append(p)
    for p in model.parameters():  # anything not covered above (kept last)
        if p.requires_grad and id(p) not in seen:
            seen.add(id(p))
            order.append(p)
    return order


class GradExchange:
    """Bucketed, overlappable DP gradient averaging over a flat gradient buffer (RCCL all-reduce with
    AVG on the nccl backend; SUM + divide on gloo, which has no AVG).  Buckets are cut at parameter
    boundaries (`offsets`) once they reach `bucket_bytes`; `on_layer_grad(i)` launches every bucket whose
    parameters all end before the end of layer i's last parameter in the flat order."""

    def __init__(self, flat_grad: torch.Tensor, offsets: List[int], bucket_bytes: int = 256 << 20,
                 process_group=None):
        self.flat = flat_grad
        self.offsets = list(offsets)
        self.numel = flat_grad.numel()
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.buckets = []
        start = 0
        cap = max(1, bucket_bytes // flat_grad.element_size())
        for i in range(len(self.offsets)):
            end = self.offsets[i + 1] if i + 1 < len(self.offsets) else self.numel
            if end - start >= cap or i + 1 == len(self.offsets):
                self.buckets.append((start, end))
                start = end
        self.layer_ready: List[int] = []
        self._pending = []
        self._launched = set()

    def on_layer_grad(self, layer_idx: int):
        last = self.layer_ready[layer_idx] if layer_idx < len(self.layer_ready) else -1
        if last < 0:
            return
        ready_end = self.offsets[last + 1] if last + 1 < len(self.offsets) else self.numel
        for bi, (s, e) in enumerate(self.buckets):
            if e <= ready_end and bi not in self._launched:
                self._launch(bi)

    def _launch(self, bi):
        s, e = self.buckets[bi]
        self._launched.add(bi)
        op = dist.ReduceOp.AVG if dist.get_backend(self.pg) == "nccl" else dist.ReduceOp.SUM
        work = dist.all_reduce(self.flat[s:e], op=op, group=self.pg, async_op=True)
        self._pending.append((bi, work, op))

    def finish(self):
        """Launch whatever is left and wait for every bucket (stream-ordered on nccl)."""
        if self.world == 1:
            return
        for bi in range(len(self.buckets)):
            if bi not in self._launched:
                self._launch(bi)
        for bi, work, op in self._pending:
            work.wait()
            if op == dist.ReduceOp.SUM:
                s, e = self.buckets[bi]
                self.flat[s:e].div_(self.world)
        self._pending.clear()
        self._launched.clear()


class TrainEngine:
    ALIGN = 64  # elements; keeps every view 128-B aligned (kernel loads are 16 B)

    def __init__(self, model, lr: float = 2e-5, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 max_grad_norm: float = 1.0, warmup_ratio: float = 0.005, total_steps: int = 1000,
                 process_group=None, bucket_bytes: int = 256 << 20, overlap: bool = True):
        self.model = model
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.warmup_steps = max(1, int(math.ceil(warmup_ratio * total_steps)))
        self.total_steps = total_steps
        self.step_count = 0
        dev = next(model.parameters()).device
        self.device = dev
        params = _forward_order(model)
        self.params = params
        offs, n = [], 0
        for p in params:
            offs.append(n)
            n += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel = n
        self.offsets = offs
        self.flat_param = torch.zeros(n, dtype=BF16, device=dev)
        self.flat_grad = torch.zeros(n, dtype=BF16, device=dev)
        self.master = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, o in zip(params, offs):
                view = self.flat_param[o:o + p.numel()].view_as(p)
                view.copy_(p.data.to(BF16))
                p.data = view
                p._svla_grad = self.flat_grad[o:o + p.numel()].view_as(p)
                p._svla_accum = False
                self.master[o:o + p.numel()].copy_(view.reshape(-1).float())
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.clip = torch.ones(1, dtype=torch.float32, device=dev)
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.exchange = GradExchange(self.flat_grad, offs, bucket_bytes, process_group)
        self.buckets = self.exchange.buckets
        if overlap and self.exchange.world > 1:
            lm = self.model.language_model.model
            pid = {id(p): i for i, p in enumerate(params)}
            ready = []
            for layer in lm.layers:
                idx = [pid[id(p)] for p in layer.parameters() if id(p) in pid]
                ready.append(max(idx) if idx else -1)
            self.exchange.layer_ready = ready
            lm._svla_layer_grad_hook = self.exchange.on_layer_grad

    # ------------------------------------------------------------------ optimizer
    def lr_at(self, step: int) -> float:
        if step <= self.warmup_steps:
            return self.lr * step / self.warmup_steps
        return self.lr * max(0.0, (self.total_steps - step) / max(1, self.total_steps - self.warmup_steps))

    def optimizer_step(self):
        self.step_count += 1
        K.sumsq(self.flat_grad, self.sumsq)
        K.clip_scale(self.sumsq, self.max_grad_norm, self.clip, self.gnorm)
        K.adamw(self.master, self.flat_param, self.flat_grad, self.m, self.v, self.lr_at(self.step_count),
                self.betas[0], self.betas[1], self.eps, self.wd, self.step_count, self.clip)

    def train_step(self, batch: Dict[str, torch.Tensor]):
        """forward + backward + DP all-reduce + clip + AdamW; returns the loss tensor (no host sync)."""
        out = self.model(**batch, return_dict=True)
        out.loss.backward()
        self.exchange.finish()
        self.optimizer_step()
        return out.loss.detach()


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
