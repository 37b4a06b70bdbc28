"""autograd Functions of the SpatialVLA hot path, each a thin shell over libsvla kernels.

Every Function documents the reference op(s) it replaces.  All tensors are bf16, 2-D row-major
[rows, features] on the GPU.  Weight gradients go either to freshly allocated tensors returned to
autograd (standard HF/torch semantics) or — when the training engine has attached a flat-buffer
view as `param._svla_grad` — straight into that view (accumulating when `param._svla_accum`),
in which case autograd receives None for that parameter (no extra copy, no autograd add).
"""
import math
import os
import weakref
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib as L
from . import kernels as K

BF16 = torch.bfloat16
F32 = torch.float32


# ------------------------------------------------------------------------------------ helpers
def _empty(*shape, dtype=BF16, like=None, device=None):
    return torch.empty(*shape, dtype=dtype, device=like.device if like is not None else device)


# Parameters whose gradients go to a TrainEngine's flat buffer, by (data_ptr, shape): a Function's saved weight can
# come back from ctx.saved_tensors as an alias without the Parameter's attributes -- torch.utils.checkpoint's
# recompute (gradient checkpointing) returns the recomputed saved tensors -- and its gradient must still land in the
# flat buffer, not in a fresh tensor autograd would put in .grad.
_FLAT_PARAMS: "weakref.WeakValueDictionary" = weakref.WeakValueDictionary()


def register_flat_param(p: torch.Tensor):
    _FLAT_PARAMS[(p.data_ptr(), tuple(p.shape))] = p


def _grad_dest(p: torch.Tensor, needed: bool):
    """(buffer, accumulate, value returned to autograd) for the gradient of parameter p."""
    if not needed:
        return None, False, None
    if not hasattr(p, "_svla_grad"):
        p = _FLAT_PARAMS.get((p.data_ptr(), tuple(p.shape)), p)
    g = getattr(p, "_svla_grad", None)
    if g is not None:
        return g, bool(getattr(p, "_svla_accum", False)), None
    buf = torch.empty_like(p)
    return buf, False, buf


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


# Weight gradients on a side stream (SVLA_WGRAD_STREAM=0: all on the current stream).  A projection's weight-gradient
# GEMM reads only dY and X, so it can run beside the input-gradient GEMM and whatever follows that on the main stream
# (the attention backward, the GeGLU derivative pass).  The GEMMs run one workgroup per CU with a tile count that
# rarely divides 256 (o dgrad: 312 tiles, the last round fills 56 CUs), so the second kernel takes the CUs the first
# leaves idle.  Outputs are independent and every kernel's reduction order is fixed by its own tiling, so results are
# bitwise those of the serial order.
# When every weight gradient of a Function goes to the engine's flat buffer (nothing returned to autograd), the main
# stream does not wait for the side stream at the Function's end (SVLA_WGRAD_DEFER=0: it does): the side work keeps
# overlapping the next layers' backward.  The tensors it reads are marked with record_stream, so the caching allocator
# does not hand their memory out again before the side stream has read them, and the main stream waits for the side
# stream at the end of the backward pass (an autograd engine callback) and wherever the engine hands gradients to
# a collective (join_side_work, TrainEngine's bucket hooks).
WGRAD_STREAM = [os.environ.get("SVLA_WGRAD_STREAM", "1") != "0"]
# CUs the side-stream weight-gradient GEMMs leave to the main stream (their stream-K persistent grid is capped at
# num_cus - reserve, svla_gemm_set_cu_cap); 0 = they may take every CU.  Without it a persistent weight-gradient grid
# holds every CU until it is done and the main stream's next kernel (the norm-pair backward, 69 us alone) waits
# ~600 us for a CU (profiles/r7a_block_breakdown.txt).  8: step 216.4-216.8 -> 214.3-214.4 ms, block 4.65-4.67 ->
# 4.61 ms (16: the same within noise); 4: 214.1-214.3 (8) -> 212.4-212.8 ms, 2: 212.9-213.0 (profiles/
# r8q_side_cu_reserve_ab.txt); a CU reserve for the Zoe forward beside SigLIP (64, 128) measured no gain
SIDE_CU_RESERVE = [int(os.environ.get("SVLA_SIDE_CU_RESERVE", "4"))]
WGRAD_DEFER = [os.environ.get("SVLA_WGRAD_DEFER", "1") != "0"]
_side_streams: dict = {}
_join_queued: dict = {}  # device -> main stream the end-of-backward callback will make wait


def side_stream(device) -> "torch.cuda.Stream":
    """The per-device side stream (_SideWork's; the forward also runs the frozen Zoe estimator on it)."""
    s = _side_streams.get(device)
    if s is None:
        s = _side_streams[device] = torch.cuda.Stream(device)
    return s


def join_side_work():
    """Make the stream that queued side-stream weight gradients wait for all of them."""
    for dev, main in list(_join_queued.items()):
        main.wait_stream(_side_streams[dev])
        del _join_queued[dev]


_NUM_CUS: dict = {}


def _num_cus(device) -> int:
    n = _NUM_CUS.get(device)
    if n is None:
        n = _NUM_CUS[device] = torch.cuda.get_device_properties(device).multi_processor_count
    return n


class _SideWork:
    """run(fn, *reads): fn on the side stream, after everything issued on the main stream so far (reads: the tensors
    fn reads); join(*returned): the main stream waits for the side stream now, or -- when no returned gradient buffer
    is given and deferral is on -- at the end of the backward pass."""
    __slots__ = ("on", "main", "side", "reads")

    def __init__(self, like: torch.Tensor):
        self.on = WGRAD_STREAM[0] and like.is_cuda and not torch.cuda.is_current_stream_capturing()
        self.reads = []
        if self.on:
            dev = like.device
            self.main = torch.cuda.current_stream(dev)
            self.side = side_stream(dev)

    def run(self, fn, *reads):
        if not self.on:
            return fn()
        self.side.wait_stream(self.main)
        self.reads.extend(reads)
        res = SIDE_CU_RESERVE[0]
        with torch.cuda.stream(self.side):
            if res <= 0:
                return fn()
            lib = L.lib()
            lib.svla_gemm_set_cu_cap(max(1, _num_cus(self.side.device) - res))
            try:
                return fn()
            finally:
                lib.svla_gemm_set_cu_cap(0)

    def join(self, *returned):
        if not self.on:
            return
        if not WGRAD_DEFER[0] or any(r is not None for r in returned):
            self.main.wait_stream(self.side)
            return
        for t in self.reads:
            if t is not None:
                t.record_stream(self.side)
        dev = self.main.device
        if dev not in _join_queued:
            _join_queued[dev] = self.main
            torch.autograd.Variable._execution_engine.queue_callback(join_side_work)


class ResidualSlot:
    """Hand-off of a residual-stream gradient between the two consumers of one tensor: the residual branch
    (add + post-norm, or a GEMM epilogue's residual input) and the pre-norm that reads the same tensor.  The
    residual branch's backward always runs first (the pre-norm feeds it), so it parks its gradient here instead
    of returning it, and the pre-norm's backward adds it inside the norm-backward kernel (dres) -- the sum
    autograd would otherwise form with a separate elementwise add over the residual stream."""
    __slots__ = ("g",)

    def __init__(self):
        self.g = None

    def put(self, g):
        self.g = g

    def take(self):
        g, self.g = self.g, None
        return g


class MXSlot:
    """Hand-off of an activation's OCP MX e4m3 copy from the kernel that produced the bf16 tensor (a norm forward) to
    the fp8 projection that reads it (configs[4]): the producer writes both in one pass, the consumer takes the copy
    instead of quantising the tensor again.  `ptr` ties the copy to the bf16 tensor it was made from."""
    __slots__ = ("val", "ptr")

    def __init__(self):
        self.val, self.ptr = None, None

    def put(self, t, val):
        self.val, self.ptr = val, t.data_ptr()

    def take(self, t):
        """The copy of t if this slot holds one (else None); the slot is emptied either way."""
        v, p = self.val, self.ptr
        self.val, self.ptr = None, None
        return v if v is not None and p == t.data_ptr() else None


def mx_slot_for(f8, site) -> Optional[MXSlot]:
    """An MXSlot when projection `site` runs in fp8 with MX scales (producers then emit the copy), else None."""
    return MXSlot() if f8 is not None and site in FP8_SITES[0] and FP8_SCALING[0] == "mx" else None


# ------------------------------------------------------------------------------------ norms
class RMSNormFn(torch.autograd.Function):
    """Gemma2RMSNorm.forward (reference model/modeling_gemma2.py:69-74).  mx: an MXSlot that receives the MX e4m3
    copy of y, made by the same launch (the fp8 q|k|v operand)."""

    @staticmethod
    def forward(ctx, x, w, eps, slot=None, mx=None):
        x = _c(x)
        y = torch.empty_like(x)
        rstd = _empty(x.shape[0], dtype=F32, like=x)
        if mx is not None and x.shape[1] % 128 == 0:
            mx.put(y, K.rmsnorm_fwd_mx(x, w, eps, y, rstd))
        else:
            K.rmsnorm_fwd(x, w, eps, y, rstd)
        ctx.save_for_backward(x, w, rstd)
        ctx.slot = slot
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dx = torch.empty_like(x)
        dw, acc, ret = _grad_dest(w, ctx.needs_input_grad[1])
        dres = ctx.slot.take() if ctx.slot is not None else None
        K.rmsnorm_bwd(x, w, rstd, _c(dy), None if dres is None else _c(dres), dx, dw, dw_accumulate=acc)
        return dx, ret, None, None, None


class AddRMSNormFn(torch.autograd.Function):
    """h = res + Gemma2RMSNorm(y)  (decoder-layer sandwich norm + residual, modeling_gemma2.py:489-496)."""

    @staticmethod
    def forward(ctx, res, y, w, eps, slot=None, mx_grad=None):
        res, y = _c(res), _c(y)
        h = torch.empty_like(y)
        rstd = _empty(y.shape[0], dtype=F32, like=y)
        K.add_rmsnorm_fwd(res, y, w, eps, h, rstd)
        ctx.save_for_backward(y, w, rstd)
        ctx.slot = slot
        ctx.mx_grad = mx_grad
        return h

    @staticmethod
    def backward(ctx, dh):
        y, w, rstd = ctx.saved_tensors
        dh = _c(dh)
        dy = torch.empty_like(y)
        dw, acc, ret = _grad_dest(w, ctx.needs_input_grad[2])
        N = y.shape[1]
        mx = ctx.mx_grad is not None and N % 128 == 0 and N > 1536
        dy_mx = K.rmsnorm_bwd(y, w, rstd, dh, None, dy, dw, dw_accumulate=acc, mx=mx)
        if dy_mx is not None:  # the MX copy of dy for the fp8 dgrad of the projection that produced y
            ctx.mx_grad.put(dy, dy_mx)
        if ctx.slot is not None:  # the pre-norm reading `res` adds dh in its backward kernel
            ctx.slot.put(dh)
            return None, dy, ret, None, None, None
        return dh, dy, ret, None, None, None


class AddRMSNorm2Fn(torch.autograd.Function):
    """(h, x) = (res + Gemma2RMSNorm_1(y), Gemma2RMSNorm_2(h)): the decoder layer's post-attention norm + residual
    and its pre-feedforward norm (modeling_gemma2.py:487-490) in one forward launch (svla_add_rmsnorm2_fwd_train,
    bitwise AddRMSNormFn then RMSNormFn).  Backward (one launch, svla_rmsnorm2_bwd): dh_total = rms_bwd_2(dx) + dh
    (dh: h's residual-branch gradient, from slot_h when its consumer parks it there), then dy = rms_bwd_1(dh_total);
    dh_total is the gradient of res (parked in slot_res for the pre-norm that also reads res, as AddRMSNormFn does)."""

    @staticmethod
    def forward(ctx, res, y, w1, w2, eps1, eps2, slot_res=None, slot_h=None, mx=None, mx_grad=None):
        res, y = _c(res), _c(y)
        h, x = torch.empty_like(y), torch.empty_like(y)
        r1 = _empty(y.shape[0], dtype=F32, like=y)
        r2 = _empty(y.shape[0], dtype=F32, like=y)
        if mx is not None and y.shape[1] % 128 == 0:  # + the MX copy of x (the fp8 gate|up operand)
            mx.put(x, K.add_rmsnorm2_fwd_train_mx(res, y, w1, w2, eps1, eps2, h, x, r1, r2))
        else:
            K.add_rmsnorm2_fwd_train(res, y, w1, w2, eps1, eps2, h, x, r1, r2)
        ctx.save_for_backward(y, h, w1, w2, r1, r2)
        ctx.slots = (slot_res, slot_h)
        ctx.mx_grad = mx_grad
        ctx.set_materialize_grads(False)  # h's residual gradient usually arrives through slot_h: no zero tensor
        return h, x

    @staticmethod
    def backward(ctx, dh, dx):
        y, h, w1, w2, r1, r2 = ctx.saved_tensors
        slot_res, slot_h = ctx.slots
        if slot_h is not None:
            parked = slot_h.take()
            if parked is not None:
                dh = parked if dh is None else dh + parked
        dw2, acc2, ret2 = _grad_dest(w2, ctx.needs_input_grad[3])
        dw1, acc1, ret1 = _grad_dest(w1, ctx.needs_input_grad[2])
        dht = torch.empty_like(h)
        dy = torch.empty_like(y)
        if dx is None:
            dx = torch.zeros_like(h)
        # both norms' backward in one pass (bitwise the two svla_rmsnorm_bwd calls)
        mx = ctx.mx_grad is not None and y.shape[1] % 128 == 0
        dy_mx = K.rmsnorm2_bwd(h, w2, r2, _c(dx), None if dh is None else _c(dh), y, w1, r1, dht, dy, dw2, dw1, acc2,
                               acc1, mx=mx)
        if dy_mx is not None:  # the MX copy of dy (the attention output's gradient) for the fp8 o dgrad
            ctx.mx_grad.put(dy, dy_mx)
        if slot_res is not None:
            slot_res.put(dht)
            return None, dy, ret1, ret2, None, None, None, None, None, None
        return dht, dy, ret1, ret2, None, None, None, None, None, None


class LayerNormFn(torch.autograd.Function):
    """nn.LayerNorm (SigLIP layer_norm1/2/post_layernorm [3p]; Ego3D head.1, modeling_spatialvla.py:61)."""

    @staticmethod
    def forward(ctx, x, w, b, eps, slot=None):
        x = _c(x)
        y = torch.empty_like(x)
        mean = _empty(x.shape[0], dtype=F32, like=x)
        rstd = _empty(x.shape[0], dtype=F32, like=x)
        K.layernorm_fwd(x, w, b, eps, y, mean, rstd)
        ctx.save_for_backward(x, w, b, mean, rstd)
        ctx.slot = slot
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, mean, rstd = ctx.saved_tensors
        dx = torch.empty_like(x)
        dw, accw, retw = _grad_dest(w, ctx.needs_input_grad[1])
        db, accb, retb = _grad_dest(b, ctx.needs_input_grad[2])
        if dw is not None and db is not None and accw != accb:
            raise RuntimeError("LayerNorm weight/bias grads must share accumulate mode")
        dres = ctx.slot.take() if ctx.slot is not None else None
        K.layernorm_bwd(x, w, mean, rstd, _c(dy), None if dres is None else _c(dres), dx, dw, db, accumulate=accw)
        return dx, retw, retb, None, None


class ReLUFn(torch.autograd.Function):
    """nn.ReLU (Ego3D position_embedding_head.2, modeling_spatialvla.py:62)."""

    @staticmethod
    def forward(ctx, x):
        x = _c(x)
        y = torch.empty_like(x)
        K.relu_fwd(x, y)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        K.relu_bwd(x, _c(dy), dx)
        return dx


# ------------------------------------------------------------------------------------ linear
def _cat_views(ts):
    """torch.cat of 1-D tensors that already sit back to back in one storage (the engine's flat buffer) as a
    view; otherwise a copy."""
    nxt, st = ts[0].data_ptr(), ts[0].untyped_storage().data_ptr()
    for t in ts:
        if t.dim() != 1 or not t.is_contiguous() or t.data_ptr() != nxt or t.untyped_storage().data_ptr() != st:
            return torch.cat(ts)
        nxt += t.numel() * t.element_size()
    return torch.as_strided(ts[0], (sum(t.numel() for t in ts),), (1,))


def _bias_grad(dy, b, needed):
    db, acc, ret = _grad_dest(b, needed)
    if db is not None:
        K.colsum_bf16(dy, db, accumulate=acc)
    return ret


class LinearFn(torch.autograd.Function):
    """y = bf16(bf16(x W^T + b) * post_scale) — nn.Linear (+ the projector's / sqrt(H),
    modeling_spatialvla.py:124,331-332).  With `res`, y = bf16(bf16(x W^T + b) + res): the residual add
    fused in the epilogue (SigLIP encoder residuals; Ego3D + vision features, modeling_spatialvla.py:328).
    K may be padded (`k_pad`): the weight is zero-padded per call (patchify, Ego3D 204-wide input)."""

    @staticmethod
    def forward(ctx, x, w, b, res, post_scale):
        x = _c(x)
        M = x.shape[0]
        N, Kw = w.shape
        wk = w
        if x.shape[1] != Kw:  # zero-padded reduction dim (ld must be a multiple of 8)
            wk = torch.zeros(N, x.shape[1], dtype=BF16, device=w.device)
            wk[:, :Kw] = w
        y = _empty(M, N, like=x)
        if res is not None:
            K.linear_fwd(x, [wk], y, kind=L.EPI_BIAS_RESID, bias=b, in0=_c(res))
        elif b is not None:
            K.linear_fwd(x, [wk], y, kind=L.EPI_BIAS, bias=b, alpha=post_scale)
        else:
            K.linear_fwd(x, [wk], y, kind=L.EPI_STORE, alpha=post_scale)
        ctx.save_for_backward(x, w, b)
        ctx.post_scale = post_scale
        ctx.has_res = res is not None
        ctx.wk = wk if wk is not w else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b = ctx.saved_tensors
        dy = _c(dy)
        if ctx.post_scale != 1.0:
            # y = bf16(z * s): dz = bf16(dy * s) (autograd of the reference's division)
            dy = (dy * ctx.post_scale).to(BF16)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _empty(*x.shape, like=x)
            K.linear_dgrad(dy, [ctx.wk if ctx.wk is not None else w], dx)
        retw = None
        if ctx.needs_input_grad[1]:
            if x.shape[1] != w.shape[1]:
                tmp = _empty(w.shape[0], x.shape[1], like=x)
                K.linear_wgrad(dy, x, [tmp])
                dw, acc, retw = _grad_dest(w, True)
                if acc:
                    dw.add_(tmp[:, :w.shape[1]])
                else:
                    dw.copy_(tmp[:, :w.shape[1]])
            else:
                dw, acc, retw = _grad_dest(w, True)
                K.linear_wgrad(dy, x, [dw], accumulate=acc)
        retb = _bias_grad(dy, b, b is not None and ctx.needs_input_grad[2])
        dres = dy if ctx.has_res else None
        return dx, retw, retb, dres, None


# ------------------------------------------------------------------------------------ fp8 projections
# Bumped by TrainEngine.optimizer_step: AdamW rewrites the bf16 weights through the C-ABI, which torch's version
# counters do not see, so the fp8 weight copies compare this epoch as well.
WEIGHT_EPOCH = [0]
# fp8 projections: the input-gradient (dgrad) GEMMs run in e4m3 too (the weight-gradient GEMMs stay bf16)
FP8_DGRAD = [True]
# scaling of the fp8 operands: "mx" = OCP MX block scales (one E8M0 scale per 32 k, applied by the MFMA; the product
# path), "row" = one fp32 scale per row applied in the epilogue (round 2-4)
FP8_SCALING = [os.environ.get("SVLA_FP8_SCALING", "mx")]
# which Gemma2 projections run in fp8 when a layer has fp8 weights (configs[4]): any of "qkv", "o", "gate_up", "down"
# (SVLA_FP8_SITES, comma-separated); the others stay on the bf16 GEMM.  tests/test_fp8_ablation_gpu.py measures each
# site's share of the logit error and of the action-row flips.
FP8_SITES = [set(os.environ.get("SVLA_FP8_SITES", "qkv,o,gate_up,down").split(","))]


def _fp8_site(f8, name):
    """f8 if projection `name` runs in fp8 (FP8_SITES), else None (the bf16 GEMM)."""
    return f8 if f8 is not None and name in FP8_SITES[0] else None


class FP8Weights:
    """e4m3 copies of one Gemma2 layer's projection weights (BASELINE configs[4]): q|k|v [4096, H], o [H, 2048],
    gate|up [2I, H], down [H, I].  MX scaling: the forward copy W (MX blocks along the input dim K) and, for dgrad,
    W^T (blocks along the output dim N: the dgrad GEMM's reduction) each quantised from bf16 (svla_quant_mx_rows);
    row scaling: per-row fp32 scales, W^T the byte transpose of the forward copy.  Rebuilt lazily when a weight
    moved, was modified in place, or the optimizer stepped (WEIGHT_EPOCH)."""

    def __init__(self):
        self._key = None
        self.mats = {}

    @staticmethod
    def _rows(mats):
        mats = K._merge_rows(list(mats))
        return mats[0] if len(mats) == 1 else torch.cat(mats, 0)

    def _entry(self, name, mats):
        key = (WEIGHT_EPOCH[0], FP8_SCALING[0]) + tuple((m.data_ptr(), m._version) for m in mats)
        hit = self.mats.get(name)
        if hit is None or hit["key"] != key:
            w = self._rows(mats)
            if FP8_SCALING[0] == "mx" and w.shape[0] % 128 == 0 and w.shape[1] % 128 == 0:
                # both layouts from one read of the bf16 weight (the forward copy and the dgrad copy W^T)
                (q, s), (qt, st) = K.quant_mx_both(w)
                hit = self.mats[name] = {"key": key, "q": q, "s": s, "qt": qt, "st": st}
            else:
                q, s = K.quant_mx_rows(w) if FP8_SCALING[0] == "mx" else K.quant_fp8_rows(w)
                hit = self.mats[name] = {"key": key, "q": q, "s": s}
        return hit

    def get(self, name, mats):
        e = self._entry(name, mats)
        return e["q"], e["s"]

    def get_t(self, name, mats):
        """The dgrad operand: MX -- (e4m3 W^T [K, N], its MX scales); row -- (the byte transpose of the forward copy,
        the forward copy's row scales s [N])."""
        e = self._entry(name, mats)
        if "qt" not in e:
            if FP8_SCALING[0] == "mx":
                e["qt"], e["st"] = K.quant_mx_cols(self._rows(mats))  # W^T's rows, no transposed copy
            else:
                e["qt"], e["st"] = K.transpose_u8(e["q"]), e["s"]
        return e["qt"], e["st"]

    def ones(self, n, device):
        o = self.mats.get(("ones", n))
        if o is None:
            o = self.mats[("ones", n)] = torch.ones(n, dtype=torch.float32, device=device)
        return o


def _fp8_linear(x, f8, name, mats, out, x_mx=None, **kw):
    """out = epi(x @ cat(mats)^T) with both operands quantised to e4m3 (x per call -- or x_mx, the MX copy x's
    producer already made -- weights cached)."""
    wq, ws = f8.get(name, mats)
    if FP8_SCALING[0] == "mx":
        xq, xs = x_mx if x_mx is not None else K.quant_mx_rows(x)
        K.gemm_mxfp8(xq, xs, wq, ws, out, **kw)
    else:
        xq, xs = K.quant_fp8_rows(x)
        K.gemm_fp8(xq, xs, wq, ws, out, **kw)


def _fp8_dgrad(dy, f8, name, mats, out, dy_mx=None):
    """out[M, K] = dy[M, N] @ cat(mats)[N, K] on the fp8 GEMM.  MX: dy quantised with blocks along N against the
    MX copy of W^T (dy_mx: that quantisation already made by dy's producer).  Row scaling: the forward's e4m3 weight
    W ~ diag(s_w) W_q reused transposed -- dy's columns are scaled by s_w before dy is quantised per row, so
    out = s_dy[m] * sum_n q_dy[m, n] W_q[n, k]."""
    wt, st = f8.get_t(name, mats)
    if FP8_SCALING[0] == "mx":
        dq, ds = dy_mx if dy_mx is not None else K.quant_mx_rows(dy)
        K.gemm_mxfp8(dq, ds, wt, st, out)
    else:
        dq, ds = K.quant_fp8_rows(dy, colscale=st)
        K.gemm_fp8(dq, ds, wt, f8.ones(wt.shape[0], dy.device), out)


# ------------------------------------------------------------------------------------ Gemma2 blocks
@dataclass
class GemmaAttnCfg:
    B: int
    L: int
    Hq: int
    Hkv: int
    D: int
    scale: float
    softcap: float
    window: int


class GemmaAttentionFn(torch.autograd.Function):
    """Gemma2Attention.forward (modeling_gemma2.py:364-413): q/k/v projections, rotary embedding
    (:95-154), eager prefix-LM GQA attention with logit softcap (:169-195), o_proj — as one fused
    QKV GEMM whose epilogue applies RoPE to q/k (bf16 rounding of the reference), one attention kernel,
    one O GEMM.  The saved qkv holds the rotated q/k; the attention backward returns dq/dk w.r.t. the
    pre-rotation q/k (RoPE transpose), which is what the projection backward needs."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, wo, cos, sin, kv_class, cfg: GemmaAttnCfg, f8: Optional[FP8Weights] = None,
                capture: Optional[dict] = None, mx_in: Optional[MXSlot] = None, mx_dout: Optional[MXSlot] = None):
        x = _c(x)
        x_mx = mx_in.take(x) if mx_in is not None else None
        M, H = x.shape
        qd, kd = cfg.Hq * cfg.D, cfg.Hkv * cfg.D
        qkv = _empty(M, qd + 2 * kd, like=x)
        rope = (cos, sin, cos.shape[0], cfg.D, qd + kd)
        if _fp8_site(f8, "qkv") is not None:
            _fp8_linear(x, f8, "qkv", (wq, wk, wv), qkv, x_mx=x_mx, kind=L.EPI_ROPE, rope=rope)
        else:
            K.linear_fwd(x, [wq, wk, wv], qkv, kind=L.EPI_ROPE, rope=rope)
        attn = _empty(M, qd, like=x)
        lse = _empty(cfg.B, cfg.Hq, cfg.L, dtype=F32, like=x)
        a = K.attn_args(cfg.B, cfg.L, cfg.Hq, cfg.Hkv, cfg.D, qkv[:, :qd], qkv.stride(0), qkv[:, qd:qd + kd],
                        qkv.stride(0), qkv[:, qd + kd:], qkv.stride(0), cfg.scale, cfg.softcap, kv_class, cfg.window)
        K.attn_fwd(a, attn, lse)
        if capture is not None:  # output_attentions: the rotated q|k|v rows (no copy)
            capture["qkv"] = qkv
        out = _empty(M, wo.shape[0], like=x)
        if _fp8_site(f8, "o") is not None:
            _fp8_linear(attn, f8, "o", (wo,), out)
        else:
            K.linear_fwd(attn, [wo], out)
        ctx.save_for_backward(x, wq, wk, wv, wo, qkv, attn, lse, cos, sin, kv_class)
        ctx.cfg = cfg
        ctx.f8 = f8
        ctx.mx_dout = mx_dout
        return out

    @staticmethod
    def backward(ctx, dout):
        x, wq, wk, wv, wo, qkv, attn, lse, cos, sin, kv_class = ctx.saved_tensors
        cfg = ctx.cfg
        if cos.shape[0] != cfg.L:  # Gemma2Attention.forward refuses this case up front (check_rope_for_grad)
            raise NotImplementedError("GemmaAttentionFn.backward: per-sequence RoPE tables (the backward's RoPE "
                                      "transpose reads table row = position in the sequence)")
        dout = _c(dout)
        M = x.shape[0]
        qd, kd = cfg.Hq * cfg.D, cfg.Hkv * cfg.D
        dattn = _empty(M, qd, like=x)
        f8 = ctx.f8 if FP8_DGRAD[0] else None
        # each weight gradient is queued on the side stream before the main-stream work it may overlap
        side = _SideWork(x)
        dwo, acc, ret_wo = _grad_dest(wo, ctx.needs_input_grad[4])
        if dwo is not None:
            side.run(lambda: K.linear_wgrad(dout, attn, [dwo], accumulate=acc), dout, attn)
        if _fp8_site(f8, "o") is not None:
            _fp8_dgrad(dout, f8, "o", (wo,), dattn, dy_mx=ctx.mx_dout.take(dout) if ctx.mx_dout is not None else None)
        else:
            K.linear_dgrad(dout, [wo], dattn)
        dqkv = torch.empty_like(qkv)
        a = K.attn_args(cfg.B, cfg.L, cfg.Hq, cfg.Hkv, cfg.D, qkv[:, :qd], qkv.stride(0), qkv[:, qd:qd + kd],
                        qkv.stride(0), qkv[:, qd + kd:], qkv.stride(0), cfg.scale, cfg.softcap, kv_class, cfg.window,
                        cos, sin)
        ld = dqkv.stride(0)
        K.attn_bwd(a, attn, dattn, lse, dqkv[:, :qd], ld, dqkv[:, qd:qd + kd], ld, dqkv[:, qd + kd:], ld)
        dx = None
        dests = [_grad_dest(w, ctx.needs_input_grad[1 + i]) for i, w in enumerate((wq, wk, wv))]

        def qkv_wgrad():
            if all(d[0] is not None for d in dests) and len({d[1] for d in dests}) == 1:
                K.linear_wgrad(dqkv, x, [d[0] for d in dests], accumulate=dests[0][1])
            else:
                off = 0
                for (dw, acc_i, _), w in zip(dests, (wq, wk, wv)):
                    n = w.shape[0]
                    if dw is not None:
                        K.linear_wgrad(_c(dqkv[:, off:off + n]), x, [dw], accumulate=acc_i)
                    off += n
        side.run(qkv_wgrad, dqkv, x)
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            if _fp8_site(f8, "qkv") is not None:
                _fp8_dgrad(dqkv, f8, "qkv", (wq, wk, wv), dx)
            else:
                K.linear_dgrad(dqkv, [wq, wk, wv], dx)
        rets = [d[2] for d in dests]
        side.join(*rets, ret_wo)
        return (dx, *rets, ret_wo, None, None, None, None, None, None, None, None)


@torch.no_grad()
def gemma_attention_weights(qkv, kv_class, cfg: GemmaAttnCfg) -> torch.Tensor:
    """output_attentions of the reference eager attention (modeling_gemma2.py:169-195): softmax probabilities
    [B, Hq, L, L] in bf16, from the rotated q / k rows the fused projection wrote.  The attention OUTPUT always comes
    from the HIP kernel, which never materialises these L x L maps; this is an introspection path (torch ops, the
    reference's op order and bf16 roundings: bf16 scores * scale, bf16 softcap, + additive mask, fp32 softmax)."""
    B, L, Hq, Hkv, D = cfg.B, cfg.L, cfg.Hq, cfg.Hkv, cfg.D
    qd, kd = Hq * D, Hkv * D
    q = qkv[:, :qd].reshape(B, L, Hq, D).transpose(1, 2)
    k = qkv[:, qd:qd + kd].reshape(B, L, Hkv, D).transpose(1, 2)
    k = k.repeat_interleave(Hq // Hkv, dim=1)                                   # repeat_kv (:157-166)
    w = torch.matmul(q, k.transpose(2, 3)) * cfg.scale
    if cfg.softcap:
        w = torch.tanh(w / cfg.softcap) * cfg.softcap
    mn = torch.finfo(w.dtype).min
    i = torch.arange(L, device=qkv.device)
    cls = (kv_class if kv_class is not None else torch.zeros(B, L, dtype=torch.uint8, device=qkv.device))[:, :L]
    vis = (cls[:, None, :] == 0) | ((cls[:, None, :] == 1) & (i[None, :, None] >= i[None, None, :]))
    if cfg.window:  # sliding layers (:461-473): keys at distance >= window are masked
        vis = vis & ((i[:, None] - i[None, :]) < cfg.window)[None]
    w = w + torch.where(vis, 0.0, mn).to(w.dtype)[:, None]
    return torch.softmax(w, dim=-1, dtype=torch.float32).to(qkv.dtype)


# decode steps run RoPE + cache append + attention as one launch (svla_attn_decode_rope); False = the two-launch
# form (svla_qkv_rope_append, then svla_attn_decode), kept for the bitwise A/B test
DECODE_FUSED = [os.environ.get("SVLA_DECODE_FUSED", "1") != "0"]


# decode steps fold the two norms between sublayers into the next projection's prologue (svla_gemv_rmsnorm2)
DECODE_NORM_FUSED = [os.environ.get("SVLA_DECODE_NORM_FUSED", "1") != "0"]


@torch.no_grad()
def gemma_attention_cached(x, wq, wk, wv, wo, cos, sin, k_cache, v_cache, kv_class, p0, cfg: GemmaAttnCfg,
                           pre=None, skip_o=False):
    """Gemma2Attention.forward with a KV cache (modeling_gemma2.py:364-413, cache update :387-395), inference
    only.  x holds the cfg.L new tokens of each of the cfg.B sequences, at absolute positions p0 .. p0+L-1;
    their rotated k and v are written into rows p0.. of k_cache/v_cache ([B, capacity, Hkv*D]).  The prefill
    (p0 == 0) runs the flash kernel of the uncached forward over the prompt, so it is bit-identical to it;
    later steps run the decode kernel over the first p0+L cache rows.  pre = (res, y, w1, w2, eps1, eps2, h_out): a
    decode step whose input x = rms(res + rms(y; w1); w2) is formed inside the q|k|v GEMV (h_out the new residual)."""
    if pre is not None:
        if p0 == 0:
            raise ValueError("gemma_attention_cached: the fused norm prologue is a decode-step path (p0 > 0)")
        M, H = pre[1].shape
        like = pre[1]
    else:
        x = _c(x)
        M, H = x.shape
        like = x
    B, Lq = cfg.B, cfg.L
    qd, kd = cfg.Hq * cfg.D, cfg.Hkv * cfg.D
    qkv = _empty(M, qd + 2 * kd, like=like)
    attn = _empty(M, qd, like=like)
    if p0 > 0:
        # decode step: plain projection, then one launch rotates q / k, appends k / v to the cache and attends;
        # the kernels read table row b*Lq+t (per-sequence positions), so a shared table is repeated per sequence
        if cos.shape[0] != B * Lq:
            cos, sin = cos.repeat(B, 1), sin.repeat(B, 1)
        if pre is not None:
            K.gemv_rmsnorm2(*pre, [wq, wk, wv], qkv)
        else:
            K.linear_fwd(x, [wq, wk, wv], qkv)
        if DECODE_FUSED[0]:
            K.attn_decode_rope(qkv, Lq, cos, sin, k_cache, v_cache, p0 + Lq, cfg.Hq, cfg.Hkv, cfg.D, cfg.scale,
                               cfg.softcap, kv_class, cfg.window, attn)
        else:
            K.qkv_rope_append(qkv, B, Lq, cfg.Hq, cfg.Hkv, cfg.D, cos, sin, k_cache, v_cache, p0)
            K.attn_decode(qkv[:, :qd], Lq, k_cache, v_cache, p0 + Lq, cfg.Hq, cfg.Hkv, cfg.D, cfg.scale,
                          cfg.softcap, kv_class, cfg.window, attn)
    elif PREFILL_ROPE_FILL[0]:
        # the plain projection, then one launch rotates q and k in place and fills cache rows 0.. with k and v
        # (svla_qkv_rope_fill: the ROPE epilogue's rounding, bitwise), instead of the RoPE epilogue + two cache copies
        if cos.shape[0] != B * Lq:
            cos, sin = cos.repeat(B, 1), sin.repeat(B, 1)
        K.linear_fwd(x, [wq, wk, wv], qkv)
        K.qkv_rope_append(qkv, B, Lq, cfg.Hq, cfg.Hkv, cfg.D, cos, sin, k_cache, v_cache, 0, k_back=True)
    else:
        K.linear_fwd(x, [wq, wk, wv], qkv, kind=L.EPI_ROPE, rope=(cos, sin, cos.shape[0], cfg.D, qd + kd))
        k_cache[:, :Lq].copy_(qkv[:, qd:qd + kd].view(B, Lq, kd))
        v_cache[:, :Lq].copy_(qkv[:, qd + kd:].view(B, Lq, kd))
    if p0 == 0:
        lse = _empty(B, cfg.Hq, Lq, dtype=F32, like=like)
        cls = kv_class[:, :Lq].contiguous()  # held until the launch: attn_args keeps only its pointer
        a = K.attn_args(B, Lq, cfg.Hq, cfg.Hkv, cfg.D, qkv[:, :qd], qkv.stride(0), qkv[:, qd:qd + kd],
                        qkv.stride(0), qkv[:, qd + kd:], qkv.stride(0), cfg.scale, cfg.softcap, cls, cfg.window)
        K.attn_fwd(a, attn, lse)
    if skip_o:  # the caller runs the o projection (gemma_mlp_decode with o=(attn, wo): inside its launch)
        return attn
    out = _empty(M, wo.shape[0], like=like)
    K.linear_fwd(attn, [wo], out)
    return out


# the prefill's q|k|v: plain GEMM + svla_qkv_rope_fill (one launch: RoPE of q and k, cache rows of k and v) instead
# of the RoPE epilogue + two cache copies; SVLA_PREFILL_ROPE_FILL=0: the latter
PREFILL_ROPE_FILL = [os.environ.get("SVLA_PREFILL_ROPE_FILL", "1") != "0"]


# ... with the o projection inside the same launch (a second grid barrier) instead of its own GEMV: opt-in, measured
# slower (1.97 vs 1.84 ms per token: 2304 rows over 2048 waves leave one row in flight a wave; profiles/r7b_*)
DECODE_O_FUSED = [os.environ.get("SVLA_DECODE_O_FUSED", "0") != "0"]


def persist_ok(y, wg, wu, wd) -> bool:
    return (DECODE_MLP_PERSIST[0] and y.shape[1] <= 2560 and wg.shape[0] <= 10240 and y.shape[0] <= 8
            and wg.stride(1) == wu.stride(1) == wd.stride(1) == 1
            and K.decode_mlp_grid(y.shape[0], y.shape[1], wg.shape[0]) > 0)


# the decode MLP as one persistent launch (svla_decode_mlp) instead of the norm-GEMV + down-GEMV pair: 1.80 vs
# 1.95 ms per decode token (profiles/r6z_decode_mlp_persist_ab.txt); SVLA_DECODE_MLP_PERSIST=0: the pair
DECODE_MLP_PERSIST = [os.environ.get("SVLA_DECODE_MLP_PERSIST", "1") != "0"]


@torch.no_grad()
def gemma_mlp_decode(res, y, w1, w2, eps1, eps2, h_out, wg, wu, wd, o=None):
    """Decode-step Gemma2 MLP (modeling_gemma2.py:91-92) whose input is the post-attention + pre-feedforward norm pair
    (:487-490), formed inside the gate|up GEMV: h_out = res + rms(y; w1) (the residual stream), returns
    down(gelu_tanh(gate x) * up x) with x = rms(h_out; w2)."""
    if o is not None:  # y = attn @ wo^T (the o projection), in the persistent launch or as its own GEMV
        attn, wo = o
        y = _empty(attn.shape[0], wo.shape[0], like=attn)
        if (not persist_ok(y, wg, wu, wd) or attn.shape[1] > 2048 or wo.stride(1) != 1
                or y.shape[1] > 8 * K.decode_mlp_grid(y.shape[0], y.shape[1], wg.shape[0])):
            K.linear_fwd(attn, [wo], y)
            o = None
    M = y.shape[0]
    I = wg.shape[0]
    out = _empty(M, wd.shape[0], like=y)
    if persist_ok(y, wg, wu, wd):
        hact = _empty(M, I, like=y)
        K.decode_mlp(res, y, w1, w2, eps1, eps2, h_out, wg, wu, wd, hact, out, o=o)  # one persistent launch, bitwise
        return out
    hact, g, u = (_empty(M, I, like=y) for _ in range(3))
    K.gemv_rmsnorm2(res, y, w1, w2, eps1, eps2, h_out, [wg, wu], hact, geglu_out=(g, u))
    K.linear_fwd(hact, [wd], out)
    return out


class GemmaMLPFn(torch.autograd.Function):
    """Gemma2MLP.forward (modeling_gemma2.py:91-92): down(gelu_tanh(gate x) * up x) — gate/up as one
    GEMM with the GeGLU in its epilogue; backward: dH GEMM, then the GeGLU derivative in one elementwise pass."""

    @staticmethod
    def forward(ctx, x, wg, wu, wd, f8: Optional[FP8Weights] = None, mx_in: Optional[MXSlot] = None,
                mx_dout: Optional[MXSlot] = None):
        x = _c(x)
        x_mx = mx_in.take(x) if mx_in is not None else None
        M = x.shape[0]
        I = wg.shape[0]
        h = _empty(M, I, like=x)
        g = _empty(M, I, like=x)
        u = _empty(M, I, like=x)
        out = _empty(M, wd.shape[0], like=x)
        h_mx = None
        if _fp8_site(f8, "gate_up") is not None:
            kw = {}
            if _fp8_site(f8, "down") is not None and FP8_SCALING[0] == "mx" and I % 128 == 0:
                # the GeGLU epilogue also writes the MX copy of h, the fp8 down operand (no quantisation pass)
                h_mx = (torch.empty(M, I, dtype=torch.float8_e4m3fn, device=x.device), K.MXScales(M, I, x.device))
                kw["mx_out"] = h_mx
            _fp8_linear(x, f8, "gate_up", (wg, wu), h, x_mx=x_mx, kind=L.EPI_GEGLU, geglu_I=I, out1=g, out2=u, **kw)
        else:
            K.linear_geglu_fwd(x, wg, wu, h, g, u)
        if _fp8_site(f8, "down") is not None:
            _fp8_linear(h, f8, "down", (wd,), out, x_mx=h_mx)
        else:
            K.linear_fwd(h, [wd], out)
        ctx.save_for_backward(x, wg, wu, wd, g, u, h)
        ctx.f8 = f8
        ctx.mx_dout = mx_dout
        return out

    @staticmethod
    def backward(ctx, dout):
        x, wg, wu, wd, g, u, h = ctx.saved_tensors
        dout = _c(dout)
        M, I = g.shape
        side = _SideWork(x)
        dwd, acc, ret_wd = _grad_dest(wd, ctx.needs_input_grad[3])
        if dwd is not None:
            side.run(lambda: K.linear_wgrad(dout, h, [dwd], accumulate=acc), dout, h)
        dgu = _empty(M, 2 * I, like=x)
        f8 = ctx.f8 if FP8_DGRAD[0] else None
        # dH by a plain-store GEMM, then the GeGLU derivative as one HBM pass in place (in the down dgrad's epilogue
        # it cost more than the pass: +60 % on the 8-phase kernel's LDS image, +0.11 ms per layer from the 4-wave
        # kernel's accumulators with the g / u loads one row block ahead, r4)
        if _fp8_site(f8, "down") is not None:
            _fp8_dgrad(dout, f8, "down", (wd,), dgu[:, :I],
                       dy_mx=ctx.mx_dout.take(dout) if ctx.mx_dout is not None else None)
        else:
            K.linear_dgrad(dout, [wd], dgu[:, :I])
        f8gu = _fp8_site(f8, "gate_up")
        dgu_mx = None
        if f8gu is not None and FP8_SCALING[0] == "mx" and I % 128 == 0 and ctx.needs_input_grad[0]:
            # the MX copy of [dg | du] for the fp8 dgrad comes out of the same pass (no quantisation pass over dgu)
            dgu_mx = K.geglu_bwd_mx(dgu[:, :I], g, u, dgu[:, :I], dgu[:, I:])
        else:
            K.geglu_bwd(dgu[:, :I], g, u, dgu[:, :I], dgu[:, I:])
        dg_, accg, retg = _grad_dest(wg, ctx.needs_input_grad[1])
        du_, accu, retu = _grad_dest(wu, ctx.needs_input_grad[2])

        def gate_up_wgrad():
            if dg_ is not None and du_ is not None and accg == accu:
                K.linear_wgrad(dgu, x, [dg_, du_], accumulate=accg)
            else:
                if dg_ is not None:
                    K.linear_wgrad(_c(dgu[:, :I]), x, [dg_], accumulate=accg)
                if du_ is not None:
                    K.linear_wgrad(_c(dgu[:, I:]), x, [du_], accumulate=accu)
        side.run(gate_up_wgrad, dgu, x)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            if f8gu is not None:
                _fp8_dgrad(dgu, f8, "gate_up", (wg, wu), dx, dy_mx=dgu_mx)
            else:
                K.linear_dgrad(dgu, [wg, wu], dx)
        side.join(retg, retu, ret_wd)
        return dx, retg, retu, ret_wd, None, None, None


# ------------------------------------------------------------------------------------ SigLIP blocks
@dataclass
class SiglipAttnCfg:
    B: int
    L: int
    H: int
    D: int
    scale: float


class SiglipAttentionFn(torch.autograd.Function):
    """SiglipAttention.forward + encoder residual (transformers siglip [3p], called from
    modeling_spatialvla.py:310): q/k/v (bias) as one GEMM, bidirectional softmax attention
    (head_dim 72), out_proj with bias and the residual add fused in its epilogue."""

    @staticmethod
    def forward(ctx, x, res, wq, bq, wk, bk, wv, bv, wo, bo, cfg: SiglipAttnCfg, slot=None):
        ctx.slot = slot
        x, res = _c(x), _c(res)
        M, Hd = x.shape
        bqkv = _cat_views([bq, bk, bv])
        qkv = _empty(M, 3 * Hd, like=x)
        K.linear_fwd(x, [wq, wk, wv], qkv, kind=L.EPI_BIAS, bias=bqkv)
        attn = _empty(M, Hd, like=x)
        lse = _empty(cfg.B, cfg.H, cfg.L, dtype=F32, like=x)
        a = K.attn_args(cfg.B, cfg.L, cfg.H, cfg.H, cfg.D, qkv[:, :Hd], qkv.stride(0), qkv[:, Hd:2 * Hd],
                        qkv.stride(0), qkv[:, 2 * Hd:], qkv.stride(0), cfg.scale)
        K.attn_fwd(a, attn, lse)
        out = _empty(M, Hd, like=x)
        K.linear_fwd(attn, [wo], out, kind=L.EPI_BIAS_RESID, bias=bo, in0=res)
        ctx.save_for_backward(x, wq, bq, wk, bk, wv, bv, wo, bo, qkv, attn, lse)
        ctx.cfg = cfg
        return out

    @staticmethod
    def backward(ctx, dout):
        x, wq, bq, wk, bk, wv, bv, wo, bo, qkv, attn, lse = ctx.saved_tensors
        cfg = ctx.cfg
        dout = _c(dout)
        M, Hd = x.shape
        nig = ctx.needs_input_grad
        dattn = torch.empty_like(attn)
        # weight and bias gradients on the side stream (_SideWork), each queued before the main-stream work it may
        # overlap; every gradient buffer is allocated here, on the main stream
        side = _SideWork(x)
        dwo, acc, ret_wo = _grad_dest(wo, nig[8])
        dbo, accbo, ret_bo = _grad_dest(bo, nig[9])

        def o_grads():
            if dwo is not None:
                K.linear_wgrad(dout, attn, [dwo], accumulate=acc)
            if dbo is not None:
                K.colsum_bf16(dout, dbo, accumulate=accbo)
        side.run(o_grads, dout, attn)
        K.linear_dgrad(dout, [wo], dattn)
        dqkv = torch.empty_like(qkv)
        a = K.attn_args(cfg.B, cfg.L, cfg.H, cfg.H, cfg.D, qkv[:, :Hd], qkv.stride(0), qkv[:, Hd:2 * Hd],
                        qkv.stride(0), qkv[:, 2 * Hd:], qkv.stride(0), cfg.scale)
        ld = dqkv.stride(0)
        K.attn_bwd(a, attn, dattn, lse, dqkv[:, :Hd], ld, dqkv[:, Hd:2 * Hd], ld, dqkv[:, 2 * Hd:], ld)
        rets = []
        dws = [_grad_dest(w, nig[2 + 2 * i]) for i, w in enumerate((wq, wk, wv))]
        bds = [_grad_dest(b, nig[3 + 2 * i]) for i, b in enumerate((bq, bk, bv))]
        cat = None
        if all(d[0] is not None for d in bds) and len({d[1] for d in bds}) == 1:
            cat = _cat_views([d[0] for d in bds])
            if cat.data_ptr() != bds[0][0].data_ptr():  # not back to back (no engine flat buffer): a copy, unusable
                cat = None

        def qkv_grads():
            if all(d[0] is not None for d in dws) and len({d[1] for d in dws}) == 1:
                # q, k and v weight gradients in one GEMM (C row segments): three 1152x1152 wgrads launched
                # separately filled ~20 of the 256 CUs each
                K.linear_wgrad(dqkv, x, [d[0] for d in dws], accumulate=dws[0][1])
            else:
                for i, (dw, accw, _r) in enumerate(dws):
                    if dw is not None:
                        K.linear_wgrad(_c(dqkv[:, i * Hd:(i + 1) * Hd]), x, [dw], accumulate=accw)
            if cat is not None:  # the q|k|v bias gradients in one column sum over dqkv (engine: adjacent in the flat grad)
                K.colsum_bf16(dqkv, cat, accumulate=bds[0][1])
            else:
                for i, (db, accb, _r) in enumerate(bds):
                    if db is not None:
                        K.colsum_bf16(dqkv[:, i * Hd:(i + 1) * Hd], db, accumulate=accb)  # strided view, no copy
        side.run(qkv_grads, dqkv, x)
        dx = torch.empty_like(x) if nig[0] else None
        if dx is not None:
            K.linear_dgrad(dqkv, [wq, wk, wv], dx)
        for i in range(3):
            rets += [dws[i][2], bds[i][2]]
        side.join(*rets, ret_wo, ret_bo)
        dres = dout
        if ctx.slot is not None:  # handed to layer_norm1's backward (ResidualSlot)
            ctx.slot.put(dout)
            dres = None
        return (dx, dres, *rets, ret_wo, ret_bo, None, None)


# SigLIP fc1 / BEiT fc1: bias GEMM + GELU pass (svla_gelu_rows) instead of the VALU-heavy GELU GEMM epilogues, which
# ran slower inside the tile loop (profiles/r3l_epi_ab.txt); bitwise the same values (test_gelu_rows_matches_epilogues)
GELU_PASS = [os.environ.get("SVLA_GELU_PASS", "1") != "0"]


class SiglipMLPFn(torch.autograd.Function):
    """SiglipMLP + residual: res + fc2(gelu_tanh(fc1 x)) (transformers siglip [3p]); fc1 bias+GELU and
    fc2 bias+residual fused in GEMM epilogues, GELU derivative fused into the fc2 dgrad epilogue."""

    @staticmethod
    def forward(ctx, x, res, w1, b1, w2, b2, slot=None):
        ctx.slot = slot
        x, res = _c(x), _c(res)
        M = x.shape[0]
        I = w1.shape[0]
        pre = _empty(M, I, like=x)
        act = _empty(M, I, like=x)
        if GELU_PASS[0]:  # bias GEMM (the 4-wave kernel's direct epilogue), then the GELU as an HBM pass
            K.linear_fwd(x, [w1], pre, kind=L.EPI_BIAS, bias=b1)
            K.gelu_rows(K.GELU_TANH, pre, act)
        else:
            K.linear_fwd(x, [w1], act, kind=L.EPI_BIAS_GELU, bias=b1, out1=pre)
        out = _empty(M, w2.shape[0], like=x)
        K.linear_fwd(act, [w2], out, kind=L.EPI_BIAS_RESID, bias=b2, in0=res)
        ctx.save_for_backward(x, w1, b1, w2, b2, pre, act)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w1, b1, w2, b2, pre, act = ctx.saved_tensors
        dout = _c(dout)
        nig = ctx.needs_input_grad
        side = _SideWork(x)  # weight / bias gradients beside the input-gradient chain (as SiglipAttentionFn)
        dw2, acc2, ret_w2 = _grad_dest(w2, nig[4])
        db2, accb2, ret_b2 = _grad_dest(b2, nig[5])

        def fc2_grads():
            if dw2 is not None:
                K.linear_wgrad(dout, act, [dw2], accumulate=acc2)
            if db2 is not None:
                K.colsum_bf16(dout, db2, accumulate=accb2)
        side.run(fc2_grads, dout, act)
        dpre = torch.empty_like(pre)
        if GELU_PASS[0]:
            K.linear_dgrad(dout, [w2], dpre)
            K.gelu_rows(K.GELU_TANH_BWD, dpre, dpre, pre=pre)
        else:
            K.linear_dgrad(dout, [w2], dpre, kind=L.EPI_GELU_BWD, in0=pre)
        dw1, acc1, ret_w1 = _grad_dest(w1, nig[2])
        db1, accb1, ret_b1 = _grad_dest(b1, nig[3])

        def fc1_grads():
            if dw1 is not None:
                K.linear_wgrad(dpre, x, [dw1], accumulate=acc1)
            if db1 is not None:
                K.colsum_bf16(dpre, db1, accumulate=accb1)
        side.run(fc1_grads, dpre, x)
        dx = torch.empty_like(x) if nig[0] else None
        if dx is not None:
            K.linear_dgrad(dpre, [w1], dx)
        side.join(ret_w1, ret_b1, ret_w2, ret_b2)
        dres = dout
        if ctx.slot is not None:  # handed to layer_norm2's backward (ResidualSlot)
            ctx.slot.put(dout)
            dres = None
        return dx, dres, ret_w1, ret_b1, ret_w2, ret_b2, None


class PatchEmbedFn(torch.autograd.Function):
    """SiglipVisionEmbeddings.forward (transformers siglip [3p]): Conv2d(3, H, k=s=14) + bias +
    position embedding, as im2col + one GEMM whose epilogue adds bias and position rows."""

    @staticmethod
    def forward(ctx, pix, w, b, pos, patch):
        pix = _c(pix)
        B, C, S, _ = pix.shape
        np_ = (S // patch) ** 2
        Kc = C * patch * patch
        Kp = K.round_up(Kc, 8)
        cols = _empty(B * np_, Kp, like=pix)
        K.im2col_patch(pix, patch, cols)
        w2 = w.reshape(w.shape[0], Kc)
        wk = torch.zeros(w.shape[0], Kp, dtype=BF16, device=w.device)
        wk[:, :Kc] = w2
        posx = pos.unsqueeze(0).expand(B, np_, pos.shape[1]).reshape(B * np_, pos.shape[1])
        y = _empty(B * np_, w.shape[0], like=pix)
        K.linear_fwd(cols, [wk], y, kind=L.EPI_BIAS_RESID, bias=b, in0=_c(posx))
        ctx.save_for_backward(cols, w, b, pos)
        ctx.B, ctx.np = B, np_
        return y

    @staticmethod
    def backward(ctx, dy):
        cols, w, b, pos = ctx.saved_tensors
        dy = _c(dy)
        Kc = w[0].numel()
        rw = None
        if ctx.needs_input_grad[1]:
            tmp = _empty(w.shape[0], cols.shape[1], like=cols)
            K.linear_wgrad(dy, cols, [tmp])
            dw, acc, rw = _grad_dest(w, True)
            src = tmp[:, :Kc].reshape(w.shape)
            dw.add_(src) if acc else dw.copy_(src)
        rb = _bias_grad(dy, b, ctx.needs_input_grad[2])
        rp = None
        if ctx.needs_input_grad[3]:
            dp, acc, rp = _grad_dest(pos, True)
            K.colsum_bf16(dy.view(ctx.B, ctx.np * pos.shape[1]), dp.view(-1), accumulate=acc)
        return None, rw, rb, rp, None


class EmbedMergeFn(torch.autograd.Function):
    """Embedding merge of SpatialVLAForConditionalGeneration.forward (modeling_spatialvla.py:361-387)
    times the Gemma2 normalizer (modeling_gemma2.py:741-742): token embeddings (frozen table), spatial
    action-token embeddings, image features scattered into the <image> slots in (b, t) order."""

    @staticmethod
    def forward(ctx, ids, img_index, img_feats, spatial_w, embed_w, a0, normalizer, sort_rows, offsets):
        ids = _c(ids).view(-1)
        H = embed_w.shape[1]
        out = _empty(ids.numel(), H, like=embed_w)
        na = spatial_w.shape[0] if spatial_w is not None else 0
        K.embed_merge(ids, img_index, embed_w, spatial_w, a0, na, img_feats, normalizer, out)
        ctx.save_for_backward(ids, img_index, sort_rows, offsets, spatial_w, img_feats)
        ctx.normalizer, ctx.na = normalizer, na
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, img_index, sort_rows, offsets, spatial_w, img_feats = ctx.saved_tensors
        dout = _c(dout)
        dimg = torch.empty_like(img_feats) if (img_feats is not None and ctx.needs_input_grad[2]) else None
        dsp, acc, rsp = (None, False, None)
        if spatial_w is not None and ctx.needs_input_grad[3]:
            dsp, acc, rsp = _grad_dest(spatial_w, True)
            if acc:
                tmp = torch.empty_like(spatial_w)
                K.embed_merge_bwd(ids, img_index, sort_rows, offsets, ctx.na, dout, ctx.normalizer, tmp, None)
                dsp.add_(tmp)
                dsp = None
        if dimg is not None or dsp is not None:
            K.embed_merge_bwd(ids, img_index, sort_rows, offsets, ctx.na, dout, ctx.normalizer, dsp, dimg)
        return None, None, dimg, rsp, None, None, None, None, None


class LMHeadCEFn(torch.autograd.Function):
    """lm_head + final logit softcap (modeling_gemma2.py:993-997) + the shifted, masked cross-entropy of
    SpatialVLAForConditionalGeneration.forward (modeling_spatialvla.py:415-430).  Logits are written once
    in bf16 (row stride padded to a multiple of 64 columns); softmax statistics come from the GEMM
    epilogue, so the fp32 [B, L, V] tensor of the reference is never materialised.
    Returns (logits [M, V] view, loss scalar fp32); argmax / lse are stashed on ctx-owned tensors."""

    @staticmethod
    def forward(ctx, h, w, target, cap, stash):
        h = _c(h)
        M = h.shape[0]
        V = w.shape[0]
        ldv = K.round_up(V, 64)
        logits_buf = _empty(M, ldv, like=h)
        ntn = K.ceil_div(V, 128)
        stats = _empty(M, ntn, 3, dtype=F32, like=h)
        # plain-store GEMM (the 4-wave kernel's direct epilogue), then softcap + statistics as one HBM pass: the
        # VALU-heavy SOFTCAP_CE epilogue inside the GEMM cost 13.4-13.9 ms per step against 9.2 + ~2 ms
        K.linear_fwd(h, [w], logits_buf[:, :V])
        K.softcap_ce_rows(logits_buf, V, stats, cap)
        lse = _empty(M, dtype=F32, like=h)
        argmax = _empty(M, dtype=torch.int64, like=h)
        loss_rows = _empty(M, dtype=F32, like=h)
        loss2 = _empty(2, dtype=F32, like=h)
        K.ce_finalize(V, ntn, stats, logits_buf[:, :V], target, lse, argmax, loss_rows, loss2)
        stash["argmax"] = argmax
        stash["lse"] = lse
        stash["n_valid"] = loss2[1:2]
        ctx.save_for_backward(h, w, logits_buf, lse, target, loss2)
        ctx.cap, ctx.V = cap, V
        ctx.row_plan = stash.pop("row_plan", None) if stash is not None else None
        ctx.mark_non_differentiable(logits_buf)
        # the logits output never receives a gradient: without this autograd hands backward a materialised zero
        # [M, V] bf16 tensor (5.3 GB at B=32, ~0.9 ms of fills per step, r4 ATen attribution)
        ctx.set_materialize_grads(False)
        return logits_buf[:, :V], loss2[0]

    @staticmethod
    def backward(ctx, dlogits_unused, dloss):
        """d(loss)/d(logits) is exactly zero on every row without a label (target < 0: the reference's
        CrossEntropyLoss ignore_index / attention-mask rows, modeling_spatialvla.py:415-430) -- at B=32 only the
        13 suffix rows of each 312-token episode carry one.  The softmax gradient and both lm_head backward GEMMs
        therefore run over the labelled rows only: dh is zero elsewhere and dW = sum over labelled rows, the same
        values as the dense products (whose other terms are exact zeros), at 1/24 of their cost."""
        h, w, logits_buf, lse, target, loss2 = ctx.saved_tensors
        if dloss is None:  # the loss did not reach the graph's output
            return None, None, None, None, None
        M, ldv = logits_buf.shape
        V = ctx.V
        gscale = (dloss.float() / torch.clamp(loss2[1], min=1.0)).reshape(1).contiguous()
        if ctx.row_plan is not None:  # labelled rows first + their count, fetched behind the forward's event
            order, cnt, ev = ctx.row_plan
            if ev is not None:
                ev.synchronize()
                cnt = int(cnt[0])
            rows = order[:cnt]
        else:
            rows = torch.nonzero(target >= 0).view(-1)
        R = int(rows.numel())
        dh = torch.zeros_like(h) if ctx.needs_input_grad[0] else None
        dw, acc, rw = _grad_dest(w, ctx.needs_input_grad[1])
        if R == 0:
            if dw is not None and not acc:
                dw.zero_()
            return dh, rw, None, None, None
        dlog = _empty(R, ldv, like=h)
        K.ce_bwd(V, logits_buf.index_select(0, rows)[:, :V], lse.index_select(0, rows),
                 target.index_select(0, rows).contiguous(), ctx.cap, gscale, dlog)
        if dh is not None:
            dh_r = _empty(R, h.shape[1], like=h)
            # reduction over the padded vocab: dlog is zero in [V, ldv); W rows beyond V read as 0 (k_valid=V)
            A = K._operand([dlog], L.LAYOUT_KC, k_valid=ldv)
            Bop = K._operand([w], L.LAYOUT_RC, k_valid=V)
            K.gemm(R, w.shape[1], ldv, A, Bop, [dh_r], [0], dh_r.stride(0), K._epi(L.EPI_STORE))
            dh.index_copy_(0, rows, dh_r)
        if dw is not None:
            K.linear_wgrad(dlog[:, :V], h.index_select(0, rows).contiguous(), [dw], accumulate=acc)
        return dh, rw, None, None, None


# ------------------------------------------------------------------------------------ attention plug-in
def kv_class_from_additive_mask(mask: Optional[torch.Tensor], B: int, Lq: int, Lk: int, device) -> torch.Tensor:
    """Per-key classes (0 visible to all queries, 1 visible to queries i >= j, 2 never visible) equivalent to
    the reference's additive [B,1,Lq,Lk] mask (modeling_spatialvla.py:258-306).  Raises ValueError when the
    mask is not of that form (the kernel never materialises an L x L mask)."""
    if mask is None:
        return torch.zeros(B, Lk, dtype=torch.uint8, device=device)
    if Lq != Lk:
        raise ValueError(f"svla attention: query length {Lq} != key length {Lk} (KV cache not supported)")
    vis = mask[:, 0, :, :Lk] == 0                                   # [B, Lq, Lk]
    all_vis = vis.all(dim=1)
    none_vis = ~vis.any(dim=1)
    cls = torch.where(all_vis, 0, torch.where(none_vis, 2, 1)).to(torch.uint8)
    i = torch.arange(Lq, device=device)
    causal = i[:, None] >= i[None, :]
    rebuilt = torch.where(cls[:, None, :] == 0, True, torch.where(cls[:, None, :] == 2, False, causal[None]))
    if not bool((rebuilt == vis).all()):
        raise ValueError("svla attention: mask is not a per-key prefix-LM/causal/padding mask")
    return cls.contiguous()


def gemma2_attention_forward(module, query, key, value, mask, **_kwargs):
    """Drop-in entry for the reference's plugin table GEMMA2_ATTENTION_FUNCTION (modeling_gemma2.py:317-322,
    called at :401-403 as fn(self, q, k, v, attention_mask, output_attentions=...)).  Same arguments and
    return as eager_attention_forward (:169-195): q [B,Hq,L,D], k/v [B,Hkv,L,D] after RoPE, additive mask
    [B,1,L,L] or None -> (out [B,L,Hq,D] contiguous, None).  Scale = module.scaling, softcap =
    module.attn_logit_softcapping; probabilities are rounded to bf16 before PV as in the reference (Q3)."""
    if _kwargs.get("output_attentions"):
        raise NotImplementedError("svla attention does not materialise attention weights")
    B, _, Lq, _ = query.shape
    cls = kv_class_from_additive_mask(mask, B, Lq, key.shape[2], query.device)
    softcap = getattr(module, "attn_logit_softcapping", None) or 0.0
    return hip_attention(query, key, value, module.scaling, softcap, cls, 0), None


def hip_attention(q, k, v, scale, softcap=0.0, kv_class=None, window=0):
    """Reference plug-in signature adapter (GEMMA2_ATTENTION_FUNCTION, modeling_gemma2.py:317-322):
    q [B, Hq, L, D], k/v [B, Hkv, L, D] (post-RoPE) -> [B, L, Hq, D].  Differentiable."""
    return _PluginAttnFn.apply(q, k, v, float(scale), float(softcap or 0.0), kv_class, int(window or 0))


class _PluginAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, softcap, kv_class, window):
        B, Hq, Lq, D = q.shape
        Hkv = k.shape[1]
        qt = q.transpose(1, 2).contiguous().view(B * Lq, Hq * D)
        kt = k.transpose(1, 2).contiguous().view(B * Lq, Hkv * D)
        vt = v.transpose(1, 2).contiguous().view(B * Lq, Hkv * D)
        out = _empty(B * Lq, Hq * D, like=q)
        lse = _empty(B, Hq, Lq, dtype=F32, like=q)
        a = K.attn_args(B, Lq, Hq, Hkv, D, qt, qt.stride(0), kt, kt.stride(0), vt, vt.stride(0), scale, softcap,
                        kv_class, window)
        K.attn_fwd(a, out, lse)
        ctx.save_for_backward(qt, kt, vt, out, lse, kv_class)
        ctx.meta = (B, Lq, Hq, Hkv, D, scale, softcap, window)
        return out.view(B, Lq, Hq, D)

    @staticmethod
    def backward(ctx, dout):
        qt, kt, vt, out, lse, kv_class = ctx.saved_tensors
        B, Lq, Hq, Hkv, D, scale, softcap, window = ctx.meta
        do = _c(dout).view(B * Lq, Hq * D)
        dq, dk, dv = torch.empty_like(qt), torch.empty_like(kt), torch.empty_like(vt)
        a = K.attn_args(B, Lq, Hq, Hkv, D, qt, qt.stride(0), kt, kt.stride(0), vt, vt.stride(0), scale, softcap,
                        kv_class, window)
        K.attn_bwd(a, out, do, lse, dq, dq.stride(0), dk, dk.stride(0), dv, dv.stride(0))
        tr = lambda t, H: t.view(B, Lq, H, D).transpose(1, 2)  # noqa: E731
        return tr(dq, Hq), tr(dk, Hkv), tr(dv, Hkv), None, None, None, None


# ------------------------------------------------------------------------------------ BEiT layer (ZoeDepth)
def _beit_weights(layer):
    """q|k|v weight [3H, H] and bias [3H] (k has none) of a BeitLayer, concatenated once and cached against the
    parameters' storage and version (the estimator is frozen)."""
    at = layer.attention
    ps = (at.q_proj.weight, at.k_proj.weight, at.v_proj.weight, at.q_proj.bias, at.v_proj.bias)
    key = tuple((p.data_ptr(), p._version) for p in ps)
    hit = getattr(layer, "_svla_qkv", None)
    if hit is not None and hit[0] == key:
        return hit[1], hit[2]
    w = torch.cat([at.q_proj.weight, at.k_proj.weight, at.v_proj.weight], 0).contiguous()
    b = torch.cat([at.q_proj.bias, torch.zeros_like(at.k_proj.weight[:, 0]), at.v_proj.bias], 0).contiguous()
    layer._svla_qkv = (key, w, b)
    return w, b


def _layer_scale(lam, H, like):
    if isinstance(lam, torch.Tensor):
        return _c(lam.to(like.dtype))
    return torch.full((H,), float(lam), dtype=like.dtype, device=like.device)


def beit_layer(layer, hidden_states, bias):
    """transformers BeitLayer.forward [3p] (the ZoeDepth backbone, called at model/modeling_spatialvla.py:314-323)
    in inference on the HIP kernels:
        h = x + lambda_1 * o_proj(attn(q_proj|k_proj|v_proj(LN_before(x)), + rel-pos bias))
        y = h + lambda_2 * fc2(gelu(fc1(LN_after(h))))
    LayerNorm: svla_layernorm_fwd; the three projections one GEMM with the [bq, 0, bv] bias epilogue; attention
    svla_attn_fwd at head_dim 64 with the additive bias (fp32 scores and softmax, P in bf16); o_proj and fc2 with
    the BIAS_SCALE_RESID epilogue (bf16(bf16(lambda * bf16(acc + b)) + residual), the module's rounding points);
    fc1 with BIAS_GELU_ERF.  bias: [heads, L, ld] bf16 or None."""
    B, Lq, H = hidden_states.shape
    at = layer.attention
    D = at.head_dim
    nh = at.num_attention_heads
    x = _c(hidden_states).view(B * Lq, H)
    M = B * Lq
    ln_before, ln_after = layer.layernorm_before, layer.layernorm_after
    mean = _empty(M, dtype=F32, like=x)
    rstd = _empty(M, dtype=F32, like=x)
    xn = _empty(M, H, like=x)
    K.layernorm_fwd(x, ln_before.weight, ln_before.bias, float(ln_before.eps), xn, mean, rstd)
    wqkv, bqkv = _beit_weights(layer)
    qkv = _empty(M, 3 * H, like=x)
    K.linear_fwd(xn, [wqkv], qkv, kind=L.EPI_BIAS, bias=bqkv)
    a = K.attn_args(B, Lq, nh, nh, D, qkv[:, :H], qkv.stride(0), qkv[:, H:2 * H], qkv.stride(0), qkv[:, 2 * H:],
                    qkv.stride(0), float(at.scaling), 0.0, None, 0, bias=bias)
    ctx = _empty(M, H, like=x)
    lse = _empty(B, nh, Lq, dtype=F32, like=x)
    K.attn_fwd(a, ctx, lse)
    h = _empty(M, H, like=x)
    K.linear_fwd(ctx, [at.o_proj.weight], h, kind=L.EPI_BIAS_SCALE_RESID, bias=at.o_proj.bias,
                 colscale=_layer_scale(layer.lambda_1, H, x), in0=x)
    K.layernorm_fwd(h, ln_after.weight, ln_after.bias, float(ln_after.eps), xn, mean, rstd)
    f1 = _empty(M, layer.mlp.fc1.weight.shape[0], like=x)
    if GELU_PASS[0]:
        K.linear_fwd(xn, [layer.mlp.fc1.weight], f1, kind=L.EPI_BIAS, bias=layer.mlp.fc1.bias)
        K.gelu_rows(K.GELU_ERF, f1, f1)
    else:
        K.linear_fwd(xn, [layer.mlp.fc1.weight], f1, kind=L.EPI_BIAS_GELU_ERF, bias=layer.mlp.fc1.bias)
    y = _empty(M, H, like=x)
    K.linear_fwd(f1, [layer.mlp.fc2.weight], y, kind=L.EPI_BIAS_SCALE_RESID, bias=layer.mlp.fc2.bias,
                 colscale=_layer_scale(layer.lambda_2, H, x), in0=h)
    return y.view(B, Lq, H)
