"""Tensor-level wrappers over the libsvla C-ABI (include/svla.h).

Every function here takes torch tensors that already live on the GPU, validates the shapes the
kernel assumes (so a bad call raises on the host instead of faulting the device), and launches on
torch's current HIP stream.  No function here has a non-HIP path.
"""
import ctypes
import os
import math
from typing import List, Optional, Sequence

import torch

from . import _lib as L

BF16 = torch.bfloat16


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _req(cond: bool, msg: str):
    if not cond:
        raise ValueError(msg)


def _chk_bf16(t: torch.Tensor, name: str):
    _req(t.is_cuda and t.dtype == BF16, f"{name}: expected a bf16 CUDA tensor, got {t.dtype} on {t.device}")


def _ld(t: torch.Tensor) -> int:
    _req(t.dim() == 2 and t.stride(1) == 1, "expected a 2-D row-major matrix view")
    return t.stride(0)


# ---------------------------------------------------------------------------------------- GEMM
def _operand(mats: Sequence[torch.Tensor], layout: int, seg_dim: int = L.SEG_OUTER, starts=None, r_valid: int = 0,
             k_valid: int = 0) -> L.Operand:
    op = L.Operand()
    op.r_valid = int(r_valid)
    op.k_valid = int(k_valid)
    ld = _ld(mats[0])
    for i, m in enumerate(mats):
        _chk_bf16(m, "gemm operand")
        _req(_ld(m) == ld, "gemm: all segments of an operand need the same leading dimension")
        op.ptr[i] = m.data_ptr()
    op.nseg = len(mats)
    op.seg_dim = seg_dim
    op.layout = layout
    op.ld = ld
    if starts is not None:
        for i, s in enumerate(starts):
            op.seg_start[i] = int(s)
    return op


def _epi(kind=L.EPI_STORE, accumulate=False, alpha=1.0, cap=0.0, bias=None, in0=None, in1=None, out1=None,
         out2=None, row_stats=None, rope=None, colscale=None, mx_out=None) -> L.Epilogue:
    e = L.Epilogue()
    if mx_out is not None:  # (q [M, I] e4m3, MXScales): the GEGLU epilogue's MX copy of h (fp8 GEMMs)
        q, sc = mx_out
        e.mx_q, e.mx_ldq, e.mx_scales, e.mx_sld = q.data_ptr(), q.stride(0), sc.buf.data_ptr(), sc.ld
    e.colscale = _ptr(colscale)
    e.kind = kind
    e.accumulate = 1 if accumulate else 0
    e.alpha = alpha
    e.cap = cap
    e.bias = _ptr(bias)
    if in0 is not None:
        e.in0, e.ld_in0 = in0.data_ptr(), _ld(in0)
    if in1 is not None:
        e.in1, e.ld_in1 = in1.data_ptr(), _ld(in1)
    if out1 is not None:
        e.out1, e.ld_out1 = out1.data_ptr(), _ld(out1)
    if out2 is not None:
        e.out2, e.ld_out2 = out2.data_ptr(), _ld(out2)
    e.row_stats = _ptr(row_stats)
    if rope is not None:  # (cos [L, D/2] bf16, sin, L, D, rotated columns)
        cos, sin, Lr, D, cols = rope
        _req(cos.stride(1) == 1 and sin.stride() == cos.stride(), "rope tables must share a row-major layout")
        e.rope_cos, e.rope_sin, e.rope_ld = cos.data_ptr(), sin.data_ptr(), cos.stride(0)
        e.rope_L, e.rope_D, e.rope_cols = int(Lr), int(D), int(cols)
    return e


_gemm_ws: dict = {}


def gemm_workspace(stream=None) -> torch.Tensor:
    """The caller-owned stream-K workspace of svla_gemm_bf16 for one (device, stream): GEMMs on different streams
    never share one (include/svla.h).  Zero-filled once; the kernels leave it zeroed."""
    s = stream if stream is not None else torch.cuda.current_stream()
    key = (s.device.index, s.cuda_stream)
    buf = _gemm_ws.get(key)
    if buf is None:
        n = int(L.lib().svla_gemm_workspace_bytes())
        buf = torch.zeros(n + 256, dtype=torch.uint8, device=s.device)
        off = (-buf.data_ptr()) % 256
        buf = buf[off:off + n]
        _gemm_ws[key] = buf
    return buf


gemm_log: Optional[list] = None  # tools: when a list, every svla_gemm_bf16 call appends its shape/layouts/epilogue
gemm_variant: int = int(os.environ.get("SVLA_GEMM_VARIANT", "0"))  # tests / tools: kernel choice (svla_gemm_bf16_ex)


def gemm(M: int, N: int, K: int, A: L.Operand, B: L.Operand, c_mats: Sequence[Optional[torch.Tensor]],
         c_starts: Sequence[int], ldc: int, epi: L.Epilogue, variant: Optional[int] = None):
    if gemm_log is not None:
        gemm_log.append((M, N, K, int(A.layout), int(B.layout), int(epi.kind), int(epi.accumulate)))
    n = len(c_mats)
    cp = (ctypes.c_void_p * 4)(*([_ptr(c) for c in c_mats] + [None] * (4 - n)))
    cs = (ctypes.c_int64 * 5)(*([int(s) for s in c_starts] + [0] * (5 - n)))
    ws = gemm_workspace()
    v = gemm_variant if variant is None else variant
    if v:
        rc = L.lib().svla_gemm_bf16_ex(M, N, K, ctypes.byref(A), ctypes.byref(B), cp, cs, n, ldc, ctypes.byref(epi),
                                       ws.data_ptr(), ws.numel(), int(v), _stream())
    else:
        rc = L.lib().svla_gemm_bf16(M, N, K, ctypes.byref(A), ctypes.byref(B), cp, cs, n, ldc, ctypes.byref(epi),
                                    ws.data_ptr(), ws.numel(), _stream())
    L.check(rc, "svla_gemm_bf16")


def _starts(sizes):
    out, acc = [], 0
    for s in sizes:
        out.append(acc)
        acc += s
    return out, acc


def _merge_rows(mats: List[torch.Tensor]) -> List[torch.Tensor]:
    """Row blocks [N_i, K] that sit back to back in one allocation (the engine's flat parameter buffer) as a
    single [sum N_i, K] view; otherwise unchanged."""
    if len(mats) < 2:
        return mats
    K = mats[0].shape[1]
    nxt = mats[0].data_ptr()
    st = mats[0].untyped_storage().data_ptr()
    for m in mats:
        if (m.dim() != 2 or m.shape[1] != K or m.stride() != (K, 1) or m.data_ptr() != nxt
                or m.untyped_storage().data_ptr() != st):
            return mats
        nxt += m.numel() * m.element_size()
    m0 = mats[0]
    return [torch.as_strided(m0, (sum(m.shape[0] for m in mats), K), (K, 1))]


def _aligned(sizes, mult):
    st, _ = _starts(sizes)
    return all(s % mult == 0 for s in st)


def linear_fwd(x: torch.Tensor, weights: List[torch.Tensor], out: torch.Tensor, kind=L.EPI_STORE, bias=None,
               alpha=1.0, in0=None, out1=None, out2=None, row_stats=None, cap=0.0, rope=None, colscale=None):
    """out[M, sum N_i] = epi(x[M,K] @ cat(weights)^T).  Weights [N_i, K] are read in place."""
    M, K = x.shape
    sizes = [w.shape[0] for w in weights]
    for w in weights:
        _req(w.shape[1] == K, f"linear: weight K {w.shape[1]} != {K}")
    weights = _merge_rows(weights)
    sizes = [w.shape[0] for w in weights]
    if len(weights) > 1 and not _aligned(sizes, 128):
        weights = [torch.cat(weights, 0)]
        sizes = [weights[0].shape[0]]
    starts, N = _starts(sizes)
    A = _operand([x], L.LAYOUT_KC)
    B = _operand(weights, L.LAYOUT_KC, L.SEG_OUTER, starts)
    gemm(M, N, K, A, B, [out], [0], _ld(out),
         _epi(kind, alpha=alpha, bias=bias, in0=in0, out1=out1, out2=out2, row_stats=row_stats, cap=cap, rope=rope,
              colscale=colscale))


GEMV_NORM_MAX_K = 2560  # svla_gemv_rmsnorm2 holds a row of up to this many features in registers (gemm.hip)


def gemv_rmsnorm2(res, y, w1, w2, eps1, eps2, h_out, weights: List[torch.Tensor], out: torch.Tensor, geglu_out=None):
    """Decode step: h_out = bf16(res + rms(y; w1)), x = rms(h_out; w2) (svla_add_rmsnorm2_fwd, bitwise), then
    out = x @ cat(weights)^T (STORE), or with geglu_out = (g, u) and weights = [w_gate, w_up]: out = GeGLU of the
    gate|up projection (svla_gemv_rmsnorm2, M <= 8 rows)."""
    M, Kd = y.shape
    _req(Kd <= GEMV_NORM_MAX_K and Kd % 8 == 0, f"gemv_rmsnorm2: K {Kd} must be a multiple of 8 <= {GEMV_NORM_MAX_K}")
    for t, nm in ((res, "res"), (y, "y"), (h_out, "h_out"), (w1, "w1"), (w2, "w2"), (out, "out")):
        _chk_bf16(t, "gemv_rmsnorm2 " + nm)
    _req(res.shape == y.shape == h_out.shape and _ld(res) == _ld(y) == _ld(h_out), "gemv_rmsnorm2: res/y/h_out rows")
    if geglu_out is not None:
        I = weights[0].shape[0]
        B = _operand(weights, L.LAYOUT_KC, L.SEG_GEGLU, [0, I])
        N = 2 * I
        e = _epi(L.EPI_GEGLU, out1=geglu_out[0], out2=geglu_out[1])
    else:
        weights = _merge_rows(weights)
        starts, N = _starts([w.shape[0] for w in weights])
        B = _operand(weights, L.LAYOUT_KC, L.SEG_OUTER, starts)
        e = _epi(L.EPI_STORE)
    L.check(L.lib().svla_gemv_rmsnorm2(M, N, Kd, res.data_ptr(), y.data_ptr(), _ld(y), w1.data_ptr(), w2.data_ptr(),
                                       float(eps1), float(eps2), h_out.data_ptr(), ctypes.byref(B), out.data_ptr(),
                                       _ld(out), ctypes.byref(e), _stream()), "svla_gemv_rmsnorm2")


# svla_decode_mlp grid-barrier words: zeroed once per (device, stream) and never freed (captured decode graphs keep
# the raw pointer; the counter is back at zero after every launch)
_DECODE_MLP_SYNC = {}


def decode_mlp_timeouts() -> int:
    """Grid-barrier waits of svla_decode_mlp that hit their bound (word 32 of each stream's sync buffer): 0 unless a
    launch's blocks could not all be resident at once (such a block writes NaN instead of its numbers)."""
    return sum(int(t.view(torch.int32)[32].item()) for t in _DECODE_MLP_SYNC.values())


_DECODE_MLP_TIMEOUTS_SEEN = [0]


def check_decode_mlp_timeouts(what: str = "decode"):
    """Raise RuntimeError if a persistent decode-MLP launch missed a grid barrier since the last check (one small
    device read per sync buffer; predict_action / generate call it once, after their last step)."""
    if not _DECODE_MLP_SYNC:
        return
    n = decode_mlp_timeouts()
    if n != _DECODE_MLP_TIMEOUTS_SEEN[0]:
        new = n - _DECODE_MLP_TIMEOUTS_SEEN[0]
        _DECODE_MLP_TIMEOUTS_SEEN[0] = n
        raise RuntimeError(f"{what}: {new} block(s) of the persistent decode MLP (svla_decode_mlp) missed a grid "
                           "barrier (its grid was not co-resident); their outputs are NaN and the tokens are invalid. "
                           "Set SVLA_DECODE_MLP_PERSIST=0 for the two-launch path.")


def gemm_cu_cap(cap: int):
    """svla_gemm_set_cu_cap: cap the persistent stream-K grid of this thread's next GEMM launches (0 = off)."""
    L.lib().svla_gemm_set_cu_cap(max(0, int(cap)))


_DECODE_MLP_GRID = {}


def decode_mlp_grid(M: int, H: int, I: int) -> int:
    """Blocks svla_decode_mlp would launch (occupancy-capped), 0 if it can not run: the two-launch path then."""
    key = (torch.cuda.current_device(), M, H, I)
    g = _DECODE_MLP_GRID.get(key)
    if g is None:
        g = _DECODE_MLP_GRID[key] = int(L.lib().svla_decode_mlp_grid(M, H, I))
    return g


def decode_mlp(res, y, w1, w2, eps1, eps2, h_out, wg, wu, wd, act, out, o=None):
    """Decode-step Gemma2 MLP in one persistent launch (svla_decode_mlp): h_out = bf16(res + rms(y; w1)),
    act = GeGLU(rms(h_out; w2) @ [wg; wu]^T), out = act @ wd^T -- bitwise gemv_rmsnorm2 (GEGLU) + the down GEMV.
    o = (attn, wo): the o projection first, in the same launch (y = attn @ wo^T is then written, bitwise the GEMV)."""
    M, H = y.shape
    I = wg.shape[0]
    _req(M <= 8 and H % 8 == 0 and I % 8 == 0 and H <= 2560 and I <= 10240,
         "decode_mlp: M <= 8, H <= 2560, I <= 10240, multiples of 8")
    for t, nm in ((res, "res"), (y, "y"), (h_out, "h_out"), (w1, "w1"), (w2, "w2"), (wg, "wg"), (wu, "wu"),
                  (wd, "wd"), (act, "act"), (out, "out")):
        _chk_bf16(t, "decode_mlp " + nm)
    _req(res.shape == y.shape == h_out.shape and _ld(res) == _ld(y) == _ld(h_out), "decode_mlp: res/y/h_out rows")
    _req(wg.shape == wu.shape == (I, H) and _ld(wg) == _ld(wu) and wd.shape == (H, I), "decode_mlp: weight shapes")
    _req(act.shape[0] >= M and act.shape[1] >= I and out.shape[0] >= M and out.shape[1] >= H, "decode_mlp: outputs")
    attn, wo = o if o is not None else (None, None)
    if attn is not None:
        _chk_bf16(attn, "decode_mlp attn")
        _chk_bf16(wo, "decode_mlp wo")
        _req(attn.shape[0] == M and wo.shape == (H, attn.shape[1]) and attn.shape[1] % 8 == 0 and
             attn.shape[1] <= 2048 and attn.stride(1) == 1 and wo.stride(1) == 1, "decode_mlp: o projection shapes")
    key = (y.device.index, _stream())
    sync = _DECODE_MLP_SYNC.get(key)
    if sync is None:
        sync = _DECODE_MLP_SYNC[key] = torch.zeros(max(16, int(L.lib().svla_decode_mlp_sync_bytes())),
                                                   dtype=torch.uint8, device=y.device)
    L.check(L.lib().svla_decode_mlp(M, H, I, res.data_ptr(), y.data_ptr(), _ld(y), w1.data_ptr(), w2.data_ptr(),
                                    float(eps1), float(eps2), h_out.data_ptr(), wg.data_ptr(), wu.data_ptr(), _ld(wg),
                                    wd.data_ptr(), _ld(wd), act.data_ptr(), _ld(act), out.data_ptr(), _ld(out),
                                    _ptr(attn), _ld(attn) if attn is not None else 0,
                                    attn.shape[1] if attn is not None else 0, _ptr(wo),
                                    _ld(wo) if wo is not None else 0, sync.data_ptr(), _stream()), "svla_decode_mlp")


# Optional live launch timing (bench.py's roofline): launch_timer["geglu"] = [] makes every GeGLU GEMM launch
# record a pair of HIP events on the stream it is launched on (the current torch stream).
launch_timer: dict = {}


def linear_geglu_fwd(x: torch.Tensor, w_gate: torch.Tensor, w_up: torch.Tensor, h: torch.Tensor, g: torch.Tensor,
                     u: torch.Tensor):
    """h = gelu_tanh(x Wg^T) * (x Wu^T); g, u saved (Gemma2MLP, modeling_gemma2.py:91-92)."""
    M, K = x.shape
    I = w_gate.shape[0]
    _req(I % 64 == 0 and w_up.shape[0] == I, "geglu: intermediate size must be a multiple of 64")
    A = _operand([x], L.LAYOUT_KC)
    B = _operand([w_gate, w_up], L.LAYOUT_KC, L.SEG_GEGLU, [0, I])
    rec = launch_timer.get("geglu")
    if rec is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
    gemm(M, 2 * I, K, A, B, [h], [0], _ld(h), _epi(L.EPI_GEGLU, out1=g, out2=u))
    if rec is not None:
        e1.record(torch.cuda.current_stream())
        rec.append((e0, e1, M, 2 * I, K))


def linear_dgrad(dy: torch.Tensor, weights: List[torch.Tensor], out: torch.Tensor, kind=L.EPI_STORE, in0=None,
                 in1=None, out1=None, out2=None, accumulate=False):
    """out[M, K] = epi(dy[M, N] @ cat(weights)[N, K])."""
    M, N = dy.shape
    K = weights[0].shape[1]
    sizes = [w.shape[0] for w in weights]
    _req(sum(sizes) == N, "dgrad: weight rows must sum to dy columns")
    weights = _merge_rows(weights)
    sizes = [w.shape[0] for w in weights]
    if len(weights) > 1 and not _aligned(sizes, 64):
        weights = [torch.cat(weights, 0)]
        sizes = [N]
    starts, _ = _starts(sizes)
    A = _operand([dy], L.LAYOUT_KC)
    B = _operand(weights, L.LAYOUT_RC, L.SEG_K, starts)
    gemm(M, K, N, A, B, [out], [0], _ld(out), _epi(kind, accumulate=accumulate, in0=in0, in1=in1, out1=out1,
                                                   out2=out2))


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, outs: List[torch.Tensor], accumulate=False):
    """outs_i[N_i, K] = dy[:, seg_i]^T @ x  (weight gradients, written in place)."""
    M, N = dy.shape
    K = x.shape[1]
    sizes = [o.shape[0] for o in outs]
    _req(sum(sizes) == N, "wgrad: out rows must sum to dy columns")
    for o in outs:
        _req(o.shape[1] == K and o.is_contiguous(), "wgrad: outputs must be contiguous [N_i, K]")
    outs = _merge_rows(outs)
    sizes = [o.shape[0] for o in outs]
    if len(outs) > 1 and not _aligned(sizes, 128):
        tmp = torch.empty(N, K, dtype=BF16, device=dy.device)
        linear_wgrad(dy, x, [tmp], accumulate=False)
        off = 0
        for o in outs:
            seg = tmp[off:off + o.shape[0]]
            if accumulate:
                o.add_(seg)
            else:
                o.copy_(seg)
            off += o.shape[0]
        return
    starts, _ = _starts(sizes)
    A = _operand([dy], L.LAYOUT_RC)
    B = _operand([x], L.LAYOUT_RC)
    gemm(N, K, M, A, B, outs, starts, K, _epi(L.EPI_STORE, accumulate=accumulate))


# ---------------------------------------------------------------------------------------- fp8 projections
FP8 = torch.float8_e4m3fn


def quant_fp8_rows(x: torch.Tensor, q: Optional[torch.Tensor] = None, scale: Optional[torch.Tensor] = None,
                   colscale: Optional[torch.Tensor] = None):
    """Row-wise OCP e4m3 quantisation (svla_quant_fp8_rows) of x * colscale (colscale fp32 [K] or None):
    q = e4m3(clamp(x' * 448/amax_row)), scale = amax_row/448.  Returns (q [rows, K] float8_e4m3fn, scale [rows])."""
    _chk_bf16(x, "quant_fp8_rows")
    rows, K = x.shape
    if q is None:
        q = torch.empty(rows, K, dtype=FP8, device=x.device)
    if scale is None:
        scale = torch.empty(rows, dtype=torch.float32, device=x.device)
    _req(q.dtype == FP8 and q.shape == (rows, K) and q.stride(1) == 1, "quant_fp8_rows: q must be [rows, K] e4m3")
    _req(scale.dtype == torch.float32 and scale.numel() >= rows and scale.is_contiguous(), "quant_fp8_rows: scale")
    if colscale is not None:
        _req(colscale.dtype == torch.float32 and colscale.is_contiguous() and colscale.numel() >= K,
             "quant_fp8_rows: colscale must be a contiguous fp32 [K]")
    L.check(L.lib().svla_quant_fp8_rows(rows, K, x.data_ptr(), _ld(x), _ptr(colscale), q.data_ptr(), q.stride(0),
                                        scale.data_ptr(), _stream()), "svla_quant_fp8_rows")
    return q, scale


class MXScales:
    """E8M0 block scales of an MX-quantised [rows, K] matrix in svla_quant_mx_rows' tile-major layout: a uint8 buffer
    of K/128 k-tiles, each `ld` bytes (4 per row, rows padded to a multiple of 256 so every 256-row tile's scale rows
    are in the buffer)."""

    def __init__(self, rows: int, K: int, device, buf: Optional[torch.Tensor] = None):
        self.rows, self.K = rows, K
        self.ld = 4 * ((rows + 255) // 256 * 256)
        n = (K // 128) * self.ld
        self.buf = buf if buf is not None else torch.empty(n, dtype=torch.uint8, device=device)
        _req(self.buf.dtype == torch.uint8 and self.buf.numel() >= n and self.buf.is_contiguous(), "MXScales: buffer")

    def exponents(self) -> torch.Tensor:
        """[rows, K/32] int32 exponents X (scale = 2^X): the layout undone, for tests."""
        t = self.buf[:(self.K // 128) * self.ld].view(self.K // 128, self.ld // 4, 4)[:, :self.rows]
        return (t.permute(1, 0, 2).reshape(self.rows, self.K // 32).to(torch.int32) - 127)


def quant_mx_rows(x: torch.Tensor, q: Optional[torch.Tensor] = None, sc: Optional[MXScales] = None):
    """OCP MX e4m3 quantisation of rows (svla_quant_mx_rows): one E8M0 scale 2^X per 32 consecutive k, X =
    clamp(floor(log2(amax)) - 8, -127, 127), q = e4m3(clamp(x * 2^-X, +-448)).  Returns (q [rows, K] e4m3,
    MXScales)."""
    _chk_bf16(x, "quant_mx_rows")
    rows, K = x.shape
    _req(K % 128 == 0, f"quant_mx_rows: K={K} must be a multiple of 128")
    if q is None:
        q = torch.empty(rows, K, dtype=FP8, device=x.device)
    if sc is None:
        sc = MXScales(rows, K, x.device)
    _req(q.dtype == FP8 and q.shape == (rows, K) and q.stride(1) == 1, "quant_mx_rows: q must be [rows, K] e4m3")
    _req(sc.rows >= rows and sc.K == K, "quant_mx_rows: scale buffer shape")
    L.check(L.lib().svla_quant_mx_rows(rows, K, x.data_ptr(), _ld(x), q.data_ptr(), q.stride(0), sc.buf.data_ptr(),
                                       sc.ld, _stream()), "svla_quant_mx_rows")
    return q, sc


def quant_mx_cols(w: torch.Tensor):
    """quant_mx_rows(w.t()) without the bf16 transpose (svla_quant_mx_cols): w [N, K] bf16 -> (q [K, N] e4m3 with MX
    blocks of 32 consecutive n, MXScales of a [K]-row matrix) -- the dgrad operand W^T of the fp8 projections."""
    _chk_bf16(w, "quant_mx_cols")
    N, Kd = w.shape
    _req(N % 128 == 0 and Kd % 64 == 0, f"quant_mx_cols: [{N}, {Kd}] needs N % 128 == 0 and K % 64 == 0")
    q = torch.empty(Kd, N, dtype=FP8, device=w.device)
    sc = MXScales(Kd, N, w.device)
    L.check(L.lib().svla_quant_mx_cols(N, Kd, w.data_ptr(), _ld(w), q.data_ptr(), q.stride(0), sc.buf.data_ptr(),
                                       sc.ld, _stream()), "svla_quant_mx_cols")
    return q, sc


def quant_mx_both(w: torch.Tensor):
    """(quant_mx_rows(w), quant_mx_cols(w)) from one read of w (svla_quant_mx_both; R, C multiples of 128):
    ((q [R, C], MXScales), (qt [C, R], MXScales))."""
    _chk_bf16(w, "quant_mx_both")
    R, C = w.shape
    _req(R % 128 == 0 and C % 128 == 0, f"quant_mx_both: [{R}, {C}] needs multiples of 128")
    q = torch.empty(R, C, dtype=FP8, device=w.device)
    sc = MXScales(R, C, w.device)
    qt = torch.empty(C, R, dtype=FP8, device=w.device)
    sct = MXScales(C, R, w.device)
    L.check(L.lib().svla_quant_mx_both(R, C, w.data_ptr(), _ld(w), q.data_ptr(), q.stride(0), sc.buf.data_ptr(), sc.ld,
                                       qt.data_ptr(), qt.stride(0), sct.buf.data_ptr(), sct.ld, _stream()),
            "svla_quant_mx_both")
    return (q, sc), (qt, sct)


def gemm_mxfp8(xq: torch.Tensor, xs: MXScales, wq: torch.Tensor, ws: MXScales, out: torch.Tensor,
               kind=L.EPI_STORE, geglu_I: int = 0, **epi_kw):
    """out = epi(sum_k 2^(Xa + Xb) xq wq^T) on the MX fp8 MFMA kernel (svla_gemm_mxfp8); wq and ws as gemm_fp8's
    (geglu_I > 0: gate rows then up rows of one matrix, one scale matrix)."""
    M, K = xq.shape
    N = wq.shape[0]
    _req(wq.shape[1] == K and xs.K == K and ws.K == K, f"gemm_mxfp8: K mismatch ({K}, {wq.shape[1]}, {xs.K}, {ws.K})")
    _req(xs.rows >= M and ws.rows >= N, "gemm_mxfp8: scale rows")
    A = _operand_fp8([xq])
    if geglu_I:
        B = _operand_fp8([wq[:geglu_I], wq[geglu_I:]], L.SEG_GEGLU, [0, geglu_I])
    else:
        B = _operand_fp8([wq])
    cp = (ctypes.c_void_p * 4)(out.data_ptr(), None, None, None)
    cs = (ctypes.c_int64 * 5)(0, 0, 0, 0, 0)
    wsp = gemm_workspace()
    e = _epi(kind, **epi_kw)
    rec = launch_timer.get("geglu_fp8") if geglu_I else None
    if rec is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
    L.check(L.lib().svla_gemm_mxfp8(M, N, K, ctypes.byref(A), xs.buf.data_ptr(), xs.ld, xs.buf.numel(),
                                    ctypes.byref(B), ws.buf.data_ptr(), ws.ld, ws.buf.numel(), cp, cs, 1, _ld(out),
                                    ctypes.byref(e), wsp.data_ptr(), wsp.numel(), _stream()), "svla_gemm_mxfp8")
    if rec is not None:
        e1.record(torch.cuda.current_stream())
        rec.append((e0, e1, M, N, K))


def transpose_u8(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[c, r] = x[r, c] for a 1-byte-element matrix (e4m3 weight copies), svla_transpose_u8."""
    _req(x.is_cuda and x.element_size() == 1 and x.dim() == 2 and x.stride(1) == 1, "transpose_u8: 1-byte matrix")
    R, C = x.shape
    if out is None:
        out = torch.empty(C, R, dtype=x.dtype, device=x.device)
    _req(out.shape == (C, R) and out.stride(1) == 1 and out.element_size() == 1, "transpose_u8: out must be [C, R]")
    L.check(L.lib().svla_transpose_u8(R, C, x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0), _stream()),
            "svla_transpose_u8")
    return out


def _operand_fp8(mats: Sequence[torch.Tensor], seg_dim: int = L.SEG_OUTER, starts=None) -> L.Operand:
    op = L.Operand()
    ld = mats[0].stride(0)
    for i, m in enumerate(mats):
        _req(m.is_cuda and m.dtype == FP8 and m.dim() == 2 and m.stride(1) == 1 and m.stride(0) == ld,
             "gemm_fp8: operands are row-major e4m3 matrices with one leading dimension")
        op.ptr[i] = m.data_ptr()
    op.nseg, op.seg_dim, op.layout, op.ld = len(mats), seg_dim, L.LAYOUT_KC, ld
    if starts is not None:
        for i, s in enumerate(starts):
            op.seg_start[i] = int(s)
    return op


def gemm_fp8(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor, out: torch.Tensor,
             kind=L.EPI_STORE, geglu_I: int = 0, **epi_kw):
    """out = epi(xs[m] * ws[n] * (xq @ wq^T)) on the fp8 MFMA kernel (svla_gemm_fp8).  geglu_I > 0: wq holds the
    gate rows [0, I) then the up rows [I, 2I), kind EPI_GEGLU, epi_kw out1=g, out2=u."""
    M, K = xq.shape
    N = wq.shape[0]
    _req(wq.shape[1] == K, f"gemm_fp8: weight K {wq.shape[1]} != {K}")
    _req(xs.numel() >= M and ws.numel() >= N and xs.dtype == ws.dtype == torch.float32, "gemm_fp8: scales")
    A = _operand_fp8([xq])
    if geglu_I:
        B = _operand_fp8([wq[:geglu_I], wq[geglu_I:]], L.SEG_GEGLU, [0, geglu_I])
    else:
        B = _operand_fp8([wq])
    cp = (ctypes.c_void_p * 4)(out.data_ptr(), None, None, None)
    cs = (ctypes.c_int64 * 5)(0, 0, 0, 0, 0)
    wsp = gemm_workspace()
    e = _epi(kind, **epi_kw)
    rec = launch_timer.get("geglu_fp8") if geglu_I else None
    if rec is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
    L.check(L.lib().svla_gemm_fp8(M, N, K, ctypes.byref(A), xs.data_ptr(), ctypes.byref(B), ws.data_ptr(), cp, cs, 1,
                                  _ld(out), ctypes.byref(e), wsp.data_ptr(), wsp.numel(), _stream()), "svla_gemm_fp8")
    if rec is not None:
        e1.record(torch.cuda.current_stream())
        rec.append((e0, e1, M, N, K))


# ---------------------------------------------------------------------------------------- norms
def rmsnorm_fwd(x, w, eps, y, rstd):
    rows, N = x.shape
    L.check(L.lib().svla_rmsnorm_fwd(rows, N, x.data_ptr(), w.data_ptr(), eps, y.data_ptr(), rstd.data_ptr(),
                                     _stream()), "rmsnorm_fwd")


def rmsnorm_fwd_mx(x, w, eps, y, rstd):
    """rmsnorm_fwd that also returns the MX e4m3 copy of y (svla_rmsnorm_fwd_mx): (q, MXScales)."""
    rows, N = x.shape
    _req(N % 128 == 0 and x.is_contiguous() and y.is_contiguous(), "rmsnorm_fwd_mx: N % 128 == 0, contiguous rows")
    q = torch.empty(rows, N, dtype=FP8, device=x.device)
    sc = MXScales(rows, N, x.device)
    L.check(L.lib().svla_rmsnorm_fwd_mx(rows, N, x.data_ptr(), w.data_ptr(), eps, y.data_ptr(), rstd.data_ptr(),
                                        q.data_ptr(), q.stride(0), sc.buf.data_ptr(), sc.ld, _stream()),
            "rmsnorm_fwd_mx")
    return q, sc


def add_rmsnorm_fwd(res, yin, w, eps, h, rstd):
    rows, N = yin.shape
    L.check(L.lib().svla_add_rmsnorm_fwd(rows, N, res.data_ptr(), yin.data_ptr(), w.data_ptr(), eps, h.data_ptr(),
                                         rstd.data_ptr(), _stream()), "add_rmsnorm_fwd")


def add_rmsnorm2_fwd_train(res, yin, w1, w2, eps1, eps2, h, x, rstd1, rstd2):
    """h = bf16(res + rms(yin; w1)), x = rms(h; w2) and both rows' rstd (svla_add_rmsnorm2_fwd_train)."""
    rows, N = yin.shape
    for t, n in ((res, "res"), (yin, "yin"), (w1, "w1"), (w2, "w2"), (h, "h"), (x, "x")):
        _chk_bf16(t, n)
    _req(res.shape == yin.shape == h.shape == x.shape and res.is_contiguous() and yin.is_contiguous()
         and h.is_contiguous() and x.is_contiguous(), "add_rmsnorm2_train: shapes")
    _req(rstd1.numel() >= rows and rstd2.numel() >= rows and rstd1.dtype == rstd2.dtype == torch.float32,
         "add_rmsnorm2_train: rstd buffers")
    L.check(L.lib().svla_add_rmsnorm2_fwd_train(rows, N, res.data_ptr(), yin.data_ptr(), w1.data_ptr(), w2.data_ptr(),
                                                float(eps1), float(eps2), h.data_ptr(), x.data_ptr(),
                                                rstd1.data_ptr(), rstd2.data_ptr(), _stream()), "add_rmsnorm2_fwd_train")


def add_rmsnorm2_fwd_train_mx(res, yin, w1, w2, eps1, eps2, h, x, rstd1, rstd2):
    """add_rmsnorm2_fwd_train that also returns the MX e4m3 copy of x (svla_add_rmsnorm2_fwd_train_mx)."""
    rows, N = yin.shape
    for t, n in ((res, "res"), (yin, "yin"), (w1, "w1"), (w2, "w2"), (h, "h"), (x, "x")):
        _chk_bf16(t, n)
    _req(res.shape == yin.shape == h.shape == x.shape and res.is_contiguous() and yin.is_contiguous()
         and h.is_contiguous() and x.is_contiguous() and N % 128 == 0, "add_rmsnorm2_train_mx: shapes")
    q = torch.empty(rows, N, dtype=FP8, device=x.device)
    sc = MXScales(rows, N, x.device)
    L.check(L.lib().svla_add_rmsnorm2_fwd_train_mx(rows, N, res.data_ptr(), yin.data_ptr(), w1.data_ptr(),
                                                   w2.data_ptr(), float(eps1), float(eps2), h.data_ptr(), x.data_ptr(),
                                                   rstd1.data_ptr(), rstd2.data_ptr(), q.data_ptr(), q.stride(0),
                                                   sc.buf.data_ptr(), sc.ld, _stream()), "add_rmsnorm2_fwd_train_mx")
    return q, sc


RPB = 16  # rows per block of the norm backward kernels (norms.hip RPB): sizes the weight-gradient partial planes
RPB2 = 8  # the norm-pair backward's (norms.hip RPB2)


def add_rmsnorm2_fwd(res, yin, w1, w2, eps1, eps2, h, x):
    rows, N = yin.shape
    for t, n in ((res, "res"), (yin, "yin"), (w1, "w1"), (w2, "w2"), (h, "h"), (x, "x")):
        _chk_bf16(t, n)
    _req(res.shape == yin.shape == h.shape == x.shape and res.is_contiguous() and yin.is_contiguous(),
         "add_rmsnorm2: shapes")
    L.check(L.lib().svla_add_rmsnorm2_fwd(rows, N, res.data_ptr(), yin.data_ptr(), w1.data_ptr(), w2.data_ptr(),
                                          float(eps1), float(eps2), h.data_ptr(), x.data_ptr(), _stream()),
            "add_rmsnorm2_fwd")


def rmsnorm_bwd(x, w, rstd, dy, dres, dx, dw_out, dw_accumulate=False, mx=False):
    """RMSNorm backward (svla_rmsnorm_bwd); mx=True: svla_rmsnorm_bwd_mx, also returning the MX e4m3 copy of dx
    (q, MXScales) -- the fp8 dgrad operand -- from the same pass (N % 128 == 0, N > 1536)."""
    rows, N = x.shape
    nb = (rows + RPB - 1) // RPB
    part = torch.empty(nb, N, dtype=torch.float32, device=x.device)
    npart = ctypes.c_int64(0)
    out = None
    if mx:
        _req(N % 128 == 0 and N > 1536 and dx.is_contiguous(), "rmsnorm_bwd_mx: N % 128 == 0, N > 1536")
        q = torch.empty(rows, N, dtype=FP8, device=x.device)
        sc = MXScales(rows, N, x.device)
        L.check(L.lib().svla_rmsnorm_bwd_mx(rows, N, x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dy.data_ptr(),
                                            _ptr(dres), dx.data_ptr(), part.data_ptr(), ctypes.byref(npart),
                                            q.data_ptr(), q.stride(0), sc.buf.data_ptr(), sc.ld, _stream()),
                "rmsnorm_bwd_mx")
        out = (q, sc)
    else:
        L.check(L.lib().svla_rmsnorm_bwd(rows, N, x.data_ptr(), w.data_ptr(), rstd.data_ptr(), dy.data_ptr(),
                                         _ptr(dres), dx.data_ptr(), part.data_ptr(), ctypes.byref(npart), _stream()),
                "rmsnorm_bwd")
    if dw_out is not None:
        colsum_f32(part[:npart.value], dw_out, dw_accumulate)
    return out


def rmsnorm2_bwd(h, w2, rstd2, dx, dres, y, w1, rstd1, dh_out, dy_out, dw2, dw1, acc2=False, acc1=False, mx=False):
    """Backward of add_rmsnorm2_fwd_train in one pass (svla_rmsnorm2_bwd); weight gradients dw2 / dw1 (or None) by
    one column-sum launch over both partial planes (two when only one is wanted or the accumulate modes differ).
    mx=True: svla_rmsnorm2_bwd_mx, returning the MX e4m3 copy of dy_out (q, MXScales) from the same pass."""
    rows, N = h.shape
    for t, n in ((h, "h"), (dx, "dx"), (y, "y"), (dh_out, "dh_out"), (dy_out, "dy_out")):
        _req(t.shape == (rows, N) and t.is_contiguous(), f"rmsnorm2_bwd: {n} must be contiguous [{rows}, {N}]")
    _req(dres is None or (dres.shape == (rows, N) and dres.is_contiguous()), "rmsnorm2_bwd: dres")
    nb = (rows + RPB2 - 1) // RPB2
    part = torch.empty(2, nb, N, dtype=torch.float32, device=h.device)
    npart = ctypes.c_int64(0)
    out = None
    if mx:
        _req(N % 128 == 0, "rmsnorm2_bwd_mx: N % 128 == 0")
        q = torch.empty(rows, N, dtype=FP8, device=h.device)
        sc = MXScales(rows, N, h.device)
        L.check(L.lib().svla_rmsnorm2_bwd_mx(rows, N, h.data_ptr(), w2.data_ptr(), rstd2.data_ptr(), dx.data_ptr(),
                                             _ptr(dres), y.data_ptr(), w1.data_ptr(), rstd1.data_ptr(),
                                             dh_out.data_ptr(), dy_out.data_ptr(), part.data_ptr(), ctypes.byref(npart),
                                             q.data_ptr(), q.stride(0), sc.buf.data_ptr(), sc.ld, _stream()),
                "rmsnorm2_bwd_mx")
        out = (q, sc)
    else:
        L.check(L.lib().svla_rmsnorm2_bwd(rows, N, h.data_ptr(), w2.data_ptr(), rstd2.data_ptr(), dx.data_ptr(),
                                          _ptr(dres), y.data_ptr(), w1.data_ptr(), rstd1.data_ptr(), dh_out.data_ptr(),
                                          dy_out.data_ptr(), part.data_ptr(), ctypes.byref(npart), _stream()),
                "rmsnorm2_bwd")
    if dw2 is not None and dw1 is not None and acc2 == acc1:
        L.check(L.lib().svla_colsum2_f32(npart.value, N, part.data_ptr(), dw2.data_ptr(), dw1.data_ptr(), int(acc2),
                                         _stream()), "colsum2_f32")
    else:
        if dw2 is not None:
            colsum_f32(part[0], dw2, acc2)
        if dw1 is not None:
            colsum_f32(part[1], dw1, acc1)
    return out


def layernorm_fwd(x, w, b, eps, y, mean, rstd):
    rows, N = x.shape
    L.check(L.lib().svla_layernorm_fwd(rows, N, x.data_ptr(), w.data_ptr(), b.data_ptr(), eps, y.data_ptr(),
                                       mean.data_ptr(), rstd.data_ptr(), _stream()), "layernorm_fwd")


def layernorm_bwd(x, w, mean, rstd, dy, dres, dx, dw_out, db_out, accumulate=False):
    rows, N = x.shape
    nb = (rows + RPB - 1) // RPB
    part = torch.empty(2, nb, N, dtype=torch.float32, device=x.device)
    npart = ctypes.c_int64(0)
    L.check(L.lib().svla_layernorm_bwd(rows, N, x.data_ptr(), w.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                       dy.data_ptr(), _ptr(dres), dx.data_ptr(), part.data_ptr(), ctypes.byref(npart),
                                       _stream()), "layernorm_bwd")
    # partial planes [2][nb][N]: dw, then db -- both reduced by one launch when both are wanted
    if dw_out is not None and db_out is not None:
        L.check(L.lib().svla_colsum2_f32(npart.value, N, part.data_ptr(), dw_out.data_ptr(), db_out.data_ptr(),
                                         int(accumulate), _stream()), "colsum2_f32")
    elif dw_out is not None:
        colsum_f32(part[0], dw_out, accumulate)
    elif db_out is not None:
        colsum_f32(part[1], db_out, accumulate)


def colsum_f32(part, out, accumulate=False):
    """out[n] = bf16(sum_p part[p, n]) (+ out), one launch, fixed order."""
    P, N = part.shape
    _req(part.is_contiguous() and out.numel() == N, "colsum_f32: contiguous [P, N] partials, [N] output")
    L.check(L.lib().svla_colsum_f32(P, N, part.data_ptr(), out.data_ptr(), int(accumulate), None, _stream()),
            "colsum_f32")


def colsum_bf16(x, out, accumulate=False):
    """out[n] = bf16(sum_m x[m, n]) (+ out) over a row-strided bf16 matrix (bias gradients): row slices into an fp32
    workspace and their reduction where one block per 32 columns would leave the chip idle, else one launch."""
    M, N = x.shape
    _req(out.numel() == N and out.is_contiguous(), "colsum_bf16: [N] contiguous output")
    nb = int(L.lib().svla_colsum_bf16_workspace_bytes(M, N))
    ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device=x.device) if nb else None
    L.check(L.lib().svla_colsum_bf16(M, N, x.data_ptr(), _ld(x), out.data_ptr(), int(accumulate),
                                     ws.data_ptr() if ws is not None else None, _stream()), "colsum_bf16")


# ---------------------------------------------------------------------------------------- attention
def attn_args(B, Lq, Hq, Hkv, D, q, ldq, k, ldk, v, ldv, scale, softcap=0.0, kv_class=None, window=0,
              cos=None, sin=None, bias=None) -> L.AttnArgs:
    a = L.AttnArgs()
    a.B, a.L, a.Hq, a.Hkv, a.D = B, Lq, Hq, Hkv, D
    a.sliding_window = int(window)
    a.scale = float(scale)
    a.softcap = float(softcap or 0.0)
    a.q, a.ldq, a.k, a.ldk, a.v, a.ldv = q.data_ptr(), ldq, k.data_ptr(), ldk, v.data_ptr(), ldv
    a.kv_class = _ptr(kv_class)
    if cos is not None:
        a.rope_cos, a.rope_sin, a.rope_ld = cos.data_ptr(), sin.data_ptr(), cos.stride(0)
    if bias is not None:  # [Hq, L, ld] bf16, rows contiguous
        _req(bias.dim() == 3 and bias.stride(2) == 1 and bias.stride(0) == Lq * bias.stride(1),
             "attn bias must be [Hq, L, ld] with contiguous rows")
        a.bias, a.bias_ld = bias.data_ptr(), bias.stride(1)
    return a


def attn_fwd(a: L.AttnArgs, out: torch.Tensor, lse: torch.Tensor):
    L.check(L.lib().svla_attn_fwd(ctypes.byref(a), out.data_ptr(), _ld(out), lse.data_ptr(), _stream()), "attn_fwd")


def attn_decode(q, Lq, k_cache, v_cache, Lk, Hq, Hkv, D, scale, softcap, kv_class, window, out):
    """Lq new queries (rows b*Lq+t of q, rotated) against the first Lk rows of the [B, cap, Hkv*D] K/V cache."""
    B = k_cache.shape[0]
    _req(q.shape[0] == B * Lq and out.shape[0] == B * Lq, "attn_decode: q/out rows != B*Lq")
    _req(k_cache.shape[1] >= Lk and v_cache.shape[1] >= Lk, "attn_decode: cache shorter than Lk")
    _req(k_cache.stride(2) == 1 and v_cache.stride(2) == 1 and q.stride(1) == 1 and out.stride(1) == 1,
         "attn_decode: rows must be contiguous")
    _req(kv_class is None or (kv_class.dtype == torch.uint8 and kv_class.shape[0] == B and kv_class.stride(1) == 1),
         "attn_decode: kv_class must be uint8 [B, >=Lk]")
    for t, n in ((q, "q"), (k_cache, "k"), (v_cache, "v"), (out, "out")):
        _chk_bf16(t, n)
    a = L.AttnDecodeArgs()
    a.B, a.Lq, a.Lk, a.Hq, a.Hkv, a.D = B, Lq, Lk, Hq, Hkv, D
    a.sliding_window, a.scale, a.softcap = int(window or 0), float(scale), float(softcap or 0.0)
    a.q, a.ldq = q.data_ptr(), q.stride(0)
    a.k, a.ldk, a.bsk = k_cache.data_ptr(), k_cache.stride(1), k_cache.stride(0)
    a.v, a.ldv, a.bsv = v_cache.data_ptr(), v_cache.stride(1), v_cache.stride(0)
    a.kv_class = _ptr(kv_class)
    a.ldc = kv_class.stride(0) if kv_class is not None else 0
    nb = L.lib().svla_attn_decode_workspace_bytes(B, Lq, Hq, Lk, D)
    ws = torch.empty((nb + 3) // 4, dtype=torch.float32, device=q.device)
    L.check(L.lib().svla_attn_decode(ctypes.byref(a), out.data_ptr(), out.stride(0), ws.data_ptr(), nb, _stream()),
            "attn_decode")


# svla_attn_decode_rope workspaces: zeroed once, one per (device, stream) -- the arrival counters at their head
# return to zero after every launch, so a buffer is reused by every later call (and by captured graph replays)
_DECODE_WS = {}
# every workspace ever handed out stays allocated: a graph captured against a smaller one keeps its raw pointer
# (and its zeroed arrival counters), so a replacement must never return the old buffer to the caching allocator
_DECODE_WS_RETIRED = []


def _decode_rope_ws(nbytes, device):
    key = (device.index, _stream())
    ws = _DECODE_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        if ws is not None:
            _DECODE_WS_RETIRED.append(ws)
        ws = torch.zeros(max(nbytes, 8 << 20), dtype=torch.uint8, device=device)
        _DECODE_WS[key] = ws
    return ws


def attn_decode_rope(qkv, Lq, cos, sin, k_cache, v_cache, Lk, Hq, Hkv, D, scale, softcap, kv_class, window, out):
    """The decode step's attention in one launch: q|k|v projection rows (b*Lq+t, unrotated) -> RoPE (table row t),
    rotated k / v appended to cache rows Lk-Lq.., attention of the Lq new queries over the first Lk cache rows."""
    B = k_cache.shape[0]
    _req(qkv.shape[0] == B * Lq and out.shape[0] == B * Lq and qkv.stride(1) == 1 and out.stride(1) == 1,
         "attn_decode_rope: qkv/out rows != B*Lq or not contiguous")
    _req(qkv.shape[1] >= (Hq + 2 * Hkv) * D, "attn_decode_rope: qkv narrower than q|k|v")
    _req(k_cache.shape[1] >= Lk and v_cache.shape[1] >= Lk and Lk > Lq, "attn_decode_rope: cache / Lk")
    _req(k_cache.stride(2) == 1 and v_cache.stride(2) == 1, "attn_decode_rope: cache rows must be contiguous")
    _req(cos.shape[0] >= B * Lq and cos.shape == sin.shape and cos.stride(1) == 1 and cos.stride(0) == sin.stride(0),
         "attn_decode_rope: tables must hold one row per token row b*Lq+t")
    _req(kv_class is None or (kv_class.dtype == torch.uint8 and kv_class.shape[0] == B and kv_class.stride(1) == 1),
         "attn_decode_rope: kv_class must be uint8 [B, >=Lk]")
    for t, n in ((qkv, "qkv"), (k_cache, "k"), (v_cache, "v"), (out, "out"), (cos, "cos"), (sin, "sin")):
        _chk_bf16(t, n)
    a = L.AttnDecodeArgs()
    a.B, a.Lq, a.Lk, a.Hq, a.Hkv, a.D = B, Lq, Lk, Hq, Hkv, D
    a.sliding_window, a.scale, a.softcap = int(window or 0), float(scale), float(softcap or 0.0)
    a.q, a.ldq = qkv.data_ptr(), qkv.stride(0)
    a.k, a.ldk, a.bsk = k_cache.data_ptr(), k_cache.stride(1), k_cache.stride(0)
    a.v, a.ldv, a.bsv = v_cache.data_ptr(), v_cache.stride(1), v_cache.stride(0)
    a.kv_class = _ptr(kv_class)
    a.ldc = kv_class.stride(0) if kv_class is not None else 0
    nb = L.lib().svla_attn_decode_rope_workspace_bytes(B, Lq, Hq, Hkv, Lk, D)
    ws = _decode_rope_ws(nb, qkv.device)
    L.check(L.lib().svla_attn_decode_rope(ctypes.byref(a), cos.data_ptr(), sin.data_ptr(), cos.stride(0),
                                          out.data_ptr(), out.stride(0), ws.data_ptr(), ws.numel(), _stream()),
            "attn_decode_rope")


def qkv_rope_append(qkv, B, Lq, Hq, Hkv, D, cos, sin, k_cache, v_cache, p0, k_back=False):
    """RoPE q in place, rotated k and v into cache rows p0.. (the decode step's q|k|v epilogue); k_back: k rotated in
    place as well (svla_qkv_rope_fill, the prefill: its flash attention reads q and k from the projection rows)."""
    _req(qkv.shape[0] == B * Lq and qkv.stride(1) == 1, "qkv_rope_append: qkv rows")
    _req(cos.shape[0] >= B * Lq and cos.shape == sin.shape and cos.stride(1) == 1,
         "qkv_rope_append: tables must hold one row per token row b*Lq+t")
    _req(k_cache.shape[1] >= p0 + Lq and v_cache.shape[1] >= p0 + Lq, "qkv_rope_append: cache too short")
    for t, n in ((qkv, "qkv"), (cos, "cos"), (sin, "sin"), (k_cache, "k_cache"), (v_cache, "v_cache")):
        _chk_bf16(t, n)
    fn = L.lib().svla_qkv_rope_fill if k_back else L.lib().svla_qkv_rope_append
    L.check(fn(B, Lq, Hq, Hkv, D, qkv.data_ptr(), qkv.stride(0), cos.data_ptr(), sin.data_ptr(), cos.stride(0),
               k_cache.data_ptr(), k_cache.stride(1), k_cache.stride(0), v_cache.data_ptr(), v_cache.stride(1),
               v_cache.stride(0), int(p0), _stream()), "qkv_rope_append")


# head_dim-256 backward with dS stored by the dK/dV kernel and dQ = dS K (svla_attn_bwd_ds) instead of the dQ kernel
# that recomputes S, P and dP (svla_attn_bwd); SVLA_ATTN_DS=0 selects the latter
ATTN_DS = [os.environ.get("SVLA_ATTN_DS", "1") != "0"]
# The stored-dS workspace is bf16 B*Hq*round64(L)^2 (52 MB at the 4B training shape, B=32, L=312) and grows with L^2
# (2 GiB per call at B=8, L=4096); above this cap the recomputing path (B*Hq*L fp32 of workspace) runs instead.
ATTN_DS_MAX_BYTES = int(os.environ.get("SVLA_ATTN_DS_MAX_MB", "512")) << 20


def attn_bwd(a: L.AttnArgs, out, dout, lse, dq, lddq, dk, lddk, dv, lddv):
    n = int(L.lib().svla_attn_bwd_ds_workspace_bytes(a.B, a.L, a.Hq)) if a.D == 256 and ATTN_DS[0] else 0
    if 0 < n <= ATTN_DS_MAX_BYTES:
        buf = torch.empty(n + 256, dtype=torch.uint8, device=out.device)
        off = (-buf.data_ptr()) % 256
        L.check(L.lib().svla_attn_bwd_ds(ctypes.byref(a), out.data_ptr(), _ld(out), dout.data_ptr(), _ld(dout),
                                         lse.data_ptr(), dq.data_ptr(), lddq, dk.data_ptr(), lddk, dv.data_ptr(), lddv,
                                         buf.data_ptr() + off, n, _stream()), "attn_bwd_ds")
        return
    ws = torch.empty(a.B * a.Hq * a.L, dtype=torch.float32, device=out.device)
    L.check(L.lib().svla_attn_bwd(ctypes.byref(a), out.data_ptr(), _ld(out), dout.data_ptr(), _ld(dout),
                                  lse.data_ptr(), dq.data_ptr(), lddq, dk.data_ptr(), lddk, dv.data_ptr(), lddv,
                                  ws.data_ptr(), _stream()), "attn_bwd")


# ---------------------------------------------------------------------------------------- glue
def embed_merge(ids, img_index, embed, spatial, a0, na, img, normalizer, out):
    rows = ids.numel()
    H = embed.shape[1]
    L.check(L.lib().svla_embed_merge(rows, H, ids.data_ptr(), _ptr(img_index), embed.data_ptr(), _ptr(spatial),
                                     a0, na, _ptr(img), normalizer, out.data_ptr(), _stream()), "embed_merge")


def embed_merge_bwd(ids, img_index, sorted_rows, offsets, na, dout, normalizer, dspatial, dimg):
    rows, H = dout.shape
    L.check(L.lib().svla_embed_merge_bwd(rows, H, ids.data_ptr(), _ptr(img_index), _ptr(sorted_rows),
                                         _ptr(offsets), na, dout.data_ptr(), normalizer, _ptr(dspatial), _ptr(dimg),
                                         _stream()), "embed_merge_bwd")


def ego3d_encode(depth, kinv, uv_h, patch, reso, n_freqs, feat, xyz_out=None):
    B, _, Hd, Wd = depth.shape
    _req(kinv.numel() == B * 9 and kinv.dtype == torch.float32 and kinv.is_contiguous(),
         f"ego3d_encode: inv(K) must be [{B}, 3, 3] fp32 (one per depth map), got {tuple(kinv.shape)}")
    _req(feat.shape[0] >= B * (Hd // patch) * (Wd // patch), "ego3d_encode: feat has fewer rows than B * patches")
    _req(xyz_out is None or xyz_out.numel() >= B * (Hd // patch) * (Wd // patch) * 3 * reso * reso,
         "ego3d_encode: xyz_out too small")
    L.check(L.lib().svla_ego3d_encode(B, Hd, Wd, depth.data_ptr(), kinv.data_ptr(), uv_h.data_ptr(), patch, reso,
                                      n_freqs, feat.data_ptr(), _ld(feat), _ptr(xyz_out), _stream()), "ego3d_encode")


def inv3x3(K: torch.Tensor) -> torch.Tensor:
    """inv(K) for [B, 3, 3] intrinsics (closed form, fp32, svla_inv3x3_f32)."""
    Kf = K.float().contiguous()
    _req(Kf.shape[-2:] == (3, 3) and Kf.is_cuda, "inv3x3: [B, 3, 3] CUDA tensor")
    out = torch.empty_like(Kf)
    L.check(L.lib().svla_inv3x3_f32(Kf.numel() // 9, Kf.data_ptr(), out.data_ptr(), _stream()), "inv3x3")
    return out


def im2col_patch(x, patch, cols):
    B, _, S, _ = x.shape
    L.check(L.lib().svla_im2col_patch(B, S, patch, x.data_ptr(), cols.data_ptr(), _ld(cols), _stream()),
            "im2col_patch")


def affine(x, scale, offset, out):
    L.check(L.lib().svla_affine_bf16(x.numel(), x.data_ptr(), scale, offset, out.data_ptr(), _stream()), "affine")


def relu_fwd(x, y):
    L.check(L.lib().svla_relu_fwd(x.numel(), x.data_ptr(), y.data_ptr(), _stream()), "relu_fwd")


def relu_bwd(x, dy, dx):
    L.check(L.lib().svla_relu_bwd(x.numel(), x.data_ptr(), dy.data_ptr(), dx.data_ptr(), _stream()), "relu_bwd")


def add(a, b, out):
    L.check(L.lib().svla_add_bf16(a.numel(), a.data_ptr(), b.data_ptr(), out.data_ptr(), _stream()), "add")


GELU_TANH, GELU_ERF, GELU_TANH_BWD = 0, 1, 2


def gelu_rows(mode: int, x: torch.Tensor, y: torch.Tensor, pre: Optional[torch.Tensor] = None):
    """y = gelu_tanh(x) / gelu_erf(x) / x * gelu_tanh'(pre) over [M, N] bf16 rows (svla_gelu_rows)."""
    _chk_bf16(x, "gelu_rows x")
    _chk_bf16(y, "gelu_rows y")
    M, N = x.shape
    _req(y.shape == x.shape and (pre is None or pre.shape == x.shape), "gelu_rows: shapes")
    L.check(L.lib().svla_gelu_rows(M, N, int(mode), x.data_ptr(), _ld(x), _ptr(pre), _ld(pre) if pre is not None else 0,
                                   y.data_ptr(), _ld(y), _stream()), "svla_gelu_rows")


def softcap_ce_rows(logits: torch.Tensor, N: int, row_stats: torch.Tensor, cap: float):
    """In place: logits[:, :N] = softcap(logits) and row_stats [M, ceil(N/128), 3] (svla_softcap_ce_rows)."""
    _chk_bf16(logits, "softcap_ce_rows")
    M, ld = logits.shape[0], _ld(logits)
    _req(row_stats.dtype == torch.float32 and row_stats.is_contiguous() and row_stats.numel() >= M * ceil_div(N, 128) * 3,
         "softcap_ce_rows: row_stats must be a contiguous fp32 [M, ceil(N/128), 3]")
    L.check(L.lib().svla_softcap_ce_rows(M, N, logits.data_ptr(), ld, float(cap), row_stats.data_ptr(), _stream()),
            "svla_softcap_ce_rows")


def ce_finalize(N, ntiles, row_stats, logits, target, lse, argmax, loss_rows, loss_out):
    M = logits.shape[0]
    L.check(L.lib().svla_ce_finalize(M, N, ntiles, row_stats.data_ptr(), logits.data_ptr(), _ld(logits),
                                     _ptr(target), lse.data_ptr(), argmax.data_ptr(), loss_rows.data_ptr(),
                                     loss_out.data_ptr(), _stream()), "ce_finalize")


def ce_bwd(N, logits, lse, target, cap, grad_scale, dlogits):
    M = logits.shape[0]
    L.check(L.lib().svla_ce_bwd(M, N, logits.data_ptr(), _ld(logits), lse.data_ptr(), target.data_ptr(), cap,
                                grad_scale.data_ptr(), dlogits.data_ptr(), _ld(dlogits), _stream()), "ce_bwd")


def action_accuracy(pred: torch.Tensor, labels: torch.Tensor, ranges, counts=None, acc=None):
    """svla_action_accuracy: pred [B, >= L-1] int64 argmax ids (pred[b, t] for logits[b, t]), labels [B, L] int64,
    ranges = 6 inclusive token-id bounds (translation, rotation, gripper).  Returns (counts int64 [8], acc fp32 [4])
    on the device: {overall, translation, rotation, gripper} accuracy (train/monkey_patch.py:267-309)."""
    B, Lp = pred.shape
    _req(labels.dim() == 2 and labels.shape[0] == B and Lp >= labels.shape[1] - 1, "action_accuracy: shapes")
    _req(pred.dtype == labels.dtype == torch.int64 and pred.is_cuda and labels.is_cuda, "action_accuracy: int64 CUDA")
    _req(pred.stride(1) == 1 and labels.stride(1) == 1, "action_accuracy: rows must be contiguous")
    if counts is None:
        counts = torch.empty(8, dtype=torch.int64, device=pred.device)
    if acc is None:
        acc = torch.empty(4, dtype=torch.float32, device=pred.device)
    rg = (ctypes.c_int64 * 6)(*[int(v) for v in ranges])
    L.check(L.lib().svla_action_accuracy(B, labels.shape[1], pred.data_ptr(), pred.stride(0), labels.data_ptr(),
                                         labels.stride(0), rg, counts.data_ptr(), acc.data_ptr(), _stream()),
            "svla_action_accuracy")
    return counts, acc


def sumsq(x_flat, out, n_partial=4096):
    part = torch.empty(n_partial, dtype=torch.float32, device=x_flat.device)
    L.check(L.lib().svla_sumsq_bf16(x_flat.numel(), x_flat.data_ptr(), part.data_ptr(), n_partial, out.data_ptr(),
                                    _stream()), "sumsq")


def clip_scale(sumsq_t, max_norm, clip, norm_out):
    L.check(L.lib().svla_clip_scale(sumsq_t.data_ptr(), max_norm, clip.data_ptr(), _ptr(norm_out), _stream()),
            "clip_scale")


def adamw(master, param, grad, m, v, lr, b1, b2, eps, wd, step, clip=None):
    bc1 = 1.0 - b1 ** step
    bc2 = 1.0 - b2 ** step
    L.check(L.lib().svla_adamw(master.numel(), master.data_ptr(), param.data_ptr(), grad.data_ptr(), m.data_ptr(),
                               v.data_ptr(), lr, b1, b2, eps, wd, bc1, bc2, _ptr(clip), _stream()), "adamw")


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def ceil_div(a: int, b: int) -> int:
    return -(-a // b)


__all__ = [n for n in dir() if not n.startswith("_")] + ["math"]


# ---------------------------------------------------------------------------------------- Zoe metric tail
def zoe_metric_tail(clb, feat, rel, emb, ctr):
    """Fused ZoeDepthMetricDepthEstimationHead tail (csrc/zoe.hip): clb = the
    ZoeDepthConditionalLogBinomialSoftmax module (its 1x1-conv MLP weights, eps and temperature bounds);
    feat [B, CF, H, W] outconv activation, rel [B, H, W] relative depth, emb [B, CE, h, w] bin embedding,
    ctr [B, NB, h, w] bin centres (any strides).  Returns the metric depth [B, 1, H, W] fp32."""
    B, CF, H, W = feat.shape
    _req(rel.shape == (B, H, W), "zoe_tail: relative depth must match the outconv activation's size")
    _, CE, h, w = emb.shape
    NB = ctr.shape[1]
    _req(ctr.shape[2:] == emb.shape[2:], "zoe_tail: bin centres and embedding must share the low resolution")
    for t in (feat, rel, emb, ctr):
        _chk_bf16(t, "zoe_tail input")
    c1, c2 = clb.mlp[0], clb.mlp[2]
    key = (feat.device, c1.weight.data_ptr(), c1.weight._version, c2.weight._version)
    hit = getattr(clb, "_svla_params", None)
    if hit is None or hit[0] != key:  # frozen: one fp32 parameter block per module
        from transformers.models.zoedepth.modeling_zoedepth import log_binom
        lbt = clb.log_binomial_transform
        lb = log_binom(lbt.k_minus_1, lbt.k_idx).reshape(-1).float()
        w1t = c1.weight.reshape(c1.out_channels, -1).float().t().contiguous()
        w2 = c2.weight.reshape(c2.out_channels, -1).float()
        prm = torch.cat([w1t.reshape(-1), w2.reshape(-1), c1.bias.float(), c2.bias.float(), lb.to(feat.device)])
        clb._svla_params = hit = (key, prm.contiguous())
    prm = hit[1]
    out = torch.empty(B, 1, H, W, dtype=torch.float32, device=feat.device)
    i64 = lambda t: (ctypes.c_int64 * t.dim())(*t.stride())  # noqa: E731
    L.check(L.lib().svla_zoe_metric_tail(B, H, W, h, w, CF, CE, NB, c1.out_channels, feat.data_ptr(), i64(feat),
                                         rel.data_ptr(), i64(rel), emb.data_ptr(), i64(emb), ctr.data_ptr(), i64(ctr),
                                         prm.data_ptr(), float(clb.p_eps), float(clb.max_temp), float(clb.min_temp),
                                         1e-4, out.data_ptr(), _stream()), "zoe_metric_tail")
    return out


def zoe_readout_cat(hidden: torch.Tensor, out: torch.Tensor):
    """svla_zoe_readout_cat: hidden [B, T + 1, C] (CLS first) -> out [B * T, 2C] rows [token, CLS]."""
    B, T1, C = hidden.shape
    _req(hidden.is_contiguous() and hidden.dtype == torch.bfloat16, "zoe_readout_cat: contiguous bf16 hidden")
    _req(out.shape == (B * (T1 - 1), 2 * C) and out.is_contiguous(), "zoe_readout_cat: out [B*T, 2C]")
    L.check(L.lib().svla_zoe_readout_cat(B, T1 - 1, C, hidden.data_ptr(), out.data_ptr(), _stream()),
            "zoe_readout_cat")


def zoe_attractor(attractors: torch.Tensor, centres: torch.Tensor, alpha: float, gamma: int, mean: bool):
    """ZoeDepthAttractorLayerUnnormed's bin update on the fused kernel (svla_zoe_attractor): attractors [B, NA, H, W],
    centres [B, NB, H, W] (bf16, any strides; channels-last for the 16-B path) -> new centres, channels-last."""
    B, NA, H, W = attractors.shape
    _, NB, h2, w2 = centres.shape
    _req(centres.shape[0] == B and (h2, w2) == (H, W), "zoe_attractor: attractors and centres must share B, H, W")
    _chk_bf16(attractors, "zoe_attractor attractors")
    _chk_bf16(centres, "zoe_attractor centres")
    _req(NB % 8 == 0, "zoe_attractor: bin count must be a multiple of 8")
    out = torch.empty(B, NB, H, W, dtype=BF16, device=centres.device, memory_format=torch.channels_last)
    i64 = lambda t: (ctypes.c_int64 * 4)(*t.stride())  # noqa: E731
    L.check(L.lib().svla_zoe_attractor(B, H, W, NA, NB, attractors.data_ptr(), i64(attractors), centres.data_ptr(),
                                       i64(centres), float(alpha), int(gamma), int(bool(mean)), out.data_ptr(),
                                       i64(out), _stream()), "zoe_attractor")
    return out


# ---------------------------------------------------------------------------------------- Zoe pre/post resize
def zoe_preprocess(x: torch.Tensor, pad: int, size, mean, std) -> torch.Tensor:
    """process_zoe (reference modeling_spatialvla.py:99-110) in one kernel: reflect pad, bicubic resize to `size`
    (align_corners=True) and (x - mean) / std with the reference's bf16 roundings.  x bf16 [B, C, H, W]."""
    _chk_bf16(x, "zoe_preprocess")
    _req(x.dim() == 4 and x.is_contiguous() and x.shape[1] <= 4, "zoe_preprocess: x must be contiguous [B, C<=4, H, W]")
    B, C, H, W = x.shape
    OH, OW = size
    out = torch.empty(B, C, OH, OW, dtype=x.dtype, device=x.device)
    m = (ctypes.c_float * C)(*[float(v) for v in mean])
    sd = (ctypes.c_float * C)(*[float(v) for v in std])
    L.check(L.lib().svla_zoe_preprocess(B, C, H, W, int(pad), OH, OW, x.data_ptr(), m, sd, out.data_ptr(), _stream()),
            "zoe_preprocess")
    return out


def zoe_depth_resize(depth: torch.Tensor, pad: int, size) -> torch.Tensor:
    """F.interpolate(depth[:, None], size + 2 pad, bicubic, align_corners=True)[..., pad:-pad, pad:-pad] (reference
    modeling_spatialvla.py:318-323) in one kernel.  depth bf16 [B, IH, IW] -> [B, 1, OH, OW]."""
    _chk_bf16(depth, "zoe_depth_resize")
    _req(depth.dim() == 3 and depth.is_contiguous(), "zoe_depth_resize: depth must be contiguous [B, IH, IW]")
    B, IH, IW = depth.shape
    OH, OW = size
    out = torch.empty(B, 1, OH, OW, dtype=depth.dtype, device=depth.device)
    L.check(L.lib().svla_zoe_depth_resize(B, IH, IW, int(pad), OH, OW, depth.data_ptr(), out.data_ptr(), _stream()),
            "zoe_depth_resize")
    return out


# ---------------------------------------------------------------------------------------- Zoe DPT neck resize
def upsample_bilinear_cl(x: torch.Tensor, size=None, scale_factor=None, align_corners: bool = False):
    """torch.nn.functional.interpolate(x, size / scale_factor, mode="bilinear", align_corners) for a channels-last
    bf16 [B, C, H, W] map (C % 8 == 0) through svla_upsample_bilinear_nhwc; returns a channels-last tensor.
    Scales follow torch's area_pixel_compute_scale (recompute_scale_factor unset)."""
    B, C, H1, W1 = x.shape
    _req(x.dtype == torch.bfloat16 and x.is_cuda and C % 8 == 0, "upsample_bilinear_cl: bf16 CUDA map, C % 8 == 0")
    _req(x.is_contiguous(memory_format=torch.channels_last), "upsample_bilinear_cl: input must be channels-last")
    if size is None:
        sf = scale_factor if isinstance(scale_factor, (tuple, list)) else (scale_factor, scale_factor)
        H2, W2 = int(math.floor(H1 * float(sf[0]))), int(math.floor(W1 * float(sf[1])))
    else:
        H2, W2 = (size, size) if isinstance(size, int) else (int(size[0]), int(size[1]))
        sf = None

    def scale(i, o, s):  # torch area_pixel_compute_scale<float>: float divisions, 1/scale in double then float
        import numpy as np
        if align_corners:
            return float(np.float32(i - 1) / np.float32(o - 1)) if o > 1 else 0.0
        return float(np.float32(1.0 / float(s))) if s is not None and float(s) > 0 else float(np.float32(i) / np.float32(o))
    rh = scale(H1, H2, sf[0] if sf is not None else None)
    rw = scale(W1, W2, sf[1] if sf is not None else None)
    out = torch.empty(B, C, H2, W2, dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    L.check(L.lib().svla_upsample_bilinear_nhwc(B, C, H1, W1, H2, W2, int(bool(align_corners)), float(rh), float(rw),
                                                x.data_ptr(), out.data_ptr(), _stream()), "upsample_bilinear_nhwc")
    return out


def geglu_bwd(dh: torch.Tensor, g: torch.Tensor, u: torch.Tensor, dg: torch.Tensor, du: torch.Tensor):
    """svla_geglu_bwd over [M, I] row-strided bf16 views (dg may be dh itself)."""
    M, I = g.shape
    for t in (dh, g, u, dg, du):
        _req(t.shape == (M, I) and t.dtype == torch.bfloat16 and t.stride(1) == 1, "geglu_bwd: [M, I] bf16 rows")
    L.check(L.lib().svla_geglu_bwd(M, I, dh.data_ptr(), dh.stride(0), g.data_ptr(), g.stride(0), u.data_ptr(),
                                   u.stride(0), dg.data_ptr(), dg.stride(0), du.data_ptr(), du.stride(0), _stream()),
            "geglu_bwd")


def geglu_bwd_mx(dh: torch.Tensor, g: torch.Tensor, u: torch.Tensor, dg: torch.Tensor, du: torch.Tensor):
    """geglu_bwd that also returns the MX e4m3 copy of [dg | du] (svla_geglu_bwd_mx): (q [M, 2I], MXScales),
    bitwise quant_mx_rows of the bf16 [dg | du] -- the fp8 gate|up dgrad operand without a separate pass."""
    M, I = g.shape
    for t in (dh, g, u, dg, du):
        _req(t.shape == (M, I) and t.dtype == torch.bfloat16 and t.stride(1) == 1, "geglu_bwd_mx: [M, I] bf16 rows")
    _req(I % 128 == 0, "geglu_bwd_mx: I must be a multiple of 128")
    q = torch.empty(M, 2 * I, dtype=FP8, device=g.device)
    sc = MXScales(M, 2 * I, g.device)
    L.check(L.lib().svla_geglu_bwd_mx(M, I, dh.data_ptr(), dh.stride(0), g.data_ptr(), g.stride(0), u.data_ptr(),
                                      u.stride(0), dg.data_ptr(), dg.stride(0), du.data_ptr(), du.stride(0),
                                      q.data_ptr(), q.stride(0), sc.buf.data_ptr(), sc.ld, _stream()), "geglu_bwd_mx")
    return q, sc


# ---------------------------------------------------------------------------------------- NHWC convolution
# split-K of the sub-wave convolution grids (the stream's GEMM workspace); SVLA_CONV_SPLIT=0: none
CONV_SPLIT = [os.environ.get("SVLA_CONV_SPLIT", "1") != "0"]


def conv_weight_khwc(weight: torch.Tensor, transposed: bool = False) -> torch.Tensor:
    """torch conv weight -> the svla_conv2d_nhwc layout: Conv2d [Cout, Cin, KH, KW] -> [Cout, KH, KW, Cin];
    ConvTranspose2d [Cin, Cout, f, f] -> [f, f, Cout, Cin]."""
    if transposed:
        return weight.permute(2, 3, 1, 0).contiguous()
    return weight.permute(0, 2, 3, 1).contiguous()


def conv2d_cl(x: torch.Tensor, w_khwc: torch.Tensor, bias: Optional[torch.Tensor] = None, stride: int = 1,
              pad: int = 0, pre_relu: bool = False, post_relu: bool = False, res1: Optional[torch.Tensor] = None,
              res2: Optional[torch.Tensor] = None, transposed: bool = False) -> torch.Tensor:
    """svla_conv2d_nhwc on channels-last bf16 maps: x [B, Cin, H, W] (channels_last memory) -> [B, Cout, OH, OW]
    channels_last.  w_khwc from conv_weight_khwc.  transposed: ConvTranspose2d with kernel == stride (w [f, f, Cout,
    Cin]).  res1 / res2: channels-last maps of the output's shape added (each rounded to bf16) after bias + relu."""
    _req(x.is_cuda and x.dtype == BF16 and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last),
         "conv2d_cl: x must be a channels-last bf16 CUDA map")
    B, Cin, H, W = x.shape
    a = L.ConvArgs()
    if transposed:
        f, f2, Cout, Cw = w_khwc.shape
        _req(f == f2 and Cw == Cin, "conv2d_cl: transposed weight must be [f, f, Cout, Cin]")
        OH, OW, KH, KW = H * f, W * f, f, f
        a.flags |= L.CONV_TRANSPOSED
        a.factor = f
    else:
        Cout, KH, KW, Cw = w_khwc.shape
        _req(Cw == Cin, f"conv2d_cl: weight Cin {Cw} != input channels {Cin}")
        OH, OW = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    _req(w_khwc.is_contiguous() and w_khwc.dtype == BF16, "conv2d_cl: weight must be contiguous bf16")
    out = torch.empty(B, Cout, OH, OW, dtype=BF16, device=x.device, memory_format=torch.channels_last)
    for r, nm in ((res1, "res1"), (res2, "res2")):
        _req(r is None or (r.shape == out.shape and r.dtype == BF16
                           and r.is_contiguous(memory_format=torch.channels_last)),
             f"conv2d_cl: {nm} must be a channels-last bf16 map of the output's shape")
    _req(bias is None or (bias.dtype == BF16 and bias.is_contiguous() and bias.numel() == Cout), "conv2d_cl: bias")
    a.B, a.H, a.W, a.Cin, a.OH, a.OW, a.Cout = B, H, W, Cin, OH, OW, Cout
    a.KH, a.KW, a.stride, a.pad = KH, KW, stride, pad
    a.flags |= (L.CONV_PRE_RELU if pre_relu else 0) | (L.CONV_POST_RELU if post_relu else 0)
    a.x, a.w, a.bias, a.res1, a.res2, a.out = (x.data_ptr(), w_khwc.data_ptr(), _ptr(bias), _ptr(res1), _ptr(res2),
                                               out.data_ptr())
    if CONV_SPLIT[0]:
        ws = gemm_workspace()
        a.workspace, a.ws_bytes = ws.data_ptr(), ws.numel()
    L.check(L.lib().svla_conv2d_nhwc(ctypes.byref(a), _stream()), "svla_conv2d_nhwc")
    return out
