"""fp8 projections (BASELINE configs[4]): row-wise OCP e4m3 quantisation and the MX-scaled fp8 MFMA
GEMM (svla_quant_fp8_rows, svla_gemm_fp8).

Tolerances (stated here):
  * quantiser: bit-exact against torch's float8_e4m3fn cast of the same scaled, clamped fp32 values;
  * GEMM kernel: against an fp32 matmul of the DEQUANTISED operands (the exact product the kernel must form) at
    relative L2 <= 4e-3 (bf16 output rounding; fp32 accumulation order);
  * GEMM vs the bf16 GEMM of the unquantised operands: relative L2 <= 6e-2 (e4m3 has a 3-bit mantissa: the
    quantisation error of random operands lands at 3.75e-2 on MI355X);
  * one Gemma2 layer (four fp8 GEMMs in sequence: q|k|v, o, gate|up, down) vs the bf16 layer: relative L2 <= 0.12
    on the residual update, dx and every weight gradient -- the single-GEMM error compounded over the chain
    (measured 8.7e-2 / 7.6e-2 / 9.8e-2).
"""
import os

import pytest
import torch

from spatialvla_amd import kernels as K, _lib as L

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def ref_quant(x):
    xf = x.float()
    amax = xf.abs().amax(1)
    inv = torch.where(amax > 0, torch.tensor(448.0, device=x.device) / amax, torch.zeros_like(amax))
    q = (xf * inv[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
    return q, amax / 448.0


@pytest.mark.parametrize("rows,k", [(37, 2304), (300, 9216), (5, 2048), (64, 208)])
def test_quant_fp8_rows_bitexact(cuda, rows, k):
    g = torch.Generator(device=cuda).manual_seed(rows + k)
    x = (torch.randn(rows, k, device=cuda, generator=g) * torch.logspace(-3, 2, rows, device=cuda)[:, None]).to(BF)
    x[1, :] = 0  # zero row -> scale 0, q 0
    q, s = K.quant_fp8_rows(x)
    qr, sr = ref_quant(x.cpu())  # CPU: correctly rounded fp32 division, as the kernel's
    assert torch.equal(q.view(torch.uint8).cpu(), qr.view(torch.uint8))
    assert torch.equal(s.cpu(), sr)


def test_quant_fp8_rows_colscale_and_transpose(cuda):
    """Quantiser with column scales (the dgrad operand) bit-exact to torch; byte transpose exact."""
    g = torch.Generator(device=cuda).manual_seed(5)
    for rows, k in ((300, 18432), (37, 4096)):
        x = torch.randn(rows, k, device=cuda, generator=g).to(BF)
        cs = torch.rand(k, device=cuda, generator=g) * 0.01 + 1e-4
        q, s = K.quant_fp8_rows(x, colscale=cs)
        xr = (x.float() * cs[None, :]).cpu()
        amax = xr.abs().amax(1)
        inv = torch.where(amax > 0, torch.tensor(448.0) / amax, torch.zeros_like(amax))
        qr = (xr * inv[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)
        assert torch.equal(q.view(torch.uint8).cpu(), qr.view(torch.uint8)) and torch.equal(s.cpu(), amax / 448.0)
    for r_, c_ in ((4096, 2304), (2304, 18432), (100, 48)):
        m = torch.randint(0, 256, (r_, c_), dtype=torch.uint8, device=cuda)
        assert torch.equal(K.transpose_u8(m), m.t().contiguous())


def test_fp8_dgrad_gemm(cuda):
    """dX = dY @ W on the fp8 path (functional._fp8_dgrad): dY scaled by the forward weight copy's row scales and
    quantised per row, against the byte-transposed e4m3 weight.  Within 4e-3 of the exact product of the
    quantised operands, within 6e-2 of the bf16 product."""
    from spatialvla_amd import functional as Fn
    g = torch.Generator(device=cuda).manual_seed(8)
    M, N, Kd = 2000, 18432, 2304
    dy = torch.randn(M, N, device=cuda, generator=g).to(BF)
    w = (torch.randn(N, Kd, device=cuda, generator=g) * 0.02).to(BF)
    f8 = Fn.FP8Weights()
    out = torch.empty(M, Kd, dtype=BF, device=cuda)
    prev, Fn.FP8_SCALING[0] = Fn.FP8_SCALING[0], "row"
    try:
        Fn._fp8_dgrad(dy, f8, "w", (w,), out)
        wq, ws = f8.get("w", (w,))
    finally:
        Fn.FP8_SCALING[0] = prev
    dq, ds = K.quant_fp8_rows(dy, colscale=ws)
    exact = (dq.float() * ds[:, None]) @ wq.float()
    bf = dy.float() @ w.float()
    e_k, e_q = rel(out, exact), rel(out, bf)
    print(f"fp8 dgrad: vs quantised-operand product {e_k:.2e}, vs bf16 {e_q:.2e}")
    assert e_k < 4e-3 and e_q < 6e-2


def _dequant(q, s):
    return q.float() * s[:, None]


@pytest.mark.parametrize("m,n,k", [(1000, 4096, 2304), (9984, 2304, 2048), (300, 2304, 9216), (256, 512, 208),
                                   (2000, 1280, 4096)])
def test_gemm_fp8_store(cuda, m, n, k):
    g = torch.Generator(device=cuda).manual_seed(m + n)
    x = torch.randn(m, k, device=cuda, generator=g).to(BF)
    w = (torch.randn(n, k, device=cuda, generator=g) * 0.02).to(BF)
    xq, xs = K.quant_fp8_rows(x)
    wq, ws = K.quant_fp8_rows(w)
    out = torch.full((m, n), float("nan"), dtype=BF, device=cuda)
    K.gemm_fp8(xq, xs, wq, ws, out)
    exact = _dequant(xq, xs) @ _dequant(wq, ws).T
    bf = x.float() @ w.float().T
    e_k, e_q = rel(out, exact), rel(out, bf)
    print(f"fp8 gemm {m}x{n}x{k}: vs dequantised fp32 {e_k:.2e}, vs unquantised {e_q:.2e}")
    assert torch.isfinite(out.float()).all()
    assert e_k < 4e-3 and e_q < 6e-2


def test_gemm_fp8_geglu_and_resid(cuda):
    """Gemma2 gate|up GeGLU epilogue (h, g, u) and the bias+residual epilogue on the fp8 kernel, against the bf16
    epilogue formulas applied to the exact dequantised products."""
    m, hdim, inter = 700, 2304, 1536
    g0 = torch.Generator(device=cuda).manual_seed(3)
    x = torch.randn(m, hdim, device=cuda, generator=g0).to(BF)
    wgu = (torch.randn(2 * inter, hdim, device=cuda, generator=g0) * 0.02).to(BF)
    xq, xs = K.quant_fp8_rows(x)
    wq, ws = K.quant_fp8_rows(wgu)
    h = torch.empty(m, inter, dtype=BF, device=cuda)
    gg, uu = torch.empty_like(h), torch.empty_like(h)
    K.gemm_fp8(xq, xs, wq, ws, h, kind=L.EPI_GEGLU, geglu_I=inter, out1=gg, out2=uu)
    ex = _dequant(xq, xs) @ _dequant(wq, ws).T
    g_ref, u_ref = ex[:, :inter].to(BF), ex[:, inter:].to(BF)
    h_ref = torch.nn.functional.gelu(g_ref.float(), approximate="tanh").to(BF).float() * u_ref.float()
    assert rel(gg, g_ref) < 4e-3 and rel(uu, u_ref) < 4e-3 and rel(h, h_ref) < 6e-3
    # bias + residual (o_proj / down-proj style output with the residual stream added)
    n = 2304
    w2 = (torch.randn(n, inter, device=cuda, generator=g0) * 0.02).to(BF)
    res = torch.randn(m, n, device=cuda, generator=g0).to(BF)
    hq, hs = K.quant_fp8_rows(h)
    w2q, w2s = K.quant_fp8_rows(w2)
    out = torch.empty(m, n, dtype=BF, device=cuda)
    K.gemm_fp8(hq, hs, w2q, w2s, out, kind=L.EPI_BIAS_RESID, in0=res)
    ref = (_dequant(hq, hs) @ _dequant(w2q, w2s).T).to(BF).float() + res.float()
    assert rel(out, ref) < 4e-3


def test_gemm_fp8_rejects_bad_args(cuda):
    x = torch.zeros(64, 200, dtype=torch.float8_e4m3fn, device=cuda)  # K = 200 is not a multiple of 16
    s = torch.ones(64, device=cuda)
    out = torch.empty(64, 64, dtype=BF, device=cuda)
    with pytest.raises(L.SvlaError, match="multiple of 16"):
        K.gemm_fp8(x, s, x, s, out)


def test_gemma2_layer_fp8_vs_bf16(cuda):
    """One Gemma2 decoder layer at SpatialVLA-4B widths (B=2, L=312, prefix 299) with the fp8 forward projections
    against the same layer in bf16: output and input gradient within the stated fp8 tolerance (rel-L2 <= 0.12),
    weight gradients too (the backward GEMMs are bf16 on the fp8 forward's saved activations).  A second call after
    an in-place weight change must requantise (stale fp8 copies would be a silent error)."""
    import json
    from spatialvla_amd import SpatialVLAConfig, presets
    from spatialvla_amd.modeling_gemma2 import Gemma2DecoderLayer, KVMask
    cfg = SpatialVLAConfig(**json.loads(json.dumps(presets.spatialvla_4b(use_vision_zoe=False)))).text_config
    torch.manual_seed(0)
    layer = Gemma2DecoderLayer(cfg, 1).to(torch.bfloat16).to(cuda)
    with torch.no_grad():
        for p in layer.parameters():
            p.normal_(0, 0.02) if p.dim() == 2 else p.normal_(0, 0.1)
    B, L, P = 2, 312, 299
    cls = torch.ones(B, L, dtype=torch.uint8, device=cuda)
    cls[:, :P] = 0
    rope = layer.self_attn.rotary_emb.tables((torch.arange(L, device=cuda) + 1)[None], torch.bfloat16)
    x = torch.randn(B, L, cfg.hidden_size, device=cuda).to(BF)
    gy = torch.randn(B, L, cfg.hidden_size, device=cuda).to(BF)

    def run():
        xi = x.clone().requires_grad_(True)
        for p in layer.parameters():
            p.grad = None
        y = layer(xi, KVMask(cls), rope)
        y.backward(gy)
        return y.detach(), xi.grad, {n: p.grad.clone() for n, p in layer.named_parameters()}

    y0, dx0, g0 = run()
    layer.set_fp8_projections(True)
    y1, dx1, g1 = run()
    e_y, e_dx = rel(y1 - x, y0 - x), rel(dx1, dx0)
    e_w = max(rel(g1[n], g0[n]) for n in g0 if g0[n].float().norm() > 0)
    print(f"fp8 layer vs bf16: update {e_y:.2e}, dx {e_dx:.2e}, worst weight grad {e_w:.2e}")
    assert e_y < 0.12 and e_dx < 0.12 and e_w < 0.12
    with torch.no_grad():
        layer.mlp.down_proj.weight.mul_(2.0)
    y2, _, _ = run()
    layer.set_fp8_projections(False)
    y3, _, _ = run()
    assert rel(y2 - x, y3 - x) < 0.12, "fp8 weight copy not refreshed after an in-place update"


# ------------------------------------------------------------------------------------------------ OCP MX scaling
def ref_quant_mx(x):
    """OCP MX (spec v1.0) e4m3 restatement on the CPU: per 32-k block, X = clamp(ceil(log2(amax / 448)), -127, 127)
    (amax = 0 or subnormal: -127), q = e4m3(clamp(x * 2^-X, +-448)).  Returns (q, X [rows, K/32] int32)."""
    xf = x.float().cpu()
    rows, k = xf.shape
    blk = xf.view(rows, k // 32, 32)
    amax = blk.abs().amax(2)
    bits = amax.view(torch.int32)
    e = ((bits >> 23) & 0xFF) - 127 - 8 + ((bits & 0x7FFFFF) > 0x600000).int()
    X = torch.where(((bits >> 23) & 0xFF) == 0, torch.full_like(e, -127), e).clamp(-127, 127)
    assert bool((blk.abs() * torch.exp2(-X.float())[..., None] <= 448).all())  # nothing saturates
    q = (blk * torch.exp2(-X.float())[..., None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(rows, k)
    return q, X


def _mx_data(rows, k, g, device):
    """Random rows whose 32-k blocks span 2^-20 .. 2^20 in magnitude (so per-block scales matter), with an all-zero
    block, a block of bf16 subnormals and a row of zeros."""
    x = torch.randn(rows, k, device=device, generator=g)
    mag = torch.exp2(torch.randint(-20, 21, (rows, k // 32), device=device, generator=g).float())
    x = (x.view(rows, k // 32, 32) * mag[..., None]).view(rows, k)
    x[0, :32] = 0
    x[1, 32:64] = 1e-39
    x[2, :] = 0
    return x.to(BF)


@pytest.mark.parametrize("rows,k", [(37, 2304), (300, 9216), (5, 2048), (64, 128), (259, 18432)])
def test_quant_mx_rows_bitexact(cuda, rows, k):
    g = torch.Generator(device=cuda).manual_seed(rows * 7 + k)
    x = _mx_data(rows, k, g, cuda)
    q, sc = K.quant_mx_rows(x)
    qr, Xr = ref_quant_mx(x)
    assert torch.equal(sc.exponents().cpu(), Xr)
    assert torch.equal(q.view(torch.uint8).cpu(), qr.view(torch.uint8))


@pytest.mark.parametrize("n,k", [(4096, 2304), (2304, 2048), (18432, 2304), (2304, 9216), (128, 64), (384, 192)])
def test_quant_mx_cols_equals_rows_of_transpose(cuda, n, k):
    """svla_quant_mx_cols(W) (the dgrad operand W^T, no bf16 transpose) is bit for bit svla_quant_mx_rows(W^T): the
    e4m3 bytes and the E8M0 scales, including zero, subnormal, NaN and Inf blocks."""
    g = torch.Generator(device=cuda).manual_seed(n + k)
    w = _mx_data(n, k, g, cuda)
    w[5, 7] = float("nan")
    w[64 + 3, k - 1] = float("inf")
    q, sc = K.quant_mx_cols(w)
    qr, scr = K.quant_mx_rows(w.t().contiguous())
    assert torch.equal(sc.exponents(), scr.exponents())
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8))


@pytest.mark.parametrize("r,c", [(4096, 2304), (2304, 2048), (18432, 2304), (2304, 9216), (128, 128), (9984, 4096)])
def test_quant_mx_both_equals_rows_and_cols(cuda, r, c):
    """svla_quant_mx_both (the fp8 weight copies from one read) is bit for bit quant_mx_rows(W) and quant_mx_cols(W)."""
    g = torch.Generator(device=cuda).manual_seed(r * 3 + c)
    w = _mx_data(r, c, g, cuda)
    w[1, 2] = float("nan")
    w[100, 127] = float("-inf")
    (q, sc), (qt, sct) = K.quant_mx_both(w)
    q0, sc0 = K.quant_mx_rows(w)
    qt0, sct0 = K.quant_mx_cols(w)
    assert torch.equal(sc.exponents(), sc0.exponents()) and torch.equal(q.view(torch.uint8), q0.view(torch.uint8))
    assert torch.equal(sct.exponents(), sct0.exponents()) and torch.equal(qt.view(torch.uint8), qt0.view(torch.uint8))


@pytest.mark.parametrize("items", ["1", "4", "8"])
def test_quant_mx_rows_items_per_wave_bitwise(cuda, items):
    """The items-per-wave variants of svla_quant_mx_rows (SVLA_QUANT_MX_ITEMS, read once per process: run in a child)
    give the bytes of the CPU restatement on a ragged shape (K = 2304: a half 512-k chunk per row)."""
    import subprocess
    import sys
    code = ("import torch, sys; sys.path.insert(0, %r); sys.path.insert(0, %r); import test_fp8_gpu as T; "
            "from spatialvla_amd import kernels as K; g = torch.Generator(device='cuda').manual_seed(3); "
            "x = T._mx_data(1001, 2304, g, 'cuda'); q, sc = K.quant_mx_rows(x); qr, Xr = T.ref_quant_mx(x); "
            "assert torch.equal(sc.exponents().cpu(), Xr); "
            "assert torch.equal(q.view(torch.uint8).cpu(), qr.view(torch.uint8)); print('ok')"
            % (os.path.dirname(os.path.abspath(__file__)), os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SVLA_QUANT_MX_ITEMS=items),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, p.stderr[-3000:]


def test_geglu_bwd_mx_equals_pass_then_quant(cuda):
    """svla_geglu_bwd_mx: the bf16 dg / du of svla_geglu_bwd bit for bit, and the MX copy of [dg | du] bit for bit
    quant_mx_rows of them (the fused producer of the fp8 gate|up dgrad operand)."""
    torch.manual_seed(41)
    M, I = 777, 1280
    dh = torch.randn(M, I, device=cuda).to(BF)
    g = (torch.randn(M, I, device=cuda) * 2).to(BF)
    u = torch.randn(M, I, device=cuda).to(BF)
    dh[3, 5] = float("nan")
    ref = torch.empty(M, 2 * I, dtype=BF, device=cuda)
    K.geglu_bwd(dh, g, u, ref[:, :I], ref[:, I:])
    got = torch.empty(M, 2 * I, dtype=BF, device=cuda)
    q, sc = K.geglu_bwd_mx(dh.clone(), g, u, got[:, :I], got[:, I:])
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    qr, scr = K.quant_mx_rows(ref)
    assert torch.equal(sc.exponents(), scr.exponents())
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8))


def test_norms_emit_mx_copy_bitwise(cuda):
    """svla_rmsnorm_fwd_mx / svla_add_rmsnorm2_fwd_train_mx: the bf16 outputs and rstd of the plain kernels bit for bit,
    and the MX copy of the normalised output bit for bit quant_mx_rows of it (the fp8 q|k|v / gate|up operands)."""
    torch.manual_seed(43)
    M, N = 1000, 2304
    res = torch.randn(M, N, device=cuda).to(BF)
    y = (torch.randn(M, N, device=cuda) * 3).to(BF)
    w1 = (torch.randn(N, device=cuda) * 0.3).to(BF)
    w2 = (torch.randn(N, device=cuda) * 0.3).to(BF)
    out0, out1 = torch.empty_like(y), torch.empty_like(y)
    r0, r1 = (torch.empty(M, dtype=torch.float32, device=cuda) for _ in range(2))
    K.rmsnorm_fwd(y, w1, 1e-6, out0, r0)
    q, sc = K.rmsnorm_fwd_mx(y, w1, 1e-6, out1, r1)
    assert torch.equal(out0, out1) and torch.equal(r0, r1)
    qr, scr = K.quant_mx_rows(out0)
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8)) and torch.equal(sc.exponents(), scr.exponents())
    h0, x0, h1, x1 = (torch.empty_like(y) for _ in range(4))
    a0, b0, a1, b1 = (torch.empty(M, dtype=torch.float32, device=cuda) for _ in range(4))
    K.add_rmsnorm2_fwd_train(res, y, w1, w2, 1e-6, 1e-6, h0, x0, a0, b0)
    q, sc = K.add_rmsnorm2_fwd_train_mx(res, y, w1, w2, 1e-6, 1e-6, h1, x1, a1, b1)
    assert torch.equal(h0, h1) and torch.equal(x0, x1) and torch.equal(a0, a1) and torch.equal(b0, b1)
    qr, scr = K.quant_mx_rows(x0)
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8)) and torch.equal(sc.exponents(), scr.exponents())


def test_norm_backwards_emit_mx_copy_bitwise(cuda):
    """svla_rmsnorm_bwd_mx / svla_rmsnorm2_bwd_mx: every output of the plain backward kernels bit for bit, and the MX
    copy of the stored input gradient bit for bit quant_mx_rows of it (the fp8 down / o dgrad operands)."""
    torch.manual_seed(47)
    M, N = 999, 2304
    x = (torch.randn(M, N, device=cuda) * 2).to(BF)
    y = torch.randn(M, N, device=cuda).to(BF)
    w1 = (torch.randn(N, device=cuda) * 0.3).to(BF)
    w2 = (torch.randn(N, device=cuda) * 0.3).to(BF)
    dy = torch.randn(M, N, device=cuda).to(BF)
    dres = torch.randn(M, N, device=cuda).to(BF)
    rs = torch.rand(M, device=cuda) + 0.5
    rs2 = torch.rand(M, device=cuda) + 0.5
    outs = []
    for mx in (False, True):
        dx = torch.empty_like(x)
        dw = torch.zeros(N, dtype=BF, device=cuda)
        cp = K.rmsnorm_bwd(x, w1, rs, dy, dres, dx, dw, mx=mx)
        outs.append((dx, dw, cp))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    qr, scr = K.quant_mx_rows(outs[0][0])
    q, sc = outs[1][2]
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8)) and torch.equal(sc.exponents(), scr.exponents())
    outs = []
    for mx in (False, True):
        dh, dyo = torch.empty_like(x), torch.empty_like(x)
        dw2, dw1 = torch.zeros(N, dtype=BF, device=cuda), torch.zeros(N, dtype=BF, device=cuda)
        cp = K.rmsnorm2_bwd(x, w2, rs2, dy, dres, y, w1, rs, dh, dyo, dw2, dw1, mx=mx)
        outs.append((dh, dyo, dw2, dw1, cp))
    for a, b in zip(outs[0][:4], outs[1][:4]):
        assert torch.equal(a, b)
    qr, scr = K.quant_mx_rows(outs[0][1])
    q, sc = outs[1][4]
    assert torch.equal(q.view(torch.uint8), qr.view(torch.uint8)) and torch.equal(sc.exponents(), scr.exponents())


def test_quant_mx_rows_nonfinite_blocks_are_nan(cuda):
    """A NaN or +-Inf element makes its whole 32-k MX block NaN -- scale byte 0xFF (OCP MX v1.0 §5.3) and e4m3 NaN
    elements (0x7F) -- instead of a finite clamp that would hide a diverging activation or dY; every other block is
    the finite quantisation; the MX GEMM then returns NaN on exactly the rows that hold such a block."""
    g = torch.Generator(device=cuda).manual_seed(77)
    rows, k = 256, 512
    x = _mx_data(rows, k, g, cuda)
    x[3, 40] = float("nan")
    x[7, 33 * 5 + 1] = float("inf")
    x[9, 300] = float("-inf")
    bad = {(3, 40 // 32), (7, (33 * 5 + 1) // 32), (9, 300 // 32)}
    q, sc = K.quant_mx_rows(x)
    X = sc.exponents().cpu()
    qb = q.view(torch.uint8).cpu().view(rows, k // 32, 32)
    xc = x.clone()
    for r, b in bad:
        xc[r, 32 * b:32 * b + 32] = 0.0
    qr, Xr = ref_quant_mx(xc)
    qrb = qr.view(torch.uint8).view(rows, k // 32, 32)
    for r in range(rows):
        for b in range(k // 32):
            if (r, b) in bad:
                assert X[r, b] == 0xFF - 127 and bool((qb[r, b] == 0x7F).all()), (r, b)
            elif r in (3, 7, 9):
                assert X[r, b] == Xr[r, b] and torch.equal(qb[r, b], qrb[r, b]), (r, b)
    others = [r for r in range(rows) if r not in (3, 7, 9)]
    assert torch.equal(X[others], Xr[others]) and torch.equal(qb[others], qrb[others])
    w = (_mx_data(384, k, g, cuda).float() * 0.02).to(BF)
    wq, ws = K.quant_mx_rows(w)
    out = torch.zeros(rows, 384, dtype=BF, device=cuda)
    K.gemm_mxfp8(q, sc, wq, ws, out)
    nanrows = torch.isnan(out.float()).all(1).cpu()
    assert nanrows[[3, 7, 9]].all() and not nanrows[others].any()


def _dequant_mx(q, sc):
    X = sc.exponents()
    rows, k = q.shape
    return (q.float().view(rows, k // 32, 32) * torch.exp2(X.float())[..., None]).view(rows, k)


@pytest.mark.parametrize("m,n,k", [(1000, 4096, 2304), (9984, 2304, 2048), (300, 2304, 9216), (256, 512, 128),
                                   (2000, 1280, 4096), (9984, 2304, 18432)])
def test_gemm_mxfp8_store(cuda, m, n, k):
    """The MX kernel against the fp32 product of the dequantised operands (block scales varying 2^-20..2^20 inside
    every row of both operands, so a wrong lane -> block scale map is an O(1) error), and against the bf16 product."""
    g = torch.Generator(device=cuda).manual_seed(m + n + k)
    x = _mx_data(m, k, g, cuda)
    w = (_mx_data(n, k, g, cuda).float() * 0.02).to(BF)
    xq, xs = K.quant_mx_rows(x)
    wq, ws = K.quant_mx_rows(w)
    out = torch.full((m, n), float("nan"), dtype=BF, device=cuda)
    K.gemm_mxfp8(xq, xs, wq, ws, out)
    exact = _dequant_mx(xq, xs) @ _dequant_mx(wq, ws).T
    bf = x.float() @ w.float().T
    e_k, e_q = rel(out, exact), rel(out, bf)
    print(f"mxfp8 gemm {m}x{n}x{k}: vs dequantised fp32 {e_k:.2e}, vs unquantised {e_q:.2e}")
    assert torch.isfinite(out.float()).all()
    assert e_k < 4e-3 and e_q < 6e-2


def test_fp8_mx_dgrad_gemm(cuda):
    """dX = dY @ W on the MX path (functional._fp8_dgrad): dY quantised with MX blocks along N against the MX copy of
    W^T (blocks along N, from the bf16 weight).  Within 4e-3 of the exact product of the quantised operands, within
    6e-2 of the bf16 product."""
    from spatialvla_amd import functional as Fn
    g = torch.Generator(device=cuda).manual_seed(9)
    M, N, Kd = 2000, 18432, 2304
    dy = torch.randn(M, N, device=cuda, generator=g).to(BF)
    w = (torch.randn(N, Kd, device=cuda, generator=g) * 0.02).to(BF)
    f8 = Fn.FP8Weights()
    out = torch.empty(M, Kd, dtype=BF, device=cuda)
    prev, Fn.FP8_SCALING[0] = Fn.FP8_SCALING[0], "mx"
    try:
        Fn._fp8_dgrad(dy, f8, "w", (w,), out)
        wt, st = f8.get_t("w", (w,))
    finally:
        Fn.FP8_SCALING[0] = prev
    dq, ds = K.quant_mx_rows(dy)
    exact = _dequant_mx(dq, ds) @ _dequant_mx(wt, st).T
    bf = dy.float() @ w.float()
    e_k, e_q = rel(out, exact), rel(out, bf)
    print(f"mx dgrad: vs quantised-operand product {e_k:.2e}, vs bf16 {e_q:.2e}")
    assert e_k < 4e-3 and e_q < 6e-2


def test_gemm_mxfp8_geglu(cuda):
    """Gemma2 gate|up GeGLU epilogue on the MX kernel (one [2I] weight and scale matrix, gate rows then up rows)."""
    m, hdim, inter = 700, 2304, 1536
    g = torch.Generator(device=cuda).manual_seed(31)
    x = torch.randn(m, hdim, device=cuda, generator=g).to(BF)
    w = (torch.randn(2 * inter, hdim, device=cuda, generator=g) * 0.02).to(BF)
    xq, xs = K.quant_mx_rows(x)
    wq, ws = K.quant_mx_rows(w)
    h, gg, uu = (torch.empty(m, inter, dtype=BF, device=cuda) for _ in range(3))
    K.gemm_mxfp8(xq, xs, wq, ws, h, kind=L.EPI_GEGLU, geglu_I=inter, out1=gg, out2=uu)
    exact = _dequant_mx(xq, xs) @ _dequant_mx(wq, ws).T
    ge, ue = exact[:, :inter].to(BF), exact[:, inter:].to(BF)
    he = (torch.nn.functional.gelu(ge.float(), approximate="tanh").to(BF).float() * ue.float()).to(BF)
    print(f"mxfp8 geglu: g {rel(gg, ge):.2e} u {rel(uu, ue):.2e} h {rel(h, he):.2e}")
    assert rel(gg, ge) < 4e-3 and rel(uu, ue) < 4e-3 and rel(h, he) < 6e-3
    # the same launch with the MX copy of h from the epilogue: h, g, u bit for bit, and the copy bit for bit
    # quant_mx_rows(h) (the fp8 down operand); M = 700 leaves a ragged last row block
    h2, g2, u2 = (torch.empty(m, inter, dtype=BF, device=cuda) for _ in range(3))
    hq = (torch.empty(m, inter, dtype=torch.float8_e4m3fn, device=cuda), K.MXScales(m, inter, cuda))
    K.gemm_mxfp8(xq, xs, wq, ws, h2, kind=L.EPI_GEGLU, geglu_I=inter, out1=g2, out2=u2, mx_out=hq)
    assert torch.equal(h2, h) and torch.equal(g2, gg) and torch.equal(u2, uu)
    qr, scr = K.quant_mx_rows(h)
    assert torch.equal(hq[0].view(torch.uint8), qr.view(torch.uint8))
    assert torch.equal(hq[1].exponents(), scr.exponents())
