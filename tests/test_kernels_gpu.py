"""Per-kernel parity of libsvla against plain PyTorch fp32 references of the same op (GPU)."""
import math
import os

import pytest
import torch
import torch.nn.functional as F

from harness import rel_l2

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _r(*shape, scale=1.0, dev="cuda"):
    return (torch.randn(*shape, device=dev) * scale).to(BF)


# ------------------------------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (200, 300, 136), (624, 577, 256), (9, 130, 72)])
@pytest.mark.parametrize("layouts", ["nt", "nn", "tn"])
def test_gemm_layouts(cuda, M, N, K, layouts):
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(0)
    if layouts == "nt":      # x[M,K] @ W[N,K]^T
        a, b = _r(M, K), _r(N, K)
        ref = a.float() @ b.float().T
        A, B = Kn._operand([a], L.LAYOUT_KC), Kn._operand([b], L.LAYOUT_KC)
    elif layouts == "nn":    # dy[M,K'] @ W[K',N]
        a, b = _r(M, K), _r(K, N + (-N) % 8)[:, :N]
        ref = a.float() @ b.float()
        A, B = Kn._operand([a], L.LAYOUT_KC), Kn._operand([b], L.LAYOUT_RC)
    else:                    # dy^T @ x : A stored [K, M], B stored [K, N]
        a, b = _r(K, M + (-M) % 8)[:, :M], _r(K, N + (-N) % 8)[:, :N]
        ref = a.float().T @ b.float()
        A, B = Kn._operand([a], L.LAYOUT_RC), Kn._operand([b], L.LAYOUT_RC)
    c = torch.empty(M, N + (-N) % 8, dtype=BF, device=cuda)[:, :N]
    Kn.gemm(M, N, K, A, B, [c], [0], c.stride(0), Kn._epi())
    torch.cuda.synchronize()
    assert rel_l2(c, ref) < 5e-3


def _variants(fn):
    """Run fn() under the GEMM dispatch variants (svla_gemm_bf16_ex): 1 = 2-barrier, 2 = 8-phase, 0 = product
    dispatch (twice), 3 = 4-wave kernel wherever both operands are KC (twice), 4 = 8-phase + stream-K, 5 = product
    dispatch without the small-M GEMV path.  Returns {variant: result}."""
    from spatialvla_amd import kernels as Kn
    outs = {}
    try:
        for v in (1, 2, 0, "0b", 3, "3b", 4, 5):
            Kn.gemm_variant = {"0b": 0, "3b": 3}.get(v, v)
            outs[v] = fn()
            torch.cuda.synchronize()
    finally:
        Kn.gemm_variant = 0
    return outs


def _flat(x):
    return torch.cat([t.float().reshape(-1) for t in x]) if isinstance(x, (tuple, list)) else x.float()


def _check_variants(outs, tol=2e-3):
    """8-phase == 2-barrier bitwise (same k order per output); stream-K reorders the fp32 sum of the k
    segments of a tile: close to the others and bitwise stable run to run."""
    f = lambda v: outs[v] if isinstance(outs[v], (tuple, list)) else (outs[v],)
    for a, b in zip(f(2), f(1)):
        assert torch.equal(a, b)
    for a, b in zip(f(0), f("0b")):
        assert torch.equal(a, b)
    for a, b in zip(f(3), f("3b")):
        assert torch.equal(a, b)
    for v in (0, 3, 4, 5):
        assert rel_l2(_flat(outs[v]), _flat(outs[1])) < tol, v


@pytest.mark.parametrize("M,N,K", [(1154, 4096, 1024), (1154, 1024, 4096), (300, 200, 64)])
def test_gemm_beit_epilogues(cuda, M, N, K):
    """BIAS_GELU_ERF: bf16(gelu_erf(bf16(acc + b))); BIAS_SCALE_RESID: bf16(bf16(s * bf16(acc + b)) + r) -- the
    rounding points of BeitLayer's fc1 + exact GELU and of lambda * sublayer + residual; vs torch on the same
    bf16 products (fp32 accumulation order differs: a bf16 ulp at most on a few elements)."""
    from spatialvla_amd import kernels as Kn, _lib as L_
    torch.manual_seed(12)
    x, w = _r(M, K), _r(N, K, scale=0.05)
    b, sc, res = _r(N, scale=0.5), _r(N, scale=0.3), _r(M, N)
    acc = (x.float() @ w.float().T)
    pre = (acc + b.float()).to(BF).float()
    ref_g = F.gelu(pre).to(BF)
    ref_s = ((sc.float() * pre).to(BF).float() + res.float()).to(BF)
    out_g = torch.empty(M, N, dtype=BF, device=cuda)
    out_s = torch.empty(M, N, dtype=BF, device=cuda)
    Kn.linear_fwd(x, [w], out_g, kind=L_.EPI_BIAS_GELU_ERF, bias=b)
    Kn.linear_fwd(x, [w], out_s, kind=L_.EPI_BIAS_SCALE_RESID, bias=b, colscale=sc, in0=res)
    assert rel_l2(out_g, ref_g) < 5e-3 and rel_l2(out_s, ref_s) < 5e-3
    ulp = lambda t: torch.abs(t.float()) * 2.0 ** -7 + 1e-6  # noqa: E731
    assert (torch.abs(out_g.float() - ref_g.float()) <= 2 * ulp(ref_g)).float().mean() > 0.999
    assert (torch.abs(out_s.float() - ref_s.float()) <= 2 * ulp(ref_s)).float().mean() > 0.999


@pytest.mark.parametrize("L", [577, 130])
def test_attention_d64_bias(cuda, L):
    """head_dim 64 MHA with an additive [heads, L, L] score bias (BEiT relative position bias): fp32 reference
    softmax(q k^T / 8 + bias) v."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(13)
    B, Hn, D = 2, 4, 64
    qkv = _r(B * L, 3 * Hn * D)
    ld = qkv.stride(0)
    q, k, v = qkv[:, :Hn * D], qkv[:, Hn * D:2 * Hn * D], qkv[:, 2 * Hn * D:]
    bias_full = _r(Hn, L, L, scale=2.0)
    bias = torch.zeros(Hn, L, (L + 7) // 8 * 8, dtype=BF, device=cuda)
    bias[:, :, :L] = bias_full
    a = Kn.attn_args(B, L, Hn, Hn, D, q, ld, k, ld, v, ld, D ** -0.5, 0.0, None, 0, bias=bias)
    out = torch.empty(B * L, Hn * D, dtype=BF, device=cuda)
    lse = torch.empty(B, Hn, L, device=cuda)
    Kn.attn_fwd(a, out, lse)
    qf, kf, vf = (t.float().view(B, L, Hn, D).transpose(1, 2) for t in (q, k, v))
    s_ = qf @ kf.transpose(-1, -2) * D ** -0.5 + bias_full.float()[None]
    ref = (torch.softmax(s_, -1) @ vf).transpose(1, 2).reshape(B * L, Hn * D)
    assert rel_l2(out, ref) < 1e-2
    assert rel_l2(lse, torch.logsumexp(s_, -1)) < 1e-4


def test_gemm_two_streams_bitwise(cuda):
    """svla_gemm_bf16 is re-entrant across streams (include/svla.h): GEMMs that use stream-K (slabs + arrival
    counters in the caller's workspace) run concurrently on two streams, each with its own workspace, and return
    exactly what they return one at a time."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(21)
    shapes = [(4096, 2304, 4096), (2048, 4608, 3072), (9984, 2304, 2304)]  # < 1 or ragged waves of tiles: stream-K
    xs = [_r(m, k) for m, n, k in shapes]
    ws = [_r(n, k, scale=0.05) for m, n, k in shapes]
    ref = []
    for x, w in zip(xs, ws):
        o = torch.empty(x.shape[0], w.shape[0], dtype=BF, device=cuda)
        Kn.linear_fwd(x, [w], o)
        ref.append(o)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [[torch.empty_like(r) for r in ref] for _ in streams]
    for rep in range(4):
        for i in range(len(shapes)):  # interleave the launches of both streams
            for si, st in enumerate(streams):
                with torch.cuda.stream(st):
                    j = (i + si) % len(shapes)
                    Kn.linear_fwd(xs[j], [ws[j]], outs[si][j])
    torch.cuda.synchronize()
    w0 = Kn.gemm_workspace(streams[0])
    w1 = Kn.gemm_workspace(streams[1])
    assert w0.data_ptr() != w1.data_ptr()
    for si in range(2):
        for j in range(len(shapes)):
            assert torch.equal(outs[si][j], ref[j]), (si, j)


@pytest.mark.parametrize("cap", [248, 200, 97])
def test_gemm_cu_cap_stream_k(cuda, cap):
    """svla_gemm_set_cu_cap (the side-stream weight-gradient GEMMs' persistent-grid cap, functional.SIDE_CU_RESERVE):
    stream-K schedules on a capped grid -- the 4-wave kernel (long K, every wgrad), the 8-phase one (short K, the B=1
    gate|up wgrad that once read a stale arrival counter when the cap moved the counters onto slab memory) -- give the
    fp32 product within bf16 rounding, are deterministic run to run, and leave the uncapped launches after them right."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(31)
    shapes = [(18432, 2304, 312), (2304, 9216, 9984), (4096, 2304, 9984), (1152, 1152, 8192)]  # wgrad: dW = dY^T X
    lib = L.lib()
    for M, N, Kd in shapes:
        dy, x = _r(Kd, M, scale=0.5), _r(Kd, N, scale=0.5)
        ref = (dy.float().t() @ x.float())
        outs = []
        try:
            lib.svla_gemm_set_cu_cap(cap)
            for _ in range(2):
                o = torch.full((M, N), float("nan"), dtype=BF, device=cuda)
                Kn.linear_wgrad(dy, x, [o])
                outs.append(o)
        finally:
            lib.svla_gemm_set_cu_cap(0)
        o0 = torch.full((M, N), float("nan"), dtype=BF, device=cuda)
        Kn.linear_wgrad(dy, x, [o0])
        assert torch.equal(outs[0], outs[1]), (M, N, Kd)
        for o in (outs[0], o0):
            assert torch.isfinite(o.float()).all(), (M, N, Kd)
            assert ((o.float() - ref).norm() / ref.norm()).item() < 8e-3, (M, N, Kd)


@pytest.mark.parametrize("M,N,K", [(2000, 16500, 200), (2304, 14336, 1000), (4100, 8200, 64), (9984, 2304, 2048),
                                   (1000, 3000, 8192)])
@pytest.mark.parametrize("layouts", ["nt", "nn", "tn"])
def test_gemm_big_tile(cuda, M, N, K, layouts):
    """Shapes that take the 256x256 tile: ragged M/N/K edges, all operand layouts, stream-K remainders
    (2304x14336: the last partial wave; 9984x2304: 351 tiles; 1000x3000: fewer tiles than CUs, ~5 k-segments
    per tile)."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(5)
    if layouts == "nt":
        a, b = _r(M, K), _r(N, K)
        ref = a.float() @ b.float().T
        A, B = Kn._operand([a], L.LAYOUT_KC), Kn._operand([b], L.LAYOUT_KC)
    elif layouts == "nn":
        a, b = _r(M, K), _r(K, N + (-N) % 8)[:, :N]
        ref = a.float() @ b.float()
        A, B = Kn._operand([a], L.LAYOUT_KC), Kn._operand([b], L.LAYOUT_RC)
    else:
        a, b = _r(K, M + (-M) % 8)[:, :M], _r(K, N + (-N) % 8)[:, :N]
        ref = a.float().T @ b.float()
        A, B = Kn._operand([a], L.LAYOUT_RC), Kn._operand([b], L.LAYOUT_RC)

    def run():
        c = torch.full((M, N + (-N) % 8), 7.0, dtype=BF, device=cuda)
        Kn.gemm(M, N, K, A, B, [c[:, :N]], [0], c.stride(0), Kn._epi())
        return c

    outs = _variants(run)
    _check_variants(outs)
    c0 = outs[0]
    assert rel_l2(c0[:, :N], ref) < 5e-3
    assert bool((c0[:, N:] == 7.0).all())  # nothing written beyond N


def test_gemm_big_tile_epilogues(cuda):
    """GeGLU, GeGLU-backward, bias+residual, softcap-CE and dW C-segments on the 256x256 tile, all main-loop
    variants."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(6)
    M, K, I = 4200, 320, 8192
    x, wg, wu = _r(M, K), _r(I, K, scale=0.1), _r(I, K, scale=0.1)

    def geglu():
        h, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
        Kn.linear_geglu_fwd(x, wg, wu, h, g, u)
        return h, g, u

    outs = _variants(geglu)
    _check_variants(outs, tol=5e-3)
    h0, g0, u0 = outs[0]
    gr, ur = x.float() @ wg.float().T, x.float() @ wu.float().T
    assert rel_l2(g0, gr) < 5e-3 and rel_l2(u0, ur) < 5e-3
    assert rel_l2(h0, F.gelu(gr, approximate="tanh") * ur) < 1e-2

    wd = _r(K, I, scale=0.1)
    dout = _r(M, K)

    def geglu_bwd():  # dgrad of down_proj with the GeGLU-backward epilogue: N = I, K' = K
        dgu = torch.empty(M, 2 * I, dtype=BF, device=cuda)
        Kn.linear_dgrad(dout, [wd], dgu[:, :I], kind=L.EPI_GEGLU_BWD, in0=g0, in1=u0, out1=dgu[:, :I],
                        out2=dgu[:, I:])
        return dgu

    _check_variants(_variants(geglu_bwd), tol=5e-3)

    bias, res = _r(I, scale=0.5), _r(M, I)

    def bias_resid():
        y = torch.empty(M, I, dtype=BF, device=cuda)
        Kn.linear_fwd(x, [wg], y, kind=L.EPI_BIAS_RESID, bias=bias, in0=res)
        return y

    outs = _variants(bias_resid)
    _check_variants(outs)
    assert rel_l2(outs[0], gr + bias.float() + res.float()) < 5e-3

    V = 30011
    wv = _r(V, K, scale=0.2)
    ldv = Kn.round_up(V, 64)
    ntn = Kn.ceil_div(V, 128)

    def softcap():
        buf = torch.empty(M, ldv, dtype=BF, device=cuda)
        stats = torch.empty(M, ntn, 3, dtype=torch.float32, device=cuda)
        Kn.linear_fwd(x, [wv], buf[:, :V], kind=L.EPI_SOFTCAP_CE, row_stats=stats, cap=30.0)
        return buf[:, :V], stats

    outs = _variants(softcap)
    _check_variants(outs)

    # wgrad into 3 gradient tensors (C row segments)
    dy, x2 = _r(M, 2 * I), _r(M, 2304)
    gs0 = [torch.zeros(s, 2304, dtype=BF, device=cuda) for s in (8192, 4096, 4096)]

    def wgrad():
        gs = [t.clone() for t in gs0]
        Kn.linear_wgrad(dy, x2, gs)
        return torch.cat(gs)

    outs = _variants(wgrad)
    _check_variants(outs)
    assert rel_l2(outs[0], dy.float().T @ x2.float()) < 5e-3


@pytest.mark.parametrize("M,N,K", [(1024, 1536, 2304), (1100, 1300, 640), (512, 768, 9984)])
def test_gemm4_direct_epilogue(cuda, M, N, K):
    """The 4-wave kernel's direct epilogue (interior tiles: stores straight from the C^T accumulators after
    v_permlane16_swap) beside its LDS-image epilogue (edge tiles of the ragged shape): STORE with alpha and
    accumulate, all operand layouts, and the GeGLU kernel, against fp32 references.  M x N multiples of 256 are
    interior-only; 1100 x 1300 mixes both paths in one launch."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(11)
    ops = {"nt": (_r(M, K), _r(N, K)), "nn": (_r(M, K), _r(K, N + (-N) % 8)[:, :N]),
           "tn": (_r(K, M + (-M) % 8)[:, :M], _r(K, N + (-N) % 8)[:, :N])}
    for lay, (a, b) in ops.items():
        A = Kn._operand([a], L.LAYOUT_RC if lay == "tn" else L.LAYOUT_KC)
        B = Kn._operand([b], L.LAYOUT_KC if lay == "nt" else L.LAYOUT_RC)
        af = a.float().T if lay == "tn" else a.float()
        bf = b.float().T if lay == "nt" else b.float()
        ref = af @ bf
        c = torch.full((M, N + (-N) % 8), 7.0, dtype=BF, device=cuda)
        Kn.gemm(M, N, K, A, B, [c[:, :N]], [0], c.stride(0), Kn._epi(alpha=0.5), variant=3)
        assert rel_l2(c[:, :N], 0.5 * ref) < 5e-3, lay
        assert bool((c[:, N:] == 7.0).all())
        c0 = c.clone()
        Kn.gemm(M, N, K, A, B, [c[:, :N]], [0], c.stride(0), Kn._epi(accumulate=True), variant=3)
        assert rel_l2(c[:, :N], c0[:, :N].float() + ref) < 5e-3, lay
        c2 = torch.empty(M, N + (-N) % 8, dtype=BF, device=cuda)[:, :N]
        Kn.gemm(M, N, K, A, B, [c2], [0], c2.stride(0), Kn._epi(), variant=3)
        c3 = torch.empty(M, N + (-N) % 8, dtype=BF, device=cuda)[:, :N]
        Kn.gemm(M, N, K, A, B, [c3], [0], c3.stride(0), Kn._epi(), variant=3)
        assert torch.equal(c2, c3) and rel_l2(c2, ref) < 5e-3, lay
    I = (N // 2 + 127) // 128 * 128
    x, wg, wu = _r(M, K), _r(I, K, scale=0.05), _r(I, K, scale=0.05)
    h, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
    try:
        Kn.gemm_variant = 3  # the GeGLU 4-wave kernel at any K
        Kn.linear_geglu_fwd(x, wg, wu, h, g, u)
    finally:
        Kn.gemm_variant = 0
    gr, ur = x.float() @ wg.float().T, x.float() @ wu.float().T
    assert rel_l2(g, gr) < 5e-3 and rel_l2(u, ur) < 5e-3
    # h from the kernel's own bf16 g, u: the epilogue's arithmetic exactly (bf16(gelu_tanh(g)) * u, rounded)
    hr = (F.gelu(g.float(), approximate="tanh").to(BF).float() * u.float()).to(BF)
    assert (h.float() - hr.float()).abs().max().item() <= 2 * hr.float().abs().max().item() * 2 ** -8
    assert rel_l2(h, F.gelu(gr, approximate="tanh") * ur) < 1e-2


def test_gemm_epilogues(cuda):
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(1)
    M, K, N = 300, 192, 264
    x, w, bias, res = _r(M, K), _r(N, K, scale=0.1), _r(N, scale=0.5), _r(M, N)
    acc = x.float() @ w.float().T
    y = torch.empty(M, N, dtype=BF, device=cuda)
    Kn.linear_fwd(x, [w], y, kind=L.EPI_BIAS, bias=bias, alpha=0.5)
    assert rel_l2(y, (acc + bias.float()) * 0.5) < 5e-3
    pre = torch.empty_like(y)
    Kn.linear_fwd(x, [w], y, kind=L.EPI_BIAS_GELU, bias=bias, out1=pre)
    assert rel_l2(pre, acc + bias.float()) < 5e-3
    assert rel_l2(y, F.gelu(acc + bias.float(), approximate="tanh")) < 1e-2
    Kn.linear_fwd(x, [w], y, kind=L.EPI_BIAS_RESID, bias=bias, in0=res)
    assert rel_l2(y, acc + bias.float() + res.float()) < 5e-3
    # accumulate
    y0 = y.clone()
    Kn.gemm(M, N, K, Kn._operand([x], L.LAYOUT_KC), Kn._operand([w], L.LAYOUT_KC), [y], [0], y.stride(0),
            Kn._epi(L.EPI_STORE, accumulate=True))
    assert rel_l2(y, y0.float() + acc) < 5e-3
    # GELU_BWD: C = acc * gelu'(pre)
    g = torch.empty_like(y)
    Kn.gemm(M, N, K, Kn._operand([x], L.LAYOUT_KC), Kn._operand([w], L.LAYOUT_KC), [g], [0], g.stride(0),
            Kn._epi(L.EPI_GELU_BWD, in0=pre))
    p = pre.float().requires_grad_(True)
    F.gelu(p, approximate="tanh").backward(acc)
    assert rel_l2(g, p.grad) < 1e-2


def test_gemm_segments_and_geglu(cuda):
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(2)
    M, K = 333, 256
    wq, wk, wv = _r(256, K, scale=0.1), _r(128, K, scale=0.1), _r(128, K, scale=0.1)
    x = _r(M, K)
    out = torch.empty(M, 512, dtype=BF, device=cuda)
    Kn.linear_fwd(x, [wq, wk, wv], out)
    ref = x.float() @ torch.cat([wq, wk, wv]).float().T
    assert rel_l2(out, ref) < 5e-3
    # dgrad over K segments and wgrad into C segments
    dy = _r(M, 512)
    dx = torch.empty(M, K, dtype=BF, device=cuda)
    Kn.linear_dgrad(dy, [wq, wk, wv], dx)
    assert rel_l2(dx, dy.float() @ torch.cat([wq, wk, wv]).float()) < 5e-3
    gs = [torch.empty_like(w) for w in (wq, wk, wv)]
    Kn.linear_wgrad(dy, x, gs)
    assert rel_l2(torch.cat(gs), dy.float().T @ x.float()) < 5e-3
    # GeGLU forward + backward epilogues
    I = 192
    wg, wu, wd = _r(I, K, scale=0.1), _r(I, K, scale=0.1), _r(K, I, scale=0.1)
    h, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
    Kn.linear_geglu_fwd(x, wg, wu, h, g, u)
    gr, ur = x.float() @ wg.float().T, x.float() @ wu.float().T
    assert rel_l2(g, gr) < 5e-3 and rel_l2(u, ur) < 5e-3
    assert rel_l2(h, F.gelu(gr, approximate="tanh") * ur) < 1e-2
    dout = _r(M, K)
    dgu = torch.empty(M, 2 * I, dtype=BF, device=cuda)
    Kn.linear_dgrad(dout, [wd], dgu[:, :I], kind=L.EPI_GEGLU_BWD, in0=g, in1=u, out1=dgu[:, :I], out2=dgu[:, I:])
    gg = g.float().requires_grad_(True)
    uu = u.float().requires_grad_(True)
    (F.gelu(gg, approximate="tanh") * uu).backward(dout.float() @ wd.float())
    assert rel_l2(dgu[:, :I], gg.grad) < 2e-2 and rel_l2(dgu[:, I:], uu.grad) < 2e-2


@pytest.mark.parametrize("M", [100, 1, 3, 8])  # M <= 8: the decode-step GEMV path
def test_gemm_softcap_ce(cuda, M):
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(3)
    K, V = 256, 1000
    h, w = _r(M, K), _r(V, K, scale=0.2)
    ldv = Kn.round_up(V, 64)
    buf = torch.empty(M, ldv, dtype=BF, device=cuda)
    ntn = Kn.ceil_div(V, 128)
    stats = torch.empty(M, ntn, 3, dtype=torch.float32, device=cuda)
    Kn.linear_fwd(h, [w], buf[:, :V], kind=L.EPI_SOFTCAP_CE, row_stats=stats, cap=30.0)
    ref = 30.0 * torch.tanh((h.float() @ w.float().T) / 30.0)
    assert rel_l2(buf[:, :V], ref) < 5e-3
    tgt = torch.randint(0, V, (M,), device=cuda)
    tgt[1::3] = -1
    lse, am = torch.empty(M, device=cuda), torch.empty(M, dtype=torch.int64, device=cuda)
    lr, lo = torch.empty(M, device=cuda), torch.empty(2, device=cuda)
    Kn.ce_finalize(V, ntn, stats, buf[:, :V], tgt, lse, am, lr, lo)
    y = buf[:, :V].float()
    assert torch.allclose(lse, torch.logsumexp(y, -1), atol=1e-3)
    assert torch.equal(am, y.argmax(-1))
    valid = tgt >= 0
    ref_loss = F.cross_entropy(y[valid], tgt[valid])
    assert abs(lo[0].item() - ref_loss.item()) < 1e-3 and lo[1].item() == valid.sum().item()
    d = torch.empty(M, ldv, dtype=BF, device=cuda)
    gscale = torch.tensor([1.0 / valid.sum().item()], device=cuda)
    Kn.ce_bwd(V, buf[:, :V], lse, tgt, 30.0, gscale, d)
    yy = y.clone().requires_grad_(True)
    F.cross_entropy(yy[valid], tgt[valid]).backward()
    ref_d = yy.grad * (1 - (y / 30.0) ** 2)
    assert rel_l2(d[:, :V], ref_d) < 1e-2
    assert d[:, V:].abs().sum().item() == 0


@pytest.mark.parametrize("M,V", [(300, 1000), (512, 30011), (9, 264)])
def test_softcap_ce_rows_matches_epilogue(cuda, M, V):
    """svla_softcap_ce_rows over plain-store logits == the SOFTCAP_CE GEMM epilogue bitwise: the softcapped logits
    and every row_stats entry {max, sumexp, argmax} (same 8-column chunks, same 16-lane group combine)."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(31)
    K = 256
    h, w = _r(M, K), _r(V, K, scale=0.3)
    ldv = Kn.round_up(V, 64)
    ntn = Kn.ceil_div(V, 128)
    fused = torch.empty(M, ldv, dtype=BF, device=cuda)
    st_f = torch.full((M, ntn, 3), float("nan"), device=cuda)
    Kn.linear_fwd(h, [w], fused[:, :V], kind=L.EPI_SOFTCAP_CE, row_stats=st_f, cap=30.0)
    raw = torch.empty(M, ldv, dtype=BF, device=cuda)
    Kn.linear_fwd(h, [w], raw[:, :V])
    st_r = torch.full((M, ntn, 3), float("nan"), device=cuda)
    Kn.softcap_ce_rows(raw, V, st_r, 30.0)
    assert torch.equal(raw[:, :V], fused[:, :V])
    assert torch.equal(st_r.view(torch.int32), st_f.view(torch.int32))


@pytest.mark.parametrize("M", [256, 4])  # 256: MFMA tile epilogue; 4: the decode GEMV path
def test_softcap_every_bf16_logit(cuda, M):
    """Every finite bf16 logit value through the SOFTCAP_CE epilogue (reciprocal-multiply divide, table tanh) against
    the reference's op-by-op bf16 softcap (modeling_gemma2.py:994-997: /cap, tanh, *cap, each cast to bf16) computed
    by torch in float64: bit-exact.  A = e_0 rows and B[n, 0] = value n, so C[m, n] = value n exactly."""
    from spatialvla_amd import kernels as Kn, _lib as L
    vals = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    vals = vals[torch.isfinite(vals.float())]
    V = vals.numel()
    ldv = Kn.round_up(V, 64)
    A = torch.zeros(M, 16, dtype=BF, device=cuda)
    A[:, 0] = 1.0
    B = torch.zeros(V, 16, dtype=BF, device=cuda)
    B[:, 0] = vals.to(cuda)
    buf = torch.empty(M, ldv, dtype=BF, device=cuda)
    stats = torch.empty(M, Kn.ceil_div(V, 128), 3, dtype=torch.float32, device=cuda)
    Kn.linear_fwd(A, [B], buf[:, :V], kind=L.EPI_SOFTCAP_CE, row_stats=stats, cap=30.0)
    x = vals.double() + 0.0  # the GEMM forms 0 + 1 * (-0.0) = +0.0
    ref = ((x / 30.0).to(torch.bfloat16).double().tanh().to(torch.bfloat16).double() * 30.0).to(torch.bfloat16)
    got = buf[:, :V].cpu()
    same = got.view(torch.int16) == ref.view(torch.int16)[None, :]
    assert bool(same.all()), (f"{int((~same).sum())} mismatches, e.g. {vals[~same[0]][:5].tolist()} -> "
                              f"{got[0][~same[0]][:5].tolist()} vs {ref[~same[0]][:5].tolist()}")


def test_softcap_rows_every_bf16_logit(cuda):
    """Every bf16 logit value (finite and +-inf) through svla_softcap_ce_rows in place -- the packed-pair table path of
    whole 16-B chunks and the scalar path of a ragged row end -- against the reference's op-by-op bf16 softcap
    (modeling_gemma2.py:994-997) in float64: bit-exact."""
    from spatialvla_amd import kernels as Kn
    vals = torch.arange(-32768, 32768, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    vals = vals[~torch.isnan(vals.float())]
    for V in (vals.numel(), vals.numel() - 3):  # ragged row ends: 2 and 7 values in the last 8-column chunk
        ldv = Kn.round_up(V, 64)
        buf = torch.zeros(2, ldv, dtype=BF, device=cuda)
        buf[:, :V] = vals[:V].to(cuda)
        stats = torch.empty(2, Kn.ceil_div(V, 128), 3, dtype=torch.float32, device=cuda)
        Kn.softcap_ce_rows(buf, V, stats, 30.0)
        x = vals[:V].double()
        ref = ((x / 30.0).to(torch.bfloat16).double().tanh().to(torch.bfloat16).double() * 30.0).to(torch.bfloat16)
        got = buf[:, :V].cpu()
        same = got.view(torch.int16) == ref.view(torch.int16)[None, :]
        assert bool(same.all()), (f"{int((~same).sum())} mismatches, e.g. {vals[:V][~same[0]][:5].tolist()} -> "
                                  f"{got[0][~same[0]][:5].tolist()} vs {ref[~same[0]][:5].tolist()}")


def test_softcap_rows_stats_special_values(cuda):
    """svla_softcap_ce_rows statistics where the full-range-table path hands a lane to the per-element path: NaN
    logits, groups whose maximum is +-0 (the max's sign follows the scan order), tied maxima (first index wins),
    +-inf and huge logits (saturate to +-cap), a ragged row end.  Softcapped values bit-exact against the reference's
    op-by-op bf16 softcap; per 128-column group max and first argmax exact, sum exp to 1e-5 (NaN where the group
    holds a NaN, as the in-order scan propagates it)."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(5)
    M, V = 48, 2048 + 5
    ldv = Kn.round_up(V, 64)
    raw = (torch.randn(M, V) * 8).to(BF)
    nan, inf = float("nan"), float("inf")
    raw[0, 5] = nan                                     # NaN in a chunk
    raw[1, 128:256] = -(torch.rand(128) * 4).to(BF)     # group max = 0 from both signs of zero
    raw[1, 130], raw[1, 200], raw[1, 131] = 0.0, -0.0, 0.0
    raw[2, 256:384] = -(torch.rand(128) * 4 + 1).to(BF)
    raw[2, 300], raw[2, 260] = -0.0, -0.0               # max -0 only
    raw[3, :128] = 2.5                                  # every value tied
    raw[4, 0:8] = torch.tensor([1.0, 7.0, 7.0, 3.0, 7.0, 0.5, 7.0, 2.0])  # ties inside one lane's chunk
    raw[4, 9], raw[4, 700] = 7.0, inf                   # tie in another lane; +inf saturates to cap
    raw[5, 3], raw[5, 4] = -inf, 1e30                   # -inf; huge -> cap
    raw[6, 512:640] = -inf                              # a whole group at -cap
    raw[7, V - 3] = nan                                 # NaN in the ragged end
    raw[8, V - 2] = 300.0                               # max in the ragged end
    buf = torch.zeros(M, ldv, dtype=BF, device=cuda)
    buf[:, :V] = raw.to(cuda)
    ntn = Kn.ceil_div(V, 128)
    stats = torch.empty(M, ntn, 3, dtype=torch.float32, device=cuda)
    Kn.softcap_ce_rows(buf, V, stats, 30.0)
    x = raw.double()
    y = ((x / 30.0).to(BF).double().tanh().to(BF).double() * 30.0).to(BF)
    got = buf[:, :V].cpu()
    same = (got.view(torch.int16) == y.view(torch.int16)) | (torch.isnan(got.float()) & torch.isnan(y.float()))
    assert bool(same.all()), f"{int((~same).sum())} softcap mismatches"
    st = stats.cpu()
    yf = y.float()
    for m in range(M):
        for g in range(ntn):
            seg = yf[m, g * 128:min(V, g * 128 + 128)]
            ok = ~torch.isnan(seg)
            mx = seg[ok].max()
            first = int(torch.nonzero(ok & (seg == mx))[0]) + g * 128
            se = float("nan") if not bool(ok.all()) else float(torch.exp(seg.double() - float(mx)).sum())
            assert float(st[m, g, 0]) == float(mx), (m, g, float(st[m, g, 0]), float(mx))
            assert int(st[m, g, 2].view(torch.int32)) == first, (m, g, int(st[m, g, 2].view(torch.int32)), first)
            if se != se:
                assert float(st[m, g, 1]) != float(st[m, g, 1]), (m, g)
            else:
                assert abs(float(st[m, g, 1]) - se) <= 1e-5 * se, (m, g, float(st[m, g, 1]), se)


@pytest.mark.parametrize("M,H,V,every", [(300, 256, 1000, 7), (9984 // 8, 2304, 4099, 24), (64, 128, 300, 0)])
def test_lm_head_ce_fn_label_rows(cuda, M, H, V, every):
    """LMHeadCEFn's backward runs the softmax gradient and both lm_head GEMMs over the labelled rows only;
    dh / dW must equal the dense fp32 reference (softcap 30, CE with ignored rows) -- including no label at
    all (every=0: zero gradients)."""
    from spatialvla_amd import functional as Fn, _lib as L
    torch.manual_seed(12)
    h = _r(M, H).requires_grad_(True)
    w = _r(V, H, scale=0.2).requires_grad_(True)
    tgt = torch.full((M,), -100, dtype=torch.int64, device=cuda)
    if every:
        tgt[::every] = torch.randint(0, V, (len(range(0, M, every)),), device=cuda)
    stash = {}
    logits, loss = Fn.LMHeadCEFn.apply(h, w, tgt, 30.0, stash)
    loss.backward()
    hf, wf = h.detach().float().requires_grad_(True), w.detach().float().requires_grad_(True)
    y = 30.0 * torch.tanh(hf @ wf.T / 30.0)
    valid = tgt >= 0
    if every:
        F.cross_entropy(y[valid], tgt[valid]).backward()
        assert rel_l2(h.grad, hf.grad) < 2e-2 and rel_l2(w.grad, wf.grad) < 2e-2
        assert h.grad[~valid].abs().sum().item() == 0
    else:
        assert h.grad.abs().sum().item() == 0 and w.grad.abs().sum().item() == 0


# ------------------------------------------------------------------------------------------ norms
def test_rmsnorm(cuda):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(4)
    R, N = 77, 2304
    x, w, res = _r(R, N), _r(N, scale=0.1), _r(R, N)
    y = torch.empty_like(x)
    rstd = torch.empty(R, device=cuda)
    Kn.rmsnorm_fwd(x, w, 1e-6, y, rstd)
    xf = x.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + wf)
    assert rel_l2(y, ref) < 5e-3
    dy = _r(R, N)
    ref.backward(dy.float())
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    Kn.rmsnorm_bwd(x, w, rstd, dy, None, dx, dw)
    assert rel_l2(dx, xf.grad) < 1e-2 and rel_l2(dw, wf.grad) < 1e-2
    h = torch.empty_like(x)
    Kn.add_rmsnorm_fwd(res, x, w, 1e-6, h, rstd)
    assert rel_l2(h, res.float() + ref.detach()) < 5e-3
    Kn.rmsnorm_bwd(x, w, rstd, dy, res, dx, None)
    assert rel_l2(dx, xf.grad + res.float()) < 1e-2


def _within_bf16_step(a, b):
    """|a - b| <= one bf16 step at b, elementwise (fp32 sums reassociated before the bf16 rounding)."""
    step = torch.finfo(torch.bfloat16).eps * b.float().abs().clamp_min(1e-30)
    return bool(((a.float() - b.float()).abs() <= step * 1.01).all())


@pytest.mark.parametrize("R,N,with_dres,acc", [(624, 2304, True, (False, False)), (77, 2304, False, (True, False)),
                                                (9, 4096, True, (False, False))])
def test_rmsnorm2_bwd_bitwise_two_calls(cuda, R, N, with_dres, acc):
    """svla_rmsnorm2_bwd (the norm pair's backward in one pass) gives dh and dy of two svla_rmsnorm_bwd calls bit
    for bit, with and without the residual gradient, accumulate modes equal or not; its weight-gradient partials
    cover 8 rows a block (16 in svla_rmsnorm_bwd), so dw agrees to fp32 reassociation: within one bf16 step."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(8)
    y, h, dx = _r(R, N), _r(R, N), _r(R, N)
    dres = _r(R, N) if with_dres else None
    w1, w2 = _r(N, scale=0.1), _r(N, scale=0.1)
    r1, r2 = torch.rand(R, device=cuda) + 0.5, torch.rand(R, device=cuda) + 0.5
    base1, base2 = _r(N), _r(N)
    dh0, dy0 = torch.empty_like(h), torch.empty_like(y)
    dw2_0, dw1_0 = base2.clone(), base1.clone()
    Kn.rmsnorm_bwd(h, w2, r2, dx, dres, dh0, dw2_0, dw_accumulate=acc[0])
    Kn.rmsnorm_bwd(y, w1, r1, dh0, None, dy0, dw1_0, dw_accumulate=acc[1])
    dh1, dy1 = torch.empty_like(h), torch.empty_like(y)
    dw2_1, dw1_1 = base2.clone(), base1.clone()
    Kn.rmsnorm2_bwd(h, w2, r2, dx, dres, y, w1, r1, dh1, dy1, dw2_1, dw1_1, acc[0], acc[1])
    torch.cuda.synchronize()
    for a, b, n in ((dh1, dh0, "dh"), (dy1, dy0, "dy")):
        assert torch.equal(a, b), n
    for a, b, n in ((dw2_1, dw2_0, "dw2"), (dw1_1, dw1_0, "dw1")):
        assert _within_bf16_step(a, b), n


def test_layernorm_colsum(cuda):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(5)
    R, N = 130, 1152
    x, w, b = _r(R, N), _r(N, scale=0.1) + 1, _r(N, scale=0.1)
    y = torch.empty_like(x)
    mu, rs = torch.empty(R, device=cuda), torch.empty(R, device=cuda)
    Kn.layernorm_fwd(x, w, b, 1e-6, y, mu, rs)
    xf, wf, bf = (t.float().requires_grad_(True) for t in (x, w, b))
    ref = F.layer_norm(xf, (N,), wf, bf, 1e-6)
    assert rel_l2(y, ref) < 5e-3
    dy = _r(R, N)
    ref.backward(dy.float())
    dx, dw, db = torch.empty_like(x), torch.empty_like(w), torch.empty_like(b)
    Kn.layernorm_bwd(x, w, mu, rs, dy, None, dx, dw, db)
    assert rel_l2(dx, xf.grad) < 1e-2 and rel_l2(dw, wf.grad) < 1e-2 and rel_l2(db, bf.grad) < 1e-2
    cs = torch.empty(N, dtype=BF, device=cuda)
    Kn.colsum_bf16(dy, cs)
    assert rel_l2(cs, dy.float().sum(0)) < 5e-3


@pytest.mark.parametrize("M,N,ld", [(8192, 1152, 3456), (8192, 4304, 4304), (624, 2304, 2304), (5, 8, 16)])
def test_colsum_single_pass(cuda, M, N, ld):
    """svla_colsum_bf16 / svla_colsum_f32 / svla_colsum2_f32 (one launch each): fp32 sums of strided bf16 and fp32
    matrices, accumulate into the bf16 output, bitwise reproducible run to run."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(6)
    x = _r(M, ld)[:, :N]
    out = torch.empty(N, dtype=BF, device=cuda)
    Kn.colsum_bf16(x, out)
    ref = x.float().sum(0)
    assert rel_l2(out, ref) < 5e-3
    again = torch.empty_like(out)
    Kn.colsum_bf16(x, again)
    assert torch.equal(out, again)
    base = _r(N)
    acc = base.clone()
    Kn.colsum_bf16(x, acc, accumulate=True)
    assert rel_l2(acc, ref + base.float()) < 5e-3
    part = torch.randn(2, M, N, device=cuda)
    o1 = torch.empty(N, dtype=BF, device=cuda)
    Kn.colsum_f32(part[0], o1)
    assert rel_l2(o1, part[0].sum(0)) < 5e-3
    o2a, o2b = torch.empty_like(o1), torch.empty_like(o1)
    L.check(L.lib().svla_colsum2_f32(M, N, part.data_ptr(), o2a.data_ptr(), o2b.data_ptr(), 0,
                                     torch.cuda.current_stream().cuda_stream), "colsum2")
    assert torch.equal(o2a, o1) and rel_l2(o2b, part[1].sum(0)) < 5e-3


# ------------------------------------------------------------------------------------------ attention
def _ref_attn(q, k, v, scale, cap, kv_class, window, cos=None, sin=None):
    """fp32 eager reference in [B, L, H, D] layout with per-key classes."""
    B, L, Hq, D = q.shape
    Hkv = k.shape[2]
    q, k, v = (t.float().transpose(1, 2) for t in (q, k, v))
    if cos is not None:
        c, s = torch.cat([cos, cos], -1).float(), torch.cat([sin, sin], -1).float()
        rh = lambda t: torch.cat((-t[..., D // 2:], t[..., :D // 2]), -1)  # noqa: E731
        q = q * c + rh(q) * s
        k = k * c + rh(k) * s
    k = k.repeat_interleave(Hq // Hkv, 1)
    v = v.repeat_interleave(Hq // Hkv, 1)
    s_ = q @ k.transpose(-1, -2) * scale
    if cap:
        s_ = cap * torch.tanh(s_ / cap)
    i = torch.arange(L, device=q.device)[:, None]
    j = torch.arange(L, device=q.device)[None, :]
    if kv_class is not None:
        c = kv_class[:, None, None, :].long()
        vis = (c == 0) | ((c == 1) & (j <= i))
    else:
        vis = torch.ones(1, 1, L, L, dtype=torch.bool, device=q.device)
    if window:
        vis = vis & ((i - j) < window)
    s_ = torch.where(vis, s_, torch.tensor(-3.3895313892515355e38, device=q.device))
    p = torch.softmax(s_, -1)
    return (p @ v).transpose(1, 2)


@pytest.mark.parametrize("ds", [True, False])
@pytest.mark.parametrize("D,Hq,Hkv,L,rope,cap", [(256, 2, 1, 140, True, 50.0), (256, 8, 4, 312, True, 50.0),
                                                 (256, 4, 1, 200, True, 50.0), (256, 3, 3, 100, True, 50.0),
                                                 (256, 2, 2, 65, False, 0.0),
                                                 (72, 2, 2, 256, False, 0.0), (72, 3, 3, 70, False, 0.0)])
def test_attention(cuda, D, Hq, Hkv, L, rope, cap, ds):
    """Forward and backward against the fp32 eager reference; head_dim 256 through both backward paths: dS stored
    by the dK/dV kernel and dQ = dS K (svla_attn_bwd_ds, ds=True, the product's) and the dQ kernel that recomputes
    S, P and dP (svla_attn_bwd)."""
    from spatialvla_amd import kernels as Kn
    if D != 256 and ds:
        pytest.skip("the stored-dS backward is the head_dim-256 path")
    Kn.ATTN_DS[0] = ds
    try:
        _attention_case(cuda, Kn, D, Hq, Hkv, L, rope, cap)
    finally:
        Kn.ATTN_DS[0] = True


def _attention_case(cuda, Kn, D, Hq, Hkv, L, rope, cap):
    torch.manual_seed(6)
    B = 2
    qkv = _r(B * L, (Hq + 2 * Hkv) * D)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    scale = 1 / 16 if D == 256 else D ** -0.5
    kv_class = None
    cos = sin = None
    if D == 256:
        P = L - 13
        kv_class = torch.zeros(B, L, dtype=torch.uint8, device=cuda)
        kv_class[:, P:] = 1
        kv_class[1, L - 3:] = 2
        if rope:
            inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
            f = (torch.arange(L, device=cuda).float() + 1)[:, None] * inv[None]
            cos, sin = f.cos().to(BF).contiguous(), f.sin().to(BF).contiguous()
    # q/k reach the kernels rotated (RoPE is the QKV GEMM's epilogue); the backward returns dq/dk w.r.t. the
    # pre-rotation q/k when given the tables
    qkv_in = qkv.clone()
    if cos is not None:
        nrot = (Hq + Hkv) * D
        qkv_in[:, :nrot] = _rope_bf16(qkv[:, :nrot].view(B, L, Hq + Hkv, D), cos, sin).view(B * L, nrot)
    qi_, ki_, vi_ = qkv_in[:, :Hq * D], qkv_in[:, Hq * D:(Hq + Hkv) * D], qkv_in[:, (Hq + Hkv) * D:]
    a = Kn.attn_args(B, L, Hq, Hkv, D, qi_, qkv.stride(0), ki_, qkv.stride(0), vi_, qkv.stride(0), scale, cap,
                     kv_class, 0)
    out = torch.empty(B * L, Hq * D, dtype=BF, device=cuda)
    lse = torch.empty(B, Hq, L, device=cuda)
    Kn.attn_fwd(a, out, lse)
    a = Kn.attn_args(B, L, Hq, Hkv, D, qi_, qkv.stride(0), ki_, qkv.stride(0), vi_, qkv.stride(0), scale, cap,
                     kv_class, 0, cos, sin)
    qr = q.view(B, L, Hq, D).float().requires_grad_(True)
    kr = k.view(B, L, Hkv, D).float().requires_grad_(True)
    vr = v.view(B, L, Hkv, D).float().requires_grad_(True)
    ref = _ref_attn(qr, kr, vr, scale, cap, kv_class, 0, cos, sin)
    assert rel_l2(out.view(B, L, Hq, D), ref) < 1e-2
    do = _r(B * L, Hq * D)
    ref.backward(do.view(B, L, Hq, D).float())
    dqkv = torch.empty_like(qkv)
    ld = dqkv.stride(0)
    Kn.attn_bwd(a, out, do, lse, dqkv[:, :Hq * D], ld, dqkv[:, Hq * D:(Hq + Hkv) * D], ld, dqkv[:, (Hq + Hkv) * D:], ld)
    assert rel_l2(dqkv[:, :Hq * D].view(B, L, Hq, D), qr.grad) < 2e-2
    assert rel_l2(dqkv[:, Hq * D:(Hq + Hkv) * D].view(B, L, Hkv, D), kr.grad) < 2e-2
    assert rel_l2(dqkv[:, (Hq + Hkv) * D:].view(B, L, Hkv, D), vr.grad) < 2e-2


@pytest.mark.parametrize("L,window", [(140, 0), (312, 100), (140, 48), (97, 0)])
def test_attention_d256_forward_window_and_classes(cuda, L, window):
    """head_dim-256 forward: sliding window, prefix / causal / never-visible key classes, a ragged last tile, and the
    lse it returns (log of the softcapped exp-sum) against fp32."""
    _d256_fwd_check(cuda, L, window)


def _d256_fwd_check(cuda, L, window):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(12)
    B, Hq, Hkv, D, cap, scale = 2, 4, 2, 256, 50.0, 1 / 16
    qkv = _r(B * L, (Hq + 2 * Hkv) * D, scale=2.0)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    cls = torch.zeros(B, L, dtype=torch.uint8, device=cuda)
    cls[:, L // 2:] = 1
    cls[0, 5:9] = 2
    cls[1, L - 4:] = 2
    a = Kn.attn_args(B, L, Hq, Hkv, D, q, qkv.stride(0), k, qkv.stride(0), v, qkv.stride(0), scale, cap, cls, window)
    out = torch.empty(B * L, Hq * D, dtype=BF, device=cuda)
    lse = torch.empty(B, Hq, L, device=cuda)
    Kn.attn_fwd(a, out, lse)
    torch.cuda.synchronize()
    ref = _ref_attn(q.view(B, L, Hq, D), k.view(B, L, Hkv, D), v.view(B, L, Hkv, D), scale, cap, cls, window)
    assert rel_l2(out.view(B, L, Hq, D), ref) < 1e-2
    qf, kf = q.view(B, L, Hq, D).float().transpose(1, 2), k.view(B, L, Hkv, D).float().transpose(1, 2)
    s_ = cap * torch.tanh(qf @ kf.repeat_interleave(Hq // Hkv, 1).transpose(-1, -2) * scale / cap)
    i, j = torch.arange(L, device=cuda)[:, None], torch.arange(L, device=cuda)[None, :]
    c = cls[:, None, None, :].long()
    vis = (c == 0) | ((c == 1) & (j <= i))
    if window:
        vis = vis & ((i - j) < window)
    lse_ref = torch.logsumexp(torch.where(vis, s_, torch.tensor(-1e30, device=cuda)), -1)
    assert (lse - lse_ref).abs().max() < 2e-2


def _rope_bf16(x, cos, sin):
    """Gemma2 apply_rotary_pos_emb in bf16 (modeling_gemma2.py:123-154): x [B, L, H, D] bf16, tables [L, D/2]."""
    c = torch.cat([cos, cos], -1)[None, :, None, :]
    s_ = torch.cat([sin, sin], -1)[None, :, None, :]
    h = x.shape[-1] // 2
    rot = torch.cat([-x[..., h:], x[..., :h]], -1)
    return (x * c) + (rot * s_)


@pytest.mark.parametrize("D,Hq,Hkv,L", [(256, 8, 4, 312), (16, 4, 1, 40)])
def test_gemm_rope_epilogue(cuda, D, Hq, Hkv, L):
    """SVLA_EPI_ROPE rotates q/k columns exactly as the reference's bf16 eager RoPE on the GEMM's own bf16
    output (bitwise), and leaves v columns alone."""
    from spatialvla_amd import kernels as Kn, _lib as L_
    torch.manual_seed(11)
    B, K = 3, 320
    N = (Hq + 2 * Hkv) * D
    x, w = _r(B * L, K), _r(N, K, scale=0.1)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    f = (torch.arange(L, device=cuda).float() + 1)[:, None] * inv[None]
    cos, sin = f.cos().to(BF).contiguous(), f.sin().to(BF).contiguous()
    nrot = (Hq + Hkv) * D
    # 0: product dispatch; 2: 8-phase kernel with the fused epilogue; 3: 4-wave kernel
    for v in ((0, 2, 3) if D == 256 else (0, 2)):
        try:
            Kn.gemm_variant = v
            plain = torch.empty(B * L, N, dtype=BF, device=cuda)
            Kn.linear_fwd(x, [w], plain)
            rot = torch.empty_like(plain)
            Kn.linear_fwd(x, [w], rot, kind=L_.EPI_ROPE, rope=(cos, sin, L, D, nrot))
            torch.cuda.synchronize()
        finally:
            Kn.gemm_variant = 0
        ref = plain.clone()
        ref[:, :nrot] = _rope_bf16(plain[:, :nrot].view(B, L, Hq + Hkv, D), cos, sin).view(B * L, nrot)
        assert torch.equal(rot, ref), v


def test_gemma2_attention_plugin_signature(cuda):
    """functional.gemma2_attention_forward as the reference's GEMMA2_ATTENTION_FUNCTION entry: same call
    (module, q, k, v, additive mask) and output layout as eager_attention_forward (modeling_gemma2.py:169-195)."""
    import types
    from spatialvla_amd.functional import gemma2_attention_forward
    torch.manual_seed(8)
    B, Hq, Hkv, L, D = 2, 8, 4, 130, 256
    q = _r(B * Hq * L, D).view(B, Hq, L, D).detach().requires_grad_(True)
    k = _r(B * Hkv * L, D).view(B, Hkv, L, D).detach().requires_grad_(True)
    v = _r(B * Hkv * L, D).view(B, Hkv, L, D).detach().requires_grad_(True)
    P = L - 13
    i = torch.arange(L, device=cuda)
    vis = (i[None, :] <= i[:, None]) | (i[None, :] < P)
    mask = torch.where(vis, 0.0, torch.finfo(BF).min).to(BF)[None, None].expand(B, 1, L, L).contiguous()
    mod = types.SimpleNamespace(scaling=1 / 16, attn_logit_softcapping=50.0, num_key_value_groups=2)
    out, w = gemma2_attention_forward(mod, q, k, v, mask, output_attentions=False)
    assert w is None and out.shape == (B, L, Hq, D) and out.is_contiguous()
    kv_class = torch.zeros(B, L, dtype=torch.uint8, device=cuda)
    kv_class[:, P:] = 1
    qr, kr, vr = (t.detach().transpose(1, 2).float().requires_grad_(True) for t in (q, k, v))
    ref = _ref_attn(qr, kr, vr, 1 / 16, 50.0, kv_class, 0, None, None)
    assert rel_l2(out, ref) < 1e-2
    do = _r(B * L, Hq * D).view(B, L, Hq, D)
    out.backward(do)
    ref.backward(do.float())
    assert rel_l2(q.grad.transpose(1, 2), qr.grad) < 2e-2
    assert rel_l2(k.grad.transpose(1, 2), kr.grad) < 2e-2
    assert rel_l2(v.grad.transpose(1, 2), vr.grad) < 2e-2


# ------------------------------------------------------------------------------------------ glue
def test_embed_merge(cuda):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(7)
    V, H, na, a0 = 600, 256, 64, 513
    emb, sp = _r(V, H), _r(na, H)
    ids = torch.randint(0, 512, (2, 40), device=cuda)
    ids[:, :10] = 512
    ids[:, 30:36] = torch.randint(a0, a0 + na, (2, 6), device=cuda)
    ids[1, 31] = ids[0, 30]
    img = _r(20, H)
    flat = ids.reshape(-1)
    m = flat == 512
    idx = torch.where(m, torch.cumsum(m.int(), 0) - 1, -1).int()
    out = torch.empty(flat.numel(), H, dtype=BF, device=cuda)
    Kn.embed_merge(flat, idx, emb, sp, a0, na, img, 16.0, out)
    ref = emb[flat].float()
    sel = (flat >= a0) & (flat < a0 + na)
    ref[sel] = sp[flat[sel] - a0].float()
    ref[m] = img.float()
    assert torch.equal(out, (ref.to(BF) * 16.0).to(BF))
    key = torch.where(sel, flat - a0, na)
    rows = torch.argsort(key, stable=True).int()
    cnt = torch.zeros(na + 1, dtype=torch.int32, device=cuda).scatter_add_(0, key, torch.ones_like(key, dtype=torch.int32))
    offs = torch.zeros(na + 2, dtype=torch.int32, device=cuda)
    offs[1:] = torch.cumsum(cnt, 0)
    dout = _r(flat.numel(), H)
    dsp, dimg = torch.empty_like(sp), torch.empty_like(img)
    Kn.embed_merge_bwd(flat, idx, rows, offs[:na + 1].contiguous(), na, dout, 16.0, dsp, dimg)
    ref_dsp = torch.zeros(na, H, device=cuda).index_add_(0, flat[sel] - a0, (dout[sel].float() * 16).to(BF).float())
    assert rel_l2(dsp, ref_dsp) < 5e-3
    assert rel_l2(dimg, dout[m].float() * 16) < 5e-3


def test_adamw_and_norm(cuda):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(8)
    n = 10007
    p = torch.randn(n, device=cuda)
    g = _r(n, scale=0.1)
    master, m, v = p.clone(), torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    pb = p.to(BF)
    ss = torch.empty(1, device=cuda)
    Kn.sumsq(g, ss, n_partial=64)
    assert abs(ss.item() - g.float().pow(2).sum().item()) / g.float().pow(2).sum().item() < 1e-4
    clip, nrm = torch.empty(1, device=cuda), torch.empty(1, device=cuda)
    Kn.clip_scale(ss, 0.5, clip, nrm)
    ref_p = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref_p], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    ref_p.grad = g.float() * clip
    opt.step()
    Kn.adamw(master, pb, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, 1, clip)
    assert torch.allclose(master, ref_p.detach(), atol=1e-6, rtol=1e-5)
    assert torch.equal(pb, master.to(BF))


@pytest.mark.parametrize("B,C,H,W,kw", [(2, 256, 24, 24, dict(scale_factor=2, align_corners=True)),
                                        (2, 128, 192, 192, dict(scale_factor=2, align_corners=True)),
                                        (3, 64, 17, 30, dict(size=(40, 33), align_corners=True)),
                                        (2, 32, 12, 20, dict(size=(24, 31), align_corners=False)),
                                        (1, 16, 9, 9, dict(scale_factor=2, align_corners=False))])
def test_upsample_bilinear_channels_last(cuda, B, C, H, W, kw):
    """svla_upsample_bilinear_nhwc reproduces torch's bilinear interpolate on channels-last bf16 maps bitwise
    (the ZoeDepth DPT neck resizes it replaces)."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(13)
    x = torch.randn(B, C, H, W, device=cuda).to(BF).contiguous(memory_format=torch.channels_last)
    ref = F.interpolate(x, mode="bilinear", **kw)
    out = Kn.upsample_bilinear_cl(x, **kw)
    assert out.shape == ref.shape
    assert torch.equal(out, ref)


def test_geglu_bwd_kernel_matches_epilogue(cuda):
    """svla_geglu_bwd (plain dH GEMM + one elementwise pass, the product path of GemmaMLPFn.backward) is
    bitwise equal to the GEGLU_BWD GEMM epilogue it replaced (same main loop, no stream-K: variant 2), in place."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(14)
    M, K, I = 1000, 320, 2048
    g, u = _r(M, I), _r(M, I)
    wd, dout = _r(K, I, scale=0.1), _r(M, K)
    try:
        Kn.gemm_variant = 2
        ref = torch.empty(M, 2 * I, dtype=BF, device=cuda)
        Kn.linear_dgrad(dout, [wd], ref[:, :I], kind=L.EPI_GEGLU_BWD, in0=g, in1=u, out1=ref[:, :I], out2=ref[:, I:])
        new = torch.empty(M, 2 * I, dtype=BF, device=cuda)
        Kn.linear_dgrad(dout, [wd], new[:, :I])
        Kn.geglu_bwd(new[:, :I], g, u, new[:, :I], new[:, I:])
        torch.cuda.synchronize()
    finally:
        Kn.gemm_variant = 0
    assert torch.equal(new, ref)
    dh = (dout.float() @ wd.float()).to(BF).float()
    gf, uf = g.float(), u.float()
    act = F.gelu(gf, approximate="tanh")
    gl = gf.clone().requires_grad_(True)
    F.gelu(gl, approximate="tanh").backward(torch.ones_like(gl))
    assert rel_l2(new[:, I:], dh * act) < 1e-2
    assert rel_l2(new[:, :I], (dh * uf) * gl.grad) < 1e-2


def test_inv3x3_closed_form(cuda):
    """svla_inv3x3_f32 vs torch.linalg.inv on scaled camera intrinsics (the backproject_patch inverse, reference
    modeling_spatialvla.py:221) and on random well-conditioned matrices: fp32 rounding only."""
    from spatialvla_amd import kernels as Kn, presets
    K0 = torch.tensor(presets.intrinsic_224(), dtype=torch.float32)
    Ks = torch.stack([K0, K0 * 1.5] + [torch.eye(3) + 0.3 * torch.randn(3, 3, generator=torch.Generator().manual_seed(i))
                                       for i in range(61)]).to(cuda)
    ref = torch.linalg.inv(Ks.double()).float()
    got = Kn.inv3x3(Ks)
    assert (got - ref).abs().max() <= 1e-5 * ref.abs().max()
    got_bf = Kn.inv3x3(K0.to(torch.bfloat16).to(cuda)[None])  # the model's bf16 intrinsic, upcast like K.float()
    assert torch.allclose(got_bf[0], torch.linalg.inv(K0.to(torch.bfloat16).float()).to(cuda), rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("M,N,K", [(300, 4304, 1152), (1024, 4096, 1024)])
def test_gelu_rows_matches_epilogues(cuda, M, N, K):
    """Bias GEMM + svla_gelu_rows == the fused BIAS_GELU / BIAS_GELU_ERF epilogues, and plain dgrad + the backward
    pass == the GELU_BWD epilogue, bit for bit.  Every GEMM here runs variant 2 (the 8-phase kernel, no stream-K):
    the dispatcher puts the plain and the fused epilogues on different kernels whose stream-K splits (and so fp32
    summation orders) differ, and the point is the epilogue arithmetic."""
    from spatialvla_amd import kernels as Kn, _lib as L
    Kn.gemm_variant = 2
    try:
        _gelu_rows_vs_epilogues(cuda, Kn, L, M, N, K)
    finally:
        Kn.gemm_variant = 0


def _gelu_rows_vs_epilogues(cuda, Kn, L, M, N, K):
    torch.manual_seed(41)
    x, w, b = _r(M, K), _r(N, K, scale=0.05), _r(N, scale=0.5)
    act_f, pre_f = torch.empty(M, N, dtype=BF, device=cuda), torch.empty(M, N, dtype=BF, device=cuda)
    Kn.linear_fwd(x, [w], act_f, kind=L.EPI_BIAS_GELU, bias=b, out1=pre_f)
    pre, act = torch.empty_like(pre_f), torch.empty_like(act_f)
    Kn.linear_fwd(x, [w], pre, kind=L.EPI_BIAS, bias=b)
    Kn.gelu_rows(Kn.GELU_TANH, pre, act)
    assert torch.equal(pre, pre_f) and torch.equal(act, act_f)
    erf_f = torch.empty_like(act_f)
    Kn.linear_fwd(x, [w], erf_f, kind=L.EPI_BIAS_GELU_ERF, bias=b)
    Kn.gelu_rows(Kn.GELU_ERF, pre, pre)
    assert torch.equal(pre, erf_f)
    dout, w2 = _r(M, K), _r(K, N, scale=0.05)
    d_f = torch.empty(M, N, dtype=BF, device=cuda)
    Kn.linear_dgrad(dout, [w2], d_f, kind=L.EPI_GELU_BWD, in0=pre_f)
    d = torch.empty_like(d_f)
    Kn.linear_dgrad(dout, [w2], d)
    Kn.gelu_rows(Kn.GELU_TANH_BWD, d, d, pre=pre_f)
    assert torch.equal(d, d_f)


@pytest.mark.parametrize("M,N,K", [(577, 3072, 1024), (256, 1152, 4304), (300, 200, 136)])
@pytest.mark.parametrize("layouts", ["nt", "nn", "tn"])
def test_gemm_tiny_tiles(cuda, M, N, K, layouts):
    """64x64 tiles of the sub-wave prefill grids (variant 9 = their dispatch; KC x KC only, the other layouts keep
    the 128x128 tiles) against fp32, plain store and the bias / bias+residual epilogues; the same values as the
    128x128 tiles (variant 1) within fp32 reordering."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(51)
    if layouts == "nt":
        a, b = _r(M, K), _r(N, K, scale=0.05)
        ref = a.float() @ b.float().T
        A, B = Kn._operand([a], L.LAYOUT_KC), Kn._operand([b], L.LAYOUT_KC)
    elif layouts == "nn":
        a, b = _r(M, K), _r(K, N + (-N) % 8, scale=0.05)[:, :N]
        ref = a.float() @ b.float()
        A, B = Kn._operand([a], L.LAYOUT_KC), Kn._operand([b], L.LAYOUT_RC)
    else:
        a, b = _r(K, M + (-M) % 8)[:, :M], _r(K, N + (-N) % 8, scale=0.05)[:, :N]
        ref = a.float().T @ b.float()
        A, B = Kn._operand([a], L.LAYOUT_RC), Kn._operand([b], L.LAYOUT_RC)
    bias, res = _r(N + (-N) % 8, scale=0.5)[:N], _r(M, N + (-N) % 8)[:, :N]
    outs = {}
    for v in (9, 1):
        c = torch.full((M, N + (-N) % 8), 7.0, dtype=BF, device=cuda)
        Kn.gemm(M, N, K, A, B, [c[:, :N]], [0], c.stride(0), Kn._epi(), variant=v)
        cb = torch.empty_like(c)
        Kn.gemm(M, N, K, A, B, [cb[:, :N]], [0], cb.stride(0), Kn._epi(L.EPI_BIAS_RESID, bias=bias, in0=res),
                variant=v)
        outs[v] = (c, cb)
    c, cb = outs[9]
    assert rel_l2(c[:, :N], ref) < 5e-3 and bool((c[:, N:] == 7.0).all())
    assert rel_l2(cb[:, :N], ref + bias.float() + res.float()) < 5e-3
    assert rel_l2(c[:, :N], outs[1][0][:, :N]) < 2e-3


@pytest.mark.parametrize("M", [600, 1024])
def test_gemm4_rope_paired_bitwise(cuda, M):
    """head_dim-256 RoPE on the paired-fragment 4-wave kernel (direct epilogue on interior tiles, LDS image on the
    ragged rows of M=600) == the 8-phase kernel's RoPE epilogue, bit for bit (q 8 heads | k 4 heads rotated, v not)."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(61)
    Kd, L_ = 512, 300
    x = _r(M, Kd)
    ws = [_r(2048, Kd, scale=0.05), _r(1024, Kd, scale=0.05), _r(1024, Kd, scale=0.05)]
    pos = torch.arange(1, L_ + 1, device=cuda).float()
    inv = 1.0 / (10000 ** (torch.arange(0, 256, 2, device=cuda).float() / 256))
    fr = pos[:, None] * inv[None]
    cos = torch.cat([fr.cos(), fr.cos()], -1).to(BF).contiguous()
    sin = torch.cat([fr.sin(), fr.sin()], -1).to(BF).contiguous()
    outs = {}
    for v in (3, 4):
        o = torch.empty(M, 4096, dtype=BF, device=cuda)
        try:
            Kn.gemm_variant = v
            Kn.linear_fwd(x, ws, o, kind=L.EPI_ROPE, rope=(cos, sin, L_, 256, 3072))
        finally:
            Kn.gemm_variant = 0
        outs[v] = o
    assert torch.equal(outs[3], outs[4])
    # against eager bf16 RoPE (rotate_half) on the bf16 projection
    y = (x.float() @ torch.cat(ws).float().T).to(BF).float()
    p = torch.arange(M, device=cuda) % L_
    c, s = cos.float()[p], sin.float()[p]
    ref = y.clone()
    for h in range(12):
        seg = y[:, 256 * h:256 * (h + 1)]
        rot = torch.cat([-seg[:, 128:], seg[:, :128]], -1)
        ref[:, 256 * h:256 * (h + 1)] = (seg * c).to(BF).float() + (rot * s).to(BF).float()
    assert rel_l2(outs[3], ref) < 5e-3


def _gelu_lut(cuda):
    """bf16 bits -> bf16 bits of the reference's gelu_tanh over all 65536 inputs (tools/gen_gelu_table.py's fp32 op
    sequence with a correctly rounded tanh; the kernels' band table + closed-form bands equal it exhaustively)."""
    import numpy as np
    from tools.gen_gelu_table import gelu_ref_bits
    lut = gelu_ref_bits(np.arange(65536, dtype=np.uint32)).astype(np.int32)
    return torch.from_numpy(lut).to(cuda)


def _apply_lut(lut, x):
    idx = x.contiguous().view(torch.int16).to(torch.int32) & 0xFFFF
    return (lut[idx.long()].to(torch.int16)).view(BF)


@pytest.mark.parametrize("M", [2048, 2085])  # interior 256 x 256 tiles (direct epilogue) / a ragged last row block
def test_geglu_gelu_table_bitwise(cuda, M):
    """Every bf16-input GELU(tanh) goes through the gelu table (svla_common.h gelu_bf16_lut): the GeGLU GEMM (4-wave
    direct epilogue from the LDS copy, LDS-path epilogue on edge tiles), the GEGLU_BWD recomputation of the
    activation, svla_geglu_bwd and svla_gelu_rows are bitwise bf16(lut(g) * u) / lut(x) of their own bf16 inputs;
    against torch's own F.gelu(approximate="tanh") (ROCm tanhf) the fraction of differing activations is printed and
    bounded."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(21)
    K, I = 512, 1024
    lut = _gelu_lut(cuda)
    x = _r(M, K)
    wg, wu = _r(I, K, scale=0.12), _r(I, K, scale=0.12)
    h, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
    Kn.linear_geglu_fwd(x, wg, wu, h, g, u)
    act = _apply_lut(lut, g)
    assert torch.equal(h, (act.float() * u.float()).to(BF))
    theirs = F.gelu(g.float(), approximate="tanh").to(BF)
    frac = (theirs != act).float().mean().item()
    print(f"gelu table vs torch F.gelu(tanh) on {g.numel()} GEMM outputs: differing {frac:.2e}")
    assert frac <= 1e-3
    # backward: svla_geglu_bwd's du = bf16(dh * act) with the same act
    dh = _r(M, I)
    dg, du = torch.empty_like(g), torch.empty_like(g)
    Kn.geglu_bwd(dh, g, u, dg, du)
    assert torch.equal(du, (dh.float() * act.float()).to(BF))
    # svla_gelu_rows mode 0
    y = torch.empty_like(g)
    Kn.gelu_rows(0, g, y)
    assert torch.equal(y, act)


@pytest.mark.parametrize("lay", ["nt", "nn"])
def test_gemm4_192_row_tiles(cuda, lay):
    """The 4-wave GEMM's 192-row tiles (launch4 picks them for forward projections of 9984 x 2304: 468 tiles instead
    of 351 on 256 CUs; nn = an input-gradient layout, which keeps the 256-row tiles): a K with a ragged last k-tile,
    STORE with alpha and accumulate (BIAS stays on the 256-row tiles), against torch in fp32 and against the same product at M = 9984 + 64 (not a multiple of 192:
    the 256-row kernel) row for row."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(31)
    M, N, K = 9984, 2304, 416
    a = _r(M + 64, K)
    if lay == "nt":
        w = _r(N, K, scale=0.1)
        B = Kn._operand([w], L.LAYOUT_KC)
        ref = a.float() @ w.float().T
    else:
        w = _r(K, N, scale=0.1)
        B = Kn._operand([w], L.LAYOUT_RC)
        ref = a.float() @ w.float()
    c = torch.empty(M, N, dtype=BF, device=cuda)
    Kn.gemm(M, N, K, Kn._operand([a[:M]], L.LAYOUT_KC), B, [c], [0], N, Kn._epi())
    big = torch.empty(M + 64, N, dtype=BF, device=cuda)
    Kn.gemm(M + 64, N, K, Kn._operand([a], L.LAYOUT_KC), B, [big], [0], N, Kn._epi())
    torch.cuda.synchronize()
    assert rel_l2(c, ref[:M]) < 5e-3
    # same k order in every tile shape (no stream-K at K = 416): bitwise the 256-row tiles' result
    assert torch.equal(c, big[:M])
    # alpha + accumulate, and BIAS
    c2 = c.clone()
    Kn.gemm(M, N, K, Kn._operand([a[:M]], L.LAYOUT_KC), B, [c2], [0], N, Kn._epi(alpha=0.5, accumulate=True))
    exp = (0.5 * c.float() + c.float()).to(BF)
    assert (c2.float() - exp.float()).abs().max().item() <= 2e-2 * c.float().abs().max().item()
    # BIAS keeps the 256-row tiles (LDS epilogue): the same values either way
    bias = _r(N)
    c3 = torch.empty_like(c)
    Kn.gemm(M, N, K, Kn._operand([a[:M]], L.LAYOUT_KC), B, [c3], [0], N, Kn._epi(L.EPI_BIAS, bias=bias))
    big3 = torch.empty_like(big)
    Kn.gemm(M + 64, N, K, Kn._operand([a], L.LAYOUT_KC), B, [big3], [0], N, Kn._epi(L.EPI_BIAS, bias=bias))
    assert torch.equal(c3, big3[:M]) and rel_l2(c3, ref[:M] + bias.float()) < 5e-3


@pytest.mark.parametrize("M,N,K", [(299, 2304, 9216), (256, 1152, 4304), (577, 1024, 4096), (37, 200, 1000),
                                   (300, 200, 136), (299, 4304, 2304)])
def test_gemm_deep_split(cuda, M, N, K):
    """The deep-pipelined small tiles (variants 10-12: 64x64, 64x128, 128x128 with NST-stage LDS rings) and their
    split-K forms (13-15: slabs + arrival counter, the last arriver sums the slabs in split order), and the short-M
    auto dispatch (variant 0) against fp32: plain store with ragged N (the columns past N untouched), bias+residual,
    GeGLU; the unsplit deep tiles bitwise the 128x128 data-parallel tiles (same k order); each split result
    reproduced bitwise by a second call (deterministic reduction order, counters reset by the reducer) and after a
    stream-K GEMM that shares the workspace's counters."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(71)
    a, b = _r(M, K), _r(N, K, scale=0.05)
    ref = a.float() @ b.float().T
    A, B = Kn._operand([a], L.LAYOUT_KC), Kn._operand([b], L.LAYOUT_KC)
    bias, res = _r(N + (-N) % 8, scale=0.5)[:N], _r(M, N + (-N) % 8)[:, :N]
    base = torch.empty(M, N + (-N) % 8, dtype=BF, device=cuda)
    Kn.gemm(M, N, K, A, B, [base[:, :N]], [0], base.stride(0), Kn._epi(), variant=1)
    # a stream-K launch on the same workspace (4-wave kernel, 9984 x 2304 x 4096 k-tiles: split tiles + counters)
    xs, ws_ = _r(2304, 4096), _r(2304, 4096, scale=0.05)
    ys = torch.empty(2304, 2304, dtype=BF, device=cuda)
    for v in (10, 11, 12, 13, 14, 15, 0):
        c = torch.full((M, N + (-N) % 8), 7.0, dtype=BF, device=cuda)
        Kn.gemm(M, N, K, A, B, [c[:, :N]], [0], c.stride(0), Kn._epi(), variant=v)
        assert rel_l2(c[:, :N], ref) < 5e-3, v
        assert bool((c[:, N:] == 7.0).all()), v
        if v in (10, 11, 12):
            assert torch.equal(c[:, :N], base[:, :N]), v
        Kn.linear_fwd(xs, [ws_], ys)
        c2 = torch.full_like(c, 7.0)
        Kn.gemm(M, N, K, A, B, [c2[:, :N]], [0], c2.stride(0), Kn._epi(), variant=v)
        assert torch.equal(c, c2), v
        cb = torch.empty_like(c)
        Kn.gemm(M, N, K, A, B, [cb[:, :N]], [0], cb.stride(0), Kn._epi(L.EPI_BIAS_RESID, bias=bias, in0=res),
                variant=v)
        assert rel_l2(cb[:, :N], ref + bias.float() + res.float()) < 5e-3, v
    if N % 64 == 0:  # GeGLU: gate rows [0, N/2), up rows [N/2, N) of the tile halves
        I = N // 2
        wg, wu = b[:I], b[I:]
        lut = _gelu_lut(cuda)
        for v in (10, 11, 12, 13, 14, 15, 0):
            h, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
            Kn.gemm_variant = v
            try:
                Kn.linear_geglu_fwd(a, wg, wu, h, g, u)
            finally:
                Kn.gemm_variant = 0
            assert rel_l2(g, ref[:, :I]) < 5e-3 and rel_l2(u, ref[:, I:]) < 5e-3, v
            assert torch.equal(h, (_apply_lut(lut, g).float() * u.float()).to(BF)), v


def test_gemm_deep_rope_pass_bitwise(cuda):
    """q|k|v + head_dim-256 RoPE at 299 rows on the 64x128 deep tiles (variant 11: product, then the in-place rope
    pass) == the 4-wave kernel's RoPE epilogue (variant 3), bit for bit; split-K (14) and the auto dispatch within
    fp32 reordering."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(73)
    M, Kd, L_ = 299, 2304, 299
    x = _r(M, Kd)
    ws = [_r(2048, Kd, scale=0.05), _r(1024, Kd, scale=0.05), _r(1024, Kd, scale=0.05)]
    pos = torch.arange(L_, device=cuda).float()
    inv = 1.0 / (10000 ** (torch.arange(0, 256, 2, device=cuda).float() / 256))
    fr = pos[:, None] * inv[None]
    cos, sin = fr.cos().to(BF).contiguous(), fr.sin().to(BF).contiguous()
    outs = {}
    for v in (3, 11, 14, 0):
        o = torch.empty(M, 4096, dtype=BF, device=cuda)
        try:
            Kn.gemm_variant = v
            Kn.linear_fwd(x, ws, o, kind=L.EPI_ROPE, rope=(cos, sin, L_, 256, 3072))
        finally:
            Kn.gemm_variant = 0
        outs[v] = o
    assert torch.equal(outs[3], outs[11])
    assert rel_l2(outs[14], outs[3]) < 2e-3 and rel_l2(outs[0], outs[3]) < 2e-3


@pytest.mark.parametrize("B,Lq", [(1, 299), (2, 37)])
def test_qkv_rope_fill_matches_rope_epilogue(cuda, B, Lq):
    """svla_qkv_rope_fill (the prefill: plain q|k|v GEMM, then q and k rotated in place and k / v written to cache
    rows 0..) == the GEMM's ROPE epilogue + copies of the k / v columns into the cache, bit for bit, per-sequence
    position tables (row b*Lq+t)."""
    from spatialvla_amd import kernels as Kn, _lib as L
    torch.manual_seed(81)
    Hq, Hkv, D, H, cap = 8, 4, 256, 512, 320
    qd, kd = Hq * D, Hkv * D
    M = B * Lq
    x = _r(M, H)
    ws = [_r(qd, H, scale=0.05), _r(kd, H, scale=0.05), _r(kd, H, scale=0.05)]
    pos = torch.cat([torch.arange(Lq, device=cuda) + 3 * b for b in range(B)]).float()
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    fr = pos[:, None] * inv[None]
    cos, sin = fr.cos().to(BF).contiguous(), fr.sin().to(BF).contiguous()
    ref = torch.empty(M, qd + 2 * kd, dtype=BF, device=cuda)
    Kn.linear_fwd(x, ws, ref, kind=L.EPI_ROPE, rope=(cos, sin, M, D, qd + kd))
    got = torch.empty_like(ref)
    Kn.linear_fwd(x, ws, got)
    kc = torch.full((B, cap, kd), 3.0, dtype=BF, device=cuda)
    vc = torch.full((B, cap, kd), 3.0, dtype=BF, device=cuda)
    Kn.qkv_rope_append(got, B, Lq, Hq, Hkv, D, cos, sin, kc, vc, 0, k_back=True)
    assert torch.equal(got, ref)
    assert torch.equal(kc[:, :Lq], ref[:, qd:qd + kd].view(B, Lq, kd))
    assert torch.equal(vc[:, :Lq], ref[:, qd + kd:].view(B, Lq, kd))
    assert bool((kc[:, Lq:] == 3.0).all()) and bool((vc[:, Lq:] == 3.0).all())
