"""KV-cached greedy decode: the decode attention kernel against an fp32 eager reference and
against the prefill flash kernel, and the cached predict_action / forward(past_key_values=...) against full
re-forwards on the same weights (reference generate path: model/modeling_spatialvla.py:440-492)."""
import os

import pytest
import torch
from safetensors.torch import load_file

import harness as H
from test_kernels_gpu import _r, _ref_attn

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.mark.parametrize("D,Hq,Hkv,Lk,Lq,window,cap", [
    (256, 8, 4, 300, 1, 0, 50.0),     # Gemma2-2B widths, one new token after a 299-token prompt
    (256, 8, 4, 303, 4, 0, 50.0),     # four new tokens at once (causal among themselves)
    (256, 2, 1, 560, 1, 0, 50.0),
    (256, 8, 2, 1000, 2, 0, 50.0),    # GQA group of 4
    (128, 2, 2, 77, 1, 16, 0.0),      # sliding window masks the far keys
    (64, 2, 1, 129, 3, 0, 0.0),
    (256, 8, 4, 9000, 1, 4096, 50.0),  # longer than the LDS-resident flash class array allows
    (256, 8, 4, 4500, 1, 4096, 50.0),  # past the Gemma2 sliding window
])
def test_attn_decode_kernel(cuda, D, Hq, Hkv, Lk, Lq, window, cap):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(11)
    B, cap_rows = 2, Lk + 7
    kd = Hkv * D
    kc = _r(B, cap_rows, kd)
    vc = _r(B, cap_rows, kd)
    qfull = _r(B, Lk, Hq * D)
    P = Lk - Lq - 5 if Lk - Lq - 5 > 0 else 0
    cls = torch.full((B, cap_rows), 2, dtype=torch.uint8, device=cuda)
    cls[:, :P] = 0
    cls[:, P:Lk] = 1
    cls[1, 3] = 2  # a padded prompt key
    q = qfull[:, Lk - Lq:].reshape(B * Lq, Hq * D).contiguous()
    out = torch.empty(B * Lq, Hq * D, dtype=BF, device=cuda)
    Kn.attn_decode(q, Lq, kc, vc, Lk, Hq, Hkv, D, 1 / 16, cap, cls, window, out)
    ref = _ref_attn(qfull.view(B, Lk, Hq, D), kc[:, :Lk].view(B, Lk, Hkv, D), vc[:, :Lk].view(B, Lk, Hkv, D),
                    1 / 16, cap, cls[:, :Lk], window)[:, Lk - Lq:]
    assert H.rel_l2(out.view(B, Lq, Hq, D), ref) < 1e-2
    if D == 256 and Lk <= 4608:
        # the same rows from the prefill flash kernel (what the uncached re-forward computes)
        qkv = torch.cat([qfull.view(B * Lk, -1), kc[:, :Lk].reshape(B * Lk, kd), vc[:, :Lk].reshape(B * Lk, kd)], 1)
        cls_l = cls[:, :Lk].contiguous()  # held: attn_args keeps only its pointer
        a = Kn.attn_args(B, Lk, Hq, Hkv, D, qkv[:, :Hq * D], qkv.stride(0), qkv[:, Hq * D:Hq * D + kd],
                         qkv.stride(0), qkv[:, Hq * D + kd:], qkv.stride(0), 1 / 16, cap, cls_l, window)
        full = torch.empty(B * Lk, Hq * D, dtype=BF, device=cuda)
        Kn.attn_fwd(a, full, torch.empty(B, Hq, Lk, device=cuda))
        rows = full.view(B, Lk, Hq * D)[:, Lk - Lq:].float()
        assert H.rel_l2(out.view(B, Lq, Hq * D), rows) < 5e-3


def test_attn_decode_rejects_bad_args(cuda):
    from spatialvla_amd import kernels as Kn
    kc = _r(1, 64, 256)
    q = _r(1, 3 * 256)  # Hq=3, Hkv=1: group 3 unsupported
    with pytest.raises(RuntimeError):
        Kn.attn_decode(q, 1, kc, kc, 10, 3, 1, 256, 1 / 16, 50.0, None, 0, torch.empty_like(q))


def _tiny_model(cuda):
    g = load_file(os.path.join(os.path.dirname(__file__), "golden", "tiny_train.safetensors"))
    model = H.build_hip_model(H.cfg_dict("tiny"), "cuda:0")
    depth = g["out.depth"].to(cuda)  # a device tensor: the captured prefill graph may not copy from the host
    model.predict_depth = lambda p: depth[:p.shape[0]]  # the golden's depth maps, one per image
    return model, g


def test_predict_action_cached_equals_uncached(cuda):
    """Greedy tokens of the KV-cached decode equal those of full re-forwards over prompt + generated tokens."""
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"][:, :-13]  # prompt only (prefix)
    inputs = {"input_ids": ids, "pixel_values": g["in.pixel_values"], "intrinsic": g["in.intrinsic"]}
    model.decode_graphs = False
    cached = model.predict_action(inputs, max_new_tokens=8, eos_token_id=-1)
    full = model.predict_action_uncached(inputs, max_new_tokens=8, eos_token_id=-1)
    assert cached.shape == (2, 8)
    assert torch.equal(cached, full), (cached, full)
    # the same steps replayed from captured HIP graphs: first call captures, second call replays
    model.decode_graphs = True
    g1 = model.predict_action(inputs, max_new_tokens=8, eos_token_id=-1)
    g2 = model.predict_action(inputs, max_new_tokens=8, eos_token_id=-1)
    assert torch.equal(g1, cached) and torch.equal(g2, cached)
    # new inputs of the same shape go through the same (replayed) prefill and decode graphs
    inputs2 = dict(inputs, pixel_values=inputs["pixel_values"].flip(-1))
    model.decode_graphs = False
    e3 = model.predict_action(inputs2, max_new_tokens=8, eos_token_id=-1)
    model.decode_graphs = True
    g3 = model.predict_action(inputs2, max_new_tokens=8, eos_token_id=-1)
    assert torch.equal(g3, e3)


def test_predict_action_image_token_mismatch_raises(cuda):
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"][:, :-13].clone()
    ids[0, 0] = 2  # one image token fewer than image features
    with pytest.raises(ValueError):
        model.predict_action({"input_ids": ids, "pixel_values": g["in.pixel_values"],
                              "intrinsic": g["in.intrinsic"]}, max_new_tokens=2, eos_token_id=-1)


def test_predict_action_eos_pads_finished(cuda):
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"][:, :-13]
    inputs = {"input_ids": ids, "pixel_values": g["in.pixel_values"], "intrinsic": g["in.intrinsic"]}
    free = model.predict_action(inputs, max_new_tokens=4, eos_token_id=-1)
    eos = int(free[0, 1])  # make sequence 0 finish at its second token
    out = model.predict_action(inputs, max_new_tokens=4, eos_token_id=eos)
    ref = model.predict_action_uncached(inputs, max_new_tokens=4, eos_token_id=eos)
    assert torch.equal(out, ref)
    assert out[0, 1] == eos and bool((out[0, 2:] == max(model.pad_token_id, 0)).all())
    # every row finished: the output stops at the token where the last row finished, as the step-by-step loop,
    # although the device-side loop only looks at the finished flags every EOS_CHECK_EVERY steps
    one = {k: v[:1] for k, v in inputs.items()}
    free1 = model.predict_action(one, max_new_tokens=12, eos_token_id=-1)
    eos1 = int(free1[0, 1])
    ref1 = model.predict_action_uncached(one, max_new_tokens=12, eos_token_id=eos1)
    assert ref1.shape[1] <= 2
    for graphs in (True, False):
        model.decode_graphs = graphs
        out1 = model.predict_action(one, max_new_tokens=12, eos_token_id=eos1)
        assert torch.equal(out1, ref1), (graphs, out1, ref1)
    model.decode_graphs = True


def test_forward_past_key_values_matches_reforward(cuda):
    """forward(use_cache=True) then forward(past_key_values=cache) on two more tokens gives the logits of a full
    forward whose appended tokens see the prompt and earlier tokens only (the HybridCache decode semantics)."""
    from spatialvla_amd.modeling_gemma2 import Gemma2KVCache, KVMask
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"].to(cuda)
    B, L = ids.shape
    P = L - 13
    pv, intr = g["in.pixel_values"].to(cuda), g["in.intrinsic"].to(cuda)
    with torch.no_grad():
        o1 = model(input_ids=ids[:, :P], pixel_values=pv, intrinsic=intr, use_cache=True)
        cache = o1.past_key_values
        assert isinstance(cache, Gemma2KVCache) and cache.get_seq_length() == P
        o2 = model(input_ids=ids[:, P:P + 1], past_key_values=cache)
        o3 = model(input_ids=ids[:, P + 1:P + 3], past_key_values=cache)
        assert cache.get_seq_length() == P + 3
        cls = torch.ones(B, P + 3, dtype=torch.uint8, device=cuda)
        cls[:, :P] = 0
        ref = model(input_ids=ids[:, :P + 3], pixel_values=pv, intrinsic=intr, kv_mask=KVMask(cls)).logits
    assert H.rel_l2(o1.logits, ref[:, :P]) < H.LOGITS_TOL  # prompt rows never see the appended tokens
    assert H.rel_l2(o2.logits, ref[:, P:P + 1]) < H.LOGITS_TOL
    assert H.rel_l2(o3.logits, ref[:, P + 1:P + 3]) < H.LOGITS_TOL
    assert torch.equal(o3.logits.float().argmax(-1), ref[:, P + 1:P + 3].float().argmax(-1))


# ------------------------------------------------------------------ small-M GEMMs of the decode step (GEMV path)
@pytest.mark.parametrize("M,N,K", [(1, 2048, 2304), (3, 2304, 9216), (8, 4096, 2304), (2, 265347 // 64 * 64, 512)])
def test_gemv_store(cuda, M, N, K):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(3)
    x, w = _r(M, K), _r(N, K, scale=0.05)
    out = torch.empty(M, N, dtype=BF, device=cuda)
    Kn.linear_fwd(x, [w], out)
    ref = x.float() @ w.float().t()
    assert H.rel_l2(out, ref) < 1e-2
    # the bf16 result matches the MFMA path on the same rows (equal up to fp32 summation order)
    big = torch.empty(64, N, dtype=BF, device=cuda)
    Kn.linear_fwd(torch.cat([x, _r(64 - M, K)]), [w], big)
    assert (out.float() - big[:M].float()).abs().max() <= 2 ** -6 * ref.abs().max()


@pytest.mark.parametrize("M", [1, 2, 5])
def test_gemv_geglu(cuda, M):
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(4)
    K, I = 2304, 1024
    x, wg, wu = _r(M, K), _r(I, K, scale=0.05), _r(I, K, scale=0.05)
    h, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
    Kn.linear_geglu_fwd(x, wg, wu, h, g, u)
    g_ref = (x.float() @ wg.float().t()).to(BF)
    u_ref = (x.float() @ wu.float().t()).to(BF)
    h_ref = (torch.nn.functional.gelu(g_ref.float(), approximate="tanh").to(BF).float() * u_ref.float())
    assert H.rel_l2(g, g_ref) < 1e-2 and H.rel_l2(u, u_ref) < 1e-2
    assert H.rel_l2(h, h_ref) < 1e-2
    # h is exactly the fused epilogue's rounding applied to the kernel's own g, u
    h_own = (torch.nn.functional.gelu(g.float(), approximate="tanh").to(BF).float() * u.float()).to(BF)
    assert (h.float() - h_own.float()).abs().max() <= 1e-2 * h_own.float().abs().max()


@pytest.mark.parametrize("M", [1, 4])
def test_gemv_rope(cuda, M):
    """The decode-step QKV projection: GEMV store + in-place RoPE pass, bitwise the reference bf16 RoPE applied
    to the GEMV's own output."""
    from spatialvla_amd import kernels as Kn, _lib as L_
    from test_kernels_gpu import _rope_bf16
    torch.manual_seed(5)
    D, Hq, Hkv, K = 256, 8, 4, 2304
    N = (Hq + 2 * Hkv) * D
    nrot = (Hq + Hkv) * D
    x, w = _r(M, K), _r(N, K, scale=0.05)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    f = (torch.arange(300, 300 + M, device=cuda).float() + 1)[:, None] * inv[None]
    cos, sin = f.cos().to(BF).contiguous(), f.sin().to(BF).contiguous()
    plain = torch.empty(M, N, dtype=BF, device=cuda)
    Kn.linear_fwd(x, [w], plain)
    rot = torch.empty_like(plain)
    Kn.linear_fwd(x, [w], rot, kind=L_.EPI_ROPE, rope=(cos, sin, M, D, nrot))
    ref = plain.clone()
    ref[:, :nrot] = _rope_bf16(plain[:, :nrot].view(1, M, Hq + Hkv, D), cos, sin).view(M, nrot)
    assert torch.equal(rot, ref)
    # q, k, v weights in three separate tensors (a B operand of 3 segments) give the same bits
    wq, wk, wv = (t.clone() for t in torch.split(w, [Hq * D, Hkv * D, Hkv * D]))
    seg = torch.empty_like(plain)
    Kn.linear_fwd(x, [wq, wk, wv], seg, kind=L_.EPI_ROPE, rope=(cos, sin, M, D, nrot))
    assert torch.equal(seg, ref)


@pytest.mark.parametrize("B,Lq,p0", [(1, 1, 299), (2, 3, 17)])
def test_qkv_rope_append(cuda, B, Lq, p0):
    """Decode-step q|k|v epilogue: bitwise the reference bf16 RoPE on q (in place) and k, k/v in cache rows p0.."""
    from spatialvla_amd import kernels as Kn
    from test_kernels_gpu import _rope_bf16
    torch.manual_seed(8)
    Hq, Hkv, D, cap = 8, 4, 256, p0 + Lq + 5
    kd = Hkv * D
    qkv = _r(B * Lq, (Hq + 2 * Hkv) * D)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    # per-sequence positions (a padded batch: sequence b is 3b tokens shorter), table row b*Lq+t
    pos = torch.cat([torch.arange(p0, p0 + Lq, device=cuda) - 3 * b for b in range(B)]).float() + 1
    f = pos[:, None] * inv[None]
    cos, sin = f.cos().to(BF).contiguous(), f.sin().to(BF).contiguous()
    kc = torch.zeros(B, cap, kd, dtype=BF, device=cuda)
    vc = torch.zeros_like(kc)
    ref = qkv.clone()
    nrot = (Hq + Hkv) * D
    for b in range(B):
        rows = slice(b * Lq, (b + 1) * Lq)
        ref[rows, :nrot] = _rope_bf16(qkv[rows, :nrot].view(1, Lq, Hq + Hkv, D), cos[rows], sin[rows]).reshape(Lq, nrot)
    Kn.qkv_rope_append(qkv, B, Lq, Hq, Hkv, D, cos, sin, kc, vc, p0)
    assert torch.equal(qkv[:, :Hq * D], ref[:, :Hq * D])
    assert torch.equal(kc[:, p0:p0 + Lq].reshape(B * Lq, kd), ref[:, Hq * D:nrot])
    assert torch.equal(vc[:, p0:p0 + Lq].reshape(B * Lq, kd), ref[:, nrot:])
    assert kc[:, :p0].abs().sum() == 0 and kc[:, p0 + Lq:].abs().sum() == 0


@pytest.mark.parametrize("B,Lq,p0,Hq,Hkv,D,window,use_cls", [
    (1, 1, 299, 8, 4, 256, 0, True), (2, 3, 61, 8, 4, 256, 0, True), (1, 1, 64, 8, 4, 256, 4096, True),
    (2, 2, 130, 4, 4, 128, 50, False), (1, 1, 7, 8, 2, 64, 0, False)])
def test_attn_decode_rope_fused_bitwise(cuda, B, Lq, p0, Hq, Hkv, D, window, use_cls):
    """svla_attn_decode_rope (one launch: RoPE + cache append + split + in-launch combine) equals
    svla_qkv_rope_append + svla_attn_decode bit for bit: output and both caches; repeated launches reuse the
    zeroed-once workspace (its counters come back to zero)."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(10)
    kd, Lk = Hkv * D, p0 + Lq
    cap = Lk + 9
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=cuda).float() / D))
    pos = torch.cat([torch.arange(p0, p0 + Lq, device=cuda) - 2 * b for b in range(B)]).float() + 1
    f = pos[:, None] * inv[None]
    emb = torch.cat([f, f], -1)  # HF layout [B*Lq, D] (the kernels read the first D/2 columns of row b*Lq+t)
    cos, sin = emb.cos().to(BF).contiguous(), emb.sin().to(BF).contiguous()
    kc0 = _r(B, cap, kd)
    vc0 = _r(B, cap, kd)
    cls = None
    if use_cls:
        cls = torch.zeros(B, cap, dtype=torch.uint8, device=cuda)
        cls[:, p0 - 3:] = 1
        cls[-1, 5:9] = 2
    for rep in range(3):
        qkv = _r(B * Lq, (Hq + 2 * Hkv) * D, scale=2.0)
        kc1, vc1, kc2, vc2 = kc0.clone(), vc0.clone(), kc0.clone(), vc0.clone()
        ref, out = torch.empty(B * Lq, Hq * D, dtype=BF, device=cuda), torch.empty(B * Lq, Hq * D, dtype=BF, device=cuda)
        q2 = qkv.clone()
        Kn.qkv_rope_append(q2, B, Lq, Hq, Hkv, D, cos, sin, kc1, vc1, p0)
        Kn.attn_decode(q2[:, :Hq * D], Lq, kc1, vc1, Lk, Hq, Hkv, D, 1 / 16, 50.0, cls, window, ref)
        Kn.attn_decode_rope(qkv, Lq, cos, sin, kc2, vc2, Lk, Hq, Hkv, D, 1 / 16, 50.0, cls, window, out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), rep
        assert torch.equal(kc2, kc1) and torch.equal(vc2, vc1), rep
    ws = Kn._DECODE_WS[(qkv.device.index, Kn._stream())]
    assert int(ws[:256].count_nonzero()) == 0  # the arrival counters are back to zero


def test_attn_decode_rope_rejects_bad_args(cuda):
    from spatialvla_amd import kernels as Kn
    qkv = _r(1, 16 * 256)
    kc = _r(1, 32, 4 * 256)
    cos = _r(1, 256)
    with pytest.raises(Exception):  # Lk must exceed Lq (a cached prefix)
        Kn.attn_decode_rope(qkv, 1, cos, cos, kc, kc, 1, 8, 4, 256, 1 / 16, 50.0, None, 0, _r(1, 8 * 256))
    with pytest.raises(Exception):  # GQA group 3
        kc3 = _r(1, 32, 3 * 256)
        Kn.attn_decode_rope(_r(1, 15 * 256), 1, cos, cos, kc3, kc3, 10, 9, 3, 256, 1 / 16, 50.0, None, 0,
                            _r(1, 9 * 256))


@pytest.mark.parametrize("rows", [1, 3, 299])
def test_add_rmsnorm2_bitwise(cuda, rows):
    """The fused residual-add + two chained RMSNorms equals the two separate norm kernels bit for bit."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(9)
    N = 2304
    res, y = _r(rows, N), _r(rows, N, scale=3.0)
    w1, w2 = _r(N, scale=0.3), _r(N, scale=0.3)
    h_ref, x_ref = torch.empty_like(res), torch.empty_like(res)
    rstd = torch.empty(rows, device=cuda)
    Kn.add_rmsnorm_fwd(res, y, w1, 1e-6, h_ref, rstd)
    Kn.rmsnorm_fwd(h_ref, w2, 1e-6, x_ref, rstd)
    h, x = torch.empty_like(res), torch.empty_like(res)
    Kn.add_rmsnorm2_fwd(res, y, w1, w2, 1e-6, 1e-6, h, x)
    assert torch.equal(h, h_ref) and torch.equal(x, x_ref)


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("geglu", [False, True])
def test_gemv_rmsnorm2_bitwise(cuda, M, geglu):
    """svla_gemv_rmsnorm2 == svla_add_rmsnorm2_fwd followed by the decode GEMV, bit for bit: h, and the q|k|v
    (three weight segments) or gate|up GeGLU outputs."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(17)
    N = 2304
    res, y = _r(M, N), _r(M, N, scale=3.0)
    w1, w2 = _r(N, scale=0.3), _r(N, scale=0.3)
    h_ref, x_ref = torch.empty_like(res), torch.empty_like(res)
    Kn.add_rmsnorm2_fwd(res, y, w1, w2, 1e-6, 1e-6, h_ref, x_ref)
    h = torch.full_like(res, 7.0)
    if geglu:
        I = 9216
        wg, wu = _r(I, N, scale=0.02), _r(I, N, scale=0.02)
        ref = [torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3)]
        Kn.linear_geglu_fwd(x_ref, wg, wu, *ref)
        out = [torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3)]
        Kn.gemv_rmsnorm2(res, y, w1, w2, 1e-6, 1e-6, h, [wg, wu], out[0], geglu_out=(out[1], out[2]))
        for a, b in zip(out, ref):
            assert torch.equal(a, b)
    else:
        ws = [_r(2048, N, scale=0.02), _r(1024, N, scale=0.02), _r(1024, N, scale=0.02)]
        ref = torch.empty(M, 4096, dtype=BF, device=cuda)
        Kn.linear_fwd(x_ref, ws, ref)
        out = torch.empty_like(ref)
        Kn.gemv_rmsnorm2(res, y, w1, w2, 1e-6, 1e-6, h, ws, out)
        assert torch.equal(out, ref)
    assert torch.equal(h, h_ref)


@pytest.fixture(params=["coop", "plain"])
def dm_launch_mode(request):
    """svla_decode_mlp launched cooperatively (the default) or with a plain launch (SVLA_DECODE_MLP_COOP=0)."""
    from spatialvla_amd import _lib as L
    L.lib().svla_decode_mlp_debug(0, 1 if request.param == "coop" else 0, 1000)
    yield request.param
    L.lib().svla_decode_mlp_debug(0, -1, 1000)


@pytest.mark.parametrize("M,H,I,KO", [(1, 2304, 9216, 2048), (3, 2304, 9216, 0), (8, 2304, 9216, 2048),
                                      (2, 256, 520, 0), (2, 256, 520, 264)])
def test_decode_mlp_persistent_bitwise(cuda, M, H, I, KO, dm_launch_mode):
    """svla_decode_mlp (one persistent launch: norm pair + gate|up GeGLU GEMV, grid barrier, down GEMV) == the
    two-launch path (svla_gemv_rmsnorm2 GEGLU, then the small-M down GEMV), bit for bit: h, act and out -- over
    repeated launches (the grid barrier's words are reused) and a ragged shape (fewer blocks than CUs).  KO > 0: the
    o projection y = attn @ wo^T inside the same launch (a second barrier), bitwise the small-M GEMV."""
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(23)
    res, y = _r(M, H), _r(M, H, scale=3.0)
    if KO:
        attn, wo = _r(M, KO), _r(H, KO, scale=0.05)
        Kn.linear_fwd(attn, [wo], y)
    w1, w2 = _r(H, scale=0.3), _r(H, scale=0.3)
    wg, wu, wd = _r(I, H, scale=0.02), _r(I, H, scale=0.02), _r(H, I, scale=0.02)
    h_ref = torch.empty_like(res)
    act_ref, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
    Kn.gemv_rmsnorm2(res, y, w1, w2, 1e-6, 1e-6, h_ref, [wg, wu], act_ref, geglu_out=(g, u))
    out_ref = torch.empty(M, H, dtype=BF, device=cuda)
    Kn.linear_fwd(act_ref, [wd], out_ref)
    t0 = Kn.decode_mlp_timeouts()
    for rep in range(3):
        h, act, out = torch.full_like(res, 7.0), torch.full_like(act_ref, 7.0), torch.full_like(out_ref, 7.0)
        if KO:
            y2 = torch.full_like(y, 7.0)
            Kn.decode_mlp(res, y2, w1, w2, 1e-6, 1e-6, h, wg, wu, wd, act, out, o=(attn, wo))
            assert torch.equal(y2, y), rep
        else:
            Kn.decode_mlp(res, y, w1, w2, 1e-6, 1e-6, h, wg, wu, wd, act, out)
        assert Kn.decode_mlp_timeouts() == t0
        assert torch.equal(h, h_ref), rep
        assert torch.equal(act, act_ref), rep
        assert torch.equal(out, out_ref), rep


def test_decode_mlp_grid_is_occupancy_capped(cuda):
    """The persistent grid never exceeds what can be resident at once: DM_BPC (2) blocks per CU at most, fewer when the
    instance's LDS (M x H bf16) or registers allow fewer, and I / 4 for small layers."""
    from spatialvla_amd import kernels as Kn
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = Kn.decode_mlp_grid(1, 2304, 9216)
    assert 0 < g <= 2 * cus
    assert Kn.decode_mlp_grid(8, 2304, 9216) <= 2 * cus
    assert Kn.decode_mlp_grid(2, 256, 520) == 130


def test_decode_mlp_oversubscribed_grid_fails_loudly(cuda):
    """A grid that can not be co-resident never yields silent numbers: launched cooperatively the runtime
    refuses it (an error, nothing runs); launched plainly, the blocks that miss the grid barrier count a timeout after
    their bounded wait (50 ms here) and write NaN, check_decode_mlp_timeouts() raises, and the barrier words are back at
    zero so the next launch is bitwise the two-launch path again."""
    from spatialvla_amd import _lib as L
    from spatialvla_amd import kernels as Kn
    torch.manual_seed(29)
    M, H, I = 1, 256, 520
    res, y = _r(M, H), _r(M, H, scale=3.0)
    w1, w2 = _r(H, scale=0.3), _r(H, scale=0.3)
    wg, wu, wd = _r(I, H, scale=0.02), _r(I, H, scale=0.02), _r(H, I, scale=0.02)
    h_ref = torch.empty_like(res)
    act_ref, g, u = (torch.empty(M, I, dtype=BF, device=cuda) for _ in range(3))
    Kn.gemv_rmsnorm2(res, y, w1, w2, 1e-6, 1e-6, h_ref, [wg, wu], act_ref, geglu_out=(g, u))
    out_ref = torch.empty(M, H, dtype=BF, device=cuda)
    Kn.linear_fwd(act_ref, [wd], out_ref)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    big = 32 * cus  # 8192 blocks of 256 threads: more than 32 waves per CU can hold
    Kn.check_decode_mlp_timeouts()  # earlier launches: nothing pending
    lib = L.lib()
    try:
        lib.svla_decode_mlp_debug(big, 1, 50)
        h, act, out = torch.empty_like(res), torch.empty_like(act_ref), torch.empty_like(out_ref)
        with pytest.raises(L.SvlaError):
            Kn.decode_mlp(res, y, w1, w2, 1e-6, 1e-6, h, wg, wu, wd, act, out)
        torch.cuda.synchronize()
        lib.svla_decode_mlp_debug(big, 0, 50)
        out.fill_(7.0)
        Kn.decode_mlp(res, y, w1, w2, 1e-6, 1e-6, h, wg, wu, wd, act, out)
        torch.cuda.synchronize()
        assert Kn.decode_mlp_timeouts() > 0
        assert torch.isnan(out.float()).any()
        with pytest.raises(RuntimeError, match="missed a grid barrier"):
            Kn.check_decode_mlp_timeouts()
    finally:
        lib.svla_decode_mlp_debug(0, -1, 1000)
    h, act, out = torch.empty_like(res), torch.empty_like(act_ref), torch.empty_like(out_ref)
    Kn.decode_mlp(res, y, w1, w2, 1e-6, 1e-6, h, wg, wu, wd, act, out)
    Kn.check_decode_mlp_timeouts()
    assert torch.equal(out, out_ref) and torch.equal(act, act_ref) and torch.equal(h, h_ref)


def test_decode_mlp_persistent_graph_tokens(cuda):
    """predict_action (graph-replayed decode steps) gives the same tokens and logits with the persistent decode MLP
    as with the two-launch MLP."""
    from spatialvla_amd import functional as Fn
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"][:, :-13]
    inputs = {"input_ids": ids, "pixel_values": g["in.pixel_values"], "intrinsic": g["in.intrinsic"]}
    outs = {}
    keep = Fn.DECODE_MLP_PERSIST[0]
    try:
        for persist in (False, True):
            Fn.DECODE_MLP_PERSIST[0] = persist  # (with it, the o projection inside the launch: DECODE_O_FUSED)
            model.clear_decode_cache()
            with torch.no_grad():
                o1 = model(input_ids=ids.to(cuda), pixel_values=inputs["pixel_values"].to(cuda),
                           intrinsic=inputs["intrinsic"].to(cuda), use_cache=True)
                o2 = model(input_ids=ids[:, -1:].to(cuda), past_key_values=o1.past_key_values)
            outs[persist] = (o2.logits.clone(), model.predict_action(inputs, max_new_tokens=6, eos_token_id=-1))
    finally:
        Fn.DECODE_MLP_PERSIST[0] = keep
        model.clear_decode_cache()
    assert torch.equal(outs[True][0], outs[False][0])
    assert torch.equal(outs[True][1], outs[False][1])


def test_decode_norm_fusion_bitwise(cuda):
    """A decode step with the norm pairs inside the projections' GEMVs gives the logits of the unfused loop, bit for
    bit (predict_action tokens as well)."""
    from spatialvla_amd import functional as Fn
    model, g = _tiny_model(cuda)
    ids = g["in.input_ids"][:, :-13]
    inputs = {"input_ids": ids, "pixel_values": g["in.pixel_values"], "intrinsic": g["in.intrinsic"]}
    model.decode_graphs = False
    outs = {}
    try:
        for fused in (False, True):
            Fn.DECODE_NORM_FUSED[0] = fused
            with torch.no_grad():
                o1 = model(input_ids=ids.to(cuda), pixel_values=inputs["pixel_values"].to(cuda),
                           intrinsic=inputs["intrinsic"].to(cuda), use_cache=True)
                o2 = model(input_ids=ids[:, -1:].to(cuda), past_key_values=o1.past_key_values)
            outs[fused] = (o2.logits.clone(), model.predict_action(inputs, max_new_tokens=6, eos_token_id=-1))
    finally:
        Fn.DECODE_NORM_FUSED[0] = True
        model.decode_graphs = True
    assert torch.equal(outs[True][0], outs[False][0])
    assert torch.equal(outs[True][1], outs[False][1])
