"""svla_conv2d_nhwc (the ZoeDepth DPT neck / head convolutions, csrc/conv.hip) against torch fp32 convolutions of
the same bf16 operands: every geometry the frozen estimator uses (3x3 stride 1 and 2, 1x1, channel counts that are
not multiples of 64, the narrow 32-channel head conv, ConvTranspose2d with kernel == stride), pre- and
post-activation ReLU and the residual adds with the eager module's bf16 rounding points."""
import pytest
import torch
import torch.nn.functional as F

from harness import rel_l2

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("B,Cin,H,W,Cout,k,s,p", [
    (2, 256, 24, 24, 256, 3, 1, 1), (3, 96, 20, 17, 256, 3, 1, 1), (2, 768, 24, 24, 768, 3, 2, 1),
    (2, 256, 12, 12, 256, 1, 1, 0), (2, 128, 40, 36, 32, 3, 1, 1), (1, 1024, 24, 24, 192, 1, 1, 0),
    (2, 256, 48, 48, 128, 3, 1, 1), (1, 32, 16, 16, 8, 1, 1, 0)])
@pytest.mark.parametrize("pre,post", [(False, False), (True, True)])
def test_conv2d_nhwc_vs_torch(cuda, B, Cin, H, W, Cout, k, s, p, pre, post):
    from spatialvla_amd import kernels as K
    torch.manual_seed(0)
    x = torch.randn(B, Cin, H, W, device=cuda).to(BF)
    w = (torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5).to(BF)
    b = torch.randn(Cout, device=cuda).to(BF)
    xr = F.relu(x) if pre else x
    ref = F.conv2d(xr.float(), w.float(), b.float(), stride=s, padding=p)
    if post:
        ref = F.relu(ref)
    got = K.conv2d_cl(_cl(x), K.conv_weight_khwc(w), b, stride=s, pad=p, pre_relu=pre, post_relu=post)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
    assert rel_l2(got, ref) < 8e-3


def test_conv2d_nhwc_residual_rounding(cuda):
    """PreActResidualLayer + FeatureFusionLayer order: out = bf16(bf16(bf16(conv + b) + res1) + res2)."""
    from spatialvla_amd import kernels as K
    torch.manual_seed(1)
    B, C, H, W = 2, 256, 24, 24
    x = torch.randn(B, C, H, W, device=cuda).to(BF)
    w = (torch.randn(C, C, 3, 3, device=cuda) / (C * 9) ** 0.5).to(BF)
    r1, r2 = torch.randn(B, C, H, W, device=cuda).to(BF), torch.randn(B, C, H, W, device=cuda).to(BF)
    conv = F.conv2d(F.relu(x).float(), w.float(), None, padding=1).to(BF)
    ref = ((conv + r1) + r2)  # bf16 ops: each add rounds
    got = K.conv2d_cl(_cl(x), K.conv_weight_khwc(w), None, pad=1, pre_relu=True, res1=_cl(r1), res2=_cl(r2))
    assert rel_l2(got, ref) < 5e-3


@pytest.mark.parametrize("B,Cin,H,W,Cout,f", [(2, 96, 24, 24, 96, 4), (2, 192, 24, 24, 192, 2), (1, 64, 5, 7, 16, 3)])
def test_conv_transpose_k_eq_s_vs_torch(cuda, B, Cin, H, W, Cout, f):
    from spatialvla_amd import kernels as K
    torch.manual_seed(2)
    x = torch.randn(B, Cin, H, W, device=cuda).to(BF)
    w = (torch.randn(Cin, Cout, f, f, device=cuda) / Cin ** 0.5).to(BF)
    b = torch.randn(Cout, device=cuda).to(BF)
    ref = F.conv_transpose2d(x.float(), w.float(), b.float(), stride=f)
    got = K.conv2d_cl(_cl(x), K.conv_weight_khwc(w, transposed=True), b, transposed=True)
    assert got.shape == ref.shape
    assert rel_l2(got, ref) < 8e-3


def test_conv2d_nhwc_rejects_bad_args(cuda):
    from spatialvla_amd import kernels as K
    x = _cl(torch.randn(1, 12, 8, 8, device=cuda).to(BF))  # Cin not a multiple of 8
    w = K.conv_weight_khwc(torch.randn(16, 12, 3, 3, device=cuda).to(BF))
    with pytest.raises(RuntimeError):
        K.conv2d_cl(x, w, None, pad=1)


@pytest.mark.parametrize("B,Cin,H,W,Cout,k,s,p", [(1, 256, 24, 24, 256, 3, 1, 1), (1, 256, 12, 12, 256, 3, 1, 1),
                                                (1, 512, 48, 48, 256, 1, 1, 0), (1, 256, 12, 12, 256, 3, 2, 1)])
def test_conv2d_split_k_matches_unsplit(cuda, B, Cin, H, W, Cout, k, s, p):
    """Sub-wave 64x64 convolution grids split K over workgroups (the B = 1 DPT neck; slabs + counters in the stream's
    GEMM workspace): against fp32 torch, within fp32 reordering of the unsplit result, and bitwise reproducible
    (deterministic reduction order, counters left zero) -- with pre-activation ReLU and two residuals."""
    from spatialvla_amd import kernels as K
    torch.manual_seed(3)
    x = torch.randn(B, Cin, H, W, device=cuda).to(BF)
    w = (torch.randn(Cout, Cin, k, k, device=cuda) / (Cin * k * k) ** 0.5).to(BF)
    b = torch.randn(Cout, device=cuda).to(BF)
    OH = (H + 2 * p - k) // s + 1
    r1 = _cl(torch.randn(B, Cout, OH, OH, device=cuda).to(BF))
    r2 = _cl(torch.randn(B, Cout, OH, OH, device=cuda).to(BF))
    wk = K.conv_weight_khwc(w)
    outs = []
    for split in (False, True, True):
        K.CONV_SPLIT[0] = split
        try:
            outs.append(K.conv2d_cl(_cl(x), wk, b, stride=s, pad=p, pre_relu=True, res1=r1, res2=r2))
        finally:
            K.CONV_SPLIT[0] = True
    torch.cuda.synchronize()
    ref = F.conv2d(F.relu(x).float(), w.float(), b.float(), stride=s, padding=p) + r1.float() + r2.float()
    assert rel_l2(outs[1], ref) < 8e-3
    assert rel_l2(outs[1], outs[0]) < 4e-3
    assert torch.equal(outs[1], outs[2])
