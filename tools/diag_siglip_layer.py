"""Diagnostic: common-mode (column-sum) error of the HIP SigLIP MLP / attention gradients vs torch on CPU and GPU."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import torch
import torch.nn.functional as F
import harness as H
from spatialvla_amd import functional as Fn

torch.manual_seed(0)
cuda = torch.device("cuda:0")
BF = torch.bfloat16
M, Hd, I = 256, 1152, 4304


def sk(x):
    x = x.float().cpu()
    return x.reshape(x.shape[0], -1).sum(0) if x.dim() >= 2 else x


def mlp_torch(x, res, w1, b1, w2, b2):
    return res + F.linear(F.gelu(F.linear(x, w1, b1), approximate="tanh"), w2, b2)


def leaves(ts, dev):
    return [t.detach().to(dev).clone().requires_grad_(True) for t in ts]


x = torch.randn(M, Hd).to(BF)
res = torch.randn(M, Hd).to(BF)
w1 = (torch.randn(I, Hd) / Hd ** 0.5).to(BF)
b1 = (torch.randn(I) * 0.02).to(BF)
w2 = (torch.randn(Hd, I) / I ** 0.5).to(BF)
b2 = (torch.randn(Hd) * 0.02).to(BF)
dout = (torch.randn(M, Hd) * 1e-3).to(BF)
outs = {}
for tag, dev in (("cpu", "cpu"), ("gpu", cuda)):
    L = leaves([x, res, w1, b1, w2, b2], dev)
    y = mlp_torch(*L)
    y.backward(dout.to(dev))
    outs[tag] = [t.grad.float().cpu() for t in L] + [y.detach().float().cpu()]
L = leaves([x, res, w1, b1, w2, b2], cuda)
y = Fn.SiglipMLPFn.apply(L[0], L[1], L[2], L[3], L[4], L[5], None)
y.backward(dout.to(cuda))
outs["hip"] = [t.grad.float().cpu() for t in L] + [y.detach().float().cpu()]
names = ["dx", "dres", "dW1", "db1", "dW2", "db2", "y"]
for i, n in enumerate(names):
    c, g, h = outs["cpu"][i], outs["gpu"][i], outs["hip"][i]
    print(f"MLP {n:5s} full rel: gpu {H.rel_l2(g, c):.2e} hip {H.rel_l2(h, c):.2e} | sketch rel: gpu "
          f"{H.rel_l2(sk(g), sk(c)):.2e} hip {H.rel_l2(sk(h), sk(c)):.2e}")
# intermediate: dpre of the reference vs HIP (HIP: recompute via the kernels)
from spatialvla_amd import kernels as Kn, _lib as Lb
xg, w1g, b1g, w2g = x.to(cuda), w1.to(cuda), b1.to(cuda), w2.to(cuda)
pre = torch.empty(M, I, dtype=BF, device=cuda); act = torch.empty_like(pre)
Kn.linear_fwd(xg, [w1g], act, kind=Lb.EPI_BIAS_GELU, bias=b1g, out1=pre)
dpre = torch.empty_like(pre)
Kn.linear_dgrad(dout.to(cuda), [w2g], dpre, kind=Lb.EPI_GELU_BWD, in0=pre)
prec = F.linear(x.float(), w1.float(), b1.float()).to(BF)
actc = F.gelu(prec, approximate="tanh")
prec_ = prec.clone().requires_grad_(True)
a_ = F.gelu(prec_, approximate="tanh")
dact = (dout @ w2)  # bf16 matmul on CPU
a_.backward(dact)
print("pre rel", H.rel_l2(pre.cpu(), prec), "act rel", H.rel_l2(act.cpu(), actc))
print("dpre rel", H.rel_l2(dpre.cpu(), prec_.grad), "rowsum rel", H.rel_l2(dpre.float().sum(1).cpu(), prec_.grad.float().sum(1)))
dact_h = torch.empty(M, I, dtype=BF, device=cuda)
Kn.linear_dgrad(dout.to(cuda), [w2g], dact_h)
print("dact rel", H.rel_l2(dact_h.cpu(), dact), "rowsum rel", H.rel_l2(dact_h.float().sum(1).cpu(), dact.float().sum(1)))
d = dact_h.float().cpu() - dact.float()
print("dact mean diff / rms", float(d.mean() / dact.float().pow(2).mean().sqrt()))
