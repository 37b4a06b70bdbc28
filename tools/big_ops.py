"""Python call sites of large ATen copies in one training step: torch.cat / Tensor.copy_ / fill_ / zero_ /
torch.zeros(_like) calls moving more than 32 MB are logged with their shapes and the innermost frames of the
caller (spatialvla_amd, transformers or bench).  python tools/big_ops.py [batch]"""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench import build_model, make_batch

LOG = []
ON = [False]


def _where():
    fr = [f for f in traceback.extract_stack()[:-2]
          if "spatialvla_amd" in f.filename or "transformers" in f.filename or "bench.py" in f.filename]
    return " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(fr[-3:]))


def _wrap(owner, name, nbytes):
    orig = getattr(owner, name)

    def f(*a, **k):
        out = orig(*a, **k)
        if ON[0]:
            try:
                n = nbytes(a, k, out)
            except Exception:  # noqa: BLE001
                n = 0
            if n > 32 << 20:
                LOG.append((name, n, _where(), tuple(out.shape) if torch.is_tensor(out) else None))
        return out
    setattr(owner, name, f)


def _tb(t):
    return t.numel() * t.element_size() if torch.is_tensor(t) else 0


def main():
    from spatialvla_amd import presets
    from spatialvla_amd.engine import TrainEngine
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dev = torch.device("cuda:0")
    cfgd = json.loads(json.dumps(presets.spatialvla_4b()))
    model = build_model(cfgd, dev)
    eng = TrainEngine(model, lr=2e-5, weight_decay=0.0, max_grad_norm=1.0, warmup_ratio=0.005, total_steps=10)
    batches = [make_batch(cfgd, B, 1234 + s, dev) for s in range(3)]
    for b in batches[:2]:
        eng.train_step(b)
    torch.cuda.synchronize()
    _wrap(torch, "cat", lambda a, k, o: _tb(o))
    _wrap(torch, "zeros", lambda a, k, o: _tb(o))
    _wrap(torch, "zeros_like", lambda a, k, o: _tb(o))
    _wrap(torch.Tensor, "copy_", lambda a, k, o: _tb(o))
    _wrap(torch.Tensor, "zero_", lambda a, k, o: _tb(o))
    _wrap(torch.Tensor, "fill_", lambda a, k, o: _tb(o))
    _wrap(torch.Tensor, "contiguous", lambda a, k, o: _tb(o) if o.data_ptr() != a[0].data_ptr() else 0)
    _wrap(torch.nn.functional, "interpolate", lambda a, k, o: _tb(o))
    ON[0] = True
    eng.train_step(batches[2])
    torch.cuda.synchronize()
    ON[0] = False
    for name, n, where, shape in LOG:
        print(f"{n / 2**20:9.1f} MB  {name:12s} {str(shape):28s} {where}")


if __name__ == "__main__":
    main()
