"""Isolated rates of the MX quantisers (svla_quant_mx_rows / svla_quant_mx_cols) on the fp8 step's shapes:
python tools/quant_bench.py   (SVLA_QUANT_MX_ITEMS selects the row kernel's items per wave).  HBM bytes = 2 B read +
1 B written per element + one scale byte per 32; rate = bytes / median time of 20 graph-free launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import kernels as K  # noqa: E402

M = 9984
ROWS = [("x qkv/gate_up [M,2304]", M, 2304), ("attn [M,2048]", M, 2048), ("dqkv [M,4096]", M, 4096),
        ("h [M,9216]", M, 9216), ("dgu [M,18432]", M, 18432), ("W gate_up [18432,2304]", 18432, 2304)]
COLS = [("W^T gate_up", 18432, 2304), ("W^T down", 2304, 9216), ("W^T qkv", 4096, 2304), ("W^T o", 2304, 2048)]


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[reps // 2]


def main():
    torch.manual_seed(0)
    print(f"items per wave: {os.environ.get('SVLA_QUANT_MX_ITEMS', '4 (default)')}")
    for name, r, k in ROWS:
        x = torch.randn(r, k, device="cuda").to(torch.bfloat16)
        q = torch.empty(r, k, dtype=torch.float8_e4m3fn, device="cuda")
        sc = K.MXScales(r, k, "cuda")
        ms = timed(lambda: K.quant_mx_rows(x, q, sc))
        print(f"rows {name:28s} {ms * 1e3:8.1f} us  {r * k * (3 + 1 / 32) / ms / 1e6:7.0f} GB/s")
    for name, n, k in COLS:
        w = torch.randn(n, k, device="cuda").to(torch.bfloat16)
        ms = timed(lambda: K.quant_mx_cols(w))
        ms2 = timed(lambda: K.quant_mx_rows(w.t().contiguous()))
        print(f"cols {name:28s} {ms * 1e3:8.1f} us  {n * k * (3 + 1 / 32) / ms / 1e6:7.0f} GB/s   "
              f"(transpose copy + rows: {ms2 * 1e3:.1f} us)")


if __name__ == "__main__":
    main()
