"""A/B of the decode-step GEMVs (M = 1..8) on one MI355X: the runtime-loop kernels (variant 6), the prefetching
kernel with one row per wave (auto, variant 0) and with two rows per wave (variant 7).  Checks the variants are
bitwise equal and prints per-shape mean launch time (HIP events over a back-to-back run) and the weight-streaming
rate.  Shapes: Gemma2-2B q|k|v (4096 x 2304), o (2304 x 2048), gate|up GeGLU (2 x 9216 x 2304), down (2304 x 9216).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatialvla_amd import _lib as L  # noqa: E402
from spatialvla_amd import kernels as K  # noqa: E402

BF = torch.bfloat16


def run(M, name, reps=200):
    dev = "cuda"
    torch.manual_seed(0)
    if name == "gateup":
        N, Kd = 9216, 2304
        wg, wu = (torch.randn(N, Kd, device=dev) * 0.02).to(BF), (torch.randn(N, Kd, device=dev) * 0.02).to(BF)
        x = torch.randn(M, Kd, device=dev).to(BF)
        g, u, h = (torch.empty(M, N, dtype=BF, device=dev) for _ in range(3))
        fn = lambda: K.linear_geglu_fwd(x, wg, wu, h, g, u)  # noqa: E731
        outs, nbytes = (h, g, u), 2 * N * Kd * 2
    else:
        N, Kd = {"qkv": (4096, 2304), "o": (2304, 2048), "down": (2304, 9216)}[name]
        w = (torch.randn(N, Kd, device=dev) * 0.02).to(BF)
        x = torch.randn(M, Kd, device=dev).to(BF)
        y = torch.empty(M, N, dtype=BF, device=dev)
        fn = lambda: K.linear_fwd(x, [w], y)  # noqa: E731
        outs, nbytes = (y,), N * Kd * 2
    res, ref = {}, None
    for v in (6, 0, 7):
        K.gemm_variant = v
        fn()
        torch.cuda.synchronize()
        got = [o.clone() for o in outs]
        if ref is None:
            ref = got
        eq = all(torch.equal(a, b) for a, b in zip(ref, got))
        # launches replayed from a HIP graph, so the host-side ctypes cost is out of the timing
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(reps):
                fn()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        res[v] = {"us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1), "bitwise": eq}
    K.gemm_variant = 0
    return res


def main():
    for M in (1, 8):
        for name in ("qkv", "o", "gateup", "down"):
            print(json.dumps({"M": M, "shape": name, **{f"v{k}": v for k, v in run(M, name).items()}}), flush=True)


if __name__ == "__main__":
    main()
