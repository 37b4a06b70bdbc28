"""A/B one Gemma2DecoderLayer fwd+bwd (bench.py's gemma2_block workload) between two libsvla builds, interleaved in
ONE process: python tools/block_lib_ab.py libA.so libB.so [rounds].  Prints fwd and fwd+bwd ms per arm and round,
the median per arm, and whether x.grad is bitwise equal between the arms."""
import os, sys
sys.argv, extra = sys.argv[:1], sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from spatialvla_amd import _lib as L
libs = [(os.path.basename(p), L.load(os.path.abspath(p), strict=False)) for p in extra[:2]]
rounds = int(extra[2]) if len(extra) > 2 else 5
L._lib = libs[0][1]
import block_ab as B  # builds the layer and inputs (module level); its CLI sections see no arguments

res, grads = {t: [] for t, _ in libs}, {}
for r in range(rounds):
    for tag, lib in libs:
        L._lib = lib
        (f, t), gx = B.run(True)
        res[tag].append(t)
        grads[tag] = gx
        print(f"round {r} {tag:24s} fwd {f:.3f} ms  fwd+bwd {t:.3f} ms", flush=True)
for tag in res:
    print(f"{tag:24s} median fwd+bwd {np.median(res[tag]):.3f} ms  min {min(res[tag]):.3f}")
t = list(grads)
print("x.grad bitwise equal:", torch.equal(grads[t[0]], grads[t[1]]))
