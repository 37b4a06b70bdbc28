"""Pair the GEMM launches of the last steady-state training step of two rocprofv3 kernel traces of bench.py
(same launch sequence, different GEMM dispatch) and compare per (kernel, grid) group:
python tools/ab_trace.py traceA.csv traceB.csv [gemm_log.json]  (bench.py with SVLA_GEMM_LOG writes the log)"""
import json
import csv
import sys
from collections import defaultdict

from ab_trace_lib import last_step


A, B = last_step(sys.argv[1]), last_step(sys.argv[2])
assert len(A) == len(B), (len(A), len(B))
log = json.load(open(sys.argv[3])) if len(sys.argv) > 3 else None
if log is not None:
    assert len(log) == len(A), (len(log), len(A))
EPI = ["store", "bias", "bias_gelu", "bias_resid", "geglu", "geglu_bwd", "gelu_bwd", "softcap_ce", "rope"]
grp = defaultdict(lambda: [0, 0.0, 0.0, ""])
for i, ((na, ga, ta), (nb, gb, tb)) in enumerate(zip(A, B)):
    shape = ""
    if log is not None:
        M, N, K, la, lb, kind, acc = log[i]
        shape = f"{M}x{N}x{K} {'KR'[la]}{'KR'[lb]} {EPI[kind] if kind < len(EPI) else kind}{'+acc' if acc else ''}"
    k = (nb, shape or gb, na)
    grp[k][0] += 1; grp[k][1] += ta; grp[k][2] += tb
tot_a = sum(t for *_, t in A); tot_b = sum(t for *_, t in B)
print(f"GEMM time per step: A {tot_a / 1e3:.2f} ms  B {tot_b / 1e3:.2f} ms")
for k, (n, ta, tb, _) in sorted(grp.items(), key=lambda kv: -kv[1][2]):
    print(f"{n:4d}x  {str(k[1]):34s} A={k[2]:28s} B={k[0]:28s} A {ta / n:8.1f} us  B {tb / n:8.1f} us  B/A {tb / ta:.3f}")
