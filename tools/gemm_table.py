"""Per-shape GEMM table of the last steady-state step of ONE rocprofv3 kernel trace of bench.py (run with
SVLA_GEMM_LOG): calls, mean us, TFLOP/s, ms per step and ms lost against 1000 TFLOP/s.
python tools/gemm_table.py trace.csv gemm_log.json"""
import json
import sys
from collections import defaultdict

from ab_trace_lib import last_step  # noqa: E402

EPI = ["store", "bias", "bias_gelu", "bias_resid", "geglu", "geglu_bwd", "gelu_bwd", "softcap_ce", "rope"]
A = last_step(sys.argv[1])
log = json.load(open(sys.argv[2]))
assert len(log) == len(A), (len(log), len(A))
grp = defaultdict(lambda: [0, 0.0, 0.0])
for (n, g, t), (M, N, K, la, lb, kind, acc) in zip(A, log):
    k = (f"{M}x{N}x{K} {'KR'[la]}{'KR'[lb]} {EPI[kind] if kind < len(EPI) else kind}{'+acc' if acc else ''}", n)
    grp[k][0] += 1; grp[k][1] += t; grp[k][2] += 2.0 * M * N * K
tot = sum(v[1] for v in grp.values())
print(f"GEMM time per step {tot / 1e3:.2f} ms over {len(A)} launches")
rows = []
for k, (c, t, f) in grp.items():
    tf = f / (t * 1e-6) / 1e12
    lost = (t - f / 1e15 * 1e6) / 1e3
    rows.append((lost, k, c, t, tf))
for lost, k, c, t, tf in sorted(rows, reverse=True):
    print(f"{c:4d}x {k[0]:36s} {k[1]:26s} {t / c:8.1f} us {tf:7.1f} TF/s  {t / 1e3:7.2f} ms  lost@1PF {lost:6.2f} ms")
