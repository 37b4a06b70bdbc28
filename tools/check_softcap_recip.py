"""Exhaustive check behind svla_common.h softcap_bf16: for every finite bf16 x, bf16(x * RN(1/cap)) == bf16(x / cap)
(correctly rounded fp32 division), at the Gemma2 caps 30 (final logits) and 50 (attention)."""
import numpy as np


def rbf(x):
    b = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    return (((b + 0x7FFF + ((b >> 16) & 1)) >> 16) << 16).astype(np.uint32)


v = (np.arange(65536, dtype=np.uint32) << 16).view(np.float32)
v = v[np.isfinite(v)]
for cap in (30.0, 50.0):
    q_div = (v / np.float32(cap)).astype(np.float32)
    q_mul = (v * (np.float32(1.0) / np.float32(cap))).astype(np.float32)
    bad = int(np.sum(rbf(q_div) != rbf(q_mul)))
    print(f"cap {cap}: {bad} mismatches of {v.size}")
    assert bad == 0
