"""The generated bf16 function tables the kernels compile in (spatialvla_amd/csrc/*_table.h) are what their generators
produce, and the gelu table's band rule equals the reference's fp32 formula on every bf16 input (CPU only)."""
import os
import re

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_values(name, sym):
    txt = open(os.path.join(REPO, "spatialvla_amd", "csrc", name)).read()
    body = txt[txt.index(sym):]
    body = body[body.index("{") + 1:body.index("};")]
    return np.array([int(v, 16) for v in re.findall(r"0x[0-9a-fA-F]+", body)], dtype=np.uint32)


def test_gelu_table_matches_generator_and_formula():
    from tools.gen_gelu_table import LO, N, gelu_ref_bits, lut_rule
    tab = _header_values("gelu_bf16_table.h", "svla_gelu_bf16_tab")
    band = np.concatenate([np.arange(LO, LO + N, dtype=np.uint32), np.arange(LO, LO + N, dtype=np.uint32) | 0x8000])
    assert len(tab) == 2 * N and np.array_equal(tab, gelu_ref_bits(band))
    allb = np.arange(65536, dtype=np.uint32)
    ref, got = gelu_ref_bits(allb), lut_rule(allb, tab.astype(np.uint16))
    nan = lambda v: ((v & 0x7F80) == 0x7F80) & ((v & 0x7F) != 0)
    assert not ((ref != got) & ~(nan(ref) & nan(got))).any()
    # spot values: gelu(1) = 0.8412 -> bf16 0x3f57; gelu(-1) = -0.1588 -> 0xbe23; zero keeps its sign
    one, mone = 0x3F80, 0xBF80
    assert got[one] == 0x3F57 and got[mone] == 0xBE23 and got[0] == 0 and got[0x8000] == 0x8000


def test_tanh_table_matches_generator():
    tab = _header_values("tanh_bf16_table.h", "svla_tanh_bf16_tab")
    e0, e1 = 119, 129
    bits = np.arange(e0 << 7, e1 << 7, dtype=np.uint32)
    a = (bits << 16).view(np.float32).astype(np.float64)
    t = np.tanh(a).astype(np.float32).view(np.uint32).astype(np.uint64)
    tb = ((t + 0x7FFF + ((t >> 16) & 1)) >> 16).astype(np.uint32)
    assert np.array_equal(tab, tb)
