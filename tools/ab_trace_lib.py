"""Shared trace parsing for tools/ab_trace.py and tools/gemm_table.py."""
import csv


def last_step(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"]]
    a, b = ends[-2] + 1, ends[-1] + 1
    out = []
    for r in rows[a:b]:
        n = r["Kernel_Name"]
        if ("gemm4_kernel" in n or "gemm8_kernel" in n or "gemm_kernel" in n) and "Cijk" not in n and "igemm" not in n:
            g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            out.append((n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:28], g,
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out
