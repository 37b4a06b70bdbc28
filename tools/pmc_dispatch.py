"""Per-dispatch PMC table of ONE iteration of tools/block_ab.py (profile mode): python tools/pmc_dispatch.py
<csv_or_dir> [...] -> for each kernel of the last iteration (found by the repeating name pattern), the counters
of every pass merged by dispatch order, plus derived values: MFMA busy share of the SIMD cycles
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)), the clock (GRBM_GUI_ACTIVE / 8 / duration),
VALU and LDS instructions per MFMA, and LDS bank-conflict cycles per LDS-array cycle."""
import csv
import glob
import os
import re
import sys
from collections import OrderedDict


def load(path):
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*counter_collection.csv"),
                                                             recursive=True)
    disp = OrderedDict()
    for f in files:
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            e = disp.setdefault(d, {"name": r["Kernel_Name"], "grid": r.get("Grid_Size", ""), "c": {},
                                    "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                                    if r.get("End_Timestamp") else None,
                                    "vgpr": r.get("VGPR_Count", ""), "agpr": r.get("Accum_VGPR_Count", ""),
                                    "lds": r.get("LDS_Block_Size", "")})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def last_iteration(ds):
    names = [d["name"] for d in ds]
    for tail in range(0, 8):
        nm = names[:len(names) - tail]
        P = next((p for p in range(1, len(nm) // 2) if nm[-p:] == nm[-2 * p:-p]), None)
        if P:
            return ds[len(names) - tail - P:len(names) - tail]
    return ds


def short(n):
    return re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))[:44]


def main():
    passes = [last_iteration(load(p)) for p in sys.argv[1:]]
    n = min(len(p) for p in passes)
    print(f"{'kernel':44s} {'grid':>9s} {'us':>7s} {'GHz':>5s} {'MFMA%':>6s} {'MFMA':>9s} {'VALU/MF':>7s} "
          f"{'LDS/MF':>6s} {'bank%':>6s} {'wait%':>6s} {'vgpr/agpr':>9s}")
    for i in range(n):
        c = {}
        for p in passes:
            c.update(p[i]["c"])
        d = passes[0][i]
        dur = next((p[i]["dur"] for p in passes if p[i]["dur"]), None)
        gui = c.get("GRBM_GUI_ACTIVE")
        ghz = gui / 8 / (dur * 1e3) if gui and dur else float("nan")
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mf = c.get("SQ_INSTS_MFMA")
        util = busy / (gui / 8 * 1024) if busy is not None and gui else float("nan")
        vpm = c["SQ_INSTS_VALU"] / mf if mf and "SQ_INSTS_VALU" in c else float("nan")
        lpm = c["SQ_INSTS_LDS"] / mf if mf and "SQ_INSTS_LDS" in c else float("nan")
        bank = (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
                if c.get("SQ_LDS_IDX_ACTIVE") else float("nan"))
        wait = (c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else float("nan"))
        print(f"{short(d['name']):44s} {d['grid']:>9s} {dur if dur else float('nan'):7.1f} {ghz:5.2f} "
              f"{100 * util:6.1f} {mf if mf is not None else float('nan'):9.3g} {vpm:7.2f} {lpm:6.2f} "
              f"{100 * bank:6.1f} {100 * wait:6.1f} {d['vgpr']:>4s}/{d['agpr']:<4s}")
    print("\nraw counters per dispatch:")
    for i in range(n):
        c = {}
        for p in passes:
            c.update(p[i]["c"])
        print(short(passes[0][i]["name"]), " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
