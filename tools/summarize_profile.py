"""Condense rocprofv3 output of a bench.py run into the small files committed under profiles/.

  python tools/summarize_profile.py trace <rocprof_dir> <out_prefix>   # --kernel-trace --stats run
  python tools/summarize_profile.py pmc   <rocprof_dir> <out_prefix>   # --pmc FETCH_SIZE / WRITE_SIZE run

trace: copies the kernel_stats summary, writes a per-step breakdown (steady-state step between the last two
AdamW launches) and the launches of the dominant kernel (the Gemma2 gate/up GeGLU GEMM, identified by its
grid: ceil(M/256) * ceil(2I/256) workgroups of 512 threads at B=32), with their mean duration.
pmc: per-launch counter values of the same kernel (FETCH_SIZE doubled: on gfx950 it reports half the bytes
of 16-B/lane streaming reads, MI355X_MICROARCH.md §HBM) -> HBM bytes per launch.
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

M, I, H = 32 * 312, 9216, 2304
DOM_TILES = ((M + 255) // 256) * ((2 * I + 255) // 256)
DOM_GRID = DOM_TILES * 512  # 8-wave kernel; the 4-wave kernel launches DOM_TILES * 256 threads
DOM_GRIDS = (DOM_TILES * 512, DOM_TILES * 256)


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def _key(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    m = re.match(r"([^(]*)", n)
    return (m.group(1) if m else n)[:110]


def _is_dom(r):
    return re.search(r"gemm[48]?_kernel", r["Kernel_Name"]) is not None and int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) in DOM_GRIDS


def trace(d, out):
    shutil.copy(_find(d, "kernel_stats.csv"), out + "_kernel_stats.csv")
    rows = list(csv.DictReader(open(_find(d, "kernel_trace.csv"))))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    lines = []
    if len(ad) >= 2:
        seg = rows[ad[-2] + 1: ad[-1] + 1]
        t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
        agg = collections.defaultdict(lambda: [0, 0])
        for r in seg:
            dd = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            agg[_key(r["Kernel_Name"])][0] += dd
            agg[_key(r["Kernel_Name"])][1] += 1
        tot = sum(v[0] for v in agg.values())
        lines.append(f"steady-state step: wall {(t1 - t0) / 1e6:.2f} ms, sum of kernel time {tot / 1e6:.2f} ms, "
                     f"{len(seg)} launches")
        # GPU idle inside the step: the union of the kernels' intervals against the wall time, and the largest gaps
        # with the kernel that ended before each one
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _key(r["Kernel_Name"])) for r in seg)
        busy, cs, ce, last = 0, iv[0][0], iv[0][1], iv[0][2]
        gaps = []
        for a, b, nm in iv[1:]:
            if a > ce:
                busy += ce - cs
                gaps.append((a - ce, (ce - t0) / 1e6, last, nm))
                cs, ce = a, b
            if b >= ce:
                ce, last = b, nm
        busy += ce - cs
        lines.append(f"GPU busy (union of kernel intervals) {busy / 1e6:.2f} ms, idle {(t1 - t0 - busy) / 1e6:.2f} ms in "
                     f"{len(gaps)} gaps")
        for g, at, before, after in sorted(gaps, reverse=True)[:12]:
            lines.append(f"   gap {g / 1e3:8.1f} us at {at:8.2f} ms  after {before[:50]}  before {after[:50]}")
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0]):
            lines.append(f"{v[0] / 1e6:9.3f} ms {100 * v[0] / tot:5.1f}% n={v[1]:5d} avg={v[0] / v[1] / 1e3:9.1f} us  {k}")
    open(out + "_step_breakdown.txt", "w").write("\n".join(lines) + "\n")
    dom = [r for r in rows if _is_dom(r)]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in dom]
    with open(out + "_dominant_kernel.json", "w") as f:
        json.dump({"kernel": _key(dom[0]["Kernel_Name"]) if dom else None, "grid_threads": DOM_GRID,
                   "launches": len(durs), "mean_ns": (sum(durs) / len(durs)) if durs else None,
                   "mean_ns_last_26": (sum(durs[-26:]) / len(durs[-26:])) if durs else None,
                   "durations_ns": durs}, f, indent=1)
    print("\n".join(lines[:40]))
    print(f"dominant kernel: {len(durs)} launches, mean {sum(durs) / max(1, len(durs)) / 1e3:.1f} us")


def pmc(d, out):
    path = _find(d, "counter_collection.csv")
    rows = list(csv.DictReader(open(path)))
    cols = rows[0].keys() if rows else []
    gcol = "Grid_Size" if "Grid_Size" in cols else "Grid_Size_X"
    per = collections.defaultdict(dict)
    for r in rows:
        if re.search(r"gemm[48]?_kernel", r["Kernel_Name"]) is None or int(float(r[gcol])) not in DOM_GRIDS:
            continue
        per[r.get("Dispatch_Id", r.get("Correlation_Id"))][r["Counter_Name"]] = float(r["Counter_Value"])
    vals = collections.defaultdict(list)
    for dsp, cv in per.items():
        for k, v in cv.items():
            vals[k].append(v)
    res = {"file": os.path.basename(path), "launches": len(per)}
    for k, v in vals.items():
        mean = sum(v) / len(v)
        res[k + "_mean"] = mean
        if k == "FETCH_SIZE":      # KiB units; x2 gfx950 correction
            res["hbm_read_bytes_per_launch"] = mean * 1024 * 2
        if k == "WRITE_SIZE":
            res["hbm_write_bytes_per_launch"] = mean * 1024
    json.dump(res, open(out + ".json", "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    {"trace": trace, "pmc": pmc}[sys.argv[1]](sys.argv[2], sys.argv[3])
