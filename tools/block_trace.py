"""Per-kernel breakdown of ONE iteration of tools/block_ab.py (profile mode) from a rocprofv3 --kernel-trace csv.
usage: python tools/block_trace.py <rocprof_dir>"""
import csv, glob, os, re, sys

d = sys.argv[1]
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
P = tail = None
for tail in range(0, 8):  # trailing non-iteration kernels (the final x.grad clone)
    nm = names[:len(names) - tail]
    P = next((p for p in range(1, len(nm) // 2) if nm[-p:] == nm[-2 * p:-p]), None)
    if P:
        break
it = rows[len(names) - tail - P:len(names) - tail]
t0, t1 = int(it[0]["Start_Timestamp"]), int(it[-1]["End_Timestamp"])
tot = 0
for r in it:
    dd = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += dd
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))[:70]
    st = (int(r["Start_Timestamp"]) - t0) / 1e3
    print(f"{dd:9.1f} us  @{st:8.1f}  grid={int(r['Grid_Size_X']):>9} wg={r['Workgroup_Size_X']:>4}  {n}")
# union of the kernels' intervals: wall time with at least one kernel running; the rest is idle GPU (launch gaps,
# host waits)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in it)
busy, cs, ce = 0, iv[0][0], iv[0][1]
gaps = []
for a, b in iv[1:]:
    if a > ce:
        busy += ce - cs
        gaps.append(((cs - t0) / 1e3, (a - ce) / 1e3))
        cs, ce = a, b
    else:
        ce = max(ce, b)
busy += ce - cs
print(f"iteration: {P} kernels, wall {(t1 - t0) / 1e3:.1f} us, kernel sum {tot:.1f} us, busy (union) {busy / 1e3:.1f} us, "
      f"idle {(t1 - t0 - busy) / 1e3:.1f} us in {len(gaps)} gaps; largest: "
      + ", ".join(f"{g:.1f} us after @{s:.0f}" for s, g in sorted(gaps, key=lambda x: -x[1])[:6]))
