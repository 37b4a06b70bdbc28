"""Per-kernel totals of a rocprofv3 kernel trace divided by a repeat count: python tools/kernel_table.py DIR N"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
n = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
agg = collections.defaultdict(lambda: [0, 0])
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:110]
    agg[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[k][1] += 1
tot = sum(v[0] for v in agg.values())
print(f"kernel time per repeat {tot / n / 1e6:.2f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"{v[0] / n / 1e6:9.3f} ms n={v[1] / n:7.1f} avg={v[0] / v[1] / 1e3:8.1f} us {k}")
