"""Kernels of one prefill (the last predict_action of a decode_bench.py --new-tokens 1 trace): the launches after the
last host gap longer than 2 ms, grouped by kernel name.  python tools/prefill_trace_summary.py <trace dir>"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
cut = 0
for i in range(1, len(rows)):
    if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 2_000_000:
        cut = i
seg = rows[cut:]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0])
for r in seg:
    k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:100]
    agg[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[k][1] += 1
tot = sum(v[0] for v in agg.values())
print(f"last prefill: wall {(t1 - t0) / 1e6:.2f} ms, kernel sum {tot / 1e6:.2f} ms, {len(seg)} launches")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:30]:
    print(f"{v[0] / 1e6:9.3f} ms n={v[1]:5d} avg={v[0] / v[1] / 1e3:8.1f} us {k}")
