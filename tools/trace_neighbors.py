"""Kernels launched around each occurrence of a kernel (by name substring) in a rocprofv3 kernel trace, to find
which host op issues it: python tools/trace_neighbors.py <trace dir> <substring> [count]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[3]) if len(sys.argv) > 3 else 6
name = lambda r: r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:70]
hits = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
for i in hits[-n:]:
    print("----")
    for j in range(max(0, i - 3), min(len(rows), i + 3)):
        print((">> " if j == i else "   ") + name(rows[j]) + f"  stream {rows[j].get('Stream_Id', '?')}")
