"""Summarise rocprofv3 --pmc CSVs per kernel: python tools/pmc_table.py dir1 [dir2 ...] -> mean counter value per
dispatch for each kernel (all dirs merged), plus the kernel-trace average duration when a *_kernel_stats.csv is
among the dirs."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))
    durs = {}
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                durs[r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]] = float(r["AverageNs"]) / 1e3
    for k in sorted(set(vals) | set(durs)):
        print(k, f"avg {durs[k]:.1f} us" if k in durs else "")
        for c, v in sorted(vals[k].items()):
            print(f"    {c:28s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
