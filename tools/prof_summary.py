"""Per-step kernel-time breakdown from a rocprofv3 kernel_trace.csv (steady-state step between the last
two AdamW launches).  Usage: python tools/prof_summary.py <kernel_trace.csv> [top]"""
import collections, csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r['Start_Timestamp']))
ad = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name']]
seg = rows[ad[-2] + 1: ad[-1] + 1]
t0, t1 = int(seg[0]['Start_Timestamp']), int(seg[-1]['End_Timestamp'])


def key(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    m = re.match(r'([^(]*)', n)
    k = m.group(1) if m else n
    return k[:100]


agg = collections.defaultdict(lambda: [0, 0])
for r in seg:
    d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    agg[key(r['Kernel_Name'])][0] += d
    agg[key(r['Kernel_Name'])][1] += 1
tot = sum(v[0] for v in agg.values())
print(f"step wall {(t1 - t0) / 1e6:.2f} ms, sum of kernel time {tot / 1e6:.2f} ms, {len(seg)} launches")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{v[0] / 1e6:8.2f} ms {100 * v[0] / tot:5.1f}% n={v[1]:5d} avg={v[0] / v[1] / 1e3:8.1f}us  {k}")
