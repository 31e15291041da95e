#!/usr/bin/env python3
"""Per-kernel ms per step of two rocprofv3 --stats kernel_stats.csv files (3-step bench runs
with one warmup step: totals / 4), largest first: tools/kernel_compare.py A.csv B.csv [N]."""
import csv, re, sys
def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        m = re.search(r'(\w+)(<[^()]*>)?\(', r['Name'])
        name = (m.group(1) + (m.group(2) or '')) if m else r['Name'][:40]
        d[name] = d.get(name, 0) + int(r['TotalDurationNs']) / 4e6   # 4 bench steps (warmup 1 + 3)
    return d
a, b = load(sys.argv[1]), load(sys.argv[2])
rows = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, 0), b.get(k, 0)))
for k in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{a.get(k,0):8.3f} {b.get(k,0):8.3f} {b.get(k,0)-a.get(k,0):+7.3f}  {k[:90]}")
print(f"{sum(a.values()):8.3f} {sum(b.values()):8.3f}  total")
