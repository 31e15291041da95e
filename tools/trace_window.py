#!/usr/bin/env python3
"""Per-kernel device time inside a window of a rocprofv3 kernel trace.

    python tools/trace_window.py TRACE.csv MARKER [--per N]

The window starts at the first dispatch whose kernel name contains MARKER (e.g.
k_tree_edges: the merges of tools/merge_probe.py, after its tree builds); times are
summed per kernel and divided by --per (default: the number of MARKER dispatches)."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("marker")
    ap.add_argument("--per", type=int, default=0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    start = next(i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"])
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows[start:]:
        name = r["Kernel_Name"].replace("sheep::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[name] += 1
    per = a.per or sum(1 for r in rows[start:] if a.marker in r["Kernel_Name"])
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1e6
    print(f"window: {len(rows) - start} dispatches, span {span / per:.3f} ms per unit, busy {sum(tot.values()) / per:.3f} ms per unit ({per} units)")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {k:60s} {v / per:8.3f} ms  {cnt[k] / per:6.1f} calls  {1e3 * v / cnt[k]:8.1f} us avg")


if __name__ == "__main__":
    main()
