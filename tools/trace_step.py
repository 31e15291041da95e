#!/usr/bin/env python3
"""Per-kernel time of the LAST path step in a rocprofv3 kernel trace (kernel_trace.csv of
a bench.py run): the dispatches from the last k_degree_fused up to the evaluator's first
kernel (k_max_part, k_pp or k_parts_jnid) or the end.  Prints ms per kernel base name, calls, and the step span.

    python tools/trace_step.py run_kernel_trace.csv [--levels] [--from KERNEL]

--from KERNEL: the step starts at the last dispatch of KERNEL instead (e.g. k_tree_count
for the last merge of tools/merge_trace.py).
"""
import csv
import re
import sys
from collections import Counter, defaultdict


def base(name):
    m = re.search(r"(k_\w+|__amd_\w+|\w+_kernel\w*)", name)
    return m.group(1) if m else name[:40]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    first = sys.argv[sys.argv.index("--from") + 1] if "--from" in sys.argv else "k_degree_fused"
    starts = [i for i, r in enumerate(rows) if base(r["Kernel_Name"]) == first]
    step = rows[starts[-1]:]
    ends = [i for i, r in enumerate(step) if base(r["Kernel_Name"]) in ("k_pp", "k_max_part", "k_parts_jnid")]
    step = step[:ends[0]] if ends else step
    tot, cnt = defaultdict(float), Counter()
    for r in step:
        b = base(r["Kernel_Name"])
        tot[b] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        cnt[b] += 1
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
    print(f"step span {span:.3f} ms, kernel time {sum(tot.values()):.3f} ms, {len(step)} dispatches")
    for k, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"{v:9.3f} ms {cnt[k]:6d}  {k}")
    if "--levels" in sys.argv:   # etree levels: each starts at a k_split_count
        lv, cur = [], None
        for r in step:
            b = base(r["Kernel_Name"])
            if b == "k_split_count":
                cur = defaultdict(float)
                lv.append(cur)
            if cur is not None and b in ("k_split_count", "k_split_write", "k_hook_round", "k_hook_finish", "k_light_top",
                                         "k_cross_find", "k_cross_find_win", "k_cross_apply", "k_level_clean", "k_pack", "k_apply", "k_reduce"):
                cur[b] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        for i, d in enumerate(lv):
            print(f"level {i:2d} {sum(d.values()):7.3f} ms  " + " ".join(f"{k[2:]}={v:.3f}" for k, v in sorted(d.items())))


if __name__ == "__main__":
    main()
