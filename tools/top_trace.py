#!/usr/bin/env python3
"""The dense-top-block kernels of the last path step in a rocprofv3 kernel trace: every
k_top_* dispatch (and the launches between them) with its duration and the idle gap before
it, from the first k_top_extract of the step to the next k_split_count.

    python tools/top_trace.py run_kernel_trace.csv
"""
import csv
import re
import sys


def base(name):
    m = re.search(r"(k_\w+|__amd_\w+|\w+_kernel\w*)", name)
    return m.group(1) if m else name[:40]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if base(r["Kernel_Name"]) == "k_degree_fused"]
step = rows[starts[-1]:]
first = next(i for i, r in enumerate(step) if base(r["Kernel_Name"]).startswith("k_top_extract"))
end = next(i for i in range(first, len(step)) if base(step[i]["Kernel_Name"]) == "k_split_count")
prev_end = int(step[first - 1]["End_Timestamp"])
t0 = int(step[first]["Start_Timestamp"])
tot = 0.0
for r in step[first:end]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev_end) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f} us  {base(r['Kernel_Name'])}")
    tot += (e - s) / 1e3
    prev_end = e
print(f"span {(prev_end - t0) / 1e3:.1f} us, kernel time {tot:.1f} us")
