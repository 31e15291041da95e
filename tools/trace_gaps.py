#!/usr/bin/env python3
"""Idle gaps of the LAST path step in a rocprofv3 kernel trace (as tools/trace_step.py cuts
it): every gap of more than --min us between one dispatch's end and the next one's start,
with the kernels on both sides, and the total idle time.

    python tools/trace_gaps.py run_kernel_trace.csv [--min 10]
"""
import csv
import sys

from trace_step import base


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    mn = float(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 10.0
    starts = [i for i, r in enumerate(rows) if base(r["Kernel_Name"]) == "k_degree_fused"]
    step = rows[starts[-1]:]
    ends = [i for i, r in enumerate(step) if base(r["Kernel_Name"]) in ("k_pp", "k_max_part", "k_parts_jnid")]
    step = step[:ends[0]] if ends else step
    idle, big = 0.0, []
    end = int(step[0]["End_Timestamp"])
    for prev, r in zip(step, step[1:]):
        s = int(r["Start_Timestamp"])
        gap = (s - end) / 1e3
        if gap > 0:
            idle += gap
        if gap > mn:
            big.append((gap, base(prev["Kernel_Name"]), base(r["Kernel_Name"])))
        end = max(end, int(r["End_Timestamp"]))
    print(f"idle {idle / 1e3:.3f} ms in {len(step)} dispatches; gaps > {mn} us: {len(big)} ({sum(g for g, _, _ in big) / 1e3:.3f} ms)")
    for g, a, b in big:
        print(f"{g:8.1f} us  {a} -> {b}")


if __name__ == "__main__":
    sys.path.insert(0, __import__("os").path.dirname(__file__))
    main()
