#!/usr/bin/env python3
"""Cut a rocprofv3 kernel trace (kernel_trace.csv) into phases at idle gaps of the device
(no kernel running for more than --gap ms, default 20) and print, per phase, its span,
kernel time, dispatch count and the per-kernel totals; with --levels also the etree
levels (each starts at a k_split_count) of every phase that has them.

    python tools/trace_phases.py run_kernel_trace.csv [--gap 20] [--levels] [--min-ms 1]

Phases shorter than --min-ms of kernel time are listed on one line each."""
import argparse
import csv
import re
from collections import Counter, defaultdict

LEVEL_KERNELS = ("k_split_count", "k_split_write", "k_hook_round", "k_hook_finish", "k_light_top", "k_cross_find",
                 "k_cross_find_win", "k_cross_apply", "k_pack")


def base(name):
    m = re.search(r"(k_\w+|__amd_\w+|\w+_kernel\w*)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=20.0)
    ap.add_argument("--levels", action="store_true")
    ap.add_argument("--min-ms", type=float, default=1.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    phases, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and (s - last_end) / 1e6 > a.gap and cur:
            phases.append(cur)
            cur = []
        cur.append(r)
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        phases.append(cur)
    for pi, ph in enumerate(phases):
        tot, cnt = defaultdict(float), Counter()
        for r in ph:
            b = base(r["Kernel_Name"])
            tot[b] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            cnt[b] += 1
        span = (int(ph[-1]["End_Timestamp"]) - int(ph[0]["Start_Timestamp"])) / 1e6
        ktime = sum(tot.values())
        if ktime < a.min_ms:
            print(f"phase {pi:2d}: span {span:8.3f} ms, kernels {ktime:8.3f} ms, {len(ph):5d} dispatches "
                  f"(first {base(ph[0]['Kernel_Name'])})")
            continue
        print(f"\nphase {pi:2d}: span {span:8.3f} ms, kernels {ktime:8.3f} ms, {len(ph):5d} dispatches")
        for k, v in sorted(tot.items(), key=lambda x: -x[1]):
            if v >= 0.005:
                print(f"  {v:9.3f} ms {cnt[k]:6d}  {k}")
        if a.levels:
            lv, cur_lv = [], None
            for r in ph:
                b = base(r["Kernel_Name"])
                if b == "k_split_count":
                    cur_lv = [defaultdict(float), 0, int(r["Start_Timestamp"]), 0]
                    lv.append(cur_lv)
                if cur_lv is not None and b in LEVEL_KERNELS:
                    cur_lv[0][b] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                    cur_lv[1] += 1
                    cur_lv[3] = int(r["End_Timestamp"])
            for i, (d, n, s, e) in enumerate(lv):
                print(f"  level {i:2d} {sum(d.values()):7.3f} ms ({n:3d} launches, span {(e - s) / 1e6:7.3f}) "
                      + " ".join(f"{k[2:]}={v:.3f}" for k, v in sorted(d.items())))


if __name__ == "__main__":
    main()
