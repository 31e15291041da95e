#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE need separate passes on gfx950).  Used to fill bench.py's roofline.traffic.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json --workload "RMAT-26 ef16, k=64" \
        [--steps S]   # path steps the profiled bench ran (warmup included)

Units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  Per MI355X_MICROARCH.md
(HBM [CDNA4]) FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads and
counts Infinity-Cache hits; other access widths are uncalibrated.  Both the raw sum and
the streaming-corrected sum (2 x FETCH + WRITE) are recorded.
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def per_kernel(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"].split("(")[0]
        acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--steps", type=int, default=1, help="path steps in the profiled run (bench --steps + --warmup)")
    a = ap.parse_args()
    f, w = per_kernel(a.fetch), per_kernel(a.write)
    res = {}
    for k in sorted(set(f) & set(w)):
        fl, wl = f[k], w[k]
        fb, wb = sum(fl) / a.steps, sum(wl) / a.steps
        res[k] = {"launches_per_step": len(fl) / a.steps, "fetch_bytes": round(fb), "write_bytes": round(wb),
                  "traffic_raw": round(fb + wb), "traffic_stream_corrected": round(2 * fb + wb)}
    json.dump({"workload": a.workload, "unit": "bytes per path step", "kernels": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
