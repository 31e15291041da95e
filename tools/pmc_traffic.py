#!/usr/bin/env python3
"""Per-kernel HBM traffic of ONE path step from rocprofv3 PMC passes, for bench.py's
roofline.traffic and path_roofline.traffic.

FETCH_SIZE and WRITE_SIZE need separate passes on gfx950, and each is collected for two
bench runs that differ only in the number of timed steps (--steps 1 and --steps 2, no
warmup, the same evaluator repetitions).  One step's traffic is the difference of the two
runs, kernel by kernel: graph generation, context set-up and the evaluator leg are
identical in both runs and cancel, so nothing outside the path is counted.  Kernels are
keyed by their full signature (template instances stay apart).  The evaluator's traffic
per run is the 1-step run's evaluator kernels divided by its repetitions.

    python tools/pmc_traffic.py OUT.json --workload "RMAT-26 ef16, k=64" --eval-reps 1 \
        --fetch F1.csv F2.csv --write W1.csv W2.csv

Units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  Per MI355X_MICROARCH.md
(HBM [CDNA4]) FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads and
counts Infinity-Cache hits; other access widths are uncalibrated.  Both the raw sum and
the streaming-corrected sum (2 x FETCH + WRITE) are recorded.
"""
import argparse
import csv
import json
from collections import defaultdict

EVAL_KERNELS = ("k_pp", "k_eval_records", "k_eval_nodes", "k_max_part", "k_parts_jnid", "k_eval_edges", "k_eval_loops",
                "k_eval_nodes_j")


def per_kernel(path):
    tot, calls = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].strip()
        tot[name] += float(r["Counter_Value"]) * 1024.0
        calls[name] += 1
    return tot, calls


def base(name):
    name = name.replace("(anonymous namespace)::", "")   # its "(" is not the argument list
    head = name.split("(")[0]
    return head.split("<")[0].split("::")[-1].replace("void ", "").strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--fetch", nargs=2, required=True, metavar=("STEPS1", "STEPS2"))
    ap.add_argument("--write", nargs=2, required=True, metavar=("STEPS1", "STEPS2"))
    ap.add_argument("--eval-reps", type=int, default=1)
    a = ap.parse_args()
    f1, c1 = per_kernel(a.fetch[0])
    f2, c2 = per_kernel(a.fetch[1])
    w1, _ = per_kernel(a.write[0])
    w2, _ = per_kernel(a.write[1])
    res = {}
    for k in sorted(set(f1) | set(f2)):
        fb, wb = f2.get(k, 0.0) - f1.get(k, 0.0), w2.get(k, 0.0) - w1.get(k, 0.0)
        ent = {"base": base(k), "launches_per_step": c2.get(k, 0) - c1.get(k, 0),
               "per_step": {"fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_raw": round(fb + wb),
                            "traffic_stream_corrected": round(2 * fb + wb)}}
        if base(k) in EVAL_KERNELS:
            fe, we = f1.get(k, 0.0) / a.eval_reps, w1.get(k, 0.0) / a.eval_reps
            ent["per_eval"] = {"fetch_bytes": round(fe), "write_bytes": round(we), "traffic_raw": round(fe + we),
                               "traffic_stream_corrected": round(2 * fe + we)}
        if ent["launches_per_step"] or "per_eval" in ent:
            res[k] = ent
    json.dump({"workload": a.workload, "unit": "bytes per path step (2-step run minus 1-step run)",
               "kernels": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
