#!/usr/bin/env python3
"""The reference CPU baseline over MPI rank counts (SURVEY §8(d) CPU baseline): the
reference's own lib/ graph2tree -r -p flow (oracle/_ref/ref_harness mpi, compiled from the
reference's sources by oracle/ref/Makefile) at P ranks x T OpenMP threads (the threads
serve __gnu_parallel::sort, sequence.h:55,85) on the GPU box's host cores, for one RMAT
scale.  Test infrastructure: it times the baseline, never the product.

    python tools/cpu_sweep.py OUT.json --scale 26 --k 64 --configs 8x1 16x1 16x4 16x16 32x8
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--ef", type=int, default=16)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--configs", nargs="+", default=["1x1", "8x1", "16x1", "16x16"])
    a = ap.parse_args()
    import bench
    import sheep_amd
    ctx = sheep_amd.default_context()
    rows = []
    for p in a.configs:
        ns = argparse.Namespace(cpu_scale=a.scale, ef=a.ef, k=a.k, cpu_configs=[p])
        t = time.time()
        r = bench.cpu_baseline(ns, ctx)
        r["wall_s_incl_generation_and_load"] = round(time.time() - t, 2)
        rows.append(r)
        print(json.dumps(r), flush=True)
    json.dump({"workload": f"RMAT-{a.scale} ef{a.ef}, k={a.k}", "runs": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
