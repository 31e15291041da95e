#!/usr/bin/env python3
"""The literal `mpiexec -n P graph2tree G -ir` sequence on the host cores:
the reference's own mpiSequence (sequence.h:65-93), whose __gnu_parallel::sort comparator
captures the whole degree vector BY VALUE (sequence.h:85), against the same flow with
degreeSequence's by-reference comparator (the form bench.py's cpu_baseline times).  Both
run in oracle/_ref/ref_harness (modes mpi_ir / mpi), built from the reference's sources by
oracle/ref/Makefile.  Test infrastructure: it times the baseline, never the product.

    python tools/cpu_ir.py OUT.json [--rmat-ranks 1 2] [--hep-ranks 1 2 4 8] [--timeout 400]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(mpiexec, harness, mode, path, k, p, threads, timeout):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    t = time.time()
    try:
        r = subprocess.run([mpiexec, "-n", str(p), harness, mode, path, str(k)], capture_output=True, text=True,
                           timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"mode": mode, "ranks": p, "threads": threads, "timed_out_after_s": timeout}
    if r.returncode != 0:
        return {"mode": mode, "ranks": p, "threads": threads, "error": r.stderr.strip()[-300:]}
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    res.update(mode=mode, wall_s=round(time.time() - t, 2))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--rmat-scale", type=int, default=20)
    ap.add_argument("--rmat-ranks", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--hep-ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--timeout", type=int, default=400)
    a = ap.parse_args()
    import sheep_amd
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    mpiexec = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
    rows = []
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        rmat = os.path.join(td, f"rmat{a.rmat_scale}.dat")
        sheep_amd.rmat_host(a.rmat_scale, 16, a.rmat_scale).tofile(rmat)   # XS1 records, host generator
        graphs = [("C1 hep-th", os.path.join(ROOT, "tests", "golden", "hep.dat"), 2, a.hep_ranks),
                  (f"RMAT-{a.rmat_scale} ef16 seed {a.rmat_scale}", rmat, 16, a.rmat_ranks)]
        for name, path, k, ranks in graphs:
            for p in ranks:
                for mode in ("mpi_ir", "mpi"):
                    res = run(mpiexec, harness, mode, path, k, p, a.threads, a.timeout)
                    res["graph"] = name
                    rows.append(res)
                    print(json.dumps(res), flush=True)
    json.dump({"what": "literal -ir (mpiSequence, by-value comparator, sequence.h:85) vs the by-reference sort",
               "threads_per_rank": a.threads, "runs": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
