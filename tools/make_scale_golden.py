#!/usr/bin/env python3
"""Oracle digests at BASELINE.json's full-size configurations (C3, C4, C5) — TEST
INFRASTRUCTURE, run once per configuration on the GPU box (its host cores run the oracle)
and committed as tests/golden/scale/<cfg>.json; tests/test_scale_parity.py compares the
GPU path's outputs against them in seconds instead of re-running the oracle for minutes.

For one configuration: the seeded synthetic records (sheep_amd's generator: the input
only), copied to the host, then the CPU oracle (oracle/sheep_oracle.cpp, pinned by
tests/test_oracle_golden.py) computes
  * the degree sequence (mpiSequence / degreeSequence, sequence.h:52-92),
  * the elimination tree in graph2tree -r's map/reduce form (JTree per contiguous record
    shard, jtree.cpp:66-110, then mpi_merge's binomial merges, jnode.cpp:174-250),
  * TREEFAQS (jnode.cpp:256-290),
  * Partition + forwardPartition for k (partition.cpp:50-157) with created / packing nodes,
  * every evaluator count (evaluate(graph) + evaluate(graph, seq), partition.cpp:428-521),
and the file records xxh3-128 digests of the records, seq, parent, pst and parts beside
the scalar results and the oracle's phase times.

    python tools/make_scale_golden.py c3|c4|c5 [--threads 16]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "c3": dict(graph="rmat", scale=26, seed=26, k=64, shards=16,
               workload="RMAT-26 ef16 seed 26, k=64 (BASELINE C3)"),
    "c4": dict(graph="powerlaw", draws=2_222_000_000, gamma=1.9, seed=2010, k=128, shards=16,
               workload="Chung-Lu power law, twitter-2010 scale (41,652,230 vertices), seed 2010, k=128 (BASELINE C4)"),
    "c5": dict(graph="rmat", scale=28, seed=28, k=256, shards=8,
               workload="RMAT-28 ef16 seed 28, k=256 + full evaluator (BASELINE C5)"),
}


def generate(cfg):
    """The configuration's records on cuda:0 (int32 N x 3 view of the XS1 records)."""
    import sheep_amd
    if cfg["graph"] == "rmat":
        return sheep_amd.rmat(cfg["scale"], 16, cfg["seed"])
    return sheep_amd.powerlaw(sheep_amd.TWITTER_VERTICES, cfg["draws"], cfg["gamma"], cfg["seed"])


def digest(a) -> str:
    import xxhash
    h = xxhash.xxh3_128()
    h.update(np.ascontiguousarray(a).view(np.uint8))
    return h.hexdigest()


def host_columns(d):
    """(tail, head) as host u32 arrays and the digest of the (tail, head) pairs, copied in
    chunks (never the whole 12-B record array on the host at once)."""
    import xxhash
    R = d.shape[0]
    t, h = np.empty(R, np.uint32), np.empty(R, np.uint32)
    x = xxhash.xxh3_128()
    step = 1 << 27
    for a in range(0, R, step):
        b = min(R, a + step)
        c = np.ascontiguousarray(d[a:b, :2].cpu().numpy()).view(np.uint32)
        t[a:b], h[a:b] = c[:, 0], c[:, 1]
        x.update(c.view(np.uint8))
    return t, h, x.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=sorted(CONFIGS))
    ap.add_argument("--threads", type=int, default=16, help="oracle OpenMP threads (the box's CPU share)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    import oracle
    oracle.set_threads(a.threads)
    times = {}

    def phase(name, fn):
        t0 = time.time()
        r = fn()
        times[name] = round(time.time() - t0, 2)
        print(f"{a.config}: {name} {times[name]:.1f} s", file=sys.stderr, flush=True)
        return r

    d = phase("generate", lambda: generate(cfg))
    R = int(d.shape[0])
    t, h, rec_digest = phase("host_copy", lambda: host_columns(d))
    del d
    import torch
    torch.cuda.empty_cache()
    seq = phase("sequence", lambda: oracle.sequence(t, h, "records"))
    parent, pst = phase("tree", lambda: oracle.build_tree_mr(t, h, seq, cfg["shards"]))
    facts = phase("facts", lambda: oracle.facts(parent, pst))
    parts, info = phase("partition", lambda: oracle.partition(parent, pst, seq, cfg["k"]))
    ev = phase("evaluate", lambda: oracle.evaluate(t, h, seq, parts))
    out = {
        "config": a.config, "workload": cfg["workload"], "generator": {k: v for k, v in cfg.items()
                                                                      if k not in ("workload", "k", "shards")},
        "k": cfg["k"], "records": R, "records_digest": rec_digest,
        "n": int(len(seq)), "pos_size": int(seq.max()) + 1 if len(seq) else 0,
        "seq_digest": digest(seq), "parent_digest": digest(parent), "pst_digest": digest(pst),
        "roots": int(np.count_nonzero(parent == oracle.INVALID)), "pst_sum": int(pst.astype(np.uint64).sum()),
        "facts": facts, "parts_digest": digest(parts), "created": info["created"],
        "packing_nodes": info["packing_nodes"], "max_component": info["max_component"],
        "first_size": int(np.count_nonzero(parts == 0)), "second_size": int(np.count_nonzero(parts == 1)),
        "evaluate": ev,
        "oracle": {"threads": a.threads, "tree_form": f"build_tree_mr: {cfg['shards']} record shards + binomial merges",
                   "phase_seconds": times},
        "digest": "xxh3-128 of the little-endian u32 arrays (records: the (tail, head) pairs; parts: i16)",
    }
    path = a.out or os.path.join(ROOT, "tests", "golden", "scale", f"{a.config}.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
