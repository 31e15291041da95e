#!/usr/bin/env python3
"""The 8-GPU per-rank work of an RMAT step, phase by phase on one GPU, for a kernel trace:
the tree of ONE 1/K edge shard (the map of one rank) and the K-way merge of the K shard
trees (rank 0's reduce), each run `reps` times with an idle gap between runs so that
tools/trace_phases.py can cut the trace into phases.

    rocprofv3 --kernel-trace -d t -o run --output-format csv -- python tools/shard_trace.py 26 2 8
    python tools/trace_phases.py t/.../run_kernel_trace.csv --levels

Prints one JSON line: host wall ms per map / merge run (after a device sync) and whether
the last merge equals the whole graph's tree."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import sheep_amd
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    ctx = sheep_amd.Context(0)
    tune = dict(kv.split("=") for kv in os.environ.get("SHEEP_TUNE", "").split())
    if tune:
        ctx.set_tuning(**{k: int(v) for k, v in tune.items()})
    rec = sheep_amd.rmat(scale, 16, scale, ctx=ctx)
    s = sheep_amd.degree_sequence(rec, ctx=ctx)
    R = rec.shape[0]
    gap = 0.05

    def timed(fn):
        torch.cuda.synchronize()
        time.sleep(gap)
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return out, (time.perf_counter() - t0) * 1e3

    maps = []
    for _ in range(reps):
        _, ms = timed(lambda: sheep_amd.build_tree(rec[:R // K], s, ctx=ctx))
        maps.append(ms)
    stacked = torch.stack([timed(lambda i=i: sheep_amd.build_tree(rec[i * R // K:(i + 1) * R // K], s, ctx=ctx))[0]
                           for i in range(K)])
    whole, _ = timed(lambda: sheep_amd.build_tree(rec, s, ctx=ctx))
    del rec
    merges = []
    for _ in range(reps):
        merged, ms = timed(lambda: sheep_amd.merge_trees_many(stacked, ctx=ctx))
        merges.append(ms)
    # mpi_merge's binomial schedule (jnode.cpp:241, MPI_Reduce): ceil(log2 K) hops, each a
    # pairwise merge per pair of ranks — on K GPUs a hop's merges run side by side, so a
    # hop costs its slowest merge
    hops, cur = [], [stacked[i] for i in range(K)]
    while len(cur) > 1:
        nxt, worst = [], 0.0
        for i in range(0, len(cur) - 1, 2):
            m, ms = timed(lambda a=cur[i], b=cur[i + 1]: sheep_amd.merge_trees(a, b, ctx=ctx))
            nxt.append(m)
            worst = max(worst, ms)
        if len(cur) % 2:
            nxt.append(cur[-1])
        hops.append(worst)
        cur = nxt
    torch.cuda.synchronize()
    time.sleep(gap)
    print(json.dumps({"scale": scale, "shards": K, "map_ms": maps, "merge_ms": merges,
                      "binomial_hop_ms": hops, "binomial_equals_whole": bool(torch.equal(cur[0], whole)),
                      "merge_equals_whole": bool(torch.equal(merged, whole))}))


if __name__ == "__main__":
    main()
