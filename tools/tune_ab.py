#!/usr/bin/env python3
"""A/B of sheep_tuning variants on the sparse etree inputs of the 8-GPU step, on one GPU:
one 1/K edge shard's map (a rank's map) and the K-way merge of the K shard trees (rank 0's
reduce), each variant run `reps` times interleaved with the others, every result checked
against the default tuning's whole-graph tree.

    python tools/tune_ab.py SCALE REPS K 'name:field=v,field=v' ...

Prints one JSON line: per variant the median host wall ms (after a device sync) of the map
and of the merge, and whether its merge equals the whole graph's tree."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import sheep_amd
    scale, reps, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    variants = [("default", {})]
    for a in sys.argv[4:]:
        name, kv = a.split(":", 1)
        variants.append((name, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
    ctx = sheep_amd.Context(0)
    rec = sheep_amd.rmat(scale, 16, scale, ctx=ctx)
    s = sheep_amd.degree_sequence(rec, ctx=ctx)
    R = rec.shape[0]
    whole = sheep_amd.build_tree(rec, s, ctx=ctx)
    shards = [rec[i * R // K:(i + 1) * R // K] for i in range(K)]
    stacked = torch.stack([sheep_amd.build_tree(sh, s, ctx=ctx) for sh in shards])

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return out, (time.perf_counter() - t0) * 1e3

    res = {name: {"map_ms": [], "merge_ms": [], "merge_ok": True, "map_ok": True} for name, _ in variants}
    for _ in range(reps):
        for name, kv in variants:
            ctx.set_tuning(**kv) if kv else ctx.set_tuning()
            t, ms = timed(lambda: sheep_amd.build_tree(shards[0], s, ctx=ctx))
            res[name]["map_ms"].append(round(ms, 3))
            res[name]["map_ok"] &= bool(torch.equal(t, stacked[0]))
            m, ms = timed(lambda: sheep_amd.merge_trees_many(stacked, ctx=ctx))
            res[name]["merge_ms"].append(round(ms, 3))
            res[name]["merge_ok"] &= bool(torch.equal(m, whole))
    for name, _ in variants:
        r = res[name]
        r["map_median"] = statistics.median(r["map_ms"])
        r["merge_median"] = statistics.median(r["merge_ms"])
    print(json.dumps({"scale": scale, "shards": K, "reps": reps, "variants": dict(variants), "results": res}))


if __name__ == "__main__":
    main()
