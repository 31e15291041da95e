#!/usr/bin/env python3
"""Time the reduce step alone on one GPU: K shard trees of RMAT-<scale> reduced to one.

    python tools/merge_probe.py [scale] [reps] [K] [nparts]

Three schedules are timed: the binomial pairwise schedule's critical path (the
ceil(log2 K) merges rank 0 performs; the other ranks' merges are precomputed,
untimed, as they would run on their own GPUs), one K-way merge
(sheep_merge_trees_many), and the split K-way merge (sheep_merge_trees_part over nparts,
a power of two, default 2): each part is timed on its own (as nparts GPUs would run them
side by side) and the slowest part is the critical path.  Every result is checked against the
whole-graph tree.
Prints wall time per reduction and the per-region device times (HIP events)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import sheep_amd
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    NP = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    ctx = sheep_amd.Context(0)
    rec = sheep_amd.rmat(scale, 16, scale, ctx=ctx)
    s = sheep_amd.degree_sequence(rec, ctx=ctx)
    R = rec.shape[0]
    parts = [sheep_amd.build_tree(rec[i * R // K:(i + 1) * R // K], s, ctx=ctx) for i in range(K)]
    whole = sheep_amd.build_tree(rec, s, ctx=ctx)
    del rec
    # binomial schedule: at hop r, rank i (i % 2r == 0) merges rank i + r's tree
    inputs = []   # rank 0's (left, right) pair per hop
    cur = list(parts)
    r = 1
    while r < K:
        nxt = list(cur)
        for i in range(0, K, 2 * r):
            if i + r < K:
                if i == 0:
                    inputs.append(cur[i + r])
                nxt[i] = sheep_amd.merge_trees(cur[i], cur[i + r], ctx=ctx)
        cur = nxt
        r *= 2
    assert torch.equal(cur[0], whole), "pairwise merge differs from the whole-graph tree"
    stacked = torch.stack(parts)
    m = sheep_amd.merge_trees_many(stacked, ctx=ctx)
    assert torch.equal(m, whole), "K-way merge differs from the whole-graph tree"
    print(f"RMAT-{scale}: n={s.n} K={K} hops={len(inputs)}")
    if NP & (NP - 1) == 0:
        asm = None
        worst = 0.0
        for p in range(NP):
            for rep in range(reps + 1):                      # the first run warms the workspaces
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                part, lo, hi = sheep_amd.merge_trees_part(stacked, p, NP, ctx=ctx)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
            worst = max(worst, dt)
            print(f"  split part {p}: nodes [{lo}, {hi}) {1e3 * dt:.2f} ms")
            if asm is None:
                asm = part.clone()
            asm[lo:hi, 0] = part[lo:hi, 0]
        assert torch.equal(asm, whole), "split merge differs from the whole-graph tree"
        print(f"split K-way merge over {NP} parts: {1e3 * worst:.2f} ms critical path (slowest part)")
    for label, fn in (("pairwise critical path", None), ("one K-way merge", None)):
        torch.cuda.synchronize()
        ctx.timing(True)
        ctx.timer_reset()
        t0 = time.perf_counter()
        for _ in range(reps):
            if label.startswith("pairwise"):
                acc = parts[0]
                for other in inputs:
                    acc = sheep_amd.merge_trees(acc, other, ctx=ctx)
            else:
                sheep_amd.merge_trees_many(stacked, ctx=ctx)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        ctx.timing(False)
        print(f"{label}: {1e3 * t:.2f} ms per reduction")
        for name in ctx.timer_names():
            ms, launches, nbytes = ctx.timer(name)
            print(f"  {name:16s} {ms / reps:8.3f} ms  launches {launches / reps:g}")


if __name__ == "__main__":
    main()
