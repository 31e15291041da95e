#!/usr/bin/env python3
"""Time the reduce step alone: two half-shard trees of RMAT-<scale> merged on one GPU.

    python tools/merge_probe.py [scale] [reps]

Prints the merge's wall time per call and the per-region device times (HIP events), and
checks the merged tree against the whole-graph tree."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import sheep_amd
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ctx = sheep_amd.Context(0)
    rec = sheep_amd.rmat(scale, 16, scale, ctx=ctx)
    s = sheep_amd.degree_sequence(rec, ctx=ctx)
    R = rec.shape[0]
    a = sheep_amd.build_tree(rec[: R // 2], s, ctx=ctx)
    b = sheep_amd.build_tree(rec[R // 2:], s, ctx=ctx)
    whole = sheep_amd.build_tree(rec, s, ctx=ctx)
    m = sheep_amd.merge_trees(a, b, ctx=ctx)
    assert torch.equal(m, whole), "merged tree differs from the whole-graph tree"
    torch.cuda.synchronize()
    ctx.timing(True)
    ctx.timer_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        m = sheep_amd.merge_trees(a, b, ctx=ctx)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    print(f"RMAT-{scale}: n={s.n} merge {1e3 * t:.2f} ms/call")
    for name in ctx.timer_names():
        ms, launches, nbytes = ctx.timer(name)
        print(f"  {name:16s} {ms / reps:8.3f} ms/call  launches {launches // reps}")


if __name__ == "__main__":
    main()
