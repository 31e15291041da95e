#!/usr/bin/env python3
"""K shard trees of RMAT-<scale>, then `reps` K-way merges (sheep_merge_trees_many), for a
kernel trace of the merge alone:

    rocprofv3 --kernel-trace -d t -o run --output-format csv -- python tools/merge_trace.py 26 3 8
    python tools/trace_step.py t/.../run_kernel_trace.csv --levels --from k_tree_count

The last merge is checked against the whole-graph tree."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import sheep_amd
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    ctx = sheep_amd.Context(0)
    rec = sheep_amd.rmat(scale, 16, scale, ctx=ctx)
    s = sheep_amd.degree_sequence(rec, ctx=ctx)
    R = rec.shape[0]
    stacked = torch.stack([sheep_amd.build_tree(rec[i * R // K:(i + 1) * R // K], s, ctx=ctx) for i in range(K)])
    whole = sheep_amd.build_tree(rec, s, ctx=ctx)
    del rec
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = sheep_amd.merge_trees_many(stacked, ctx=ctx)
        torch.cuda.synchronize()
        print(f"K-way merge of {K} trees: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
    assert torch.equal(m, whole), "K-way merge differs from the whole-graph tree"
    print("merged tree == whole-graph tree")


if __name__ == "__main__":
    main()
