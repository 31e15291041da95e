#!/usr/bin/env python3
"""Times the record shuffle (bench.shuffled), the degree pass and the tree on a shuffled copy of a BASELINE graph (C3 RMAT-26 or C4 Chung-Lu): a debugging
probe for the unsorted-records paths.

    python tools/shuffled_probe.py rmat26|c4
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import sheep_amd
    which = sys.argv[1]
    t0 = time.time()

    def mark(what):
        torch.cuda.synchronize()
        print(f"{time.time() - t0:8.2f} s  {what}", file=sys.stderr, flush=True)

    if which == "c4":
        d = sheep_amd.powerlaw(sheep_amd.TWITTER_VERTICES, 2_222_000_000, 1.9, 2010)
        cap = sheep_amd.TWITTER_VERTICES
    else:
        d = sheep_amd.rmat(26, 16, 26)
        cap = 1 << 26
    mark(f"generated {d.shape[0]} records")
    from bench import shuffled
    out = shuffled(d, 4010)
    mark("shuffled")
    del d
    t1 = time.time()
    s = sheep_amd.degree_sequence(out, vs_cap=cap)
    mark(f"degree_sequence {time.time() - t1:.2f} s n={s.n}")
    t1 = time.time()
    tree = sheep_amd.build_tree(out, s)
    mark(f"build_tree {time.time() - t1:.2f} s")


if __name__ == "__main__":
    main()
