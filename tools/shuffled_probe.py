#!/usr/bin/env python3
"""Times the degree pass and the rest of the path on a shuffled copy of a BASELINE graph
(C3 RMAT-26 or C4 Chung-Lu): a debugging probe for the unsorted-records paths.

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
    if which == "c4":
        d = sheep_amd.powerlaw(sheep_amd.TWITTER_VERTICES, 2_222_000_000, 1.9, 2010)
        cap = sheep_amd.TWITTER_VERTICES
    else:
        d = sheep_amd.rmat(26, 16, 26)
        cap = 1 << 26
    g = torch.Generator(device=d.device)
    g.manual_seed(4010)
    d = d[torch.randperm(d.shape[0], device=d.device, generator=g, dtype=torch.int32)]
    flip = torch.rand(d.shape[0], device=d.device, generator=g) < 0.5
    tail, head = d[:, 0].clone(), d[:, 1].clone()
    d[:, 0] = torch.where(flip, head, tail)
    d[:, 1] = torch.where(flip, tail, head)
    del tail, head, flip
    torch.cuda.synchronize()
    print(f"{which}: {d.shape[0]} records shuffled", file=sys.stderr, flush=True)
    t0 = time.time()
    s = sheep_amd.degree_sequence(d, vs_cap=cap)
    print(f"degree_sequence {time.time() - t0:.2f} s n={s.n}", file=sys.stderr, flush=True)
    t0 = time.time()
    tree = sheep_amd.build_tree(d, s)
    torch.cuda.synchronize()
    print(f"build_tree {time.time() - t0:.2f} s", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
