"""Worker of tests/test_tuning.py (one GPU process for every configuration): the map (and,
with "merge", the K-way merge of two half trees) of one graph under each sheep_tuning
variant, every tree compared with the oracle's; SHEEP_DEBUG=etree (set by the parent)
writes the etree's branch statistics to stderr, each configuration's block behind a
"=== config i" line.  Prints one JSON line: per configuration, whether the tree (and the
merge) equal the oracle's.

    python tests/tuning_worker.py GRAPH.npz CONFIGS.json
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch
    import oracle
    import sheep_amd
    g = np.load(sys.argv[1])
    configs = json.load(open(sys.argv[2]))
    tail, head = g["tail"].astype(np.uint32), g["head"].astype(np.uint32)
    rec = np.zeros((len(tail), 3), np.uint32)
    rec[:, 0], rec[:, 1] = tail, head
    rec[:, 2] = np.float32(1.0).view(np.uint32)
    d = torch.from_numpy(rec.view(np.int32)).cuda()
    seq = oracle.sequence(tail, head)
    op, ow = oracle.build_tree(tail, head, seq)
    R = len(tail)
    halves = [oracle.build_tree(tail, head, seq, i + 1, 2) for i in range(2)]
    ctx = sheep_amd.Context(0)
    s = sheep_amd.degree_sequence(d, ctx=ctx)
    assert np.array_equal(s.numpy(), seq)
    out = []
    for i, cfg in enumerate(configs):
        print(f"=== config {i} {json.dumps(cfg)}", file=sys.stderr, flush=True)
        ctx.set_tuning(**cfg.get("tune", {}))
        tree = sheep_amd.build_tree(d, s, ctx=ctx)
        torch.cuda.synchronize()
        t = tree.cpu().numpy().view(np.uint32)
        r = {"config": cfg, "tree": bool(np.array_equal(t[:, 0], op) and np.array_equal(t[:, 1], ow))}
        if cfg.get("merge"):
            hs = torch.stack([sheep_amd.build_tree(d[(k * R) // 2:((k + 1) * R) // 2], s, ctx=ctx) for k in range(2)])
            ht = hs.cpu().numpy().view(np.uint32)
            r["halves"] = all(np.array_equal(ht[k][:, 0], halves[k][0]) and np.array_equal(ht[k][:, 1], halves[k][1])
                              for k in range(2))
            m = sheep_amd.merge_trees_many(hs, ctx=ctx).cpu().numpy().view(np.uint32)
            r["merge"] = bool(np.array_equal(m[:, 0], op) and np.array_equal(m[:, 1], ow))
        sys.stderr.flush()
        out.append(r)
    ctx.set_tuning()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
