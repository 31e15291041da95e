#!/usr/bin/env python3
"""The 8-GPU RMAT-26 step projected from one-GPU measurements.

    python tools/projection.py BENCH_8SHARDS.json SHARD_TRACE.json [--ranks 8]

BENCH_8SHARDS.json: `bench.py --scale 26 --shards 8` (the eight shard maps one after another
on one GPU, then the K-way merge, kids and partition): its per-shard regions divided by the
shard count are one rank's share.  SHARD_TRACE.json: `tools/shard_trace.py 26 2 8` (one
shard's map and the K-way merge timed alone, and the binomial schedule's pairwise merges hop
by hop).  The two transfers (the degree all-reduce and the partial trees' way to rank 0) are
not measurable on one GPU: they are modelled from MI355X_MICROARCH.md's xGMI figures and
marked as such.  Prints a markdown table per schedule and one JSON line."""
import argparse
import json

LINK_GBS = 50.0      # one xGMI link, one direction, as achieved by a 262 MB point-to-point copy (model)
RING_GBS = 350.0     # all-reduce bus bandwidth per GPU over 7 links (model)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench")
    ap.add_argument("trace")
    ap.add_argument("--ranks", type=int, default=8)
    a = ap.parse_args()
    b = json.load(open(a.bench))
    t = json.load(open(a.trace))
    P = a.ranks
    ph = {k: v["ms_per_step"] for k, v in b["phases"].items()}
    S = b["config"]["shards"]
    assert S == P, f"the bench line maps {S} shards, the projection is for {P} ranks"
    vs = b["config"]["vertex_slots"]
    n = b["config"]["tree_nodes"]
    tree_mb = n * 8 / 1e6
    deg_mb = vs * 4 / 1e6
    one = lambda k: ph.get(k, 0.0) / S   # one rank's share of a per-shard region
    rows = [
        ("degree count of the shard", "every rank", one("degree"), f"`degree` {ph.get('degree', 0):.2f} / {S}"),
        (f"degree all-reduce, {deg_mb:.0f} MB", "all (RCCL ring)", 2 * (P - 1) / P * deg_mb / RING_GBS,
         f"model: 2 x {P - 1}/{P} x {deg_mb:.0f} MB at {RING_GBS:.0f} GB/s per GPU"),
        ("heads histogram + sequence sort", "every rank (replicated)", one("degree_heads") + ph.get("sequence", 0.0),
         f"`degree_heads` {ph.get('degree_heads', 0):.2f} / {S} + `sequence` {ph.get('sequence', 0):.2f}"),
        ("relabel + pst + elimination tree of the shard", "every rank",
         one("relabel") + one("pst_group") + one("etree"),
         f"(`relabel` {ph.get('relabel', 0):.2f} + `pst_group` {ph.get('pst_group', 0):.2f} + `etree` "
         f"{ph.get('etree', 0):.2f}) / {S}"),
    ]
    tail = [("kids + partition", "rank 0", ph.get("kids", 0.0) + ph.get("partition", 0.0),
             f"`kids` {ph.get('kids', 0):.2f} + `partition` {ph.get('partition', 0):.2f}")]
    par_mb = n * 4 / 1e6
    kway = rows + [
        (f"gather of {P - 1} partial trees' parents, {P - 1} x {par_mb:.0f} MB", "into rank 0", par_mb / LINK_GBS,
         f"model: one transfer per xGMI link at {LINK_GBS:.0f} GB/s"),
        (f"pst reduce to rank 0, {par_mb:.0f} MB", "all (RCCL)", (P - 1) / P * par_mb / RING_GBS,
         f"model: {P - 1}/{P} x {par_mb:.0f} MB at {RING_GBS:.0f} GB/s per GPU"),
        (f"K-way merge of {P} trees", "rank 0", ph.get("merge", 0.0), f"`merge` {ph.get('merge', 0):.2f}"),
    ] + tail
    hops = t.get("binomial_hop_ms", [])
    binom = rows + [(f"binomial hop {i + 1}: send {tree_mb:.0f} MB + pairwise merge", "half the remaining ranks",
                     tree_mb / LINK_GBS + h, f"shard_trace `binomial_hop_ms`[{i}] {h:.2f} + model transfer")
                    for i, h in enumerate(hops)] + tail
    single = b.get("single_gpu_ms")
    out = {}
    for name, tab in (("kway", kway), ("binomial", binom)):
        tot = sum(r[2] for r in tab)
        out[name] = round(tot, 2)
        print(f"\n**{name}** (projected step {tot:.1f} ms)\n")
        print("| part of the step | on whom | ms (projected) | from |")
        print("|---|---|---|---|")
        for r in tab:
            print(f"| {r[0]} | {r[1]} | {r[2]:.2f} | {r[3]} |")
    print()
    print(json.dumps({"projected_ms": out, "map_alone_ms": t.get("map_ms"), "merge_alone_ms": t.get("merge_ms"),
                      "binomial_hop_ms": hops}))


if __name__ == "__main__":
    main()
