#!/usr/bin/env python3
"""bench.py — Sheep's map/reduce partitioning path on MI355X (BASELINE.json metric).

One step = the whole hot path over one synthetic graph already resident in HBM:

  degree count (per edge shard) -> [RCCL all-reduce of degrees] -> degree sequence
  -> per-shard elimination tree (map) -> [gather to rank 0 + one K-way tree merge]
  -> makeKids + partition_tree forwardPartition (k parts) on rank 0

(reference: graph2tree.cpp:161-216 `-ir` + partition_tree.cpp:130-143).
Every computation runs in libsheep_hip.so's HIP kernels; the CPU oracle is only timed
as the `cpu_baseline` leg (rank 0, N=1) on a bounded sample.

    python bench.py [--gpus N --steps K --warmup W --scale 26 --ef 16 --k 64]

For N > 1 launch with torch.distributed.run (one process per GPU, RCCL over xGMI).
The graph is fixed as N grows (edge shards of one RMAT graph): "scaling": "strong".
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level table)
# Leaf regions (one kernel or one fused kernel family per launch); aggregates such as
# "etree" / "partition" / "sequence" are reported in phases but not rooflined.
LEAF = ("degree", "degree_heads", "relabel", "pst_group", "etree_split", "etree_union", "etree_cross",
        "etree_apply", "etree_compact", "evaluate")
# kernels of a region, for roofline.traffic from the committed PMC passes (tools/pmc_traffic.py);
# regions whose kernels are shared with other regions (histograms, packs) get traffic null
REGION_KERNELS = {"relabel": ["k_relabel_scatter", "k_relabel_gather"], "degree": ["k_degree"], "etree_split": ["k_split_count", "k_split_write"],
                  "etree_cross": ["k_cross_find"], "etree_apply": ["k_cross_apply", "k_level_clean"],
                  "etree_compact": ["k_compact_edges"], "etree_bucket": ["k_bucket_count", "k_bucket_scatter"]}
PMC_FILE = os.path.join(ROOT, "profiles", "r1", "pmc_traffic_rmat{scale}.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--ef", type=int, default=16)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--seed", type=int, default=None, help="RMAT seed (default: the scale, SURVEY §8d)")
    ap.add_argument("--cpu-scale", type=int, default=22, help="RMAT scale of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo stages the exchanges through host memory (rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearse N ranks on a 1-GPU box; needs gloo)")
    ap.add_argument("--reduce", default="kway", choices=("kway", "binomial"),
                    help="kway: gather the partial trees to rank 0 and merge them in one pass; "
                         "binomial: ceil(log2 N) send/recv hops with a pairwise merge each")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 also builds the whole-graph tree and checks the merged one against it")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist
    import sheep_amd
    from sheep_amd import dist as sdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    if a.same_device:
        if a.dist_backend != "gloo":
            raise SystemExit("--same-device needs --dist-backend gloo (RCCL wants one rank per GPU)")
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    seed = a.scale if a.seed is None else a.seed

    ctx = sheep_amd.Context(local)
    rec = sheep_amd.rmat(a.scale, a.ef, seed, ctx=ctx)          # whole graph, identical on every rank
    R = rec.shape[0]
    beg, end = sdist.shard_bounds(R, rank, world)               # contiguous edge shard (graph2tree -l)
    shard = rec[beg:end]
    vs_cap = 1 << a.scale
    deg = torch.zeros(vs_cap, dtype=torch.int32, device="cuda")

    def step():
        deg.zero_()
        _, max_slot = sheep_amd.degree_count(shard, mode="llama", deg=deg, ctx=ctx)
        vs = max_slot
        if world > 1:                                           # sequence.h:72,78 MPI_Allreduce
            vs = sdist.allreduce_degrees(deg, max_slot)
        s = sheep_amd.sequence_from_degrees(deg, vs, ctx=ctx)
        tree = sheep_amd.build_tree(shard, s, ctx=ctx)
        if world > 1 and a.reduce == "kway":                    # reduce to rank 0 (jnode.cpp:241) in one pass
            tree = sdist.reduce_trees_kway(tree, lambda t: sheep_amd.merge_trees_many(t, ctx=ctx), rank, world)
        elif world > 1:                                         # binomial reduce to rank 0 (jnode.cpp:241)
            tree = sdist.reduce_trees(tree, lambda x, y: sheep_amd.merge_trees(x, y, ctx=ctx), rank, world)
        res = None
        if rank == 0:
            kids = sheep_amd.KidTable(tree, ctx)
            res = sheep_amd.partition(s, tree, a.k, kids=kids, ctx=ctx)
            kids.close()
        return s, tree, res

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    barrier()
    ctx.timing(True)
    ctx.timer_reset()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s, tree, res = step()
    barrier()
    t = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64, device="cuda" if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())

    # per-region device timings (HIP events on the context stream)
    phases = {}
    for name in ctx.timer_names():
        ms, launches, nbytes = ctx.timer(name)
        phases[name] = {"ms_per_step": round(ms / a.steps, 4), "launches": launches, "alg_bytes": nbytes}
    ctx.timing(False)
    roof = None
    leaf = [(phases[n]["ms_per_step"], n) for n in LEAF if n in phases and phases[n]["launches"]]
    if leaf:
        _, dom = max(leaf)
        p = phases[dom]
        ms_launch = p["ms_per_step"] * a.steps / p["launches"]
        b_launch = p["alg_bytes"] / p["launches"]
        ach = b_launch / (ms_launch * 1e-3) / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "alg_bytes_per_launch": int(b_launch), "ms_per_launch": round(ms_launch, 4)}
        roof.update(pmc_traffic(a, dom, p["launches"] / a.steps))

    verified = None
    if a.verify and rank == 0:                                  # merged tree == whole-graph tree
        whole = sheep_amd.build_tree(rec, s, ctx=ctx)
        verified = bool(torch.equal(whole, tree))
        del whole
        if not verified:
            print("bench: merged tree differs from the whole-graph tree", file=sys.stderr, flush=True)

    out = None
    if rank == 0:
        n = s.n
        b_alg = 32 * R + 14 * s.pos_size + 20 * n
        value = R * a.steps / t
        out = {
            "metric": "edges/s seq+tree+partition",
            "value": round(value, 1),
            "unit": "edges/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * t / a.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (Graph500 RMAT, seeded, self-loops/duplicates removed)",
            "config": {"workload": f"RMAT-{a.scale} ef{a.ef}, k={a.k}", "records": R, "vertex_slots": s.pos_size,
                       "tree_nodes": n, "k": a.k, "created": res.created, "packing_nodes": res.packing_nodes,
                       "heavy_nodes": res.heavy_nodes, "seed": seed,
                       "parallelism": f"edge-shards x{world}" + (f", {a.reduce} reduce" if world > 1 else "")
                       + ("" if a.dist_backend == "nccl" else f" ({a.dist_backend}"
                          + (", one device" if a.same_device else "") + ")")},
            "path_roofline": {"alg_bytes": b_alg, "achieved_GBs": round(b_alg * a.steps / t / 1e9, 2),
                              "frac": round(b_alg * a.steps / t / 1e9 / (HBM_PEAK_GBS * world), 4)},
            "roofline": roof,
            "phases": phases,
        }
        if verified is not None:
            out["verified_vs_whole_graph"] = verified
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a, ctx)
    del rec, shard
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def pmc_traffic(a, region, launches_per_step):
    """roofline.traffic: HBM bytes per launch of the region's kernels from the committed
    rocprofv3 PMC passes for this workload (FETCH_SIZE and WRITE_SIZE, separate passes);
    null when there is no profile for it or the kernels are shared between regions."""
    path = PMC_FILE.format(scale=a.scale)
    ks = REGION_KERNELS.get(region)
    if not ks or not os.path.exists(path):
        return {}
    prof = json.load(open(path))
    if prof.get("workload") != f"RMAT-{a.scale} ef{a.ef}, k={a.k}" or any(k not in prof["kernels"] for k in ks):
        return {}
    raw = sum(prof["kernels"][k]["traffic_raw"] for k in ks) / launches_per_step
    cor = sum(prof["kernels"][k]["traffic_stream_corrected"] for k in ks) / launches_per_step
    return {"traffic": int(raw), "traffic_stream_corrected": int(cor),
            "traffic_source": os.path.relpath(path, ROOT) + " (FETCH_SIZE + WRITE_SIZE; Infinity-Cache hits included)"}


def cpu_baseline(a, ctx):
    """CPU baseline on a bounded sample: RMAT-<cpu-scale> from the same generator,
    seq + tree + partition(k), one core, graph already in memory.

    kind "reference": the reference's own lib/ code (degreeSequence, JTree + makeKids,
    Partition -- the graph2tree.cpp:185-208 flow) compiled from /root/reference into
    oracle/_ref/ref_harness (`time` mode).  The oracle restatement (oracle/sheep_oracle.cpp)
    is timed beside it as `port`.  Test infrastructure timed as a baseline; never the
    measured path."""
    import subprocess
    import tempfile
    import numpy as np
    import sheep_amd
    import oracle
    sc = a.cpu_scale
    d = sheep_amd.rmat(sc, a.ef, sc, ctx=ctx)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    del d
    tail, head = np.ascontiguousarray(h[:, 0]), np.ascontiguousarray(h[:, 1])
    R = len(tail)
    sample = f"RMAT-{sc} ef{a.ef} seed {sc} ({R} records), seq+tree+partition k={a.k}, single-threaded"
    t0 = time.perf_counter()
    seq = oracle.sequence(tail, head)
    p, w = oracle.build_tree(tail, head, seq)
    oracle.partition(p, w, seq, a.k)
    tp = time.perf_counter() - t0
    port = {"value": round(R / tp, 1), "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"{sample}, oracle/sheep_oracle.cpp, {tp:.2f} s"}
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return port
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, f"rmat{sc}.dat")
        h.tofile(path)
        del h
        r = subprocess.run([harness, "time", path, str(a.k)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        port["reference_error"] = r.stderr.strip()[-300:]
        return port
    tr = json.loads(r.stdout.strip().splitlines()[-1])["seconds"]
    return {"value": round(R / tr, 1), "unit": "edges/s", "cores": 1, "kind": "reference",
            "sample": f"{sample}, reference lib/ (degreeSequence + JTree + makeKids + Partition, "
                      f"graph2tree.cpp:185-208) built by oracle/ref/Makefile, {tr:.2f} s",
            "port": port}


if __name__ == "__main__":
    main()
