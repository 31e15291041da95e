#!/usr/bin/env python3
"""bench.py — Sheep's map/reduce partitioning path on MI355X (BASELINE.json metric).

One step = the whole hot path over one synthetic graph already resident in HBM:

  degree count (per edge shard) -> [RCCL all-reduce of degrees] -> degree sequence
  -> per-shard elimination tree (map) -> [gather to rank 0 + one K-way tree merge]
  -> makeKids + partition_tree forwardPartition (k parts) on rank 0

(reference: graph2tree.cpp:161-216 `-ir` + partition_tree.cpp:130-143).
After the timed steps the ECV(down)/balance evaluator (partition.cpp:475-521) is timed
on its own ("timed and rooflined separately"): on one GPU over all
records; on N GPUs sharded — parts broadcast (Partition::mpi_sync), per-shard owner
bitsets, a binomial OR-reduction to rank 0, one node pass.

Every computation runs in libsheep_hip.so's HIP kernels; the reference's own lib/ code
(oracle/_ref, built from /root/reference) is only timed as the `cpu_baseline` leg
(rank 0, N=1) on a bounded sample.

    python bench.py [--gpus N --steps K --warmup W --scale 26 --ef 16 --k 64 --shuffle]

For N > 1 launch with torch.distributed.run (one process per GPU, RCCL over xGMI).
The graph is fixed as N grows (edge shards of one RMAT graph): "scaling": "strong".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level table)
# Leaf regions (one kernel family per region, HIP events on the context stream) and the
# kernels each runs, for roofline.traffic from the committed PMC file (tools/pmc_traffic.py).
# Algorithmic bytes per region: DESIGN.md §5 (a stated per-region extension of SURVEY
# §8(d), whose B_alg covers the whole path).  Regions whose kernels are shared with other
# regions (scans, radix passes) get traffic null.
LEAF = ("degree", "degree_heads", "sequence", "relabel", "pst_group", "etree_split", "etree_union", "etree_cross",
        "etree_apply", "merge", "kids", "partition")
REGION_KERNELS = {"degree": ["k_degree_fused"], "relabel": ["k_relabel_scatter", "k_relabel_gather"],
                  "etree_split": ["k_split_count", "k_split_write"], "etree_union": ["k_hook_round", "k_hook_finish", "k_light_top"],
                  "etree_cross": ["k_cross_find"], "etree_apply": ["k_cross_apply", "k_level_clean"],
                  "evaluate": ["k_pp", "k_eval_records", "k_eval_nodes"]}
PMC_FILE = os.path.join(ROOT, "profiles", "r2", "pmc_traffic_rmat{scale}_k{k}.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--ef", type=int, default=16)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--seed", type=int, default=None, help="generator seed (default: the RMAT scale; 2010 for powerlaw)")
    ap.add_argument("--graph", default="rmat", choices=("rmat", "powerlaw"),
                    help="rmat: Graph500 RMAT (C2/C3/C5); powerlaw: Chung-Lu at twitter-2010 scale (C4)")
    ap.add_argument("--draws", type=int, default=2_222_000_000,
                    help="powerlaw edge draws (about 1.468e9 records survive the dedup, twitter-2010's count)")
    ap.add_argument("--shards", type=int, default=1,
                    help="one GPU: edge shards mapped one after another and merged K-way (graphs of >= 2^32 "
                         "records, e.g. RMAT-28; C5 on one GPU)")
    ap.add_argument("--shuffle", action="store_true",
                    help="records in a random order, half with tail/head swapped (a generic edge list)")
    ap.add_argument("--eval-reps", type=int, default=3, help="timed evaluator runs (0: skip)")
    ap.add_argument("--cpu-scale", type=int, default=22, help="RMAT scale of the CPU-baseline sample")
    ap.add_argument("--cpu-ranks", type=int, default=16, help="MPI ranks of the reference CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="gloo stages the exchanges through host memory (rehearsal)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (rehearse N ranks on a 1-GPU box; needs gloo)")
    ap.add_argument("--reduce", default="kway", choices=("kway", "split", "binomial"),
                    help="kway: gather the partial trees to rank 0 and merge them in one pass; "
                         "split: ranks 0 and 1 receive every partial tree and each merges one half of the "
                         "position range (rank 0 the heavier upper half), rank 1 sends its half's parents; "
                         "binomial: ceil(log2 N) send/recv hops with a pairwise merge each")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 also builds the whole-graph tree and checks the merged one against it")
    return ap.parse_args()


def shuffled(d, seed):
    """The records in a random order, half of them with tail and head swapped."""
    import torch
    g = torch.Generator(device=d.device)
    g.manual_seed(seed)
    out = d[torch.randperm(d.shape[0], device=d.device, generator=g)]
    flip = torch.rand(out.shape[0], device=d.device, generator=g) < 0.5
    tail = out[:, 0].clone()
    out[flip, 0] = out[flip, 1]
    out[flip, 1] = tail[flip]
    return out


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
    seed = (a.scale if a.graph == "rmat" else 2010) if a.seed is None else a.seed
    if a.shards > 1 and world > 1:
        raise SystemExit("--shards is the one-GPU form of the edge-shard path")

    reduce = a.reduce
    ctx = sheep_amd.Context(local)
    if a.graph == "rmat":                                       # whole graph, identical on every rank
        rec = sheep_amd.rmat(a.scale, a.ef, seed, ctx=ctx)
        vs_cap, workload = 1 << a.scale, f"RMAT-{a.scale} ef{a.ef}, k={a.k}"
    else:
        rec = sheep_amd.powerlaw(sheep_amd.TWITTER_VERTICES, a.draws, 1.9, seed, ctx=ctx)
        vs_cap, workload = sheep_amd.TWITTER_VERTICES, f"Chung-Lu power law (twitter-2010 scale), k={a.k}"
    if a.shards > 1:
        workload += f", {a.shards} shards on 1 GPU"
    if a.shuffle:
        rec = shuffled(rec, 1000 + seed)
    R = rec.shape[0]
    beg, end = sdist.shard_bounds(R, rank, world)               # contiguous edge shard (graph2tree -l)
    shard = rec[beg:end].contiguous() if world > 1 else rec
    del rec
    torch.cuda.empty_cache()
    deg = torch.zeros(vs_cap, dtype=torch.int32, device=f"cuda:{local}")
    subs = [shard[i * shard.shape[0] // a.shards:(i + 1) * shard.shape[0] // a.shards] for i in range(a.shards)]
    stack = [None]

    def step():
        deg.zero_()
        vs = 0
        for sub in subs:                                        # shards accumulate into one histogram
            _, max_slot = sheep_amd.degree_count(sub, mode="llama", deg=deg, ctx=ctx)
            vs = max(vs, max_slot)
        if world > 1:                                           # sequence.h:72,78 MPI_Allreduce
            vs = sdist.allreduce_degrees(deg, vs)
        s = sheep_amd.sequence_from_degrees(deg, vs, ctx=ctx)
        if a.shards > 1:                                        # map per shard, then ONE K-way merge
            if stack[0] is None or stack[0].shape[1] != s.n:
                stack[0] = torch.empty((a.shards, s.n, 2), dtype=torch.int32, device=f"cuda:{local}")
            for i, sub in enumerate(subs):
                sheep_amd.build_tree(sub, s, ctx=ctx, out=stack[0][i])
            tree = sheep_amd.merge_trees_many(stack[0], ctx=ctx)
        else:
            tree = sheep_amd.build_tree(shard, s, ctx=ctx)
        if world > 1 and reduce == "split":                     # the K-way merge split over the ranks
            tree = sdist.reduce_trees_split(tree, lambda st, p, q: sheep_amd.merge_trees_part(st, p, q, ctx=ctx),
                                            rank, world)
        elif world > 1 and reduce == "kway":                    # reduce to rank 0 (jnode.cpp:241) in one pass
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

    def max_over_ranks(t):
        if world > 1:
            tt = torch.tensor([t], dtype=torch.float64, device=f"cuda:{local}" if a.dist_backend == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
        return t

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
    t = max_over_ranks(time.perf_counter() - t0)

    # per-region device timings (HIP events on the context stream), timed steps only
    phases = {}
    for name in ctx.timer_names():
        ms, launches, nbytes = ctx.timer(name)
        phases[name] = {"ms_per_step": round(ms / a.steps, 4), "launches": launches, "alg_bytes": nbytes}
    ctx.timer_reset()

    evaluator = None
    if a.eval_reps > 0:
        evaluator = time_evaluator(a, ctx, shard, subs, s, res, rank, world, local, barrier, max_over_ranks)
    ctx.timing(False)

    verified = None
    if a.verify and rank == 0:                                  # merged tree == whole-graph tree
        if world == 1 and a.shards == 1:
            verified = True
        elif world == 1:
            verified = bool(torch.equal(sheep_amd.build_tree(shard, s, ctx=ctx), tree)) if R < (1 << 32) else None
        else:
            whole = sheep_amd.build_tree(sheep_amd.rmat(a.scale, a.ef, seed, ctx=ctx) if not a.shuffle else
                                         shuffled(sheep_amd.rmat(a.scale, a.ef, seed, ctx=ctx), 1000 + seed), s, ctx=ctx)
            verified = bool(torch.equal(whole, tree))
            del whole
        if not verified:
            print("bench: merged tree differs from the whole-graph tree", file=sys.stderr, flush=True)

    out = None
    if rank == 0:
        n = s.n
        b_alg = 32 * R + 14 * s.pos_size + 20 * n
        value = R * a.steps / t
        leaf = [(phases[x]["ms_per_step"], x) for x in LEAF if x in phases and phases[x]["launches"]]
        roof = None
        if leaf:
            _, dom = max(leaf)
            p = phases[dom]
            ms_launch = p["ms_per_step"] * a.steps / p["launches"]
            b_launch = p["alg_bytes"] / p["launches"]
            ach = b_launch / (ms_launch * 1e-3) / 1e9
            roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                    "alg_bytes_per_launch": int(b_launch), "ms_per_launch": round(ms_launch, 4)}
            roof.update(pmc_region(a, world, dom, p["launches"] / a.steps))
        path = {"alg_bytes": b_alg, "achieved_GBs": round(b_alg * a.steps / t / 1e9, 2),
                "frac": round(b_alg * a.steps / t / 1e9 / (HBM_PEAK_GBS * world), 4)}
        path.update(pmc_path(a, world, b_alg))
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
            "data": ("synthetic (Graph500 RMAT, seeded" if a.graph == "rmat" else
                     f"synthetic (Chung-Lu power law, gamma 1.9, {sheep_amd.TWITTER_VERTICES} vertices, seeded")
                    + ", self-loops/duplicates removed"
                    + (", records shuffled and half of them reversed)" if a.shuffle else ", records (tail, head)-sorted)"),
            "config": {"workload": workload, "records": R, "vertex_slots": s.pos_size,
                       "tree_nodes": n, "k": a.k, "created": res.created, "packing_nodes": res.packing_nodes,
                       "heavy_nodes": res.heavy_nodes, "seed": seed, "shuffled": a.shuffle, "shards": a.shards,
                       "parallelism": f"edge-shards x{world}" + (f", {reduce} reduce" if world > 1 else "")
                       + ("" if a.dist_backend == "nccl" else f" ({a.dist_backend}"
                          + (", one device" if a.same_device else "") + ")")},
            "roofline": roof,
            "path_roofline": path,
            "evaluator": evaluator,
            "phases": phases,
        }
        if verified is not None:
            out["verified_vs_whole_graph"] = verified
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a, ctx)
    del shard
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


def time_evaluator(a, ctx, shard, subs, s, res, rank, world, local, barrier, max_over_ranks):
    """ECV(down) + balance (evaluate(graph, seq), partition.cpp:475-521), timed on its own:
    one GPU — sheep_evaluate over all records; N GPUs — parts broadcast, per-shard
    bitsets, binomial OR-reduction to rank 0, node pass there.  B_eval per SURVEY §8(d)."""
    import torch
    import sheep_amd
    from sheep_amd import dist as sdist
    R_total = shard.shape[0] * world if world > 1 else shard.shape[0]
    times, ev = [], None
    parts0 = res.parts if rank == 0 else None
    for _ in range(a.eval_reps):
        barrier()
        t0 = time.perf_counter()
        if world == 1 and a.shards == 1:
            ev = sheep_amd.evaluate(shard, s, parts0, what=sheep_amd.EVAL_DOWN, ctx=ctx)
        elif world == 1:                                         # the shards' bitsets, then one node pass
            e = sheep_amd.ShardedEvaluator(s, parts0, sheep_amd.EVAL_DOWN, ctx=ctx)
            for sub in subs:
                e.add(sub)
            ev = e.finish()
        else:
            parts = sdist.sync_parts(parts0, s.pos_size, torch.device("cuda", local))
            nparts = torch.tensor([0 if rank else sheep_amd.ShardedEvaluator.num_parts(parts, s, ctx)],
                                  dtype=torch.int64, device=f"cuda:{local}" if a.dist_backend == "nccl" else "cpu")
            dist_broadcast(nparts)
            e = sheep_amd.ShardedEvaluator(s, parts, sheep_amd.EVAL_DOWN, nparts=int(nparts.item()), ctx=ctx)
            e.add(shard)
            e = sdist.reduce_eval(e, rank, world)
            ev = e.finish() if rank == 0 else None
        barrier()
        times.append(max_over_ranks(time.perf_counter() - t0))
    if rank != 0:
        return None
    k = res.created
    b_eval = 24 * R_total + 4 * R_total + 2 * s.pos_size * ((k + 7) // 8)
    best = min(times)
    out = {"what": "ECV(down) + down balance", "ecv_down": ev.ecv_down, "max_down_bal": ev.max_down_bal,
           "ms": round(1e3 * best, 3), "reps": a.eval_reps, "alg_bytes": b_eval,
           "achieved_GBs": round(b_eval / best / 1e9, 2), "peak": HBM_PEAK_GBS * world,
           "frac": round(b_eval / best / 1e9 / (HBM_PEAK_GBS * world), 4),
           "edges_per_s": round(R_total / best, 1)}
    if world == 1:   # device time of the region (HIP events), beside the wall time
        ms, launches, _ = ctx.timer("evaluate")
        if launches:
            out["device_ms"] = round(ms / launches, 3)
    out.update(pmc_region(a, world, "evaluate", 1))
    return out


def dist_broadcast(t):
    import torch.distributed as dist
    from sheep_amd import dist as sdist
    if sdist._host_staged() and t.is_cuda:
        h = t.cpu()
        dist.broadcast(h, 0)
        t.copy_(h)
    else:
        dist.broadcast(t, 0)


def _pmc(a, world):
    path = PMC_FILE.format(scale=a.scale, k=a.k)
    if world != 1 or a.shuffle or a.graph != "rmat" or a.shards != 1 or not os.path.exists(path):
        return None, path
    prof = json.load(open(path))
    if prof.get("workload") != f"RMAT-{a.scale} ef{a.ef}, k={a.k}":
        return None, path
    return prof, path


def pmc_region(a, world, region, launches_per_step):
    """roofline.traffic: HBM bytes per launch of the region's kernels from the committed
    rocprofv3 PMC passes for this workload (FETCH_SIZE and WRITE_SIZE, separate passes,
    per path step as the difference of a 2-step and a 1-step run); null when there is no
    profile for it or the kernels are shared between regions."""
    prof, path = _pmc(a, world)
    ks = REGION_KERNELS.get(region)
    if prof is None or not ks:
        return {}
    sel = [v for v in prof["kernels"].values() if v["base"] in ks]
    if not sel:
        return {}
    key = "per_eval" if region == "evaluate" else "per_step"
    sel = [v for v in sel if key in v]
    if not sel:
        return {}
    raw = sum(v[key]["traffic_raw"] for v in sel) / launches_per_step
    cor = sum(v[key]["traffic_stream_corrected"] for v in sel) / launches_per_step
    return {"traffic": int(raw), "traffic_stream_corrected": int(cor),
            "traffic_source": os.path.relpath(path, ROOT) + " (FETCH_SIZE + WRITE_SIZE; Infinity-Cache hits included)"}


def pmc_path(a, world, b_alg):
    """The whole step's measured HBM traffic (every kernel of one path step) against B_alg."""
    prof, path = _pmc(a, world)
    if prof is None:
        return {}
    raw = sum(v["per_step"]["traffic_raw"] for v in prof["kernels"].values())
    cor = sum(v["per_step"]["traffic_stream_corrected"] for v in prof["kernels"].values())
    return {"traffic": int(raw), "traffic_stream_corrected": int(cor), "traffic_over_alg": round(raw / b_alg, 3),
            "traffic_source": os.path.relpath(path, ROOT)}


def cpu_info():
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_baseline(a, ctx):
    """CPU baseline on a bounded sample: RMAT-<cpu-scale> from the same generator.

    kind "reference": the reference's own lib/ code, compiled from /root/reference into
    oracle/_ref/ref_harness by oracle/ref/Makefile, run as the graph2tree `-r -p k` flow
    over MPI ranks (mpiexec -n P ref_harness mpi ...): each rank loads its edge shard
    (graph2tree -l semantics, untimed), then mpiSequence's degree all-reduce with
    degreeSequence's sort, JTree on the shard (map), JNodeTable::mpi_merge (the custom-op
    MPI_Reduce), makeKids + Partition(k) + mpi_sync on rank 0.  The timed region starts at
    a barrier after the load.  Test infrastructure timed as a baseline; never the
    measured path."""
    import shutil
    import subprocess
    import tempfile
    import numpy as np
    import sheep_amd
    sc = a.cpu_scale
    d = sheep_amd.rmat(sc, a.ef, sc, ctx=ctx)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    del d
    R = len(h)
    model, ncpu = cpu_info()
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    mpiexec = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
    if not os.path.exists(harness) or not mpiexec:
        return {"value": None, "unit": "edges/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/ref_harness or mpiexec missing on this host"}
    ranks = max(1, min(a.cpu_ranks, ncpu or 1))
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, f"rmat{sc}.dat")
        h.tofile(path)
        del h
        env = dict(os.environ, OMP_NUM_THREADS="1")
        r = subprocess.run([mpiexec, "-n", str(ranks), harness, "mpi", path, str(a.k)], capture_output=True,
                           text=True, timeout=900, env=env)
    if r.returncode != 0:
        return {"value": None, "unit": "edges/s", "cores": ranks, "kind": "reference",
                "sample": f"mpiexec failed: {r.stderr.strip()[-300:]}"}
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    sec = res["seconds"]
    return {"value": round(R / sec, 1), "unit": "edges/s", "cores": ranks, "kind": "reference",
            "cpu_model": model, "host_cpus": ncpu,
            "sample": f"RMAT-{sc} ef{a.ef} seed {sc} ({R} records), k={a.k}: reference lib/ graph2tree -r -p flow "
                      f"(mpiSequence all-reduce + degreeSequence sort, JTree per shard, JNodeTable::mpi_merge, "
                      f"makeKids + Partition + mpi_sync) on {ranks} MPI ranks x 1 thread, shards loaded untimed, "
                      f"{sec:.2f} s",
            "phases_s": {k: round(v, 3) for k, v in res.get("phases", {}).items()}}


if __name__ == "__main__":
    main()
