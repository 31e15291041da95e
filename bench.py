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
        "etree_apply", "etree_top", "merge", "kids", "partition")
REGION_KERNELS = {"degree": ["k_degree_fused"], "relabel": ["k_relabel_scatter", "k_relabel_gather"],
                  "etree_split": ["k_split_count", "k_split_write"], "etree_union": ["k_hook_round", "k_hook_finish", "k_light_top"],
                  "etree_cross": ["k_cross_find"], "etree_apply": ["k_cross_apply", "k_level_clean"],
                  "etree_top": ["k_top_extract_multi", "k_top_sum_counts", "k_top_init", "k_top_min0_lds", "k_top_hook0",
                                "k_top_round", "k_top_hook"],
                  "evaluate": ["k_pp", "k_eval_records", "k_eval_nodes", "k_parts_jnid", "k_eval_edges", "k_eval_loops",
                               "k_eval_nodes_j"]}
# the newest round's profile of this workload (profiles/rNN/), collected by tools/gpu/gpuprof.sh
PMC_DIRS = ("r6", "r5", "r4", "r3")
PMC_FILE = os.path.join(ROOT, "profiles", "{round}", "pmc_traffic_rmat{scale}_k{k}.json")


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
    ap.add_argument("--streams", type=int, default=1,
                    help="one GPU with --shards: the shards' degree counts and maps run on this many contexts, each "
                         "on a stream of its own driven by a host thread of its own (independent shards overlap on "
                         "the GPU, as the ranks of an N-GPU run do across GPUs); the merge runs on the first")
    ap.add_argument("--concurrent", type=int, default=0, metavar="N",
                    help="one GPU, one shard: whole steps on N contexts at once, each context's steps in a host "
                         "thread of its own (a stream of graphs; 0: off)")
    ap.add_argument("--shuffle", action="store_true",
                    help="records in a random order, half with tail/head swapped (a generic edge list)")
    ap.add_argument("--eval-reps", type=int, default=3, help="timed evaluator runs (0: skip)")
    ap.add_argument("--eval-records", action="store_true",
                    help="one GPU: also time the record evaluator (sheep_evaluate) beside the step-edge one")
    ap.add_argument("--cpu-scale", type=int, default=None,
                    help="RMAT scale of the CPU-baseline sample (default: the bench's own RMAT scale up to 26, else 22)")
    ap.add_argument("--cpu-same-graph", action="store_true",
                    help="run the CPU baseline on the bench's own records (any graph or scale; C4, C5) instead of "
                         "an RMAT sample, so `matches_gpu` compares the reference's results with this run's")
    ap.add_argument("--cpu-configs", nargs="+", default=["8x1", "16x1"],
                    help="PxT configurations of the reference CPU baseline: P MPI ranks x T OpenMP threads each "
                         "(the threads serve the reference's __gnu_parallel::sort, sequence.h:55,85); P x T is capped "
                         "by the host cores this process may use (affinity mask and cgroup quota) and the best is "
                         "reported.  The GPU box grants 16 CPUs' worth of time: at RMAT-26 8x1 / 16x1 / 16x4 / 16x16 / "
                         "32x1 / 32x8 ran 30.6 / 25.9 / 27.9 / 28.9 / 58.1 / 60.3 s "
                         "(profiles/r4/cpu_sweep_rmat26_k64.json, tools/cpu_sweep.py)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0: rehearse N ranks on a 1-GPU box (the world's host link over TCP "
                         "carries the exchanges instead of RCCL)")
    ap.add_argument("--reduce", default="kway", choices=("kway", "binomial"),
                    help="kway: gather the partial trees to rank 0 and merge them in one pass; "
                         "binomial: ceil(log2 N) send/recv hops with a pairwise merge each (mpi_merge's schedule)")
    ap.add_argument("--tune", nargs="+", default=[], metavar="FIELD=VALUE",
                    help="algorithm variants for A/B runs (include/sheep_hip.h sheep_tuning, e.g. fin_map_bits=12); "
                         "every variant gives the same bit-exact result")
    ap.add_argument("--no-verify", dest="verify", action="store_false",
                    help="skip the after-timing check of the merged tree (N > 1: against the whole-graph tree; "
                         "--shards: against the binomial pairwise merges of the same shard trees)")
    return ap.parse_args()


def make_records(a, seed, ctx):
    """The workload's records in HBM: (records, vertex-slot capacity, workload name)."""
    import sheep_amd
    if a.graph == "rmat":
        rec = sheep_amd.rmat(a.scale, a.ef, seed, ctx=ctx)
        vs_cap, workload = 1 << a.scale, f"RMAT-{a.scale} ef{a.ef}, k={a.k}"
    else:
        rec = sheep_amd.powerlaw(sheep_amd.TWITTER_VERTICES, a.draws, 1.9, seed, ctx=ctx)
        vs_cap, workload = sheep_amd.TWITTER_VERTICES, f"Chung-Lu power law (twitter-2010 scale), k={a.k}"
    if a.shuffle:
        rec = shuffled(rec, 1000 + seed)
    return rec, vs_cap, workload


def shuffled(d, seed):
    """The records in a scrambled order, half of them with tail and head swapped: record i
    of the output is record (a * i + b) mod R of the input (a odd, coprime to R, and b drawn
    from the seed) — consecutive outputs lie a apart, so the tails lose their order — and a
    hash of its source index decides the swap.  Built column by column in chunks:
    torch.randperm stalls above 2^30 elements on this stack (the C4 records), and whole-
    tensor indexing of an R x 3 tensor past 2^32 elements is slow."""
    import math
    import random
    import torch
    R = d.shape[0]
    rng = random.Random(seed)
    a = rng.randrange(R // 3, R) | 1 if R > 3 else 1
    while math.gcd(a, R) != 1:
        a += 2
    b = rng.randrange(R) if R else 0
    out = torch.empty_like(d)
    cols = [d[:, j].contiguous() for j in range(3)]
    step = 1 << 26
    for s in range(0, R, step):
        e = min(R, s + step)
        src = (torch.arange(s, e, device=d.device, dtype=torch.int64) * a + b) % R
        flip = ((src * 0x2545F4914F6CDD1D) >> 40) & 1 == 1
        tail, head = cols[0][src], cols[1][src]
        out[s:e, 0] = torch.where(flip, head, tail)
        out[s:e, 1] = torch.where(flip, tail, head)
        out[s:e, 2] = cols[2][src]
    return out


def spawn_ranks(a):
    """`--gpus N` without a torch.distributed launcher: start one rank per GPU with
    torch.distributed.run as a CHILD process (nothing here has touched the GPU: device
    counting does not initialise it) and exit with its status.  Fewer than N visible
    devices is an error, never a silent one-GPU run."""
    import socket
    import subprocess
    import torch
    have = torch.cuda.device_count()
    if have < a.gpus and not a.same_device:
        print(f"bench: --gpus {a.gpus} but only {have} HIP device(s) visible", file=sys.stderr, flush=True)
        sys.exit(2)
    with socket.socket() as sk:                                   # a free rendezvous port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(a)
    import torch
    import sheep_amd
    from sheep_amd import dist as sdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    if a.shards > 1 and world > 1:
        raise SystemExit("--shards is the one-GPU form of the edge-shard path")
    if a.concurrent and (world > 1 or a.shards > 1):
        raise SystemExit("--concurrent is a one-GPU, one-shard form")
    torch.cuda.set_device(local)
    seed = (a.scale if a.graph == "rmat" else 2010) if a.seed is None else a.seed
    group = None
    json_out = sys.stdout
    if world > 1:
        # stdout carries rank 0's JSON line only: the launcher's and gloo's banners and every
        # other rank's output go to stderr (the saved descriptor keeps rank 0's line)
        sys.stdout.flush()
        json_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        # torch.distributed (gloo, host) is the control plane only: the rendezvous port,
        # barriers and the max over ranks of the wall time.  The data path is the world of
        # include/sheep_hip.h (sheep_group_join, group.hip): RCCL over xGMI between the
        # ranks' GPUs, the same code graph2tree -i -r runs under mpiexec.
        # a rank that dies or stalls ends the run within this many seconds (group.hip's RCCL
        # failure path: abort, one stderr line per rank, non-zero exit) instead of wedging it
        os.environ.setdefault("SHEEP_JOIN_TIMEOUT", "180")
        sdist.init_control()
        group = sheep_amd.Group.join(local, rank, world, "127.0.0.1", sdist.shared_port(),
                                     link="host" if a.same_device else "rccl")
        ctx = group.ctx[0]
    else:
        ctx = sheep_amd.Context(local)
    tune = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.tune}
    if tune:
        (group or ctx).set_tuning(**tune)
    rec, vs_cap, workload = make_records(a, seed, ctx)          # whole graph, identical on every rank
    ctx.trim()                                                  # the generator's sort buffers are not the path's
    if a.shards > 1:
        workload += f", {a.shards} shards on 1 GPU"
    R = rec.shape[0]
    beg, end = sdist.shard_bounds(R, rank, world)               # contiguous edge shard (graph2tree -l)
    shard = rec[beg:end].contiguous() if world > 1 else rec
    del rec
    torch.cuda.empty_cache()
    dev = f"cuda:{local}"
    ctxs = [ctx]   # --streams: more contexts on this device, each with a stream of its own
    if a.shards > 1 and world == 1:
        ctxs += [sheep_amd.Context(local, stream=torch.cuda.Stream(local)) for _ in range(max(1, a.streams) - 1)]
        for cx in ctxs[1:]:
            if tune:
                cx.set_tuning(**tune)
    conc = None   # --concurrent N: N contexts, each running whole steps in a host thread of its own
    if a.concurrent > 0:
        cstreams = [torch.cuda.Stream(local) for _ in range(a.concurrent)]
        ctxs = [sheep_amd.Context(local, stream=st) for st in cstreams]
        for cx in ctxs:
            if tune:
                cx.set_tuning(**tune)
        conc = {"streams": cstreams, "last": [None] * a.concurrent,
                "deg": [torch.zeros(vs_cap, dtype=torch.int32, device=dev) for _ in range(a.concurrent)]}
    deg = torch.zeros(vs_cap, dtype=torch.int32, device=dev)
    subs = [shard[i * shard.shape[0] // a.shards:(i + 1) * shard.shape[0] // a.shards] for i in range(a.shards)]
    stack = [None]
    bufs = {}
    walls = {}   # N ranks: this rank's host wall time per part of the step (the group calls return complete)

    def lap(name, t0):
        t1 = time.perf_counter()
        walls[name] = walls.get(name, 0.0) + (t1 - t0)
        return t1

    def on_contexts(fn):
        """fn(i) for every shard i, shard i on context i mod len(ctxs): one host thread per
        context (the library's calls release the GIL and synchronise their own stream), the
        contexts' streams complete on return."""
        if len(ctxs) == 1:
            for i in range(len(subs)):
                fn(i)
            return
        import threading
        torch.cuda.synchronize()                                 # inputs written on other streams
        err = []

        def run(j):
            try:
                for i in range(j, len(subs), len(ctxs)):
                    fn(i)
                ctxs[j].sync()
            except Exception as e:                               # (re-raised below)
                err.append(e)
        th = [threading.Thread(target=run, args=(j,)) for j in range(len(ctxs))]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()
        if err:
            raise err[0]

    def step():
        deg.zero_()
        if group is not None:                                   # graph2tree -i -r over the world
            t0 = time.perf_counter()
            if "seq" not in bufs:
                bufs["seq"] = torch.empty(vs_cap, dtype=torch.int32, device=dev)
                bufs["pos"] = torch.empty(vs_cap, dtype=torch.int32, device=dev)
            s = group.sequence([shard], vs_cap, deg=[deg], seq=[bufs["seq"]], pos=[bufs["pos"]])[0]
            t0 = lap("sequence", t0)                            # incl. the wait for the slowest rank
            if "tree" not in bufs or bufs["tree"].shape[0] < s.n:
                bufs["tree"] = torch.empty((max(s.n, 1), 2), dtype=torch.int32, device=dev)
            tree = group.build_tree([shard], [s], "none", trees=[bufs["tree"]])[0]
            t0 = lap("map", t0)
            tree = group.reduce_trees([bufs["tree"][:s.n]], a.reduce)[0]
            t0 = lap("reduce", t0)                              # gather + merge on rank 0, the send elsewhere
        else:
            slots = [0] * len(subs)

            def count(i):                                       # shards accumulate into one histogram
                slots[i] = sheep_amd.degree_count(subs[i], mode="llama", deg=deg, ctx=ctxs[i % len(ctxs)])[1]

            on_contexts(count)
            s = sheep_amd.sequence_from_degrees(deg, max(slots), ctx=ctx)
            if a.shards > 1:                                    # map per shard, then ONE K-way merge
                if stack[0] is None or stack[0].shape[1] != s.n:
                    stack[0] = torch.empty((a.shards, s.n, 2), dtype=torch.int32, device=dev)
                on_contexts(lambda i: sheep_amd.build_tree(subs[i], s, ctx=ctxs[i % len(ctxs)], out=stack[0][i]))
                tree = sheep_amd.merge_trees_many(stack[0], ctx=ctx)
            else:
                tree = sheep_amd.build_tree(shard, s, ctx=ctx)
        res = None
        if rank == 0:                                           # graph2tree.cpp:203-208
            t0 = time.perf_counter()
            kids = sheep_amd.KidTable(tree, ctx)
            res = sheep_amd.partition(s, tree, a.k, kids=kids, ctx=ctx)
            kids.close()
            if group is not None:
                ctx.sync()
                lap("kids_partition", t0)
        return s, tree, res

    def conc_run(nsteps):
        """nsteps whole steps, step i on context i mod N, each context's steps in a thread."""
        import threading
        N, err = len(ctxs), []

        def worker(j):
            try:
                c, dg = ctxs[j], conc["deg"][j]
                for _ in range(j, nsteps, N):
                    with torch.cuda.stream(conc["streams"][j]):
                        dg.zero_()
                    s_ = sheep_amd.sequence_from_degrees(
                        dg, sheep_amd.degree_count(shard, mode="llama", deg=dg, ctx=c)[1], ctx=c)
                    tree_ = sheep_amd.build_tree(shard, s_, ctx=c)
                    kids = sheep_amd.KidTable(tree_, c)
                    res_ = sheep_amd.partition(s_, tree_, a.k, kids=kids, ctx=c)
                    kids.close()
                    conc["last"][j] = (s_, tree_, res_, c)
                c.sync()
            except Exception as e:                              # (re-raised below)
                err.append(e)
        th = [threading.Thread(target=worker, args=(j,)) for j in range(N)]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()
        if err:
            raise err[0]

    def barrier():
        torch.cuda.synchronize()
        ctx.sync()
        if world > 1:
            sdist.barrier()

    if conc is not None:
        conc_run(max(a.warmup, len(ctxs)))                      # every context warmed up
    else:
        for _ in range(a.warmup):
            step()
    barrier()
    for cx in ctxs:
        cx.timing(True)
        cx.timer_reset()
    walls.clear()
    barrier()
    t0 = time.perf_counter()
    if conc is not None:
        conc_run(a.steps)
    else:
        for _ in range(a.steps):
            s, tree, res = step()
    barrier()
    t = sdist.max_over_ranks(time.perf_counter() - t0) if world > 1 else time.perf_counter() - t0
    # device memory in use after the timed steps: the library's workspaces only grow and
    # torch's caching allocator keeps its blocks, so this is the step's high-water mark
    free_b, total_b = torch.cuda.mem_get_info(local)
    hbm_used = total_b - free_b

    # per-region device timings (HIP events on the context stream), timed steps only
    # (--streams: summed over the contexts; their regions overlap in time)
    phases = {}
    for cx in ctxs:
        for name in cx.timer_names():
            ms, launches, nbytes = cx.timer(name)
            p = phases.setdefault(name, {"ms_per_step": 0.0, "launches": 0, "alg_bytes": 0})
            p["ms_per_step"] = round(p["ms_per_step"] + ms / a.steps, 4)
            p["launches"] += launches
            p["alg_bytes"] += nbytes
        cx.timer_reset()
    if conc is not None:                                        # context 0's last step
        s, tree, res, ctx_last = conc["last"][0]
    for cx in ctxs[1:]:
        cx.timing(False)
    per_rank = None
    if world > 1:   # every rank's split of the step, for diagnosing the N-rank run (rank 0 reports)
        mine = {"rank": rank, "wall_ms_per_step": {k: round(1e3 * v / a.steps, 3) for k, v in walls.items()},
                "device_ms_per_step": {k: phases[k]["ms_per_step"] for k in ("gather", "merge", "etree", "relabel")
                                       if k in phases}}
        per_rank = sdist.gather_objects(mine)

    evaluator = None
    if a.eval_reps > 0:
        evaluator = time_evaluator(a, ctx_last if conc is not None else ctx, group, shard, subs, s, res, rank, world,
                                   dev, barrier)
    ctx.timing(False)
    if conc is not None:
        ctxs[0].timing(False)

    verified = None
    checks = {}
    if a.verify and (world > 1 or a.shards > 1):
        if rank == 0:
            checks = verify_tree(a, seed, ctx, shard, subs, s, tree, stack[0], world)
            verified = all(checks.values())
            if not verified:
                print("bench: merged tree differs from its cross-check", file=sys.stderr, flush=True)
        if world > 1:
            sdist.barrier()

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
            if world > 1:
                roof["note"] = "rank 0's leaf regions (rank 0 also runs the merge, kids and partition)"
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
            "config": {"workload": workload + (f", steps on {len(ctxs)} concurrent contexts" if conc is not None else
                                               f", {len(ctxs)} streams" if len(ctxs) > 1 else ""), "records": R,
                       "vertex_slots": s.pos_size,
                       "tree_nodes": n, "k": a.k, "created": res.created, "packing_nodes": res.packing_nodes,
                       "heavy_nodes": res.heavy_nodes, "event_launches": res.event_launches, "seed": seed, "shuffled": a.shuffle, "shards": a.shards,
                       "tuning": ctx.tuning() if tune else "defaults",
                       "parallelism": f"edge-shards x{world}" + (
                           f", {a.reduce} reduce, sheep_group over {'RCCL' if group.rccl else 'host TCP (one device)'}"
                           if world > 1 else "")},
            "roofline": roof,
            "path_roofline": path,
            "evaluator": evaluator,
            "phases": phases,
            "hbm_peak_bytes": hbm_used,
            "hbm_workspace_top": dict(list((ctxs[0] if conc is not None else ctx).workspace().items())[:12]),
            "hbm_peak_note": "device memory in use after the timed steps (hipMemGetInfo: total - free); the "
                             "library's workspaces only grow, so this is the step's high-water mark",
        }
        if per_rank is not None:
            out["per_rank"] = per_rank
        out.update(checks)   # verified_vs_whole_graph / verified_vs_pairwise_merges: the checks that ran
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a, ctx, (s, tree, res), seed, shard)
    del shard
    if group is not None:
        sdist.barrier()
        group.close()
        sdist.shutdown()
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if verified is False:
        sys.exit(1)


def verify_tree(a, seed, ctx, shard, subs, s, tree, stacked, world):
    """After the timed steps, rank 0 checks the reduced tree; returns {check: passed} for
    the checks that ran.  N ranks: against the whole graph's tree built on rank 0 alone.
    One GPU with --shards: against the whole graph's tree when its workspace fits the
    device (about 72 B per record: C5's 4.24 G records do not), and always against the
    binomial pairwise merges (mpi_merge's schedule, jnode.cpp:203-250) of the same shard
    trees."""
    import torch
    import sheep_amd
    if world > 1:
        rec, _, _ = make_records(a, seed, ctx)
        whole = sheep_amd.build_tree(rec, s, ctx=ctx)
        del rec
        ok = bool(torch.equal(whole, tree))
        del whole
        torch.cuda.empty_cache()
        return {"verified_vs_whole_graph": ok}
    checks = {}
    ctx.trim()
    torch.cuda.empty_cache()
    if shard.shape[0] < (1 << 32) and shard.shape[0] * 72 < torch.cuda.mem_get_info()[0]:
        checks["verified_vs_whole_graph"] = bool(torch.equal(sheep_amd.build_tree(shard, s, ctx=ctx), tree))
    cur = [stacked[i] for i in range(len(subs))]
    d = 1
    while d < len(cur):
        for i in range(0, len(cur), 2 * d):
            if i + d < len(cur):
                cur[i] = sheep_amd.merge_trees(cur[i], cur[i + d], ctx=ctx)
        d *= 2
    checks["verified_vs_pairwise_merges"] = bool(torch.equal(cur[0], tree))
    return checks


def time_evaluator(a, ctx, group, shard, subs, s, res, rank, world, dev, barrier):
    """ECV(down) + balance (evaluate(graph, seq), partition.cpp:475-521), timed on its own:
    one GPU — sheep_evaluate over all records (or the shards' bitsets with --shards); N
    GPUs — rank 0's parts broadcast (Partition::mpi_sync), per-shard bitsets, the binomial
    OR-reduction to rank 0 and the node pass there (sheep_group_broadcast_parts +
    sheep_group_evaluate).  B_eval per SURVEY §8(d)."""
    import torch
    import sheep_amd
    from sheep_amd import dist as sdist
    R_total = shard.shape[0] * world if world > 1 else shard.shape[0]
    times, ev = [], None
    for _ in range(a.eval_reps):
        barrier()
        t0 = time.perf_counter()
        if world == 1 and a.shards == 1:   # from the position-space edges the step's map left in HBM
            ev = sheep_amd.evaluate(shard, s, res.parts, what=sheep_amd.EVAL_DOWN, ctx=ctx, from_step=True)
        elif world == 1:                                         # the shards' bitsets, then one node pass
            e = sheep_amd.ShardedEvaluator(s, res.parts, sheep_amd.EVAL_DOWN, ctx=ctx)
            for sub in subs:
                e.add(sub)
            ev = e.finish()
        else:
            parts = res.parts.clone() if rank == 0 else torch.empty(s.pos_size, dtype=torch.int16, device=dev)
            parts = group.broadcast_parts([parts], s.pos_size)[0]
            ev = group.evaluate([shard], [s], [parts], what=sheep_amd.EVAL_DOWN)
        barrier()
        dt = time.perf_counter() - t0
        times.append(sdist.max_over_ranks(dt) if world > 1 else dt)
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
    if world == 1 and a.shards == 1:
        out["source"] = "the step's position-space edges (sheep_evaluate_step)"
        # the bytes this form moves: per edge the 8-B edge, the lo's 2-B part and the hi's 8-B
        # owner word; per node the part lookup (seq 4 + pos check 4 + part 2 + pj 2) and the
        # node pass (owner word 8 + pj 2 + pst 4)
        b_step = 18 * R_total + 26 * s.n
        out["own_model"] = {"alg_bytes": b_step, "achieved_GBs": round(b_step / best / 1e9, 2),
                            "frac": round(b_step / best / 1e9 / HBM_PEAK_GBS, 4),
                            "model": "18 B per edge + 26 B per tree node (what sheep_evaluate_step reads and "
                                     "writes; B_eval above prices the record evaluator's reads)"}
        if a.eval_records:   # the record evaluator (sheep_evaluate) on the same parts, for comparison
            rt = []
            for _ in range(a.eval_reps):
                barrier()
                t0 = time.perf_counter()
                er = sheep_amd.evaluate(shard, s, res.parts, what=sheep_amd.EVAL_DOWN, ctx=ctx)
                barrier()
                rt.append(time.perf_counter() - t0)
            assert er == ev, (er, ev)
            out["records_ms"] = round(1e3 * min(rt), 3)
    out.update(pmc_region(a, world, "evaluate", 1))
    return out


def _pmc(a, world):
    path = PMC_FILE.format(round=PMC_DIRS[-1], scale=a.scale, k=a.k)
    for r in PMC_DIRS:
        p = PMC_FILE.format(round=r, scale=a.scale, k=a.k)
        if os.path.exists(p):
            path = p
            break
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
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    # a cgroup CPU quota caps what the affinity mask shows (the GPU box: 256 CPUs visible,
    # cpu.max = 16 CPUs' worth of time; profiles/r4/cpu_quota.txt)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return model, os.cpu_count(), usable


def run_group(cmd, env, timeout):
    """Runs cmd in a process group of its own and kills whatever of the group is left when it
    returns (mpiexec's hydra proxies can outlive it): nothing the baseline started survives
    bench.py."""
    import signal
    import subprocess
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
    finally:
        try:
            os.killpg(p.pid, signal.SIGKILL)   # (the group's leftovers; the leader has exited)
        except (ProcessLookupError, PermissionError):
            pass
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


def cpu_baseline(a, ctx, gpu=None, seed=None, records=None):
    """The reference CPU path on the same workload (RMAT-26 by default), on this host.

    kind "reference": the reference's own lib/ code, compiled from /root/reference into
    oracle/_ref/ref_harness by oracle/ref/Makefile, run as the graph2tree `-r -p k` flow
    over MPI ranks (mpiexec -n P ref_harness mpi ...): each rank loads its edge shard
    (graph2tree -l semantics, untimed), then mpiSequence's degree all-reduce with
    degreeSequence's sort, JTree on the shard (map), JNodeTable::mpi_merge (the custom-op
    MPI_Reduce), makeKids + Partition(k) + mpi_sync on rank 0.  The timed region starts at
    a barrier after the load.  (P ranks, T OpenMP threads each) runs over --cpu-configs,
    P x T capped by the cores this process may run on (os.sched_getaffinity); the fastest
    is the value and `cores` = its P x T.  When the sample is the bench's own graph, the
    reference flow's sequence, merged tree and parts (the harness's FNV-1a digests) are
    compared with the GPU step's (`matches_gpu`): a full-size check against the reference's
    own code in every bench run.  The literal `-ir` is not used: its sort copies
    the whole degree vector with every comparator copy (sequence.h:85; its box record is
    profiles/r4/cpu_ir_literal.json, tools/cpu_ir.py).  Test infrastructure timed as a baseline; never the measured path."""
    import shutil
    import subprocess
    import tempfile
    import sheep_amd
    sc = a.cpu_scale if a.cpu_scale is not None else (min(a.scale, 26) if a.graph == "rmat" else 22)
    model, ncpu, usable = cpu_info()
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    mpiexec = shutil.which("mpiexec", path="/opt/conda/bin") or shutil.which("mpiexec")
    if not os.path.exists(harness) or not mpiexec:
        return {"value": None, "unit": "edges/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/ref_harness or mpiexec missing on this host"}
    configs = []
    for c in a.cpu_configs:
        p, t = (int(x) for x in str(c).split("x"))
        p = max(1, min(p, usable or 1))
        t = max(1, min(t, (usable or 1) // p))
        if (p, t) not in configs:
            configs.append((p, t))
    runs = []
    same = a.cpu_same_graph and records is not None
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "same.dat" if same else f"rmat{sc}.dat")
        d = records if same else sheep_amd.rmat(sc, a.ef, sc, ctx=ctx)
        R = d.shape[0]
        with open(path, "wb") as f:                               # XS1 records, streamed in chunks
            step = 1 << 26
            for b in range(0, R, step):
                f.write(sheep_amd.to_numpy_u32(d[b:b + step]).tobytes())
        del d
        ctx.sync()
        for p, th in configs:
            env = dict(os.environ, OMP_NUM_THREADS=str(th))
            r = run_group([mpiexec, "-n", str(p), harness, "mpi", path, str(a.k)], env, 900)
            if r.returncode != 0:
                runs.append({"ranks": p, "threads": th, "error": r.stderr.strip()[-300:]})
                continue
            res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            runs.append({"ranks": p, "threads": th, "seconds": round(res["seconds"], 3),
                         "edges_per_s": round(R / res["seconds"], 1),
                         "phases_s": {k: round(v, 3) for k, v in res.get("phases", {}).items()},
                         "fnv": res.get("fnv")})
            print(f"cpu_baseline: {p} ranks x {th} threads {res['seconds']:.2f} s", file=sys.stderr, flush=True)
    ok = [x for x in runs if "seconds" in x]
    if not ok:
        return {"value": None, "unit": "edges/s", "cores": 0, "kind": "reference", "sample": f"failed: {runs}"}
    best = min(ok, key=lambda x: x["seconds"])
    matches = None
    if gpu is not None and (same or (a.graph == "rmat" and sc == a.scale and seed == sc)) and \
            all(x.get("fnv") for x in ok):
        import oracle                                            # (the checker: FNV-1a over the GPU's arrays)
        gs, gtree, gres = gpu
        mine = {"seq": oracle.fnv1a(sheep_amd.to_numpy_u32(gs.seq[:gs.n])),
                "tree": oracle.fnv1a(gtree.cpu().numpy()),
                "parts": oracle.fnv1a(gres.parts.cpu().numpy())}
        matches = {k: all(x["fnv"][k] == v for x in ok) for k, v in mine.items()}
        matches["gpu_fnv"] = mine
    return {"value": best["edges_per_s"], "unit": "edges/s", "cores": best["ranks"] * best["threads"],
            "kind": "reference", "cpu_model": model, "host_cpus": ncpu, "usable_cpus": usable,
            "sample": (f"the bench's own records ({R})" if same else f"RMAT-{sc} ef{a.ef} seed {sc} ({R} records)")
                      + f", k={a.k}: reference lib/ graph2tree -r -p flow "
                      f"(mpiSequence all-reduce + degreeSequence sort, JTree per shard, JNodeTable::mpi_merge, "
                      f"makeKids + Partition + mpi_sync) on P MPI ranks x T OpenMP threads, PxT in "
                      f"{['%dx%d' % c for c in configs]} (best {best['ranks']}x{best['threads']}, "
                      f"{best['seconds']:.2f} s), shards loaded untimed",
            "phases_s": best["phases_s"], "sweep": runs, "matches_gpu": matches}


if __name__ == "__main__":
    main()
