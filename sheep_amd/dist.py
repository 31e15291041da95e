"""Edge-shard schedule over N ranks: the MI355X replacement of graph2tree's MPI `-ir`
path (graph2tree.cpp:161-216).

  * shard_bounds      — contiguous record shards, like `-l part/num_parts`;
  * allreduce_degrees — one all-reduce of the per-shard degree histograms plus a max of
                        max_slot (sequence.h:70-78 `mpiSequence`'s MPI_Allreduce);
  * sync_parts        — rank 0's part array to every rank (Partition::mpi_sync,
                        partition.cpp:69-79), so each rank can write its shard's files;
  * reduce_trees      — binomial reduction of the partial trees to rank 0 (the shape of
                        MPI_Reduce with mpi_merge_reduction, jnode.cpp:203-250): at hop r,
                        rank i with i % 2r == r sends to i - r, which merges.  Merging is
                        associative and commutative (the elimination tree of the union of
                        the parent edges), so the tree at rank 0 equals the serial one.
  * reduce_eval       — the evaluator's per-shard part bitsets ORed (and its counts
                        summed) to rank 0 in the same binomial shape;
  * reduce_trees_kway — the same reduction as ONE gather + ONE K-way merge on rank 0
                        (sheep_merge_trees_many): every rank sends its tree straight to
                        rank 0 (each over its own xGMI link, all at once), and the merge
                        runs once over all K parent-edge sets instead of ceil(log2 K)
                        merges in sequence on rank 0's critical path;
  * reduce_trees_split— the K-way merge split over nparts ranks (sheep_merge_trees_part):
                        the part ranks receive every tree, each runs the merge's top levels
                        in full and then one subproblem, and they send their node ranges'
                        parents to rank 0 (measured: little gain, see the function).

One process per GPU.  With the "nccl" backend (RCCL over xGMI) device tensors are sent
as they are.  With "gloo" they are staged through host memory, which lets the schedule
run on CPUs (tests/test_dist.py) and lets several ranks share one GPU for a rehearsal.
The compute is injected (`merge`), so the same schedule drives the HIP kernels in
bench.py and the CPU oracle in the tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_bounds(nrec: int, rank: int, world: int) -> tuple[int, int]:
    return rank * nrec // world, (rank + 1) * nrec // world


def _host_staged() -> bool:
    return dist.get_backend() == "gloo"


def _send(t: torch.Tensor, dst: int) -> None:
    dist.send(t.cpu() if _host_staged() and t.is_cuda else t, dst)


def _recv_like(like: torch.Tensor, src: int) -> torch.Tensor:
    if _host_staged() and like.is_cuda:
        buf = torch.empty(like.shape, dtype=like.dtype, device="cpu")
        dist.recv(buf, src)
        return buf.to(like.device)
    buf = torch.empty_like(like)
    dist.recv(buf, src)
    return buf


def _all_reduce(t: torch.Tensor, op) -> None:
    if _host_staged() and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)


def allreduce_degrees(deg: torch.Tensor, max_slot: int) -> int:
    """Sum the shards' degree histograms in place; returns the global max_slot."""
    mx = torch.tensor([max_slot], dtype=torch.int64, device=deg.device)
    _all_reduce(deg, dist.ReduceOp.SUM)
    _all_reduce(mx, dist.ReduceOp.MAX)
    return int(mx.item())


def reduce_trees(tree: torch.Tensor, merge, rank: int, world: int):
    """Binomial reduction to rank 0.  Returns the merged tree on rank 0, None elsewhere
    (a rank is done once it has sent)."""
    r = 1
    while r < world:
        if rank % (2 * r) == r:
            _send(tree, rank - r)
            return None
        if rank + r < world:
            tree = merge(tree, _recv_like(tree, rank + r))
        r *= 2
    return tree


def gather_trees(tree: torch.Tensor, rank: int, world: int):
    """Every rank's (n, 2) tree stacked on rank 0 as (world, n, 2); None elsewhere."""
    if rank != 0:
        if _host_staged():
            _send(tree, 0)
        else:   # the same batched P2P API on both sides (RCCL groups the transfers)
            for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, tree, 0)]):
                q.wait()
        return None
    out = torch.empty((world,) + tuple(tree.shape), dtype=tree.dtype, device=tree.device)
    out[0].copy_(tree)
    if _host_staged() and tree.is_cuda:
        host = torch.empty((world,) + tuple(tree.shape), dtype=tree.dtype, device="cpu")
        reqs = [dist.irecv(host[r], r) for r in range(1, world)]
        for q in reqs:
            q.wait()
        out[1:].copy_(host[1:])
    else:
        ops = [dist.P2POp(dist.irecv, out[r], r) for r in range(1, world)]
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    return out


def reduce_trees_kway(tree: torch.Tensor, merge_many, rank: int, world: int):
    """Gather to rank 0, then one K-way merge there.  Returns the merged tree on rank 0,
    None elsewhere."""
    stacked = gather_trees(tree, rank, world)
    return None if stacked is None else merge_many(stacked)


def gather_trees_to(tree: torch.Tensor, rank: int, world: int, receivers) -> torch.Tensor | None:
    """Every rank's (n, 2) tree stacked as (world, n, 2) on each rank in `receivers`
    (None elsewhere): one batch of point-to-point transfers, each sender's copies on
    different xGMI links."""
    recv_here = rank in receivers
    staged = _host_staged() and tree.is_cuda
    src = tree.cpu().contiguous() if staged else tree.contiguous()
    out = None
    ops = []
    if recv_here:
        out = torch.empty((world,) + tuple(tree.shape), dtype=tree.dtype, device="cpu" if staged else tree.device)
        out[rank].copy_(src)
        ops += [dist.P2POp(dist.irecv, out[r], r) for r in range(world) if r != rank]
    ops += [dist.P2POp(dist.isend, src, q) for q in receivers if q != rank]
    if ops:
        if _host_staged():
            reqs = [op.op(op.tensor, op.peer) for op in ops]
        else:
            reqs = dist.batch_isend_irecv(ops)
        for q in reqs:
            q.wait()
    if out is not None and staged:
        out = out.to(tree.device)
    return out


def reduce_trees_split(tree: torch.Tensor, merge_part, rank: int, world: int, nparts: int = 2):
    """The K-way merge split over `nparts` ranks (a power of two <= world): ranks
    0..nparts-1 receive every tree, each runs one part (merge_part(stacked, part, nparts)
    -> (tree, lo, hi): every pst and the parents of nodes [lo, hi) are the merged tree's)
    and ranks 1..nparts-1 send their parent slices to rank 0.  Rank 0 takes the LAST part:
    contractions move every level's work into right halves, so the part of the highest
    positions is by far the largest — which is also why the split gains little (RMAT-26,
    8 trees: 2 parts 4.1 / 17.3 ms, 8 parts 7.4 ... 16.1 ms, against 17.8 ms for the
    whole merge on one GPU), so bench.py keeps the K-way gather by default.
    Returns the merged tree on rank 0, None elsewhere."""
    nparts = max(1, min(nparts, world))
    if nparts & (nparts - 1):
        raise ValueError("split reduce needs a power-of-two number of parts")
    stacked = gather_trees_to(tree, rank, world, range(nparts))
    if rank >= nparts:
        return None
    part_id = nparts - 1 if rank == 0 else rank - 1
    part, lo, hi = merge_part(stacked, part_id, nparts)
    del stacked
    staged = _host_staged() and part.is_cuda
    if rank != 0:
        rng = torch.tensor([lo, hi], dtype=torch.int64, device="cpu" if _host_staged() else part.device)
        sl = part[lo:hi, 0].contiguous()
        _send(rng, 0)
        if hi > lo:
            _send(sl, 0)
        return None
    for r in range(1, nparts):
        rng = torch.empty(2, dtype=torch.int64, device="cpu" if _host_staged() else part.device)
        dist.recv(rng, r)
        a, b = int(rng[0]), int(rng[1])
        if b > a:
            buf = torch.empty(b - a, dtype=part.dtype, device="cpu" if staged else part.device)
            dist.recv(buf, r)
            part[a:b, 0] = buf.to(part.device)
    return part


def reduce_eval(ev, rank: int, world: int):
    """Binomial reduction of ShardedEvaluator states to rank 0: at
    hop r, rank i with i % 2r == r sends its bitsets and counts to i - r, which ORs / adds
    them in (sheep_eval_combine; RCCL has no bitwise-OR reduction).  Returns the combined
    evaluator on rank 0, None elsewhere."""
    r = 1
    while r < world:
        if rank % (2 * r) == r:
            _send(ev.bits, rank - r)
            _send(ev.acc, rank - r)
            return None
        if rank + r < world:
            bits = _recv_like(ev.bits, rank + r)
            acc = _recv_like(ev.acc, rank + r)
            ev.combine(bits, acc)
            del bits, acc
        r *= 2
    return ev


def sync_parts(parts: torch.Tensor | None, pos_size: int, device) -> torch.Tensor:
    """Partition::mpi_sync: broadcast rank 0's vid-indexed int16 parts (created on the
    other ranks with the size rank 0 has)."""
    if dist.get_rank() != 0:
        parts = torch.empty(pos_size, dtype=torch.int16, device=device)
    raw = parts.view(torch.uint8)   # gloo has no int16 collectives
    if _host_staged() and raw.is_cuda:
        h = raw.cpu()
        dist.broadcast(h, 0)
        raw.copy_(h)
    else:
        dist.broadcast(raw, 0)
    return parts
