"""Control plane of bench.py's N-rank run (one process per GPU, launched by
torch.distributed.run): the MI355X replacement of graph2tree's MPI `-ir` world
(graph2tree.cpp:134-216) keeps its DATA path in libsheep_hip.so — sheep_group_join
(group.hip): RCCL over xGMI for the degree all-reduce, the partial-tree gather / binomial
reduce and the parts broadcast — and uses torch.distributed over gloo (host TCP) only for:

  * shard_bounds   — contiguous record shards, like `-l part/num_parts`;
  * init_control   — the gloo process group from torchrun's env (RANK / WORLD_SIZE /
                     MASTER_ADDR / MASTER_PORT);
  * shared_port    — a free TCP port chosen by rank 0 for sheep_group_join's rendezvous;
  * barrier        — MPI_Barrier around the timed region;
  * max_over_ranks — the wall time of the slowest rank (bench.py's contract);
  * gather_objects — every rank's timing split, collected on rank 0.
"""
from __future__ import annotations

import datetime
import os
import socket

import torch
import torch.distributed as dist


def shard_bounds(nrec: int, rank: int, world: int) -> tuple[int, int]:
    return rank * nrec // world, (rank + 1) * nrec // world


def init_control(**kw) -> None:
    """The gloo group; its collectives give up after max(300 s, SHEEP_JOIN_TIMEOUT) instead of
    torch's 30 minutes, so a dead rank ends the run (the sheep world has its own deadline)."""
    if not dist.is_initialized():
        t = max(300, int(os.environ.get("SHEEP_JOIN_TIMEOUT", "300")))
        kw.setdefault("timeout", datetime.timedelta(seconds=t))
        dist.init_process_group("gloo", **kw)


def shared_port() -> int:
    """Rank 0 picks a free port on this host; every rank returns it."""
    box = [0]
    if dist.get_rank() == 0:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            box[0] = s.getsockname()[1]
    dist.broadcast_object_list(box, src=0)
    return int(box[0])


def barrier() -> None:
    dist.barrier()


def max_over_ranks(t: float) -> float:
    x = torch.tensor([float(t)], dtype=torch.float64)
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    return float(x.item())


def gather_objects(obj):
    """Rank 0 gets the list of every rank's `obj` (in rank order); the others get None."""
    out = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(obj, out, dst=0)
    return out


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
