"""The N-rank schedule (sheep_amd/dist.py) on CPUs over gloo: edge shards -> degree
all-reduce -> per-shard trees -> binomial tree reduction to rank 0, with the CPU oracle
as the per-rank compute.  The sequence and the tree at rank 0 must equal the reference's
serial outputs (golden .seq / .tre) for every world size, odd ones included; this is the
same schedule bench.py drives with the HIP kernels over RCCL."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import golden_records, golden_seq, golden_tree


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_merge(x, y):
    import oracle
    xa, ya = x.numpy().view(np.uint32), y.numpy().view(np.uint32)
    po, wo = oracle.merge(xa[:, 0], xa[:, 1], ya[:, 0], ya[:, 1])
    return torch.from_numpy(np.stack([po, wo], axis=1).view(np.int32))


def _oracle_merge_many(stacked):
    """K-way merge = any fold of pairwise merges (the oracle has the pairwise one)."""
    acc = stacked[0]
    for t in stacked[1:]:
        acc = _oracle_merge(acc, t)
    return acc


def _rank_main(rank, world, port, name, out_path, reduce="binomial", split_parts=2):
    import oracle
    from sheep_amd import dist as sdist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        rec = golden_records(name)
        beg, end = sdist.shard_bounds(len(rec), rank, world)
        tail = rec["tail"][beg:end].astype(np.int64)
        head = rec["head"][beg:end].astype(np.int64)
        vs_cap = int(max(rec["tail"].max(), rec["head"].max())) + 1
        # LLAMA degrees of this shard (graph_wrapper.h:87-89): +1 per endpoint, a self-loop once
        deg = np.bincount(tail, minlength=vs_cap) + np.bincount(head[head != tail], minlength=vs_cap)
        max_slot = int(max(tail.max(), head.max())) + 1 if len(tail) else 0
        deg_t = torch.from_numpy(deg.astype(np.int32))
        vs = sdist.allreduce_degrees(deg_t, max_slot)
        d = deg_t.numpy()[:vs]
        slots = np.nonzero(d)[0]
        seq = slots[np.lexsort((slots, d[slots]))].astype(np.uint32)   # (degree, vid), sequence.h:52-63

        p, w = oracle.build_tree(tail, head, seq)
        tree = torch.from_numpy(np.stack([p, w], axis=1).view(np.int32))

        if reduce == "split":
            def merge_part(stacked, part, nparts):
                # the split merge's contract: every pst, and parents only in the part's
                # range (the rest scrambled, so rank 0 must take them from their owners)
                full = _oracle_merge_many(stacked).clone()
                n = full.shape[0]
                lo, hi = part * n // nparts, (part + 1) * n // nparts
                full[:lo, 0] = -7
                full[hi:, 0] = -7
                return full, lo, hi
            tree = sdist.reduce_trees_split(tree, merge_part, rank, world, nparts=split_parts)
        elif reduce == "kway":
            stacked = sdist.gather_trees(tree, rank, world)
            if rank == 0:   # the gather itself is exact: row r is rank r's own tree
                assert stacked.shape == (world,) + tuple(tree.shape)
                assert torch.equal(stacked[0], tree)
            tree = None if stacked is None else _oracle_merge_many(stacked)
        else:
            tree = sdist.reduce_trees(tree, _oracle_merge, rank, world)
        assert (tree is None) == (rank != 0)
        # Partition::mpi_sync: rank 0 partitions, every rank gets the parts
        parts = None
        if rank == 0:
            t0 = tree.numpy().view(np.uint32)
            parts = torch.from_numpy(oracle.partition(t0[:, 0], t0[:, 1], seq, 4)[0])
        n_slots = int(seq.max()) + 1
        parts = sdist.sync_parts(parts, n_slots, "cpu")
        gp, gw = golden_tree(name)
        assert np.array_equal(parts.numpy(), oracle.partition(gp, gw, seq, 4)[0])
        if rank == 0:
            t = tree.numpy().view(np.uint32)
            json.dump({"seq": seq.tolist(), "parent": t[:, 0].tolist(), "pst": t[:, 1].tolist()}, open(out_path, "w"))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("name", ["hep", "rmat10"])
def test_sharded_schedule_matches_serial(tmp_path, name, world):
    out = str(tmp_path / "rank0.json")
    mp.spawn(_rank_main, args=(world, _free_port(), name, out), nprocs=world, join=True)
    got = json.load(open(out))
    assert np.array_equal(np.array(got["seq"], np.uint32), golden_seq(name))
    parent, pst = golden_tree(name)
    assert np.array_equal(np.array(got["parent"], np.uint32), parent)
    assert np.array_equal(np.array(got["pst"], np.uint32), pst)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_kway_schedule_matches_serial(tmp_path, world):
    """Gather to rank 0 + one K-way reduction (bench.py's default --reduce kway)."""
    out = str(tmp_path / "rank0.json")
    mp.spawn(_rank_main, args=(world, _free_port(), "rmat10", out, "kway"), nprocs=world, join=True)
    got = json.load(open(out))
    parent, pst = golden_tree("rmat10")
    assert np.array_equal(np.array(got["parent"], np.uint32), parent)
    assert np.array_equal(np.array(got["pst"], np.uint32), pst)


@pytest.mark.parametrize("world,nparts", [(2, 2), (3, 2), (4, 2), (4, 4)])
def test_split_schedule_matches_serial(tmp_path, world, nparts):
    """Every tree to the part ranks + one part of the split merge each + the parts' node
    ranges gathered to rank 0 (bench.py's --reduce split)."""
    out = str(tmp_path / "rank0.json")
    mp.spawn(_rank_main, args=(world, _free_port(), "rmat10", out, "split", nparts), nprocs=world, join=True)
    got = json.load(open(out))
    parent, pst = golden_tree("rmat10")
    assert np.array_equal(np.array(got["parent"], np.uint32), parent)
    assert np.array_equal(np.array(got["pst"], np.uint32), pst)


def test_shard_bounds_cover():
    from sheep_amd.dist import shard_bounds
    for R in (0, 1, 7, 1000):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(R, r, world) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == R
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
