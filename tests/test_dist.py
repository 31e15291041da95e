"""The N-rank run on CPUs (no device): the pieces of bench.py's and graph2tree -i -r's
one-process-per-rank world that are host code.

* the TCP links every joined world is built on (sheep_group_join -> mesh.hip): the
  rendezvous, rank 0's bytes to everyone, a ring shift, a gather to rank 0 and the
  all-reduces, at world sizes 1-4 (sheep_mesh_selftest, one process per rank);
* bench.py's control plane (sheep_amd/dist.py) over gloo at world 2-3: the shared
  rendezvous port, the barrier and the max over ranks of the wall time;
* the contiguous edge shards of `-l part/num_parts`.

The world's data path (the degree all-reduce, the tree gather / binomial reduce, the parts
broadcast, the sharded evaluator) runs in HIP kernels: tests/test_gpu_parity.py runs it as
processes joined over these links on one GPU, tests/test_cli.py under mpiexec."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

LIB = os.path.join(ROOT, "sheep_amd", "lib", "libsheep_hip.so")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pattern(rank, nbytes):
    out = np.empty(nbytes, np.uint8)
    x = (0x9E3779B97F4A7C15 * (rank + 1)) & 0xFFFFFFFFFFFFFFFF
    for i in range(nbytes):
        x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
        x ^= x >> 7
        x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
        out[i] = x & 0xFF
    return out


def _fnv(b):
    h = 1469598103934665603
    for x in b.tolist():
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def _mesh_rank(rank, world, port, nbytes, q):
    L = ctypes.CDLL(LIB)
    L.sheep_mesh_selftest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    cs, mx = ctypes.c_uint64(), ctypes.c_uint64()
    rc = L.sheep_mesh_selftest(rank, world, b"127.0.0.1", port, nbytes, ctypes.byref(cs), ctypes.byref(mx))
    q.put((rank, rc, cs.value, mx.value))


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_mesh_links(world):
    if not os.path.exists(LIB):
        pytest.skip("libsheep_hip.so not built")
    nbytes = 3000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mesh_rank, args=(r, world, port, nbytes, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    h = [_fnv(_pattern(r, nbytes)) for r in range(world)]
    want = sum(h[0] + (h[(r - 1) % world] if world > 1 else 0) for r in range(world))
    want += sum(h[1:]) if world > 1 else 0
    want &= 0xFFFFFFFFFFFFFFFF
    for rank, rc, cs, mx in got:
        assert rc == 0, rank
        assert cs == want, rank
        assert mx == max(h), rank


def _stall_rank(rank, world, port, stall, timeout_s, q):
    L = ctypes.CDLL(LIB)
    L.sheep_mesh_selftest_stall.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    L.sheep_last_error.restype = ctypes.c_char_p
    waited = ctypes.c_double()
    rc = L.sheep_mesh_selftest_stall(rank, world, b"127.0.0.1", port, stall, timeout_s, ctypes.byref(waited))
    q.put((rank, rc, waited.value, L.sheep_last_error().decode() if rc else ""))


@pytest.mark.parametrize("world,stall", [(2, 1), (3, 1), (3, 0)])
def test_mesh_deadline_when_a_rank_stalls(world, stall):
    """A rank that joins and then stops taking part (alive, sockets open) must surface as an
    error on the others within SHEEP_JOIN_TIMEOUT, not as a hang: rank 0 waiting on the
    stalled rank times out naming it; a rank waiting on rank 0 instead learns when rank 0
    gives up and closes its links (or times out itself when rank 0 is the stalled one)."""
    if not os.path.exists(LIB):
        pytest.skip("libsheep_hip.so not built")
    timeout_s = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stall_rank, args=(r, world, port, stall, timeout_s, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, rc, waited, msg in got:
        if rank == stall:
            assert rc == 0
            continue
        assert rc != 0, rank
        assert waited <= timeout_s + 1.5, (rank, waited)
        if rank == 0 or stall == 0:   # the waiter on the stalled rank itself: a timeout naming it
            assert f"timed out waiting for rank {stall}" in msg, msg
        else:                         # rank 0 gave up and closed its links
            assert "rank 0" in msg, msg


def _control_rank(rank, world, port, q):
    import torch.distributed as dist
    from sheep_amd import dist as sdist
    sdist.init_control(init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    p = sdist.shared_port()
    sdist.barrier()
    t = sdist.max_over_ranks(0.5 + rank)
    q.put((rank, p, t, dist.get_backend()))
    sdist.shutdown()


@pytest.mark.parametrize("world", [2, 3])
def test_control_plane(world):
    """bench.py's N-rank control plane over gloo: every rank gets rank 0's rendezvous
    port for sheep_group_join, and the wall time is the slowest rank's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_control_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    ports = {g[1] for g in got}
    assert len(ports) == 1 and 0 < ports.pop() < 65536
    assert all(g[2] == 0.5 + world - 1 for g in got)
    assert all(g[3] == "gloo" for g in got)


def test_shard_bounds_cover():
    from sheep_amd.dist import shard_bounds
    for R in (0, 1, 7, 1000):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(R, r, world) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == R
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
