"""Partition files (partition.cpp:588-670 writePartitionedGraph).

CPU: the fixtures written by the reference's own writer (oracle/_ref ref_harness
`write` / `writefile`, tests/golden/G.k<K>.{g,f}NNNN) are restated from the oracle's
partition and the records — graph order (graph2tree -p -o: X ascending, adjacency in
record order, X < Y) and input-file order (partition_tree -o: every record, an XS1 file
repeating its last one); an edge goes to the part of its earlier-positioned endpoint.
GPU: both CLIs reproduce the fixture files byte for byte (the owners come from the
sheep_edge_parts kernel)."""
import filecmp
import os
import subprocess

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, ROOT, golden_records, golden_seq, golden_tree, manifest

BIN = os.path.join(ROOT, "sheep_amd", "bin")


def write_cases():
    return sorted(manifest()["_write_k"].items())


def fixture_files(name, k, tag):
    files = sorted(f for f in os.listdir(GOLDEN) if f.startswith(f"{name}.k{k}.{tag}"))
    return [open(os.path.join(GOLDEN, f)).read() for f in files]


def restate(name, k, file_order):
    r = golden_records(name)
    seq = golden_seq(name)
    p, w = golden_tree(name)
    parts, _ = oracle.partition(p, w, seq, k)   # a fresh kid table, as in one CLI call
    pos = np.full(len(parts), -1, np.int64)
    pos[seq] = np.arange(len(seq))
    t, h = r["tail"].astype(np.int64), r["head"].astype(np.int64)
    owner = np.where(pos[t] < pos[h], parts[t], parts[h])
    if file_order:
        idx = list(range(len(t))) + [len(t) - 1]   # XS1Reader reads the last record twice
        lines = [(int(t[i]), int(h[i]), int(owner[i])) for i in idx]
    else:
        keep = np.nonzero(t != h)[0]
        lo, hi = np.minimum(t, h)[keep], np.maximum(t, h)[keep]
        order = np.argsort(lo, kind="stable")
        lines = [(int(lo[i]), int(hi[i]), int(owner[keep[i]])) for i in order]
    out = [""] * (int(parts.max()) + 1)
    for x, y, q in lines:
        out[q] += f"{x} {y}\n"
    return out


@pytest.mark.parametrize("name,k", write_cases())
@pytest.mark.parametrize("file_order", [False, True])
def test_reference_files_restated(name, k, file_order):
    got = restate(name, k, file_order)
    assert got == fixture_files(name, k, "f" if file_order else "g")


def run(*args):
    p = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("name,k", write_cases())
def test_graph2tree_partition_files(gpu_ctx, tmp_path, name, k):
    """graph2tree G -p K -o PREFIX (graph2tree.cpp:203-214): graph-order files."""
    run(os.path.join(BIN, "graph2tree"), os.path.join(GOLDEN, f"{name}.dat"), "-p", k, "-o", tmp_path / "p")
    ref = sorted(f for f in os.listdir(GOLDEN) if f.startswith(f"{name}.k{k}.g"))
    got = sorted(os.listdir(tmp_path))
    assert len(got) == len(ref)
    for g, f in zip(got, ref):
        assert g == "p" + f[-4:]
        assert filecmp.cmp(tmp_path / g, os.path.join(GOLDEN, f), shallow=False), f


@pytest.mark.gpu
@pytest.mark.parametrize("name,k", write_cases())
def test_partition_tree_partition_files(gpu_ctx, tmp_path, name, k):
    """partition_tree -g G -o PREFIX SEQ TREE K (partition_tree.cpp:146-163): input-order files."""
    out = run(os.path.join(BIN, "partition_tree"), "-g", os.path.join(GOLDEN, f"{name}.dat"), "-o", tmp_path / "p",
              os.path.join(GOLDEN, f"{name}.seq"), os.path.join(GOLDEN, f"{name}.tre"), k)
    assert "Actually created " in out
    ref = sorted(f for f in os.listdir(GOLDEN) if f.startswith(f"{name}.k{k}.f"))
    got = sorted(os.listdir(tmp_path))
    assert len(got) == len(ref)
    for g, f in zip(got, ref):
        assert filecmp.cmp(tmp_path / g, os.path.join(GOLDEN, f), shallow=False), f
