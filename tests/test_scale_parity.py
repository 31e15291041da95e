"""Parity at BASELINE.json's configurations:

* C2 — RMAT-22 ef16 seed 22, k = 16, one GPU: the whole path against the CPU oracle
  (sequence, parent + pst, parts, created / first-two sizes, every evaluator count,
  TREEFAQS), bit-exact;
* C3 — RMAT-26 ef16 seed 26, k = 64, at full size (1.05e9 records): the oracle's
  sequence; the whole-graph tree equals the one-pass merge of 8 contiguous shard trees;
  parent[v] > v and pst = the histogram of each record's lower position (computed by
  torch, independently of the HIP path); the oracle's forwardPartition on the GPU tree
  gives the GPU's parts; the oracle's evaluators give the GPU's counts.

Each configuration also runs on a SHUFFLED copy of its records (random order, half the
records with tail and head swapped): the generator's (tail, head)-sorted order is not a
property of a generic edge list, and every result must be identical.

The oracle (test infrastructure) runs with OpenMP threads here; its threaded form is
pinned to the golden fixtures by tests/test_oracle_golden.py."""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _shuffled(d, seed):
    """Records in a random order, half of them with tail and head swapped."""
    import torch
    g = torch.Generator(device=d.device)
    g.manual_seed(seed)
    perm = torch.randperm(d.shape[0], device=d.device, generator=g)
    out = d[perm]
    del perm
    flip = torch.rand(out.shape[0], device=d.device, generator=g) < 0.5
    tail = out[:, 0].clone()
    out[flip, 0] = out[flip, 1]
    out[flip, 1] = tail[flip]
    return out


def _host(d):
    import sheep_amd
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    return np.ascontiguousarray(h[:, 0]), np.ascontiguousarray(h[:, 1])


# ---------------------------------------------------------------------------------
# C2: RMAT-22, k = 16
# ---------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c2(gpu_ctx):
    import sheep_amd
    oracle.set_threads(THREADS)
    d = sheep_amd.rmat(22, 16, 22)
    t, h = _host(d)
    seq = oracle.sequence(t, h)
    op, ow = oracle.build_tree(t, h, seq)
    oparts, oinfo = oracle.partition(op, ow, seq, 16)
    oev = oracle.evaluate(t, h, seq, oparts)
    yield dict(d=d, seq=seq, op=op, ow=ow, oparts=oparts, oinfo=oinfo, oev=oev, facts=oracle.facts(op, ow))
    oracle.set_threads(1)


@pytest.mark.parametrize("variant", ["generated", "shuffled"])
def test_c2_rmat22_k16_full_path(c2, variant):
    import sheep_amd
    d = c2["d"] if variant == "generated" else _shuffled(c2["d"], 2022)
    s = sheep_amd.degree_sequence(d, vs_cap=1 << 22)
    assert np.array_equal(s.numpy(), c2["seq"]), "sequence"
    tree = sheep_amd.build_tree(d, s)
    p, w = sheep_amd.tree_to_numpy(tree)
    assert np.array_equal(p, c2["op"]), "parent"
    assert np.array_equal(w, c2["ow"]), "pst_weight"
    assert sheep_amd.facts(tree).__dict__ == c2["facts"]
    kids = sheep_amd.KidTable(tree)
    res = sheep_amd.partition(s, tree, 16, kids=kids)
    parts = res.numpy()
    assert np.array_equal(parts, c2["oparts"]), "parts"
    assert res.created == c2["oinfo"]["created"]
    assert res.first_size == np.count_nonzero(parts == 0) and res.second_size == np.count_nonzero(parts == 1)
    ev = sheep_amd.evaluate(d, s, res.parts)
    assert ev.__dict__ == c2["oev"]
    kids.close()


# ---------------------------------------------------------------------------------
# C3: RMAT-26, k = 64, full size
# ---------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c3(gpu_ctx):
    import sheep_amd
    import torch
    oracle.set_threads(THREADS)
    state = {"d": sheep_amd.rmat(26, 16, 26)}
    state["s"] = sheep_amd.degree_sequence(state["d"], vs_cap=1 << 26)
    state["tree"] = sheep_amd.build_tree(state["d"], state["s"])
    yield state
    state.clear()
    oracle.set_threads(1)
    torch.cuda.empty_cache()


def test_c3_rmat26_sequence_vs_oracle(c3):
    t, h = _host(c3["d"])
    seq = oracle.sequence(t, h, "records")
    assert np.array_equal(c3["s"].numpy(), seq)


def test_c3_rmat26_tree_properties(c3):
    """parent[v] > v for every non-root, and pst_weight = the histogram of each record's
    lower sequence position (SURVEY §0 invariants 1-2), the latter computed with torch."""
    import torch
    d, s, tree = c3["d"], c3["s"], c3["tree"]
    n = s.n
    parent = tree[:, 0].to(torch.int64) & 0xFFFFFFFF
    v = torch.arange(n, device=parent.device)
    root = parent == 0xFFFFFFFF
    assert bool(torch.all(root | ((parent > v) & (parent < n))))
    pos = s.pos[: s.pos_size].to(torch.int64) & 0xFFFFFFFF
    lo = torch.minimum(pos[d[:, 0].to(torch.int64)], pos[d[:, 1].to(torch.int64)])
    want = torch.bincount(lo, minlength=n)
    del lo, pos
    assert int(want.sum()) == d.shape[0]                    # no self-loops: every record counts
    assert torch.equal(tree[:, 1].to(torch.int64), want)


def test_c3_rmat26_eight_shards_merge_to_whole_tree(c3):
    import sheep_amd
    import torch
    d, s, whole = c3["d"], c3["s"], c3["tree"]
    R = d.shape[0]
    parts = torch.stack([sheep_amd.build_tree(d[i * R // 8:(i + 1) * R // 8], s) for i in range(8)])
    merged = sheep_amd.merge_trees_many(parts)
    del parts
    assert torch.equal(merged, whole)


def test_c3_rmat26_k64_partition_and_evaluate_vs_oracle(c3):
    import sheep_amd
    d, s, tree = c3["d"], c3["s"], c3["tree"]
    p, w = sheep_amd.tree_to_numpy(tree)
    seq = s.numpy()
    oparts, oinfo = oracle.partition(p, w, seq, 64)
    res = sheep_amd.partition(s, tree, 64)
    assert np.array_equal(res.numpy(), oparts)
    assert res.created == oinfo["created"]
    c3["parts"] = res
    ev = sheep_amd.evaluate(d, s, res.parts)
    t, h = _host(d)
    oev = oracle.evaluate(t, h, seq, oparts)
    assert ev.__dict__ == oev


def test_c3_rmat26_shuffled_records_same_results(c3):
    """The whole path on the shuffled records: same sequence, tree, parts and counts."""
    import sheep_amd
    import torch
    d = _shuffled(c3["d"], 2026)
    s = sheep_amd.degree_sequence(d, vs_cap=1 << 26)
    assert torch.equal(s.seq[: s.n], c3["s"].seq[: c3["s"].n])
    tree = sheep_amd.build_tree(d, s)
    assert torch.equal(tree, c3["tree"])
    res = sheep_amd.partition(s, tree, 64)
    ref = c3.get("parts") or sheep_amd.partition(c3["s"], c3["tree"], 64)
    assert torch.equal(res.parts, ref.parts)
    ev = sheep_amd.evaluate(d, s, res.parts, what=sheep_amd.EVAL_DOWN)
    ev0 = sheep_amd.evaluate(c3["d"], c3["s"], ref.parts, what=sheep_amd.EVAL_DOWN)
    assert ev == ev0
