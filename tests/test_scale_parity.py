"""Parity at BASELINE.json's configurations, at FULL size, against
the CPU oracle (test infrastructure, OpenMP threads):

* C2 — RMAT-22 ef16 seed 22, k = 16, one GPU: sequence, every parent and pst, parts,
  created / first-two sizes, every evaluator count, TREEFAQS.
* C3 — RMAT-26 ef16 seed 26, k = 64 (1.05e9 records): the oracle's sequence; every
  parent and pst against the oracle's tree (graph2tree -r form: 16 shard trees + the
  binomial mpi_merge, pinned to the golden trees by tests/test_oracle_golden.py); the
  whole tree == the one-pass merge of 8 contiguous shard trees; parts, created and every
  evaluator count against the oracle.
* C4 — Chung-Lu power law at twitter-2010 scale (41.65 M vertices, ~1.47e9 records,
  seed 2010), k = 128: the same set, plus the 8-shard merge, on the generated and on a
  shuffled copy of the records.
* C5 — RMAT-28 ef16 seed 28 (4.24e9 records: more than 2^32), k = 256, as 8 edge shards
  on one GPU (the one-GPU form of the 8-GPU configuration): the sequence from the
  shards' summed degrees, the K-way merge of the 8 shard trees against the oracle's
  tree AND against the binomial pairwise merges of the same shard trees, parts and
  created against the oracle, the full evaluator (edges cut, Vcom, ECV(hash/down/up),
  every balance) accumulated shard by shard against the oracle's.

Each configuration's GPU state lives in a class-scoped fixture so it is freed before
the next one is built."""
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
    """(tail, head) as host u32 arrays, copied column-wise in chunks (no 12-B/record
    host staging of the whole record array)."""
    R = d.shape[0]
    t, h = np.empty(R, np.uint32), np.empty(R, np.uint32)
    step = 1 << 27
    for a in range(0, R, step):
        b = min(R, a + step)
        c = d[a:b, :2].contiguous().cpu().numpy().view(np.uint32)
        t[a:b], h[a:b] = c[:, 0], c[:, 1]
    return t, h


def _free():
    """Give the device memory back: torch's cache and the context's kernel workspace (sized
    by the largest graph so far, sheep_ctx_trim)."""
    import gc
    import torch
    import sheep_amd
    gc.collect()
    torch.cuda.empty_cache()
    sheep_amd.default_context().trim()


def _check_tree(tree, op, ow):
    import sheep_amd
    p, w = sheep_amd.tree_to_numpy(tree)
    bad = np.flatnonzero(p != op)
    assert bad.size == 0, f"parent differs at {bad.size} nodes, first {bad[:5]}: {p[bad[:5]]} vs {op[bad[:5]]}"
    assert np.array_equal(w, ow), "pst_weight"


# ---------------------------------------------------------------------------------
# C2: RMAT-22, k = 16
# ---------------------------------------------------------------------------------
class TestC2:
    @pytest.fixture(scope="class")
    def c2(self, gpu_ctx):
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
        _free()

    @pytest.mark.parametrize("variant", ["generated", "shuffled"])
    def test_c2_rmat22_k16_full_path(self, c2, variant):
        import sheep_amd
        d = c2["d"] if variant == "generated" else _shuffled(c2["d"], 2022)
        s = sheep_amd.degree_sequence(d, vs_cap=1 << 22)
        assert np.array_equal(s.numpy(), c2["seq"]), "sequence"
        tree = sheep_amd.build_tree(d, s)
        _check_tree(tree, c2["op"], c2["ow"])
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
class TestC3:
    @pytest.fixture(scope="class")
    def c3(self, gpu_ctx):
        import sheep_amd
        oracle.set_threads(THREADS)
        state = {"d": sheep_amd.rmat(26, 16, 26)}
        state["s"] = sheep_amd.degree_sequence(state["d"], vs_cap=1 << 26)
        state["tree"] = sheep_amd.build_tree(state["d"], state["s"])
        state["t"], state["h"] = _host(state["d"])
        yield state
        state.clear()
        oracle.set_threads(1)
        _free()

    def test_c3_rmat26_sequence_vs_oracle(self, c3):
        c3["seq"] = oracle.sequence(c3["t"], c3["h"], "records")
        assert np.array_equal(c3["s"].numpy(), c3["seq"])

    def test_c3_rmat26_tree_vs_oracle(self, c3):
        """Every parent and pst against the oracle's tree (jtree.cpp:66-110 per shard,
        jnode.cpp:174-250 reduce), and parent[v] > v (SURVEY §0 invariant 1)."""
        seq = c3.get("seq")
        if seq is None:
            seq = c3["s"].numpy()
        c3["op"], c3["ow"] = oracle.build_tree_mr(c3["t"], c3["h"], seq, 16)
        _check_tree(c3["tree"], c3["op"], c3["ow"])
        op = c3["op"].astype(np.int64)
        v = np.arange(len(op))
        assert np.all((op == 0xFFFFFFFF) | (op > v))

    def test_c3_rmat26_eight_shards_merge_to_whole_tree(self, c3):
        import sheep_amd
        import torch
        d, s, whole = c3["d"], c3["s"], c3["tree"]
        R = d.shape[0]
        parts = torch.stack([sheep_amd.build_tree(d[i * R // 8:(i + 1) * R // 8], s) for i in range(8)])
        merged = sheep_amd.merge_trees_many(parts)
        del parts
        assert torch.equal(merged, whole)

    def test_c3_rmat26_k64_partition_and_evaluate_vs_oracle(self, c3):
        import sheep_amd
        d, s, tree = c3["d"], c3["s"], c3["tree"]
        p, w = c3.get("op"), c3.get("ow")
        if p is None:
            p, w = sheep_amd.tree_to_numpy(tree)
        seq = s.numpy()
        oparts, oinfo = oracle.partition(p, w, seq, 64)
        res = sheep_amd.partition(s, tree, 64)
        assert np.array_equal(res.numpy(), oparts)
        assert res.created == oinfo["created"]
        c3["parts"] = res
        ev = sheep_amd.evaluate(d, s, res.parts)
        oev = oracle.evaluate(c3["t"], c3["h"], seq, oparts)
        assert ev.__dict__ == oev

    def test_c3_rmat26_shuffled_records_same_results(self, c3):
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


# ---------------------------------------------------------------------------------
# C4: Chung-Lu power law at twitter-2010 scale, k = 128
# ---------------------------------------------------------------------------------
class TestC4:
    @pytest.fixture(scope="class")
    def c4(self, gpu_ctx):
        import sheep_amd
        oracle.set_threads(THREADS)
        d = sheep_amd.powerlaw(sheep_amd.TWITTER_VERTICES, 2_222_000_000, 1.9, 2010)
        t, h = _host(d)
        seq = oracle.sequence(t, h, "records")
        op, ow = oracle.build_tree_mr(t, h, seq, 16)
        oparts, oinfo = oracle.partition(op, ow, seq, 128)
        state = dict(d=d, t=t, h=h, seq=seq, op=op, ow=ow, oparts=oparts, oinfo=oinfo)
        yield state
        state.clear()
        oracle.set_threads(1)
        _free()

    def test_c4_size_is_twitter_scale(self, c4):
        R = c4["d"].shape[0]
        assert 1.40e9 < R < 1.55e9, R       # twitter-2010: 1,468,365,182 records
        assert len(c4["seq"]) > 0.5 * 41_652_230

    @pytest.mark.parametrize("variant", ["generated", "shuffled"])
    def test_c4_powerlaw_k128_full_path(self, c4, variant):
        import sheep_amd
        import torch
        _free()
        d = c4["d"] if variant == "generated" else _shuffled(c4["d"], 2010)
        s = sheep_amd.degree_sequence(d, vs_cap=sheep_amd.TWITTER_VERTICES)
        assert np.array_equal(s.numpy(), c4["seq"]), "sequence"
        tree = sheep_amd.build_tree(d, s)
        _check_tree(tree, c4["op"], c4["ow"])
        if variant == "generated":
            R = d.shape[0]
            stack = torch.stack([sheep_amd.build_tree(d[i * R // 8:(i + 1) * R // 8], s) for i in range(8)])
            assert torch.equal(sheep_amd.merge_trees_many(stack), tree), "8-shard K-way merge"
            del stack
        kids = sheep_amd.KidTable(tree)
        res = sheep_amd.partition(s, tree, 128, kids=kids)
        kids.close()
        assert np.array_equal(res.numpy(), c4["oparts"]), "parts"
        assert res.created == c4["oinfo"]["created"]
        ev = sheep_amd.evaluate(d, s, res.parts)
        if "oev" not in c4:
            c4["oev"] = oracle.evaluate(c4["t"], c4["h"], c4["seq"], c4["oparts"])
        assert ev.__dict__ == c4["oev"]
        del d, tree
        _free()


# ---------------------------------------------------------------------------------
# C5: RMAT-28, k = 256, 8 edge shards on one GPU, full evaluator
# ---------------------------------------------------------------------------------
class TestC5:
    SHARDS = 8

    @pytest.fixture(scope="class")
    def c5(self, gpu_ctx):
        import sheep_amd
        import torch
        oracle.set_threads(THREADS)
        d = sheep_amd.rmat(28, 16, 28)
        R = d.shape[0]
        subs = [d[i * R // self.SHARDS:(i + 1) * R // self.SHARDS] for i in range(self.SHARDS)]
        deg = torch.zeros(1 << 28, dtype=torch.int32, device="cuda")
        vs = 0
        for sub in subs:                                   # mpiSequence's summed degrees
            _, ms = sheep_amd.degree_count(sub, deg=deg)
            vs = max(vs, ms)
        s = sheep_amd.sequence_from_degrees(deg, vs)
        del deg
        stack = torch.empty((self.SHARDS, s.n, 2), dtype=torch.int32, device="cuda")
        for i, sub in enumerate(subs):
            sheep_amd.build_tree(sub, s, out=stack[i])
        tree = sheep_amd.merge_trees_many(stack)
        t, h = _host(d)
        state = dict(d=d, subs=subs, s=s, stack=stack, tree=tree, t=t, h=h)
        yield state
        state.clear()
        oracle.set_threads(1)
        _free()

    def test_c5_rmat28_more_than_2e32_records(self, c5):
        assert c5["d"].shape[0] > (1 << 32) - (1 << 28)
        assert all(sub.shape[0] < (1 << 32) for sub in c5["subs"])

    def test_c5_rmat28_sequence_vs_oracle(self, c5):
        c5["seq"] = oracle.sequence(c5["t"], c5["h"], "records")
        assert np.array_equal(c5["s"].numpy(), c5["seq"])

    def test_c5_rmat28_kway_merge_vs_oracle_tree(self, c5):
        seq = c5.get("seq")
        if seq is None:
            seq = c5["s"].numpy()
        c5["op"], c5["ow"] = oracle.build_tree_mr(c5["t"], c5["h"], seq, self.SHARDS)
        _check_tree(c5["tree"], c5["op"], c5["ow"])

    def test_c5_rmat28_kway_equals_binomial_pairwise(self, c5):
        """mpi_merge's binomial schedule (pairwise sheep_merge_trees) == the K-way merge."""
        import sheep_amd
        import torch
        cur = [c5["stack"][i] for i in range(self.SHARDS)]
        d = 1
        while d < self.SHARDS:
            for i in range(0, self.SHARDS, 2 * d):
                if i + d < self.SHARDS:
                    cur[i] = sheep_amd.merge_trees(cur[i], cur[i + d])
            d *= 2
        assert torch.equal(cur[0], c5["tree"])

    def test_c5_rmat28_k256_partition_and_full_evaluator_vs_oracle(self, c5):
        import sheep_amd
        s, tree = c5["s"], c5["tree"]
        p, w = c5.get("op"), c5.get("ow")
        if p is None:
            p, w = sheep_amd.tree_to_numpy(tree)
        seq = s.numpy()
        c5.pop("stack", None)
        _free()
        kids = sheep_amd.KidTable(tree)
        res = sheep_amd.partition(s, tree, 256, kids=kids)
        kids.close()
        oparts, oinfo = oracle.partition(p, w, seq, 256)
        assert np.array_equal(res.numpy(), oparts), "parts"
        assert res.created == oinfo["created"]
        ev = sheep_amd.ShardedEvaluator(s, res.parts, sheep_amd.EVAL_GRAPH | sheep_amd.EVAL_DOWN | sheep_amd.EVAL_UP)
        for sub in c5["subs"]:
            ev.add(sub)
        got = ev.finish()
        oev = oracle.evaluate(c5["t"], c5["h"], seq, oparts)
        assert got.__dict__ == oev


# ---------------------------------------------------------------------------------
# Packing-event-heavy partitions on a smaller Chung-Lu graph (the shape on which the
# event search once came back empty): many k in one kid table, against the oracle.
# ---------------------------------------------------------------------------------
def test_powerlaw_event_heavy_partitions(gpu_ctx):
    import sheep_amd
    d = sheep_amd.powerlaw(2_000_000, 40_000_000, 1.9, 77)
    t, h = _host(d)
    s = sheep_amd.degree_sequence(d, vs_cap=2_000_000)
    tree = sheep_amd.build_tree(d, s)
    p, w = sheep_amd.tree_to_numpy(tree)
    seq = s.numpy()
    kids = sheep_amd.KidTable(tree)
    okids = oracle.Kids(p)
    # forwardPartition never ends when one node alone outweighs max_component
    # (partition.cpp:109-131): only the k it can pack
    total, wmax = int(w.astype(np.int64).sum()), int(w.max())
    ks = [k for k in (64, 256, 1024, 4096, 128, 2048) if int((total // k) * 1.03) > 2 * wmax]
    assert len(ks) >= 3, (total, wmax)
    events = 0
    for k in ks:
        res = sheep_amd.partition(s, tree, k, kids=kids)
        oparts, oinfo = oracle.partition(p, w, seq, k, kids=okids)
        assert np.array_equal(res.numpy(), oparts), f"k={k}"
        assert res.created == oinfo["created"] and res.packing_nodes == oinfo["packing_nodes"], f"k={k}"
        events += res.packing_nodes
    kids.close()
    assert events > 2000
