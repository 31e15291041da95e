"""Parity at BASELINE.json's configurations, at FULL size, against
the CPU oracle (test infrastructure, OpenMP threads):

* C2 — RMAT-22 ef16 seed 22, k = 16, one GPU, the oracle run live: sequence, every
  parent and pst, parts, created / first-two sizes, every evaluator count, TREEFAQS.
* C3-C5 — against the oracle's recorded digests (tests/golden/scale/, made by
  tools/make_scale_golden.py on the GPU box: the oracle takes minutes per configuration
  there, more than the GPU suite's time budget):
* C3 — RMAT-26 ef16 seed 26, k = 64 (1.05e9 records): the oracle's sequence; every
  parent and pst against the oracle's tree (graph2tree -r form: 16 shard trees + the
  binomial mpi_merge, pinned to the golden trees by tests/test_oracle_golden.py); the
  whole tree == the one-pass merge of 8 contiguous shard trees; parts, created and every
  evaluator count against the oracle; the same on the shuffled records.
* C4 — Chung-Lu power law at twitter-2010 scale (41.65 M vertices, ~1.47e9 records,
  seed 2010), k = 128: the same set.
* C5 — RMAT-28 ef16 seed 28 (4.24e9 records: more than 2^32), k = 256, as 8 edge shards
  on one GPU (the one-GPU form of the 8-GPU configuration): the sequence from the
  shards' summed degrees, the K-way merge of the 8 shard trees against the oracle's
  tree AND against the binomial pairwise merges of the same shard trees, parts and
  created against the oracle, the full evaluator (edges cut, Vcom, ECV(hash/down/up),
  every balance) accumulated shard by shard against the oracle's.

Each configuration's GPU state lives in a class-scoped fixture so it is freed before
the next one is built."""
import json
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
GOLDEN_SCALE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scale")
THREADS = min(16, os.cpu_count() or 1)


def _shuffled(d, seed):
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
# C3-C5 at full size against the oracle's digests.  tools/make_scale_golden.py ran the
# oracle on each configuration's seeded records on the GPU box's host cores (minutes per
# configuration; the run logs are in profiles/r3/) and tests/golden/scale/<cfg>.json
# holds xxh3-128 digests of its sequence, parent, pst and parts arrays with every scalar
# result.  Each test regenerates the same records (their digest is checked first), runs
# the GPU path through the C ABI and compares digests and counts: bit-exact, in seconds.
# ---------------------------------------------------------------------------------
def _golden(cfg):
    return json.load(open(os.path.join(GOLDEN_SCALE, f"{cfg}.json")))


def _digest(a):
    import xxhash
    h = xxhash.xxh3_128()
    h.update(np.ascontiguousarray(a).view(np.uint8))
    return h.hexdigest()


def _records_digest(d):
    """xxh3-128 of the (tail, head) pairs, streamed to the host in chunks."""
    import xxhash
    x = xxhash.xxh3_128()
    step = 1 << 27
    for a in range(0, d.shape[0], step):
        x.update(np.ascontiguousarray(d[a:a + step, :2].cpu().numpy()).view(np.uint8))
    return x.hexdigest()


def _check_seq(s, g):
    assert s.n == g["n"] and s.pos_size == g["pos_size"]
    assert _digest(s.numpy()) == g["seq_digest"], "sequence"


def _check_tree_digest(tree, g):
    import sheep_amd
    p, w = sheep_amd.tree_to_numpy(tree)
    assert len(p) == g["n"]
    assert _digest(w) == g["pst_digest"], "pst_weight"
    assert _digest(p) == g["parent_digest"], "parent"
    # SURVEY §0 invariant 1 on the GPU's own array: every parent is a later node
    v = np.arange(len(p), dtype=np.int64)
    assert np.all((p == 0xFFFFFFFF) | (p.astype(np.int64) > v))
    assert int(np.count_nonzero(p == 0xFFFFFFFF)) == g["roots"]


def _check_parts(res, g):
    parts = res.numpy()
    assert _digest(parts) == g["parts_digest"], "parts"
    assert res.created == g["created"] and res.packing_nodes == g["packing_nodes"]
    assert res.first_size == g["first_size"] and res.second_size == g["second_size"]


def _gen(g):
    import sheep_amd
    gen = g["generator"]
    if gen["graph"] == "rmat":
        return sheep_amd.rmat(gen["scale"], 16, gen["seed"])
    return sheep_amd.powerlaw(sheep_amd.TWITTER_VERTICES, gen["draws"], gen["gamma"], gen["seed"])


class _FullSize:
    """The whole path at one BASELINE configuration on one GPU against its digests."""
    CFG = None

    @pytest.fixture(scope="class")
    def st(self, gpu_ctx):
        import sheep_amd
        g = _golden(self.CFG)
        d = _gen(g)
        state = {"g": g, "d": d}
        state["s"] = sheep_amd.degree_sequence(d, vs_cap=g["pos_size"])
        state["tree"] = sheep_amd.build_tree(d, state["s"])
        yield state
        state.clear()
        _free()

    def test_records_are_the_oracle_input(self, st):
        assert st["d"].shape[0] == st["g"]["records"]
        assert _records_digest(st["d"]) == st["g"]["records_digest"]

    def test_sequence_and_tree_vs_oracle(self, st):
        """degreeSequence (sequence.h:52-92); every parent and pst against the oracle's
        map/reduce tree (jtree.cpp:66-110 per shard, jnode.cpp:174-250); TREEFAQS."""
        import sheep_amd
        _check_seq(st["s"], st["g"])
        _check_tree_digest(st["tree"], st["g"])
        assert sheep_amd.facts(st["tree"]).__dict__ == st["g"]["facts"]

    def test_eight_shards_merge_to_whole_tree(self, st):
        import sheep_amd
        import torch
        d, s = st["d"], st["s"]
        R = d.shape[0]
        parts = torch.stack([sheep_amd.build_tree(d[i * R // 8:(i + 1) * R // 8], s) for i in range(8)])
        merged = sheep_amd.merge_trees_many(parts)
        del parts
        assert torch.equal(merged, st["tree"])

    def test_partition_and_full_evaluator_vs_oracle(self, st):
        """Partition + forwardPartition (partition.cpp:50-157), every evaluator count
        (partition.cpp:428-521)."""
        import sheep_amd
        g = st["g"]
        kids = sheep_amd.KidTable(st["tree"])
        res = sheep_amd.partition(st["s"], st["tree"], g["k"], kids=kids)
        kids.close()
        _check_parts(res, g)
        st["parts"] = res
        ev = sheep_amd.evaluate(st["d"], st["s"], res.parts)
        assert ev.__dict__ == g["evaluate"]

    def test_shuffled_records_same_results(self, st):
        """The whole path on the records in a random order, half of them reversed."""
        import sheep_amd
        g = st["g"]
        _free()
        d = _shuffled(st["d"], 2000 + g["generator"]["seed"])
        s = sheep_amd.degree_sequence(d, vs_cap=g["pos_size"])
        _check_seq(s, g)
        tree = sheep_amd.build_tree(d, s)
        _check_tree_digest(tree, g)
        res = sheep_amd.partition(s, tree, g["k"])
        _check_parts(res, g)
        ev = sheep_amd.evaluate(d, s, res.parts, what=sheep_amd.EVAL_DOWN)
        assert (ev.ecv_down, ev.max_down_bal) == (g["evaluate"]["ecv_down"], g["evaluate"]["max_down_bal"])
        del d, tree
        _free()


class TestC3(_FullSize):
    """C3: RMAT-26 ef16 seed 26, k = 64 (1.05e9 records)."""
    CFG = "c3"


class TestC4(_FullSize):
    """C4: Chung-Lu power law at twitter-2010 scale (41.65 M vertices, ~1.47e9 records,
    seed 2010), k = 128."""
    CFG = "c4"

    def test_size_is_twitter_scale(self, st):
        R = st["d"].shape[0]
        assert 1.40e9 < R < 1.55e9, R       # twitter-2010: 1,468,365,182 records
        assert st["g"]["n"] > 0.5 * 41_652_230


class TestC5:
    """C5: RMAT-28 ef16 seed 28 (4.24e9 records: more than 2^32), k = 256, as 8 edge
    shards on one GPU (the one-GPU form of the 8-GPU configuration): the sequence from the
    shards' summed degrees (mpiSequence), the K-way merge of the 8 shard trees against the
    oracle's tree AND against the binomial pairwise merges of the same shard trees
    (mpi_merge's schedule), parts, and the full evaluator accumulated shard by shard."""
    SHARDS = 8

    @pytest.fixture(scope="class")
    def c5(self, gpu_ctx):
        import sheep_amd
        import torch
        g = _golden("c5")
        d = _gen(g)
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
        state = dict(g=g, d=d, subs=subs, s=s, stack=stack, tree=tree)
        yield state
        state.clear()
        _free()

    def test_c5_records_are_the_oracle_input(self, c5):
        assert c5["d"].shape[0] == c5["g"]["records"] > (1 << 32) - (1 << 28)
        assert all(sub.shape[0] < (1 << 32) for sub in c5["subs"])
        assert _records_digest(c5["d"]) == c5["g"]["records_digest"]

    def test_c5_sequence_and_kway_tree_vs_oracle(self, c5):
        import sheep_amd
        _check_seq(c5["s"], c5["g"])
        _check_tree_digest(c5["tree"], c5["g"])
        assert sheep_amd.facts(c5["tree"]).__dict__ == c5["g"]["facts"]

    def test_c5_kway_equals_binomial_pairwise(self, c5):
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

    def test_c5_two_shards_same_tree(self, c5):
        """The one-GPU bench line's form: the fewest shards the 32-bit record index allows
        (2 x 2.1e9 records), mapped under the same sequence and merged K-way (K = 2): the
        same tree as the 8 shards' (the elimination tree is unique), against the oracle."""
        import sheep_amd
        import torch
        d, s = c5["d"], c5["s"]
        R = d.shape[0]
        halves = [d[:R // 2], d[R // 2:]]
        assert all(h.shape[0] < (1 << 32) for h in halves)
        two = torch.empty((2, s.n, 2), dtype=torch.int32, device="cuda")
        for i, h in enumerate(halves):
            sheep_amd.build_tree(h, s, out=two[i])
        tree = sheep_amd.merge_trees_many(two)
        del two
        _check_tree_digest(tree, c5["g"])
        assert torch.equal(tree, c5["tree"])

    def test_c5_partition_and_full_evaluator_vs_oracle(self, c5):
        import sheep_amd
        g = c5["g"]
        c5.pop("stack", None)
        _free()
        kids = sheep_amd.KidTable(c5["tree"])
        res = sheep_amd.partition(c5["s"], c5["tree"], g["k"], kids=kids)
        kids.close()
        _check_parts(res, g)
        ev = sheep_amd.ShardedEvaluator(c5["s"], res.parts, sheep_amd.EVAL_GRAPH | sheep_amd.EVAL_DOWN | sheep_amd.EVAL_UP)
        for sub in c5["subs"]:
            ev.add(sub)
        assert ev.finish().__dict__ == g["evaluate"]


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
