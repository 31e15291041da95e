"""GPU parity: every stage of the HIP path, called through the C ABI, against the
reference's golden fixtures (tests/golden, produced by oracle/_ref) and, at sizes the
golden files do not cover, against the CPU oracle.  Bit-exact throughout (integer /
index work)."""
import os

import numpy as np
import pytest

import oracle
from conftest import (GRAPHS, golden_part_text, golden_parts, golden_records, golden_seq, golden_tree, ks)

pytestmark = pytest.mark.gpu


def _dev_records(rec):
    import sheep_amd
    return sheep_amd.records_to_device(rec["tail"], rec["head"], rec["weight"])


def _tree_np(tree):
    import sheep_amd
    return sheep_amd.tree_to_numpy(tree)


@pytest.mark.parametrize("scale,seed", [(10, 10), (14, 14), (17, 3)])
def test_rmat_gpu_matches_host(gpu_ctx, scale, seed):
    import sheep_amd
    d = sheep_amd.to_numpy_u32(sheep_amd.rmat(scale, 16, seed)).reshape(-1, 3)
    h = sheep_amd.rmat_host(scale, 16, seed)
    assert d.shape == h.shape and np.array_equal(d, h)


@pytest.mark.parametrize("name", GRAPHS)
@pytest.mark.parametrize("mode,kind", [("llama", "seq"), ("dat", "fileseq")])
def test_degree_sequence(gpu_ctx, name, mode, kind):
    import sheep_amd
    rec = golden_records(name)
    s = sheep_amd.degree_sequence(_dev_records(rec), mode=mode)
    assert np.array_equal(s.numpy(), golden_seq(name, kind))
    # pos is the inverse permutation, INVALID on degree-0 slots
    pos = sheep_amd.to_numpy_u32(s.pos[: s.pos_size])
    seq = s.numpy()
    assert np.array_equal(pos[seq], np.arange(len(seq), dtype=np.uint32))
    assert np.count_nonzero(pos != 0xFFFFFFFF) == len(seq)


@pytest.mark.parametrize("mode", ["llama", "dat"])
def test_degree_sequence_unsorted_records(gpu_ctx, mode):
    """Records in no particular order (tails bucketed with the heads instead of run-added)
    give the oracle's sequence in both degree modes, the FILE_DAT last record included."""
    import sheep_amd
    import torch
    d = sheep_amd.rmat(15, 16, 15)
    g = torch.Generator(device=d.device)
    g.manual_seed(5)
    d = d[torch.randperm(d.shape[0], device=d.device, generator=g)].contiguous()
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    s = sheep_amd.degree_sequence(d, mode=mode)
    assert np.array_equal(s.numpy(), oracle.sequence(h[:, 0], h[:, 1], mode))


@pytest.mark.parametrize("name", GRAPHS)
def test_tree(gpu_ctx, name):
    import sheep_amd
    rec = golden_records(name)
    s = sheep_amd.sequence_from_host(golden_seq(name))
    p, w = _tree_np(sheep_amd.build_tree(_dev_records(rec), s))
    gp, gw = golden_tree(name)
    assert np.array_equal(p, gp), "parent"
    assert np.array_equal(w, gw), "pst_weight"


@pytest.mark.parametrize("name", GRAPHS)
def test_partial_trees_and_merge(gpu_ctx, name):
    """graph2tree -l 1/2, 2/2 (contiguous record halves) + merge_trees."""
    import sheep_amd
    rec = golden_records(name)
    R = len(rec)
    s = sheep_amd.sequence_from_host(golden_seq(name))
    d = _dev_records(rec)
    trees = []
    for part, which in ((1, "h1.tre"), (2, "h2.tre")):
        beg, end = (part - 1) * R // 2, part * R // 2
        t = sheep_amd.build_tree(d[beg:end], s)
        p, w = _tree_np(t)
        gp, gw = golden_tree(name, which)
        assert np.array_equal(p, gp) and np.array_equal(w, gw), which
        trees.append(t)
    p, w = _tree_np(sheep_amd.merge_trees(*trees))
    gp, gw = golden_tree(name, "merge.tre")
    assert np.array_equal(p, gp) and np.array_equal(w, gw)


@pytest.mark.parametrize("use_pos", [True, False])
@pytest.mark.parametrize("name", GRAPHS)
def test_partition_evaluate_facts(gpu_ctx, name, use_pos):
    """partition_tree -f -g SEQ TREE k1 k2 ...: one kid table for all k (the FFD sort
    order persists across k), printed lines byte-exact; the parts reach their vid slots
    through the sequence's index (sheep_partition_pos) or by the per-jnid scatter."""
    import sheep_amd
    rec = golden_records(name)
    s = sheep_amd.sequence_from_host(golden_seq(name))
    gp, gw = golden_tree(name)
    tree = sheep_amd.tree_to_device(gp, gw)
    facts_txt, blocks = golden_part_text(name)
    assert sheep_amd.facts(tree).text() == facts_txt
    kids = sheep_amd.KidTable(tree)
    d = _dev_records(rec)
    for k, block in zip(ks(name), blocks):
        res = sheep_amd.partition(s, tree, k, kids=kids, use_pos=use_pos)
        assert np.array_equal(res.numpy(), golden_parts(name, k)), f"k={k}"
        ev = sheep_amd.evaluate(d, s, res.parts)
        assert res.print_text() + ev.text(k) == block, f"k={k}"


@pytest.mark.parametrize("scale,seed,k", [(16, 5, 16), (18, 7, 64)])
def test_rmat_vs_oracle(gpu_ctx, scale, seed, k):
    """Beyond the committed fixtures: the whole path on larger RMAT graphs vs the oracle."""
    import sheep_amd
    d = sheep_amd.rmat(scale, 16, seed)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    t_, h_ = h[:, 0], h[:, 1]
    s = sheep_amd.degree_sequence(d)
    seq = oracle.sequence(t_, h_)
    assert np.array_equal(s.numpy(), seq)
    tree = sheep_amd.build_tree(d, s)
    p, w = _tree_np(tree)
    op, ow = oracle.build_tree(t_, h_, seq)
    assert np.array_equal(p, op) and np.array_equal(w, ow)
    assert sheep_amd.facts(tree).__dict__ == oracle.facts(op, ow)
    res = sheep_amd.partition(s, tree, k)
    oparts, oinfo = oracle.partition(op, ow, seq, k)
    assert np.array_equal(res.numpy(), oparts)
    assert res.created == oinfo["created"]
    ev = sheep_amd.evaluate(d, s, res.parts)
    oev = oracle.evaluate(t_, h_, seq, oparts)
    assert ev.__dict__ == oev


def test_timed_trees_count_their_levels(gpu_ctx):
    """With timing on, the elimination tree's per-level list sizes travel to a pinned
    buffer on the stream and are counted into the regions' algorithmic bytes when the
    timers are read (no host round trip inside the timed trees): the bytes of two identical
    maps are about twice one map's (the contraction dedup is lossy under races, so a level's
    list length varies a little between runs), they survive timing being switched off
    before the read, and a reset clears them.  The trees stay the oracle's."""
    import sheep_amd
    ctx = gpu_ctx
    d = sheep_amd.rmat(17, 16, 13)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    s = sheep_amd.degree_sequence(d)
    op, ow = oracle.build_tree(h[:, 0], h[:, 1], oracle.sequence(h[:, 0], h[:, 1]))
    regions = ("etree_split", "etree_union", "etree_cross", "etree_apply")
    ctx.timer_reset()
    ctx.timing(True)
    try:
        p, w = _tree_np(sheep_amd.build_tree(d, s))
        assert np.array_equal(p, op) and np.array_equal(w, ow)
        one = {r: ctx.timer(r)[2] for r in regions}
        assert all(v > 0 for v in one.values()), one
        ctx.timer_reset()
        for _ in range(2):
            p, w = _tree_np(sheep_amd.build_tree(d, s))
            assert np.array_equal(p, op) and np.array_equal(w, ow)
    finally:
        ctx.timing(False)
    two = {r: ctx.timer(r)[2] for r in regions}   # read after timing went off
    assert all(abs(two[r] - 2 * one[r]) <= 0.05 * 2 * one[r] for r in regions), (one, two)
    ctx.timer_reset()
    assert all(ctx.timer(r)[2] == 0 for r in regions)


def test_relabel_layout_reuse_and_stale(gpu_ctx):
    """The bucketed relabel reuses the degree pass's head-bucket offsets; records changed
    in place after degree_sequence (same pointer and count, other head buckets) must be
    detected in-kernel and recounted.  Swapping tail/head keeps the undirected graph, so
    the tree is the oracle's tree of the original records."""
    import sheep_amd
    d = sheep_amd.rmat(16, 16, 21)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    t_, h_ = h[:, 0].copy(), h[:, 1].copy()
    s = sheep_amd.degree_sequence(d)
    seq = oracle.sequence(t_, h_)
    op, ow = oracle.build_tree(t_, h_, seq)
    p, w = _tree_np(sheep_amd.build_tree(d, s))          # cached layout
    assert np.array_equal(p, op) and np.array_equal(w, ow)
    sw = d[::3, 0].clone()
    d[::3, 0] = d[::3, 1]
    d[::3, 1] = sw                                      # stale layout: same ptr, same nrec
    p, w = _tree_np(sheep_amd.build_tree(d, s))
    assert np.array_equal(p, op) and np.array_equal(w, ow)
    p, w = _tree_np(sheep_amd.build_tree(d, s))          # the recounted layout, reused
    assert np.array_equal(p, op) and np.array_equal(w, ow)


def test_relabel_records_in_any_order(gpu_ctx):
    """Records in no order (the degree pass's probe sees descents: both endpoints are
    bucketed, and the endpoint count's head columns are the relabel's head layout), with
    self-loops and repeated records: the tree and pst must be the oracle's; a layout made
    stale in place (heads moved to other buckets) is detected and recounted, same tree."""
    import sheep_amd
    import torch
    d = sheep_amd.rmat(16, 16, 31)
    loops = d[:4000].clone()
    loops[:, 1] = loops[:, 0]                            # self-loops
    d = torch.cat([d, loops, d[:2000]])                  # and repeated records
    g = torch.Generator(device=d.device)
    g.manual_seed(9)
    d = d[torch.randperm(d.shape[0], device=d.device, generator=g)].contiguous()
    sw = d[::2, 0].clone()
    d[::2, 0] = d[::2, 1]
    d[::2, 1] = sw
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    t_, h_ = h[:, 0].copy(), h[:, 1].copy()
    s = sheep_amd.degree_sequence(d)
    seq = oracle.sequence(t_, h_)
    assert np.array_equal(s.numpy(), seq)
    op, ow = oracle.build_tree(t_, h_, seq)
    p, w = _tree_np(sheep_amd.build_tree(d, s))
    assert np.array_equal(p, op) and np.array_equal(w, ow)
    sw = d[::3, 0].clone()
    d[::3, 0] = d[::3, 1]
    d[::3, 1] = sw                                      # stale layouts: same ptr, same nrec
    p, w = _tree_np(sheep_amd.build_tree(d, s))
    assert np.array_equal(p, op) and np.array_equal(w, ow)


def test_shards_merge_to_whole_tree(gpu_ctx):
    """Shard independence: 4 contiguous shards, pairwise merges == the whole tree."""
    import sheep_amd
    d = sheep_amd.rmat(18, 16, 11)
    s = sheep_amd.degree_sequence(d)
    whole = _tree_np(sheep_amd.build_tree(d, s))
    R = d.shape[0]
    parts = [sheep_amd.build_tree(d[i * R // 4:(i + 1) * R // 4], s) for i in range(4)]
    m = sheep_amd.merge_trees(sheep_amd.merge_trees(parts[0], parts[1]), sheep_amd.merge_trees(parts[2], parts[3]))
    p, w = _tree_np(m)
    assert np.array_equal(p, whole[0]) and np.array_equal(w, whole[1])


@pytest.mark.parametrize("name", GRAPHS)
def test_merge_many_golden_halves(gpu_ctx, name):
    """sheep_merge_trees_many over the two golden half-shard trees == the golden merge."""
    import sheep_amd
    import torch
    h = [sheep_amd.tree_to_device(*golden_tree(name, w)) for w in ("h1.tre", "h2.tre")]
    p, w = _tree_np(sheep_amd.merge_trees_many(torch.stack(h)))
    gp, gw = golden_tree(name, "merge.tre")
    assert np.array_equal(p, gp) and np.array_equal(w, gw)


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 70])
def test_merge_many_shards_to_whole_tree(gpu_ctx, k):
    """k contiguous shards merged in ONE pass == the whole tree == pairwise merges (k = 70:
    more trees than one merge pass takes, so a second pass merges the first's result)."""
    import sheep_amd
    import torch
    d = sheep_amd.rmat(17, 16, 7)
    s = sheep_amd.degree_sequence(d)
    whole = _tree_np(sheep_amd.build_tree(d, s))
    R = d.shape[0]
    parts = [sheep_amd.build_tree(d[i * R // k:(i + 1) * R // k], s) for i in range(k)]
    p, w = _tree_np(sheep_amd.merge_trees_many(torch.stack(parts)))
    assert np.array_equal(p, whole[0]) and np.array_equal(w, whole[1])
    acc = parts[0]
    for t in parts[1:]:
        acc = sheep_amd.merge_trees(acc, t)
    p2, w2 = _tree_np(acc)
    assert np.array_equal(p2, whole[0]) and np.array_equal(w2, whole[1])


@pytest.mark.parametrize("scale,k", [(17, 8), (17, 4), (17, 2), (12, 8)])
def test_split_merge_parts_tile_whole_tree(gpu_ctx, scale, k):
    """sheep_merge_trees_part: each part's node range of parents (plus every pst) is the
    merged tree's, the k ranges tile [0, n) and together they are the whole-graph tree
    (RMAT-12: too few levels to split, every part runs the whole merge)."""
    import sheep_amd
    import torch
    d = sheep_amd.rmat(scale, 16, 9)
    s = sheep_amd.degree_sequence(d)
    whole = sheep_amd.build_tree(d, s)
    R = d.shape[0]
    stacked = torch.stack([sheep_amd.build_tree(d[i * R // k:(i + 1) * R // k], s) for i in range(k)])
    asm, covered = None, 0
    for p in range(k):
        part, lo, hi = sheep_amd.merge_trees_part(stacked, p, k)
        assert torch.equal(part[:, 1], whole[:, 1])
        assert torch.equal(part[lo:hi, 0], whole[lo:hi, 0])
        if asm is None:
            asm = part.clone()
        asm[lo:hi, 0] = part[lo:hi, 0]
        covered += hi - lo
        assert lo <= hi
    assert covered == whole.shape[0] or covered == k * whole.shape[0]   # a tiling, or every part whole
    assert torch.equal(asm, whole)
    with pytest.raises(ValueError):
        sheep_amd.merge_trees_part(stacked, 0, 3)   # parts must be a power of two


def test_merge_many_rejects_bad_parent(gpu_ctx):
    import sheep_amd
    import torch
    a = sheep_amd.tree_to_device(np.array([1, 2, 0xFFFFFFFF], np.uint32), np.zeros(3, np.uint32))
    b = sheep_amd.tree_to_device(np.array([2, 0, 0xFFFFFFFF], np.uint32), np.zeros(3, np.uint32))   # 1 -> 0: not later
    with pytest.raises(ValueError, match="not a later node"):   # SHEEP_ERR_ARG
        sheep_amd.merge_trees_many(torch.stack([a, b]))


def test_unsequenced_and_out_of_range(gpu_ctx):
    """A neighbour missing from the sequence counts as POSTORDER forever (jtree.cpp:84-90);
    a neighbour beyond max(seq) makes index.at() throw (jtree.cpp:75)."""
    import sheep_amd
    rec = golden_records("edge")
    seq = golden_seq("edge")
    drop = seq[seq != 3]                    # vertex 3 unsequenced, max(seq) unchanged
    s = sheep_amd.sequence_from_host(drop)
    p, w = _tree_np(sheep_amd.build_tree(_dev_records(rec), s))
    op, ow = oracle.build_tree(rec["tail"], rec["head"], drop)
    assert np.array_equal(p, op) and np.array_equal(w, ow)
    short = seq[seq < 10]                   # max(seq) = 9 while record (10, 0) exists
    s2 = sheep_amd.sequence_from_host(short)
    with pytest.raises(IndexError):
        sheep_amd.build_tree(_dev_records(rec), s2)
    swapped = rec.copy()                    # the same record as (0, 10): head beyond max(seq)
    swapped["tail"], swapped["head"] = rec["head"], rec["tail"]
    with pytest.raises(IndexError):
        sheep_amd.build_tree(_dev_records(swapped), s2)


@pytest.mark.parametrize("stretch", [40000, 150000])
def test_wide_vertex_ids(gpu_ctx, stretch):
    """Vertex ids up to 1.6e8 (above 2^27: more than 4087 LDS buckets of 2^15 slots, the
    staged heads histogram and 4K-record relabel sub-tiles) and up to 6e8 (above 2^28:
    beyond the bucket layout, the unbucketed kernels k_degree + scattered head atomics and
    the one-pass k_relabel).  Same results as the oracle."""
    import sheep_amd
    h = sheep_amd.rmat_host(12, 16, 12)
    t_ = h[:, 0].astype(np.uint64) * stretch + 7
    h_ = h[:, 1].astype(np.uint64) * stretch + 7
    assert h_.max() >= (1 << 27)
    t_, h_ = t_.astype(np.uint32), h_.astype(np.uint32)
    w = np.ones(len(t_), np.float32)
    d = sheep_amd.records_to_device(t_, h_, w)
    s = sheep_amd.degree_sequence(d)
    seq = oracle.sequence(t_, h_)
    assert np.array_equal(s.numpy(), seq)
    p, pw = _tree_np(sheep_amd.build_tree(d, s))
    op, ow = oracle.build_tree(t_, h_, seq)
    assert np.array_equal(p, op) and np.array_equal(pw, ow)


def test_empty_and_tiny(gpu_ctx):
    import sheep_amd
    import torch
    # one record, a self-loop: one node, no tree edge, pst 0
    rec = np.zeros(1, dtype=[("tail", "<u4"), ("head", "<u4"), ("weight", "<f4")])
    rec["tail"] = rec["head"] = 4
    d = _dev_records(rec)
    s = sheep_amd.degree_sequence(d)
    assert list(s.numpy()) == [4]
    p, w = _tree_np(sheep_amd.build_tree(d, s))
    assert list(p) == [0xFFFFFFFF] and list(w) == [0]
    res = sheep_amd.partition(s, sheep_amd.tree_to_device(p, w), 2)
    assert res.created == 1


def test_tree_above_2e27_nodes(gpu_ctx):
    """A path of 1.4e8 vertices: 1.4e8 tree nodes, so the pst grouping's padded lo range
    needs more than 4087 LDS buckets (staged scatter with 8K-edge sub-tiles); vertex ids
    above 2^27 also take the staged heads histogram and 4K-record relabel sub-tiles.  Tree
    vs the oracle."""
    import sheep_amd
    N = 140_000_000
    t_ = np.arange(N, dtype=np.uint32)
    h_ = t_ + 1
    d = sheep_amd.records_to_device(t_, h_)
    s = sheep_amd.degree_sequence(d)
    seq = oracle.sequence(t_, h_)
    assert np.array_equal(s.numpy(), seq)
    p, w = _tree_np(sheep_amd.build_tree(d, s))
    del d
    op, ow = oracle.build_tree(t_, h_, seq)
    assert np.array_equal(p, op) and np.array_equal(w, ow)


@pytest.mark.parametrize("what", [0, 1, 2, 4, 6])
def test_evaluate_masks_and_shards(gpu_ctx, what):
    """sheep_evaluate computes only the metrics its mask asks for (the others come back 0),
    and the sharded evaluator (shards ORed into one state, or two states combined as
    another device's would be) gives the same counts as one call over all records."""
    import sheep_amd
    d = sheep_amd.rmat(16, 16, 9)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    s = sheep_amd.degree_sequence(d)
    tree = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, tree, 100)
    full = oracle.evaluate(h[:, 0], h[:, 1], s.numpy(), res.numpy())
    ev = sheep_amd.evaluate(d, s, res.parts, what=what)
    m = what or 7
    keep = {"edges", "nodes"}
    if m & 1:
        keep |= {"edges_cut", "vcom_vol", "max_vertex_bal", "ecv_hash", "max_hash_bal"}
    if m & 2:
        keep |= {"ecv_down", "max_down_bal"}
    if m & 4:
        keep |= {"ecv_up", "max_up_bal"}
    assert ev.__dict__ == {k: (v if k in keep else 0) for k, v in full.items()}
    R = d.shape[0]
    a = sheep_amd.ShardedEvaluator(s, res.parts, what)
    b = sheep_amd.ShardedEvaluator(s, res.parts, what, nparts=a.nparts)
    for i in range(5):
        (a if i % 2 else b).add(d[i * R // 5:(i + 1) * R // 5])
    a.combine(b.bits, b.acc)
    assert a.finish() == ev


def test_evaluate_wide_parts(gpu_ctx):
    """More than 64 parts (several bitset words per vertex), against the oracle."""
    import sheep_amd
    d = sheep_amd.rmat(15, 16, 4)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    s = sheep_amd.degree_sequence(d)
    tree = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, tree, 300)
    assert res.created > 128
    assert sheep_amd.evaluate(d, s, res.parts).__dict__ == oracle.evaluate(h[:, 0], h[:, 1], s.numpy(), res.numpy())


@pytest.mark.parametrize("use_pos", [True, False])
def test_partition_sequence_length(gpu_ctx, use_pos):
    """Partition(seq, jnodes, k) (partition.cpp:62-66): a sequence longer than the tree is
    the reference's parts.at() throw; a shorter one converts only its own entries, and
    the printed counts come from the vid-indexed vector (partition.h:135-143)."""
    import sheep_amd
    seq = golden_seq("hep")
    p, w = golden_tree("hep")
    tree = sheep_amd.tree_to_device(p, w)
    longer = sheep_amd.sequence_from_host(np.append(seq, np.uint32(seq.max() + 1)))
    with pytest.raises(IndexError):
        sheep_amd.partition(longer, tree, 4, use_pos=use_pos)
    short = seq[:-100]
    res = sheep_amd.partition(sheep_amd.sequence_from_host(short), tree, 4, use_pos=use_pos)
    oparts, oinfo = oracle.partition(p, w, short, 4)
    assert np.array_equal(res.numpy(), oparts)
    assert res.created == oinfo["created"]
    assert res.first_size == np.count_nonzero(oparts == 0) and res.second_size == np.count_nonzero(oparts == 1)


@pytest.mark.parametrize("name", GRAPHS)
def test_evaluate_from_step_edges(gpu_ctx, name):
    """sheep_evaluate_step: every count from the map's position-space edges equals the record
    evaluator's (and the golden stdout), for each metric set — the golden graphs include
    self-loops, repeated records and isolated slots (`edge`)."""
    import sheep_amd
    rec = golden_records(name)
    s = sheep_amd.sequence_from_host(golden_seq(name))
    d = _dev_records(rec)
    tree = sheep_amd.build_tree(d, s)
    assert np.array_equal(_tree_np(tree)[0], golden_tree(name)[0])
    kids = sheep_amd.KidTable(tree)
    _, blocks = golden_part_text(name)
    for k, block in zip(ks(name), blocks):
        res = sheep_amd.partition(s, tree, k, kids=kids)
        for what in (1, 2, 4, 6, 0):
            a = sheep_amd.evaluate(d, s, res.parts, what=what)
            b = sheep_amd.evaluate(d, s, res.parts, what=what, from_step=True)
            assert a == b, (k, what, a, b)
        assert res.print_text() + b.text(k) == block, f"k={k}"   # (b: every metric)


def test_evaluate_from_step_edges_needs_that_map(gpu_ctx):
    """The step edges belong to the last map over these records and this sequence: other
    records, another sequence, or a trimmed context are an argument error, not a result."""
    import sheep_amd
    rec, rec2 = golden_records("rmat12"), golden_records("rmat14")
    s, s2 = sheep_amd.sequence_from_host(golden_seq("rmat12")), sheep_amd.sequence_from_host(golden_seq("rmat14"))
    d, d2 = _dev_records(rec), _dev_records(rec2)
    tree = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, tree, 4)
    ok = sheep_amd.evaluate(d, s, res.parts, from_step=True)
    assert ok == sheep_amd.evaluate(d, s, res.parts)
    tree2 = sheep_amd.build_tree(d2, s2)   # the context's last map is now another graph's
    with pytest.raises(ValueError):
        sheep_amd.evaluate(d, s, res.parts, from_step=True)
    res2 = sheep_amd.partition(s2, tree2, 4)
    assert sheep_amd.evaluate(d2, s2, res2.parts, from_step=True) == sheep_amd.evaluate(d2, s2, res2.parts)
    # the same index with another sequence of the same length (two entries swapped)
    sw = golden_seq("rmat14").copy()
    sw[[0, 1]] = sw[[1, 0]]
    s2x = sheep_amd.Sequence(sheep_amd.sequence_from_host(sw).seq, s2.pos, s2.n, s2.pos_size)
    with pytest.raises(ValueError):
        sheep_amd.evaluate(d2, s2x, res2.parts, from_step=True)
    gpu_ctx.trim()
    with pytest.raises(ValueError):
        sheep_amd.evaluate(d2, s2, res2.parts, from_step=True)


@pytest.mark.parametrize("what", [0, 1, 2, 4])
def test_evaluate_unassigned_part(gpu_ctx, what):
    """A part of -1 (INVALID_PART) on an edge endpoint is the reference's throw in both
    evaluators (the step-edge one must not index with it); on a sequenced vertex that is no
    endpoint it is ignored by both, with the same counts."""
    import sheep_amd
    rec = golden_records("rmat12")
    seq = golden_seq("rmat12")
    d = _dev_records(rec)
    # one extra sequenced vid past every record: sequenced, never an endpoint
    extra = np.uint32(int(seq.max()) + 5)
    s = sheep_amd.sequence_from_host(np.concatenate([seq, [extra]]))
    tree = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, tree, 8)
    for victim in (int(rec["tail"][0]), int(rec["head"][0]), int(rec["head"][-1])):   # a tail, a head, another head
        parts = res.parts.clone()
        parts[victim] = -1
        with pytest.raises(IndexError):
            sheep_amd.evaluate(d, s, parts, what=what)
        with pytest.raises(IndexError):
            sheep_amd.evaluate(d, s, parts, what=what, from_step=True)
    parts = res.parts.clone()
    parts[int(extra)] = -1
    a = sheep_amd.evaluate(d, s, parts, what=what)
    assert a == sheep_amd.evaluate(d, s, parts, what=what, from_step=True)
    assert a == sheep_amd.evaluate(d, s, res.parts, what=what)


@pytest.mark.parametrize("scale,seed,k", [(16, 5, 16), (18, 7, 64)])
def test_evaluate_from_step_edges_rmat(gpu_ctx, scale, seed, k):
    """Larger RMAT graphs, with the records' self-loops and repeats added: the step-edge
    evaluator against the record evaluator and the oracle's counts."""
    import sheep_amd
    h = sheep_amd.rmat_host(scale, 16, seed)
    t_, h_ = h[:, 0].astype(np.uint32), h[:, 1].astype(np.uint32)
    extra = np.arange(0, 1 << scale, 97, dtype=np.uint32)   # self-loops on some vertices with edges
    extra = extra[np.isin(extra, np.concatenate([t_, h_]))]
    t_ = np.concatenate([t_, extra, t_[:1000]])
    h_ = np.concatenate([h_, extra, h_[:1000]])
    d = sheep_amd.records_to_device(t_, h_, np.ones(len(t_), np.float32))
    s = sheep_amd.degree_sequence(d)
    tree = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, tree, k)
    a = sheep_amd.evaluate(d, s, res.parts)
    b = sheep_amd.evaluate(d, s, res.parts, from_step=True)
    assert a == b
    o = oracle.evaluate(t_, h_, s.numpy(), res.numpy())
    assert (b.edges_cut, b.vcom_vol, b.ecv_hash, b.ecv_down, b.ecv_up) == \
        (o["edges_cut"], o["vcom_vol"], o["ecv_hash"], o["ecv_down"], o["ecv_up"])


def _star_plus_rmat(scale, seed, leaves):
    """RMAT records plus a star of `leaves` degree-1 vertices on a new centre: the centre's
    elimination-tree node has `leaves` kids (above the event kernel's 4096 staged inline)."""
    import sheep_amd
    r = sheep_amd.rmat_host(scale, 16, seed)
    t, h = r[:, 0].astype(np.uint32), r[:, 1].astype(np.uint32)
    c = np.uint32(1 << scale)
    lv = np.arange(c + 1, c + 1 + leaves, dtype=np.uint32)
    return np.concatenate([t, lv]), np.concatenate([h, np.full(leaves, c, np.uint32)])


@pytest.mark.parametrize("event_loop", [0, 1, 3, 4096])
def test_partition_event_loop_variants(gpu_ctx, event_loop):
    """sheep_tuning event_loop: one k_event launch per packing event (0), the persistent
    k_event_loop handing over to per-event launches once its table outgrows 1 or 3 entries,
    and the default (one launch, relaunched only behind a node whose kids k_event_kids
    stages), each against the oracle's forwardPartition (partition.cpp:86-157)."""
    import sheep_amd
    t, h = _star_plus_rmat(16, 9, 6000)
    w = np.ones(len(t), np.float32)
    d = sheep_amd.records_to_device(t, h, w)
    seq = oracle.sequence(t, h)
    s = sheep_amd.degree_sequence(d)
    assert np.array_equal(s.numpy(), seq)
    tree = sheep_amd.build_tree(d, s)
    p, pw = _tree_np(tree)
    gpu_ctx.set_tuning(event_loop=event_loop)
    try:
        for k in (4, 64, 512):
            res = sheep_amd.partition(s, tree, k)
            oparts, oinfo = oracle.partition(p, pw, seq, k)
            assert np.array_equal(res.numpy(), oparts), f"k={k}"
            assert res.created == oinfo["created"] and res.packing_nodes == oinfo["packing_nodes"], f"k={k}"
            if event_loop == 0:   # one k_event per event and one for the empty search
                assert res.event_launches >= res.packing_nodes + 1
            elif event_loop == 4096:   # k_event_loop, k_event_kids for the star's centre, k_event_loop again
                assert res.event_launches <= 3, res.event_launches
    finally:
        gpu_ctx.set_tuning()


def test_context_on_another_device(gpu_ctx):
    """Calls run on the context's device whatever device the calling thread has current."""
    import torch
    import sheep_amd
    if torch.cuda.device_count() < 2:
        pytest.skip("one HIP device")
    ctx1 = sheep_amd.Context(1)
    torch.cuda.set_device(0)
    with torch.cuda.device(1):
        d = sheep_amd.rmat(12, 16, 12, ctx=ctx1)
        deg = torch.zeros(1 << 12, dtype=torch.int32, device="cuda:1")
    torch.cuda.set_device(0)
    _, vs = sheep_amd.degree_count(d, deg=deg, ctx=ctx1)
    s = sheep_amd.sequence_from_degrees(deg, vs, ctx=ctx1)
    h = sheep_amd.to_numpy_u32(d).reshape(-1, 3)
    assert np.array_equal(s.numpy(), oracle.sequence(h[:, 0], h[:, 1]))


@pytest.mark.parametrize("ranks", [2, 3, 4])
def test_group_rehearsal_matches_single_gpu(gpu_ctx, ranks):
    """sheep_group_* (graph2tree -i -r without MPI) with `ranks` edge shards rehearsed on
    device 0 (device copies stand in for RCCL): the all-reduced sequence, the K-way and
    the binomial reduce, the parts broadcast and the sharded evaluator all equal the
    single-GPU results."""
    import torch
    import sheep_amd
    d = sheep_amd.rmat(16, 16, 16)
    s = sheep_amd.degree_sequence(d)
    whole = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, whole, 32)
    ev = sheep_amd.evaluate(d, s, res.parts)
    g = sheep_amd.Group([0] * ranks)
    assert not g.rccl
    R = d.shape[0]
    shards = [d[r * R // ranks:(r + 1) * R // ranks].contiguous() for r in range(ranks)]
    seqs = g.sequence(shards, 1 << 16)
    for q in seqs:
        assert q.n == s.n and torch.equal(q.seq[: q.n], s.seq[: s.n])
    for mode in ("kway", "binomial"):
        assert torch.equal(g.build_tree(shards, seqs, mode)[0], whole), mode
    partial = g.build_tree(shards, seqs, "none")
    assert torch.equal(sheep_amd.merge_trees_many(torch.stack(partial)), whole)
    parts = g.broadcast_parts([res.parts.clone()] + [torch.full_like(res.parts, 7) for _ in range(ranks - 1)],
                              s.pos_size)
    for p in parts:
        assert torch.equal(p, res.parts)
    assert g.evaluate(shards, seqs, parts) == ev
    g.close()


def test_rccl_world_of_one(gpu_ctx):
    """The RCCL transport on the one-GPU box: a joined world of ONE with link=rccl forced
    opens a one-rank communicator (ncclGetUniqueId + ncclCommInitRank), and then the
    degree ncclAllReduce (mpiSequence, sequence.h:72,78), the parts ncclBroadcast
    (mpi_sync, partition.cpp:69-79) and a grouped self ncclSend/ncclRecv of a tree (the hop
    of mpi_merge's MPI_Reduce, jnode.cpp:238-241) all run through RCCL.  Each result equals
    the host-link world's and the single-GPU path's."""
    import torch
    import sheep_amd
    d = sheep_amd.rmat(16, 16, 16)
    s = sheep_amd.degree_sequence(d)
    whole = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, whole, 32)
    ev = sheep_amd.evaluate(d, s, res.parts)
    out = {}
    for link in ("rccl", "host"):
        g = sheep_amd.Group.join(0, 0, 1, link=link)
        assert g.rccl == (link == "rccl"), link
        seqs = g.sequence([d], 1 << 16)
        assert seqs[0].n == s.n and torch.equal(seqs[0].seq[: s.n], s.seq[: s.n]), link
        tree = g.build_tree([d], seqs, "kway")[0]
        assert torch.equal(tree, whole), link
        got = torch.full_like(whole, -1)
        g.transfer(0, 0, whole, got)
        assert torch.equal(got, whole), link
        parts = g.broadcast_parts([res.parts.clone()], s.pos_size)
        assert torch.equal(parts[0], res.parts), link
        out[link] = g.evaluate([d], seqs, parts)
        g.close()
    assert out["rccl"] == out["host"] == ev


def test_rccl_world_of_one_abort(gpu_ctx, capfd):
    """The failure path's RCCL side on one GPU: a non-blocking one-rank communicator runs a
    collective through the polled wait, then sheep_group_abort ends the world
    (ncclCommAbort): one stderr line names the rank, bus id and cause, every later
    collective raises at once, and destroying the world does not hang."""
    import time
    import sheep_amd
    d = sheep_amd.rmat(12, 16, 12)
    g = sheep_amd.Group.join(0, 0, 1, link="rccl")
    assert g.rccl and not g.failed
    seqs = g.sequence([d], 1 << 12)
    assert seqs[0].n == sheep_amd.degree_sequence(d).n
    g.abort("test abort")
    assert g.failed
    t0 = time.time()
    with pytest.raises(RuntimeError, match="failed before"):
        g.sequence([d], 1 << 12)
    with pytest.raises(RuntimeError, match="failed before"):
        g.barrier()
    assert time.time() - t0 < 5
    g.close()
    err = capfd.readouterr().err
    assert "sheep: rank 0 of 1 (bus " in err and "abort of 0 bytes failed: test abort" in err, err


def test_group_join_rank_stalls(gpu_ctx, tmp_path):
    """A joined world of 3 processes on one GPU (host links) whose rank 2 joins and then
    never takes part: ranks 0 and 1 get an error from their first collective within
    SHEEP_JOIN_TIMEOUT instead of hanging, print the one-line report (rank, bus id,
    collective, bytes), and then every call is refused at once."""
    import socket
    import subprocess
    import sys
    timeout = 4
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "group_worker.py")
    env = dict(os.environ, SHEEP_JOIN_TIMEOUT=str(timeout))
    procs = [subprocess.Popen([sys.executable, worker, str(r), "3", str(port), str(tmp_path), "stall"],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env) for r in range(3)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    for r in (0, 1):
        out = outs[r]
        waited = float(out.split("failed after ")[1].split(" s")[0])
        assert waited <= timeout + 2, out
        assert f"sheep: rank {r} of 3 (bus " in out and "failed: mesh:" in out, out
        assert "refused after" in out and "failed before" in out, out
    assert "timed out waiting for rank 2" in outs[0], outs[0]


@pytest.mark.parametrize("ranks", [2, 3])
def test_group_join_processes_match_single_gpu(gpu_ctx, tmp_path, ranks):
    """sheep_group_join: `ranks` PROCESSES, one rank each (the mpiexec / torch.distributed
    form), sharing device 0, so the host link over TCP carries the exchanges.  Every rank
    runs tests/group_worker.py; rank 0's sequence, K-way and binomial trees, broadcast parts
    and evaluator equal the single-GPU results."""
    import socket
    import subprocess
    import sys
    import torch
    import sheep_amd
    d = sheep_amd.rmat(16, 16, 16)
    s = sheep_amd.degree_sequence(d)
    whole = sheep_amd.build_tree(d, s)
    res = sheep_amd.partition(s, whole, 32)
    ev = sheep_amd.evaluate(d, s, res.parts)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "group_worker.py")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(ranks), str(port), str(tmp_path)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(ranks)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    got = np.load(tmp_path / "rank0.npz")
    assert np.array_equal(got["seq"], s.numpy())
    p, w = sheep_amd.tree_to_numpy(whole)
    for mode in ("kway", "binomial"):
        assert np.array_equal(got[f"parent_{mode}"], p) and np.array_equal(got[f"pst_{mode}"], w), mode
    for r in range(ranks):
        assert np.array_equal(np.load(tmp_path / f"rank{r}.npz")["parts"], res.numpy()), r
    assert got["ecv"].tolist() == [ev.ecv_down, ev.max_down_bal, ev.edges_cut, ev.ecv_hash, ev.ecv_up]
    assert "link=host" in outs[0]


def _skip_comment_lines(text: bytes) -> bytes:
    """The graph loader's SNAP header handling (LLAMA's, un-vendored: parity unpinned):
    lines whose first token starts with '#' or '%' are dropped before reading."""
    keep = [ln for ln in text.split(b"\n") if not (ln.split() and ln.split()[0][:1] in (b"#", b"%"))]
    return b"\n".join(keep)


def _snap_cases():
    import json
    from conftest import GOLDEN
    return json.load(open(os.path.join(GOLDEN, "snap_cases.json")))


@pytest.mark.parametrize("case", range(len(_snap_cases())))
def test_parse_net_vs_reference_snapreader(gpu_ctx, case):
    """sheep_parse_net against the reference's own SNAPReader (readerwriter.h:78-90,
    compiled from /root/reference: tests/golden/make_snap_golden.py): signs, wrap-around,
    leading zeros, overflow, a number with trailing characters, '#' as a bad token."""
    import sheep_amd
    c = _snap_cases()[case]
    text = c["text"].encode()
    want = np.array(c["pairs"], dtype=np.uint64).reshape(-1, 2)
    got = sheep_amd.to_numpy_u32(sheep_amd.parse_net(text, False)).reshape(-1, 3)
    assert np.array_equal(got[:, :2].astype(np.uint64), want)
    assert np.all(got[:, 2].view(np.float32) == 1.0)


@pytest.mark.parametrize("case", range(len(_snap_cases())))
def test_parse_net_skip_comments(gpu_ctx, case):
    """skip_comments = the same reading after the comment lines are dropped."""
    import sheep_amd
    c = _snap_cases()[case]
    text = c["text"].encode()
    stripped = sheep_amd.to_numpy_u32(sheep_amd.parse_net(_skip_comment_lines(text), False)).reshape(-1, 3)
    got = sheep_amd.to_numpy_u32(sheep_amd.parse_net(text, True)).reshape(-1, 3)
    assert np.array_equal(got, stripped)


@pytest.mark.parametrize("text", [b"# header\n% more\n1 2\n3 4\n", b"1 2\n# mid comment 7 8\n3 4\n"])
def test_parse_net_comment_lines(gpu_ctx, text):
    import sheep_amd
    got = sheep_amd.to_numpy_u32(sheep_amd.parse_net(text, True)).reshape(-1, 3)
    assert got[:, :2].tolist() == [[1, 2], [3, 4]]
    raw = sheep_amd.to_numpy_u32(sheep_amd.parse_net(text, False)).reshape(-1, 3)
    assert raw.shape[0] == (0 if text.startswith(b"#") else 1)


def test_parse_net_large_vs_dat(gpu_ctx):
    """RMAT-16 written as SNAP text parses back to the same records."""
    import sheep_amd
    h = sheep_amd.rmat_host(16, 16, 3)
    text = "".join(f"{t} {u}\n" for t, u in h[:, :2]).encode()
    got = sheep_amd.to_numpy_u32(sheep_amd.parse_net(text)).reshape(-1, 3)
    assert np.array_equal(got[:, :2], h[:, :2])


def test_shard_maps_on_concurrent_contexts(gpu_ctx):
    """bench.py --streams: the shards' degree counts and maps on two contexts of one device,
    each on a stream of its own driven by a host thread of its own, at the same time: the
    shard trees and their K-way merge equal the one-context results (and the whole graph's
    tree)."""
    import threading
    import torch
    import sheep_amd
    d = sheep_amd.rmat(17, 16, 17)
    R, K = d.shape[0], 4
    subs = [d[i * R // K:(i + 1) * R // K] for i in range(K)]
    s = sheep_amd.degree_sequence(d)
    want = [sheep_amd.build_tree(x, s) for x in subs]
    whole = sheep_amd.build_tree(d, s)
    ctxs = [sheep_amd.Context(0, stream=torch.cuda.Stream(0)) for _ in range(2)]
    torch.cuda.synchronize()
    degs = [torch.zeros(1 << 17, dtype=torch.int32, device="cuda") for _ in range(2)]
    out = torch.empty((K, s.n, 2), dtype=torch.int32, device="cuda")
    err = []

    def run(j):
        try:
            for i in range(j, K, 2):
                sheep_amd.degree_count(subs[i], mode="llama", deg=degs[j], ctx=ctxs[j])
                sheep_amd.build_tree(subs[i], s, ctx=ctxs[j], out=out[i])
            ctxs[j].sync()
        except Exception as e:
            err.append(e)
    th = [threading.Thread(target=run, args=(j,)) for j in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not err, err
    torch.cuda.synchronize()
    for i in range(K):
        assert torch.equal(out[i], want[i]), i
    assert torch.equal(sheep_amd.merge_trees_many(out), whole)
    deg_all = degs[0] + degs[1]
    assert torch.equal(sheep_amd.sequence_from_degrees(deg_all, s.pos_size).seq[: s.n], s.seq[: s.n])
    for c in ctxs:
        c.close()


def test_steps_on_concurrent_contexts(gpu_ctx):
    """bench.py --concurrent N: whole steps (degree count, sequence, tree, kids, partition) on
    three contexts of one device at once, each context's steps in a host thread of its own:
    every step's sequence, tree and parts equal the one-context results."""
    import threading
    import torch
    import sheep_amd
    d = sheep_amd.rmat(18, 16, 18)
    k = 16
    s0 = sheep_amd.degree_sequence(d)
    t0 = sheep_amd.build_tree(d, s0)
    kids = sheep_amd.KidTable(t0)
    want = sheep_amd.partition(s0, t0, k, kids=kids)
    kids.close()
    N = 3
    streams = [torch.cuda.Stream(0) for _ in range(N)]
    ctxs = [sheep_amd.Context(0, stream=st) for st in streams]
    degs = [torch.zeros(1 << 18, dtype=torch.int32, device="cuda") for _ in range(N)]
    torch.cuda.synchronize()
    got, err = [], []

    def worker(j):
        try:
            for _ in range(2):
                with torch.cuda.stream(streams[j]):
                    degs[j].zero_()
                ms = sheep_amd.degree_count(d, mode="llama", deg=degs[j], ctx=ctxs[j])[1]
                s = sheep_amd.sequence_from_degrees(degs[j], ms, ctx=ctxs[j])
                tree = sheep_amd.build_tree(d, s, ctx=ctxs[j])
                kt = sheep_amd.KidTable(tree, ctxs[j])
                got.append((s, tree, sheep_amd.partition(s, tree, k, kids=kt, ctx=ctxs[j])))
                kt.close()
        except Exception as e:
            err.append(e)
    th = [threading.Thread(target=worker, args=(j,)) for j in range(N)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not err, err
    assert len(got) == 2 * N
    for s, tree, res in got:
        assert torch.equal(s.seq[: s0.n], s0.seq[: s0.n])
        assert torch.equal(tree, t0)
        assert torch.equal(res.parts, want.parts)
        assert res.created == want.created
    for c in ctxs:
        c.close()
