"""Every algorithm variant of sheep_tuning (include/sheep_hip.h) on small graphs, each one
forced onto the branch it exists for, against the oracle (advisor round 4: the dense-block
cuts, the early cut and their fallbacks only switch on at scale with the default knobs).

The variants must not change a single parent: etree(G) = etree(MSF(G)) makes the cuts
exact, and the finishes are the same divide and conquer (or Liu's sweep) per block.  One
worker process runs every configuration of a graph (tests/tuning_worker.py) with
SHEEP_DEBUG=etree, and each configuration's debug lines show that its branch ran."""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

HERE = os.path.dirname(os.path.abspath(__file__))


def rmat_graph(scale, ef, seed):
    import sheep_amd
    r = sheep_amd.rmat_host(scale, ef, seed)
    return r[:, 0].astype(np.uint32), r[:, 1].astype(np.uint32)


def pairs_graph():
    """2^17 vertices of equal degree 64 (so positions are vid order): the top 2^16
    positions hold 20,000 pairs (64 parallel records each: 19.5 group edges per vertex,
    above the top block's density rule) and 25,536 vertices whose only edges go below the
    block (singletons there).  Round 0 leaves 45,536 components: the Borůvka rounds keep
    their minima in HBM (> 2048 components beside 2^16 labels) and the hooks their
    component ids in HBM (> 2^15)."""
    half = 1 << 16
    t, h = [], []
    for i in range(20000):                       # pairs inside the top block
        t.append(half + 2 * i + 1), h.append(half + 2 * i)
    for j in range(25536):                       # top singletons, each tied to one bottom vertex
        t.append(half + 40000 + j), h.append(j)
    for i in range(20000):                       # the rest of the bottom half in pairs
        t.append(25536 + 2 * i + 1), h.append(25536 + 2 * i)
    t = np.repeat(np.array(t, np.uint32), 64)
    h = np.repeat(np.array(h, np.uint32), 64)
    return t, h


def with_sequence_path(t, h):
    """The graph plus an edge between every two vertices adjacent in its degree sequence:
    every degree grows by 2 (the ends' by 1), so the order barely moves and every vertex
    but the first has a neighbour right below it."""
    import oracle
    seq = oracle.sequence(t, h)
    a, b = seq[:-1], seq[1:]
    return np.concatenate([t, np.maximum(a, b)]), np.concatenate([h, np.minimum(a, b)])


def cliques_graph(scale, size=34):
    """Disjoint cliques of `size` vertices over [0, 2^scale): every degree is size - 1, so
    positions are vid order; 16.5 edges per vertex in every block of positions (dense enough
    for the top-block cut), and no block is one tree."""
    g = np.arange(0, (1 << scale) - size + 1, size, dtype=np.uint32)
    t, h = [], []
    for a in range(size):
        for b in range(a + 1, size):
            t.append(g + b), h.append(g + a)
    return np.concatenate(t), np.concatenate(h)


# (graph, configurations): each configuration's "expect" lists regexes its debug block
# must match (the branch it forces)
TOP = r"etree top blocks after s (\d+): (\d+) block"
CASES = {
    "rmat18": (lambda: rmat_graph(18, 16, 18), [
        {"tune": {}, "merge": True, "expect": []},
        {"tune": {"top_bits": 14, "top_blocks": 9}, "expect": [r"etree top blocks after s 14: \d block"]},
        {"tune": {"top_bits": 10, "fin_map_bits": 8, "top_blocks": 4}, "expect": [r"etree top blocks after s 10:"]},
        {"tune": {"top_bits": 14, "big_bits": 17, "big_dense": 1}, "expect": [r"etree big cut after s 17:"]},
        {"tune": {"top_bits": 14, "big_bits": 17, "big_dense": 1, "big_hot16": 1},
         "expect": [r"etree big cut after s 17:"]},
        {"tune": {"top_bits": 14, "big_bits": 17, "big_dense": 1, "big_hot_bits": 10},
         "expect": [r"etree big cut after s 17:"]},
        {"tune": {"top_bits": 0}, "expect": []},
        {"tune": {"fin_dc": 0, "fin_map_bits": 8, "fin_merge_bits": 8}, "merge": True,
         "expect": [r"etree finish B 8 "]},
        {"tune": {"fin_dc": 0, "fin_map_bits": 10, "fin_merge_bits": 11}, "merge": True,
         "expect": [r"etree finish B 10 "]},
        {"tune": {"fin_map_bits": 9, "fin_merge_bits": 13}, "merge": True, "expect": [r"etree finish B 9 "]},
        {"tune": {"fin_map_bits": 11, "fin_merge_bits": 8}, "merge": True, "expect": [r"etree finish B 11 "]},
        {"tune": {"relabel_planes": 0}, "expect": []},
        {"tune": {"relabel_per": 12}, "expect": []},
        {"tune": {"relabel_per": 15}, "expect": []},
        {"tune": {"cross_win_levels": 0}, "merge": True, "expect": []},
        {"tune": {"cross_win_levels": 8}, "merge": True, "expect": []},
        {"tune": {"hook_batch": 1}, "merge": True, "expect": []},
        {"tune": {"hook_batch": 2}, "merge": True, "expect": []},
        {"tune": {"hook_up": 1}, "merge": True, "expect": []},
        {"tune": {"hook_up": 2, "hook_batch": 2}, "merge": True, "expect": []},
        {"tune": {"merge_cut_bits": 16}, "merge": True, "expect": [r"etree big cut after s 16:"]},
    ]),
    # four times denser: the blocks right below the top one pass the density rule too
    "rmat18ef64": (lambda: rmat_graph(18, 64, 18), [
        {"tune": {"top_bits": 14, "top_blocks": 9}, "merge": True,
         "expect": [r"etree top blocks after s 14: [2-9] block"]},
        {"tune": {"top_bits": 12, "top_blocks": 9, "fin_map_bits": 10},
         "expect": [r"etree top blocks after s 12: [2-9] block"]},
        {"tune": {"top_bits": 14, "big_bits": 17, "big_dense": 1}, "expect": [r"etree big cut after s 17: .*-> kept"]},
    ]),
    # the same with a path through the sequence: every vertex but the lowest then has a
    # lower neighbour, so the early cut's round 0 leaves one tree and the cut is made (small
    # RMAT graphs alone leave thousands of trees: the cut is abandoned, above)
    "rmat18ef64path": (lambda: with_sequence_path(*rmat_graph(18, 64, 18)), [
        {"tune": {"top_bits": 14, "big_bits": 17, "big_dense": 1}, "merge": True,
         "expect": [r"etree top blocks after s 14:", r"etree big cut after s 17: .*-> cut"]},
    ]),
    "pairs": (pairs_graph, [
        {"tune": {"top_bits": 16, "top_blocks": 1}, "merge": True,
         "expect": [r"etree top blocks after s 16: 1 block",
                    r"etree top round 0 block 0: components 45536 done 0 \(minima hbm\)"]},
    ]),
    # the early cut over the top half: round 0 leaves ~3,900 separate cliques there, so the
    # cut is abandoned and the levels run as without it
    "cliques18": (lambda: cliques_graph(18), [
        {"tune": {"top_bits": 14, "big_bits": 17, "big_dense": 1}, "merge": True,
         "expect": [r"etree top blocks after s 14:", r"etree big cut after s 17: .*-> kept"]},
    ]),
}


@pytest.mark.gpu
@pytest.mark.parametrize("graph", sorted(CASES))
def test_tuning_variants_match_oracle(gpu_ctx, tmp_path, graph):
    make, configs = CASES[graph]
    t, h = make()
    np.savez(tmp_path / "g.npz", tail=t, head=h)
    json.dump(configs, open(tmp_path / "c.json", "w"))
    env = dict(os.environ, SHEEP_DEBUG="etree")
    p = subprocess.run([sys.executable, os.path.join(HERE, "tuning_worker.py"), str(tmp_path / "g.npz"),
                        str(tmp_path / "c.json")], capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    results = json.loads(p.stdout.strip().splitlines()[-1])
    blocks = re.split(r"^=== config \d+ .*$", p.stderr, flags=re.M)[1:]
    assert len(blocks) == len(configs) == len(results)
    bad = []
    for cfg, res, dbg in zip(configs, results, blocks):
        if not res["tree"] or (cfg.get("merge") and not (res["halves"] and res["merge"])):
            bad.append(("parity", cfg, res))
        for pat in cfg["expect"]:
            if not re.search(pat, dbg, re.M):
                bad.append(("branch not taken", cfg, pat, dbg[-1500:]))
    assert not bad, bad


def test_tuning_cases_are_well_formed():
    """CPU: every configuration names real fields with in-range values (the GPU test's
    sheep_ctx_set_tuning would reject them at run time)."""
    import sheep_amd
    for _, configs in CASES.values():
        for cfg in configs:
            sheep_amd.Tuning.of(**cfg["tune"])
    t, h = pairs_graph()
    deg = np.bincount(np.concatenate([t, h]), minlength=1 << 17)
    assert np.all(deg == 64)
