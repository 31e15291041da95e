"""CPU model of the per-block D&C finish (sheep_amd/csrc/etree.hip k_fin_dc): the level
rules it runs inside one workgroup — hook the light edges, tops and right-half minima,
parent(top(r)) = m_r, the next list = entries that stay plus the first-seen contractions
(m_r, b) — restated in Python over one block of 2^B positions and checked against Liu's
sequential elimination tree (the reference's JTree sweep, jtree.cpp:66-110) on random
multigraphs, with the list shuffled between levels (the kernel's list order is arbitrary).
The GPU kernel itself is pinned by the parity tests (tests/test_gpu_parity.py)."""
import random


def liu(n, edges):
    parent, anc = [-1] * n, list(range(n))

    def find(x):
        while anc[x] != x:
            anc[x] = anc[anc[x]]
            x = anc[x]
        return x

    lower = [[] for _ in range(n)]
    for lo, hi in edges:
        lower[hi].append(lo)
    for v in range(n):
        for a in lower[v]:
            r = find(a)
            if r != v:
                parent[r] = v
                anc[r] = v
    return parent


def one_tree_msf(n, edges):
    """Round 0 of Borůvka as k_fin_dc runs it on a long list: every vertex's lowest lower
    neighbour; when at most one root has an edge the picks {(minlo(x), x)} are the minimum
    spanning forest under (hi, lo) (else None: the block keeps its list)."""
    minlo, up = [None] * n, [False] * n
    for lo, hi in edges:
        minlo[hi] = lo if minlo[hi] is None else min(minlo[hi], lo)
        up[lo] = True
    if sum(1 for x in range(n) if minlo[x] is None and up[x]) > 1:
        return None
    return [(minlo[x], x) for x in range(n) if minlo[x] is not None]


def block_dc(n, edges, B, rng, msf=False):
    parent = [-1] * n
    cur = list(edges)
    if msf and one_tree_msf(n, cur) is not None:
        cur = one_tree_msf(n, cur)
    for s in range(B - 1, -1, -1):
        rng.shuffle(cur)
        uf, top, mt, claim = list(range(n)), list(range(n)), [None] * n, [None] * n

        def find(x):
            while uf[x] != x:
                x = uf[x]
            return x

        for lo, hi in cur:   # (1) light edges: both ends in the left half
            if ((lo ^ hi) >> s) == 0 and not (hi >> s) & 1:
                a, b = find(lo), find(hi)
                if a != b:
                    uf[max(a, b)] = min(a, b)
        for lo, hi in cur:   # (2) tops and right-half minima
            d = (lo ^ hi) >> s
            if d == 0 and (hi >> s) & 1:
                continue
            r = find(lo)
            if d == 0:
                top[r] = max(top[r], hi)
            else:
                mt[r] = hi if mt[r] is None else min(mt[r], hi)
        for x in range(n):   # (3) adoption
            if mt[x] is not None:
                parent[top[x]] = mt[x]
        nxt = []
        for lo, hi in cur:   # (3) the next list
            if ((lo ^ hi) >> s) == 0:
                nxt.append((lo, hi))
                continue
            m = mt[find(lo)]
            if hi == m or claim[hi] == m:
                continue
            if claim[hi] is None:
                claim[hi] = m
            nxt.append((m, hi))
        cur = nxt
    return parent


def test_block_dc_equals_liu_on_random_multigraphs():
    rng = random.Random(2026)
    for _ in range(300):
        B = rng.randint(1, 7)
        n = 1 << B
        pairs = set()
        for _ in range(rng.randint(0, 4 * n)):
            a, b = rng.randrange(n), rng.randrange(n)
            if a != b:
                pairs.add((min(a, b), max(a, b)))
        edges = sorted(pairs)
        edges += rng.sample(edges, min(len(edges), 5))   # repeated edges, as contractions produce
        assert block_dc(n, edges, B, rng) == liu(n, edges)
        assert block_dc(n, edges, B, rng, msf=True) == liu(n, edges)


def test_any_lower_neighbour_picks_that_form_one_tree_keep_the_etree():
    """The early cut of the top subproblem (etree.hip k_big_min0 / k_big_emit) keeps, per
    vertex, ANY lower neighbour (the first one a racing store leaves), not the lowest: under
    the weight hi the picks lie in some minimum spanning forest, so when at most one root
    has an edge they are one and the elimination tree is Liu's of the whole edge set."""
    rng = random.Random(77)
    cut = 0
    for _ in range(1500):
        n = rng.randint(2, 64)
        pairs = set()
        for _ in range(rng.randint(n, 8 * n)):
            a, b = rng.randrange(n), rng.randrange(n)
            if a != b:
                pairs.add((min(a, b), max(a, b)))
        edges = sorted(pairs)
        lower = [[] for _ in range(n)]
        up = [False] * n
        for lo, hi in edges:
            lower[hi].append(lo)
            up[lo] = True
        picks = [(rng.choice(lower[x]), x) for x in range(n) if lower[x]]
        if sum(1 for x in range(n) if not lower[x] and up[x]) > 1:
            continue
        cut += 1
        assert liu(n, picks) == liu(n, edges)
    assert cut > 100   # (one-tree blocks: about one case in eight here)
