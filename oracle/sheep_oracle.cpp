// =====================================================================================
//  sheep_oracle.cpp — CPU restatement of Sheep's partitioning path.
//
//  TEST INFRASTRUCTURE ONLY.  This file is the parity CHECKER for the MI355X
//  product in sheep_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
//  `cpu_baseline` leg may load it.  The product path never links, calls or falls
//  back to anything here.
//
//  Every function restates one piece of the reference (chan150/sheep, read-only at
//  /root/reference) and cites the file:line it follows.  Pinning: the restatement is
//  checked (tests/test_oracle_golden.py) against
//    * the authors' golden log data/quality/hep.degree.raw:8-38 (TREEFAQS + ECV(down)),
//    * fixtures produced by oracle/_ref (the reference's own lib/ headers compiled
//      from /root/reference through its GraphType template plug point; see
//      oracle/ref/Makefile and DESIGN.md §Oracle).
//
//  Third-party dependency: LLAMA (goatdb/llama, un-vendored, unpinned version;
//  reference README:3-8, Makefile:14).  Its loader semantics are restated in
//  LlamaGraph below and documented as pinned / unpinned in DESIGN.md.
// =====================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include <omp.h>

namespace oracle {

static constexpr uint32_t INVALID = 0xFFFFFFFFu;   // defs.h:82, jnode.h:43
typedef int16_t part_t;                             // partition.h:43
static constexpr part_t INVALID_PART = -1;          // partition.h:44

// -------------------------------------------------------------------------------------
// LLAMA-semantics graph (graph_wrapper.h:43-163 over ll_mlcsr_ro_graph).
//   * undirected doubling: record (u,v) puts v in adj[u] and u in adj[v]
//     (LL_L_UNDIRECTED_DOUBLE, graph_wrapper.h:50-51);
//   * a self-loop is stored ONCE (out-degree +1) — pinned by the twitter log
//     arithmetic in SURVEY.md §8(c);
//   * max_nodes = 1 + max vid over the loaded records; degree-0 slots are not nodes
//     (graph_wrapper.h:61-62, 83-85, NodeItr :97-110);
//   * getEdges = max_edges / 2 (graph_wrapper.h:79-81);
//   * partial load part/num_parts (1-indexed): contiguous record range
//     [(p-1)R/k, pR/k) — LLAMA's own split is unpinned, but the final tree is
//     shard-independent (SURVEY.md §0 invariant 3).
// -------------------------------------------------------------------------------------
struct LlamaGraph {
  uint32_t max_nodes = 0;
  std::vector<uint64_t> off;   // CSR offsets, size max_nodes + 1
  std::vector<uint32_t> adj;   // neighbours in record order
  uint64_t num_nodes = 0;

  // With more than one OpenMP thread (or_set_threads) the adjacency lists are filled
  // concurrently, so their order is not record order; nothing the oracle computes from
  // a graph (degrees, the elimination tree, the evaluators) depends on that order.
  LlamaGraph(const uint32_t *tail, const uint32_t *head, uint64_t R,
             uint64_t part = 0, uint64_t num_parts = 0) {
    uint64_t beg = 0, end = R;
    if (num_parts != 0) {
      beg = (part - 1) * R / num_parts;
      end = part * R / num_parts;
    }
    uint32_t mx = 0;
#pragma omp parallel for reduction(max : mx) schedule(static)
    for (uint64_t i = beg; i < end; ++i) mx = std::max(mx, std::max(tail[i], head[i]) + 1);
    max_nodes = mx;
    off.assign((size_t)max_nodes + 1, 0);
    uint64_t *o = off.data();
#pragma omp parallel for schedule(static)
    for (uint64_t i = beg; i < end; ++i) {
      __atomic_fetch_add(&o[tail[i] + 1], 1, __ATOMIC_RELAXED);
      if (tail[i] != head[i]) __atomic_fetch_add(&o[head[i] + 1], 1, __ATOMIC_RELAXED);
    }
    for (uint32_t v = 0; v < max_nodes; ++v) off[v + 1] += off[v];
    adj.resize(off[max_nodes]);
    std::vector<uint64_t> cur(off.begin(), off.end() - 1);
    uint64_t *c = cur.data();
    uint32_t *a = adj.data();
    if (omp_get_max_threads() == 1) {
      for (uint64_t i = beg; i < end; ++i) {
        a[c[tail[i]]++] = head[i];
        if (tail[i] != head[i]) a[c[head[i]]++] = tail[i];
      }
    } else {
#pragma omp parallel for schedule(static)
      for (uint64_t i = beg; i < end; ++i) {
        a[__atomic_fetch_add(&c[tail[i]], 1, __ATOMIC_RELAXED)] = head[i];
        if (tail[i] != head[i]) a[__atomic_fetch_add(&c[head[i]], 1, __ATOMIC_RELAXED)] = tail[i];
      }
    }
    uint64_t nn = 0;
#pragma omp parallel for reduction(+ : nn) schedule(static)
    for (uint32_t v = 0; v < max_nodes; ++v) nn += deg(v) != 0;
    num_nodes = nn;
  }
  uint64_t deg(uint32_t v) const { return v < max_nodes ? off[v + 1] - off[v] : 0; }
  bool isNode(uint32_t v) const { return v < max_nodes && deg(v) != 0; }   // :83-85
  uint64_t getEdges() const { return adj.size() / 2; }                      // :79-81
  uint64_t getNodes() const { return num_nodes; }                           // :75-77
};

// -------------------------------------------------------------------------------------
// Sequences (sequence.h)
// -------------------------------------------------------------------------------------
// degreeSequence (sequence.h:52-63) == mpiSequence (sequence.h:65-93) on the union of
// the shards: node slots in ascending vid, sorted by (degree, vid).  A total order,
// so any correct sort gives the same vector.
static std::vector<uint32_t> sort_by_degree(const std::vector<uint64_t> &degree) {
  std::vector<uint32_t> seq;
  uint64_t maxdeg = 0;
  for (uint32_t x = 0; x < degree.size(); ++x)
    if (degree[x] != 0) {
      seq.push_back(x);
      maxdeg = std::max(maxdeg, degree[x]);
    }
  if (maxdeg > 4 * (uint64_t)degree.size() + 1024) {
    std::sort(seq.begin(), seq.end(), [&degree](uint32_t a, uint32_t b) {
      return degree[a] != degree[b] ? degree[a] < degree[b] : a < b;
    });
    return seq;
  }
  // The same total order by a counting sort over the degree (vids stay ascending within
  // one degree): linear time for the BASELINE-size sequences (C3-C5).
  std::vector<uint64_t> at(maxdeg + 2, 0);
  for (uint32_t x : seq) ++at[degree[x] + 1];
  for (uint64_t d = 0; d <= maxdeg; ++d) at[d + 1] += at[d];
  std::vector<uint32_t> out(seq.size());
  for (uint32_t x : seq) out[at[degree[x]]++] = x;
  return out;
}

std::vector<uint32_t> degreeSequence(const LlamaGraph &g) {
  std::vector<uint64_t> degree(g.max_nodes);
  for (uint32_t x = 0; x < g.max_nodes; ++x) degree[x] = g.deg(x);
  return sort_by_degree(degree);
}

// The same sequence without building the adjacency: LLAMA's getDeg(v) (graph_wrapper.h:
// 87-89) is the number of adjacency entries of v = records with tail v plus records with
// head v that are not self-loops.
std::vector<uint32_t> degreeSequenceFromRecords(const uint32_t *tail, const uint32_t *head, uint64_t R) {
  uint32_t mx = 0;
#pragma omp parallel for reduction(max : mx) schedule(static)
  for (uint64_t i = 0; i < R; ++i) mx = std::max(mx, std::max(tail[i], head[i]) + 1);
  std::vector<uint64_t> degree(mx, 0);
  uint64_t *d = degree.data();
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < R; ++i) {
    __atomic_fetch_add(&d[tail[i]], 1, __ATOMIC_RELAXED);
    if (tail[i] != head[i]) __atomic_fetch_add(&d[head[i]], 1, __ATOMIC_RELAXED);
  }
  return sort_by_degree(degree);
}

// fileSequence_template (sequence.h:95-122): degree[X]++ and degree[Y]++ per record
// read, so a self-loop counts +2; XS1Reader::read (readerwriter.h:138-146) hands the
// last record out twice (eof is only seen after a failed read), SNAPReader does not.
std::vector<uint32_t> fileSequence(const uint32_t *tail, const uint32_t *head, uint64_t R,
                                   bool xs1_last_twice) {
  std::vector<uint64_t> degree;
  auto count = [&degree](uint32_t X, uint32_t Y) {
    size_t need = (size_t)std::max(X, Y) + 1;
    if (degree.size() < need) degree.resize(need, 0);
    degree[X] += 1;
    degree[Y] += 1;
  };
  for (uint64_t i = 0; i < R; ++i) count(tail[i], head[i]);
  if (xs1_last_twice && R != 0) count(tail[R - 1], head[R - 1]);
  return sort_by_degree(degree);
}

// -------------------------------------------------------------------------------------
// Elimination tree (Liu) — JTree::insert (jtree.cpp:66-110 / parameterised form used by
// default because Options::isDefault() is never true, jtree.h:89 vs :96), adopt
// (jnode.h:158-162) on FastUnionFind (unionfind.h:46-102).
// The union-find here keeps, at each set root, the set's newest tree node (the
// "representative" the reference stores in the root's parent slot); link by size.
// The tree is unique given (edge multiset, order), so the union-find's internal
// policy does not affect the output.
// -------------------------------------------------------------------------------------
struct UnionFind {
  std::vector<uint32_t> up, rep, size;
  explicit UnionFind(size_t n) : up(n), rep(n), size(n, 1) {
    std::iota(up.begin(), up.end(), 0u);
    std::iota(rep.begin(), rep.end(), 0u);
  }
  uint32_t root(uint32_t x) {
    uint32_t r = x;
    while (up[r] != r) r = up[r];
    while (up[x] != r) { uint32_t nx = up[x]; up[x] = r; x = nx; }
    return r;
  }
  // unionfind.h:82-102 contract: returns the representative of `lesser`'s set before
  // the union; afterwards the merged set's representative is `greater`'s.
  uint32_t unify(uint32_t lesser, uint32_t greater) {
    uint32_t rl = root(lesser), rg = root(greater);
    uint32_t old = rep[rl];
    if (rl != rg) {
      uint32_t keep_rep = rep[rg];
      if (size[rl] > size[rg]) std::swap(rl, rg);
      up[rl] = rg;
      size[rg] += size[rl];
      rep[rg] = keep_rep;
    }
    return old;
  }
};

struct Tree {
  std::vector<uint32_t> parent;   // JNode::parent (jnode.h:57)
  std::vector<uint32_t> pst;      // JNode::pst_weight (jnode.h:58)
};

// JTree(graph, seq, opts) (jtree.h:111-122) + insertSequence (jtree.cpp:112-145).
// Throws std::out_of_range where the reference's index.at() would (jtree.cpp:75).
Tree buildTree(const LlamaGraph &g, const std::vector<uint32_t> &seq) {
  Tree t;
  size_t n = seq.size();
  t.parent.assign(n, INVALID);
  t.pst.assign(n, 0);
  if (n == 0) return t;
  std::vector<uint32_t> index((size_t)*std::max_element(seq.begin(), seq.end()) + 1, INVALID);
  UnionFind uf(n);
  for (uint32_t cur = 0; cur < n; ++cur) {
    uint32_t X = seq[cur];
    if (g.isNode(X)) {
      for (uint64_t e = g.off[X]; e < g.off[X + 1]; ++e) {
        uint32_t nbr = g.adj[e];
        uint32_t nid = index.at(nbr);
        if (nid != INVALID) {                       // PREORDER edge -> adopt
          uint32_t kid = uf.unify(nid, cur);
          if (kid != cur) t.parent[kid] = cur;
        } else if (nbr != X) {                      // POSTORDER edge
          ++t.pst[cur];
        }
      }
    }
    index.at(X) = cur;                              // jtree.h:165-168
  }
  return t;
}

// -------------------------------------------------------------------------------------
// Map/reduce form of the same tree, for the BASELINE-size checks (C3-C5):
// graph2tree -r (graph2tree.cpp:185-196) — every MPI rank builds JTree over its
// contiguous edge shard (`-l part/num_parts`, graph_wrapper.h:47-49) and
// JNodeTable::mpi_merge reduces the partial trees pairwise in binomial rounds
// (jnode.cpp:203-250; merge :174-201).  Here the ranks are OpenMP threads.
//
// A partial tree is Liu's algorithm written per record instead of per adjacency list: a
// record (u, v) with positions p(u) != p(v) is, in JTree::insert (jtree.cpp:72-91), a
// PREORDER entry of the later endpoint (adopt the earlier one's component top) and a
// POSTORDER entry of the earlier one (++pst).  The adopts are grouped by the later
// position (the reference's outer loop over seq); their order inside one group does not
// change the tree.  The union-find is Liu's ancestor forest with path compression (a
// find re-points the visited path at the current node), the textbook form of the
// union-find sweep in unionfind.h:46-102: the elimination tree is unique given (edge
// multiset, order), so either gives the reference's tree.
// pst adds under merge (jnode.cpp:193), so the whole graph's pst is counted once.
//
// Both forms are pinned against each other and the golden trees in
// tests/test_oracle_golden.py.
// -------------------------------------------------------------------------------------

// Liu over adopt edges grouped by the later position: lo[off[k] .. off[k+1]) are the
// earlier endpoints of node k's PREORDER entries.  parent[] must be INVALID-filled.
// Union-find as unionfind.h:46-102 (union by rank, the set's newest node kept at its
// root as the representative), with path halving.
static void liuGrouped(uint64_t n, const uint64_t *off, const uint32_t *lo, uint32_t *parent) {
  struct Slot { uint32_t up, rep; };
  std::vector<Slot> uf(n);
  std::vector<uint8_t> rank(n, 0);
  Slot *u = uf.data();
  for (uint64_t i = 0; i < n; ++i) u[i] = Slot{(uint32_t)i, (uint32_t)i};
  auto find = [u](uint32_t x) {
    while (u[x].up != x) {
      const uint32_t g = u[u[x].up].up;
      u[x].up = g;
      x = g;
    }
    return x;
  };
  for (uint64_t k = 0; k < n; ++k) {
    uint32_t rk = find((uint32_t)k);
    const uint64_t e = off[k + 1];
    for (uint64_t j = off[k]; j < e; ++j) {
      if (j + 16 < e) __builtin_prefetch(&u[lo[j + 16]]);
      const uint32_t r = find(lo[j]);
      if (r == rk) continue;
      parent[u[r].rep] = (uint32_t)k;           // adopt (jnode.h:158-162)
      if (rank[r] > rank[rk]) { u[rk].up = r; rk = r; }
      else { u[r].up = rk; if (rank[r] == rank[rk]) ++rank[rk]; }
      u[rk].rep = (uint32_t)k;
    }
  }
}

// Counting sort of adopt edges (lo, hi) by hi over items [0, N): `emit(f, a, b)` calls
// f(lo, hi) for the edges of items [a, b).  Outside a parallel region the two passes run
// on all threads (atomic counts and cursors: the order inside one group is free).
template <class Emit>
static void groupByHi(uint64_t n, uint64_t N, Emit emit, std::vector<uint64_t> &off, std::vector<uint32_t> &lo) {
  off.assign(n + 1, 0);
  uint64_t *o = off.data();
  const bool par = !omp_in_parallel() && omp_get_max_threads() > 1;
  if (par) {
#pragma omp parallel for schedule(static)
    for (uint64_t c = 0; c < (N + 65535) / 65536; ++c)
      emit([&](uint32_t, uint32_t h) { __atomic_fetch_add(&o[(uint64_t)h + 1], 1, __ATOMIC_RELAXED); },
           c * 65536, std::min(N, (c + 1) * 65536));
  } else {
    emit([&](uint32_t, uint32_t h) { ++o[(uint64_t)h + 1]; }, 0, N);
  }
  for (uint64_t k = 0; k < n; ++k) o[k + 1] += o[k];
  lo.resize(o[n]);
  std::vector<uint64_t> cur(off.begin(), off.end() - 1);
  uint64_t *c = cur.data();
  uint32_t *l = lo.data();
  if (par) {
#pragma omp parallel for schedule(static)
    for (uint64_t b = 0; b < (N + 65535) / 65536; ++b)
      emit([&](uint32_t x, uint32_t h) { l[__atomic_fetch_add(&c[h], 1, __ATOMIC_RELAXED)] = x; },
           b * 65536, std::min(N, (b + 1) * 65536));
  } else {
    emit([&](uint32_t x, uint32_t h) { l[c[h]++] = x; }, 0, N);
  }
}

// One shard's partial tree (parent only): records [beg, end).
static void shardTree(const uint32_t *tail, const uint32_t *head, uint64_t beg, uint64_t end,
                      const std::vector<uint32_t> &pos, uint64_t n, uint32_t *parent) {
  std::fill(parent, parent + n, INVALID);
  const uint32_t *p = pos.data();
  const uint64_t ps = pos.size();
  std::vector<uint64_t> off;
  std::vector<uint32_t> lo;
  groupByHi(n, end - beg, [&](auto f, uint64_t a, uint64_t b) {
    for (uint64_t i = beg + a; i < beg + b; ++i) {
      const uint32_t u = tail[i], v = head[i];
      if (u >= ps || v >= ps) continue;   // range errors are reported by the caller
      const uint32_t pu = p[u], pv = p[v];
      if (pu == INVALID || pv == INVALID || pu == pv) continue;
      f(std::min(pu, pv), std::max(pu, pv));
    }
  }, off, lo);
  liuGrouped(n, off.data(), lo.data(), parent);
}

// JNodeTable::merge (jnode.cpp:174-201) on parent arrays: Liu over the union of both
// trees' parent edges (kid, parent).  `out` may alias `a`.
static void mergeParents(const uint32_t *a, const uint32_t *b, uint64_t n, uint32_t *out) {
  std::vector<uint64_t> off;
  std::vector<uint32_t> lo;
  groupByHi(n, n, [&](auto f, uint64_t lo_id, uint64_t hi_id) {
    for (uint64_t id = lo_id; id < hi_id; ++id) {
      if (a[id] != INVALID) f((uint32_t)id, a[id]);
      if (b[id] != INVALID) f((uint32_t)id, b[id]);
    }
  }, off, lo);
  std::fill(out, out + n, INVALID);
  liuGrouped(n, off.data(), lo.data(), out);
}

// graph2tree -r over `shards` contiguous record shards + the binomial mpi_merge.
Tree buildTreeMapReduce(const uint32_t *tail, const uint32_t *head, uint64_t R,
                        const std::vector<uint32_t> &seq, uint64_t shards) {
  Tree t;
  const uint64_t n = seq.size();
  t.parent.assign(n, INVALID);
  t.pst.assign(n, 0);
  if (n == 0) return t;
  if (shards < 1) shards = 1;
  std::vector<uint32_t> pos((size_t)*std::max_element(seq.begin(), seq.end()) + 1, INVALID);
  for (uint64_t i = 0; i < n; ++i) pos[seq[i]] = (uint32_t)i;
  const uint64_t ps = pos.size();
  // index.at(nbr) (jtree.cpp:75) throws when a sequenced vertex has a neighbour beyond
  // max(seq); pst counts POSTORDER entries (jtree.cpp:84-90), unsequenced neighbours
  // included (their index is INVALID); self-loops count nowhere.
  bool oor = false;
  uint32_t *w = t.pst.data();
#pragma omp parallel for schedule(static) reduction(|| : oor)
  for (uint64_t i = 0; i < R; ++i) {
    const uint32_t u = tail[i], v = head[i];
    const uint32_t pu = u < ps ? pos[u] : INVALID, pv = v < ps ? pos[v] : INVALID;
    if ((pu != INVALID && v >= ps) || (pv != INVALID && u >= ps)) { oor = true; continue; }
    if (u == v) continue;
    if (pu != INVALID && (pv == INVALID || pu < pv)) __atomic_fetch_add(&w[pu], 1, __ATOMIC_RELAXED);
    else if (pv != INVALID) __atomic_fetch_add(&w[pv], 1, __ATOMIC_RELAXED);
  }
  if (oor) throw std::out_of_range("vector::_M_range_check: index.at()");
  std::vector<std::vector<uint32_t>> part(shards);
#pragma omp parallel for schedule(dynamic, 1)
  for (uint64_t s = 0; s < shards; ++s) {
    part[s].resize(n);
    shardTree(tail, head, s * R / shards, (s + 1) * R / shards, pos, n, part[s].data());
  }
  for (uint64_t d = 1; d < shards; d *= 2) {   // MPI_Reduce's binomial rounds
    std::vector<uint64_t> pairs;
    for (uint64_t i = 0; i + d < shards; i += 2 * d) pairs.push_back(i);
    auto merge = [&](uint64_t i) {
      mergeParents(part[i].data(), part[i + d].data(), n, part[i].data());
      std::vector<uint32_t>().swap(part[i + d]);
    };
    if (pairs.size() == 1) {
      merge(pairs[0]);   // the last round groups its edges on every thread
    } else {
#pragma omp parallel for schedule(dynamic, 1)
      for (uint64_t j = 0; j < pairs.size(); ++j) merge(pairs[j]);
    }
  }
  t.parent.swap(part[0]);
  return t;
}

// makeKids (jnode.h:190-204): child lists in ascending child id.
std::vector<std::vector<uint32_t>> makeKids(const std::vector<uint32_t> &parent) {
  std::vector<std::vector<uint32_t>> kids(parent.size());
  for (uint32_t id = 0; id < parent.size(); ++id)
    if (parent[id] != INVALID) kids.at(parent[id]).push_back(id);
  return kids;
}

// JNodeTable::merge (jnode.cpp:174-201): Liu over the union of both parent edge sets,
// visiting lhs' kids then rhs' kids of each node; pst adds.
Tree mergeTrees(const Tree &lhs, const Tree &rhs) {
  size_t n = lhs.parent.size();
  if (rhs.parent.size() != n) throw std::invalid_argument("tree sizes differ");
  auto lk = makeKids(lhs.parent), rk = makeKids(rhs.parent);
  Tree t;
  t.parent.assign(n, INVALID);
  t.pst.assign(n, 0);
  UnionFind uf(n);
  for (uint32_t cur = 0; cur < n; ++cur) {
    for (auto *src : {&lk, &rk})
      for (uint32_t kid : (*src)[cur]) {
        uint32_t r = uf.unify(kid, cur);
        if (r != cur) t.parent[r] = cur;
      }
    t.pst[cur] = lhs.pst[cur] + rhs.pst[cur];
  }
  return t;
}

// JNodeTable::Facts (jnode.cpp:256-290), width = 1 + pst (no jxn table).
struct Facts {
  uint64_t vert_cnt = 0, edge_cnt = 0, width = 0, fill = 0, vert_height = 0,
           edge_height = 0, root_cnt = 0, halo_id = INVALID, core_id = INVALID;
};
Facts getFacts(const Tree &t) {
  Facts f;
  size_t n = t.parent.size();
  std::vector<uint64_t> vh(n, 0), eh(n, 0);
  for (uint32_t id = 0; id < n; ++id) {
    uint64_t w = 1 + (uint64_t)t.pst[id];
    f.vert_cnt++;
    f.edge_cnt += t.pst[id];
    f.width = std::max(f.width, w);
    f.fill += w - t.pst[id] - 1;
    vh[id]++;
    eh[id] += t.pst[id];
    uint32_t p = t.parent[id];
    if (p != INVALID) {
      vh.at(p) = std::max(vh.at(p), vh[id]);
      eh.at(p) = std::max(eh.at(p), eh[id]);
    } else {
      f.vert_height = std::max(f.vert_height, vh[id]);
      f.edge_height = std::max(f.edge_height, eh[id]);
      f.root_cnt++;
    }
    if (f.halo_id == INVALID && w > 3) f.halo_id = id;
    if (f.core_id == INVALID && w >= f.width) f.core_id = id;
  }
  return f;
}

std::string factsText(const Facts &f) {   // jnode.h:285-291
  char buf[512];
  snprintf(buf, sizeof buf,
           "TREEFAQS: width:%zu\troots:%zu\n\tvheight:%zu\teheight:%zu\n\tverts:%zu\tedges:%zu\n"
           "\thalo:%zu\tcore:%zu\n\tfill:%zu\n",
           (size_t)f.width, (size_t)f.root_cnt, (size_t)f.vert_height, (size_t)f.edge_height,
           (size_t)f.vert_cnt, (size_t)f.edge_cnt, (size_t)f.halo_id, (size_t)f.core_id,
           (size_t)f.fill);
  return buf;
}

// -------------------------------------------------------------------------------------
// Partition (partition.cpp:50-157, partition.h:135-143)
// -------------------------------------------------------------------------------------
struct PartitionResult {
  std::vector<part_t> parts;   // vid-indexed, size max(seq)+1, INVALID_PART elsewhere
  part_t num_parts = 0;        // the requested k (partition.cpp:52)
  size_t max_component = 0;
  uint32_t packing_nodes = 0;  // diagnostics: nodes where FFD ran
};

// get_weight (partition.cpp:38-48); pre_weight is always 0 (USE_PRE_WEIGHT off).
static inline size_t nodeWeight(const Tree &t, uint32_t id, bool vtx, bool pstw) {
  return (vtx ? 1 : 0) + (pstw ? (size_t)t.pst[id] : 0);
}

// `kids` is the persistent JNodeTable kid table: forwardPartition std::sorts it in
// place (partition.cpp:104-106) and the mutation carries over to the next k of the
// same partition_tree run.
PartitionResult partitionTree(const std::vector<uint32_t> &seq, const Tree &t,
                              std::vector<std::vector<uint32_t>> &kids, part_t np,
                              double balance, bool vtx, bool pstw) {
  size_t n = t.parent.size();
  PartitionResult res;
  res.num_parts = np;
  size_t total = 0;
  for (uint32_t id = 0; id < n; ++id) total += nodeWeight(t, id, vtx, pstw);
  const size_t max_component = (size_t)((double)(total / (size_t)(long)np) * balance);
  res.max_component = max_component;

  std::vector<part_t> parts(n, INVALID_PART);
  std::vector<size_t> part_size;
  std::vector<size_t> cb(n, 0);   // component_below
  for (uint32_t id = 0; id < n; ++id) {          // ascending pass (:97-135)
    cb[id] += nodeWeight(t, id, vtx, pstw);
    if (cb[id] > max_component) {
      res.packing_nodes++;
      std::vector<uint32_t> &k = kids[id];
      std::sort(k.begin(), k.end(), [&cb](uint32_t a, uint32_t b) { return cb[a] > cb[b]; });
      do {
        for (auto it = k.begin(); cb[id] > max_component && it != k.end(); ++it) {
          uint32_t kid = *it;
          if (cb[kid] > max_component)
            throw std::runtime_error("forwardPartition: kid exceeds max_component");
          if (parts[kid] != INVALID_PART) continue;
          for (size_t p = 0; p != part_size.size(); ++p) {
            if (part_size[p] + cb[kid] <= max_component) {
              cb[id] -= cb[kid];
              part_size[p] += cb[kid];
              parts[kid] = (part_t)p;
              break;
            }
          }
        }
        if (cb[id] > max_component) {
          bool any_unassigned = false;
          for (uint32_t kid : k) any_unassigned |= parts[kid] == INVALID_PART;
          if (!any_unassigned || part_size.size() > 32767)
            throw std::runtime_error("forwardPartition: cannot pack (reference loops forever)");
          part_size.push_back(0);
        }
      } while (cb[id] > max_component);
    }
    if (t.parent[id] != INVALID) cb.at(t.parent[id]) += cb[id];
  }
  for (uint32_t id = (uint32_t)n - 1; id != INVALID; --id) {   // descending pass (:139-156)
    if (parts[id] == INVALID_PART && t.parent[id] != INVALID) parts[id] = parts[t.parent[id]];
    while (parts[id] == INVALID_PART) {
      for (long p = (long)part_size.size() - 1; p != -1; --p) {
        if (part_size[p] + cb[id] <= max_component) {
          part_size[p] += cb[id];
          parts[id] = (part_t)p;
          break;
        }
      }
      if (parts[id] == INVALID_PART) part_size.push_back(0);
    }
  }
  // jnid -> vid re-index (:62-66)
  res.parts.assign(seq.empty() ? 0 : (size_t)*std::max_element(seq.begin(), seq.end()) + 1,
                   INVALID_PART);
  for (size_t i = 0; i < seq.size(); ++i) res.parts.at(seq[i]) = parts.at(i);
  return res;
}

std::string partitionPrintText(const PartitionResult &r) {   // partition.h:135-143
  part_t max_part = r.parts.empty() ? 0 : (part_t)(*std::max_element(r.parts.begin(), r.parts.end()) + 1);
  size_t first = std::count(r.parts.begin(), r.parts.end(), 0);
  size_t second = std::count(r.parts.begin(), r.parts.end(), 1);
  char buf[256];
  snprintf(buf, sizeof buf, "Actually created %d partitions.\nFirst two partition sizes: %zu and %zu\n",
           (int)max_part, first, second);
  return buf;
}

// -------------------------------------------------------------------------------------
// Evaluators (partition.cpp:423-521)
// -------------------------------------------------------------------------------------
struct EvalResult {
  uint64_t edges_cut = 0, vcom_vol = 0, max_vertex_bal = 0, ecv_hash = 0, max_hash_bal = 0;
  uint64_t ecv_down = 0, max_down_bal = 0, ecv_up = 0, max_up_bal = 0;
  uint64_t edges = 0, nodes = 0;
};

static inline uint32_t cormen_hash(uint32_t k) {            // partition.cpp:423-427
  double A = 0.5 * (std::sqrt(5.0) - 1);
  uint32_t s = (uint32_t)std::floor(A * std::pow(2.0, 32));
  return k * s;
}

// The reference inserts owners into a std::unordered_set<part_t> per node and takes its
// size(); PartSet is the same distinct count over a bitset of the part ids.
struct PartSet {
  std::vector<uint64_t> w;
  std::vector<uint32_t> touched;
  size_t n = 0;
  explicit PartSet(size_t nparts) : w((nparts + 63) / 64, 0) {}
  void insert(part_t p) {
    uint64_t &x = w.at((size_t)(uint16_t)p >> 6);
    const uint64_t b = 1ull << (p & 63);
    if (!(x & b)) {
      if (!x) touched.push_back((uint32_t)((size_t)(uint16_t)p >> 6));
      x |= b;
      ++n;
    }
  }
  size_t size() const { return n; }
  void clear() {
    for (uint32_t i : touched) w[i] = 0;
    touched.clear();
    n = 0;
  }
};

EvalResult evaluate(const LlamaGraph &g, const std::vector<part_t> &parts,
                    const std::vector<uint32_t> &seq, bool with_seq) {
  EvalResult r;
  r.edges = g.getEdges();
  r.nodes = g.getNodes();
  part_t max_part = *std::max_element(parts.begin(), parts.end());
  const size_t np = (size_t)max_part + 1;
  std::vector<uint64_t> vbal(np, 0), hbal(np, 0);
  uint64_t cut = 0, vcom = 0, ecvh = 0;
  bool bad = false;
#pragma omp parallel reduction(+ : cut, vcom, ecvh) reduction(|| : bad)
  {
    std::vector<uint64_t> lv(np, 0), lh(np, 0);
    PartSet vc(np), eh(np);
#pragma omp for schedule(dynamic, 4096)
    for (uint32_t X = 0; X < g.max_nodes; ++X) {             // evaluate(graph) :428-473
      if (!g.isNode(X)) continue;
      part_t Xp = parts.at(X);
      if (Xp == INVALID_PART) { bad = true; continue; }
      lv.at(Xp) += 1;
      vc.clear(); eh.clear();
      vc.insert(Xp);
      for (uint64_t e = g.off[X]; e < g.off[X + 1]; ++e) {
        uint32_t Y = g.adj[e];
        part_t Yp = parts.at(Y);
        if (Yp == INVALID_PART) { bad = true; continue; }
        if (X < Y && Xp != Yp) ++cut;
        vc.insert(Yp);
        part_t hp = cormen_hash(X) < cormen_hash(Y) ? Xp : Yp;
        eh.insert(hp);
        if (X < Y) lh.at(hp) += 1;
      }
      vcom += vc.size() - 1;
      ecvh += eh.size() - 1;
    }
#pragma omp critical
    for (size_t p = 0; p < np; ++p) { vbal[p] += lv[p]; hbal[p] += lh[p]; }
  }
  if (bad) throw std::runtime_error("unassigned vertex");
  r.edges_cut = cut; r.vcom_vol = vcom; r.ecv_hash = ecvh;
  r.max_vertex_bal = *std::max_element(vbal.begin(), vbal.end());
  r.max_hash_bal = *std::max_element(hbal.begin(), hbal.end());
  if (!with_seq) return r;

  std::vector<uint32_t> pos((size_t)*std::max_element(seq.begin(), seq.end()) + 1, INVALID);
  for (uint32_t i = 0; i < seq.size(); ++i) pos[seq[i]] = i;
  std::vector<uint64_t> dbal(np, 0), ubal(np, 0);
  uint64_t down = 0, upc = 0;
  bool oor = false;
#pragma omp parallel reduction(+ : down, upc) reduction(|| : oor)
  {
    std::vector<uint64_t> ld(np, 0), lu(np, 0);
    PartSet dn(np), up(np);
#pragma omp for schedule(dynamic, 4096)
    for (uint32_t X = 0; X < g.max_nodes; ++X) {             // evaluate(graph, seq) :475-521
      if (!g.isNode(X)) continue;
      if (X >= pos.size()) { oor = true; continue; }          // pos.at(X) throws
      uint32_t Xpos = pos[X];
      part_t Xp = parts.at(X);
      dn.clear(); up.clear();
      for (uint64_t e = g.off[X]; e < g.off[X + 1]; ++e) {
        uint32_t Y = g.adj[e];
        if (Y >= pos.size()) { oor = true; continue; }
        uint32_t Ypos = pos[Y];
        part_t Yp = parts.at(Y);
        dn.insert(Xpos < Ypos ? Xp : Yp);
        up.insert(Xpos > Ypos ? Xp : Yp);
        if (Xpos < Ypos) ld.at(Xp) += 1;
        if (Xpos > Ypos) lu.at(Xp) += 1;
      }
      down += dn.size() - 1;
      upc += up.size() - 1;
    }
#pragma omp critical
    for (size_t p = 0; p < np; ++p) { dbal[p] += ld[p]; ubal[p] += lu[p]; }
  }
  if (oor) throw std::out_of_range("vector::_M_range_check: pos.at()");
  r.ecv_down = down; r.ecv_up = upc;
  r.max_down_bal = *std::max_element(dbal.begin(), dbal.end());
  r.max_up_bal = *std::max_element(ubal.begin(), ubal.end());
  return r;
}

std::string evalText(const EvalResult &r, part_t num_parts, bool with_seq) {
  char buf[1024];
  size_t E = r.edges, N = r.nodes;
  size_t Ek = E / (size_t)(long)num_parts, Nk = N / (size_t)(long)num_parts;
  int len = snprintf(buf, sizeof buf,
      "edges cut: %zu (%f%%)\nVcom. vol: %zu (%f%%)\n  balance: %zu (%f%%)\nECV(hash): %zu (%f%%)\n  balance: %zu (%f%%)\n",
      (size_t)r.edges_cut, (double)r.edges_cut / E, (size_t)r.vcom_vol, (double)r.vcom_vol / E,
      (size_t)r.max_vertex_bal, (double)r.max_vertex_bal / Nk, (size_t)r.ecv_hash,
      (double)r.ecv_hash / E, (size_t)r.max_hash_bal, (double)r.max_hash_bal / Ek);
  if (with_seq)
    snprintf(buf + len, sizeof buf - len,
        "ECV(down): %zu (%f%%)\n  balance: %zu (%f%%)\nECV(up)  : %zu (%f%%)\n  balance: %zu (%f%%)\n",
        (size_t)r.ecv_down, (double)r.ecv_down / E, (size_t)r.max_down_bal, (double)r.max_down_bal / Ek,
        (size_t)r.ecv_up, (double)r.ecv_up / E, (size_t)r.max_up_bal, (double)r.max_up_bal / Ek);
  return buf;
}

}  // namespace oracle

// =====================================================================================
// C ABI for ctypes (tests / bench cpu_baseline only).  All functions return 0 on
// success, -1 on error (message via or_last_error()).
// =====================================================================================
using namespace oracle;
static thread_local std::string g_err;

#define OR_TRY(...)                                    \
  try { __VA_ARGS__; return 0; }                      \
  catch (const std::exception &e) { g_err = e.what(); return -1; }

extern "C" {
const char *or_last_error() { return g_err.c_str(); }

// FNV-1a over n bytes: the digest oracle/ref/ref_harness prints of the reference flow's
// sequence, merged tree and parts, so a GPU result can be compared with it.
uint64_t or_fnv1a(const unsigned char *p, uint64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

// OpenMP threads for the graph build and the evaluators (default 1; tests raise it for
// BASELINE-size parity checks).
void or_set_threads(int n) { omp_set_num_threads(n < 1 ? 1 : n); }

// mode 0: LLAMA degree sequence (degreeSequence / mpiSequence); mode 1: file sequence
// over .dat records (last record twice); mode 2: file sequence over .net pairs.
int or_sequence(const uint32_t *tail, const uint32_t *head, uint64_t R, int mode,
                uint32_t *seq_out, uint64_t cap, uint64_t *n_out) {
  OR_TRY({
    std::vector<uint32_t> s;
    if (mode == 0) s = degreeSequence(LlamaGraph(tail, head, R));
    else if (mode == 3) s = degreeSequenceFromRecords(tail, head, R);
    else s = fileSequence(tail, head, R, mode == 1);
    if (s.size() > cap) throw std::length_error("seq capacity");
    std::copy(s.begin(), s.end(), seq_out);
    *n_out = s.size();
  })
}

// JTree over the (optionally partial) graph; parent/pst arrays of length n.
int or_build_tree(const uint32_t *tail, const uint32_t *head, uint64_t R, uint64_t part,
                  uint64_t num_parts, const uint32_t *seq, uint64_t n, uint32_t *parent,
                  uint32_t *pst) {
  OR_TRY({
    LlamaGraph g(tail, head, R, part, num_parts);
    Tree t = buildTree(g, std::vector<uint32_t>(seq, seq + n));
    std::copy(t.parent.begin(), t.parent.end(), parent);
    std::copy(t.pst.begin(), t.pst.end(), pst);
  })
}

// graph2tree -r form (shard trees on OpenMP threads + binomial merges); parent/pst of
// length n.
int or_build_tree_mr(const uint32_t *tail, const uint32_t *head, uint64_t R, const uint32_t *seq, uint64_t n,
                     uint64_t shards, uint32_t *parent, uint32_t *pst) {
  OR_TRY({
    Tree t = buildTreeMapReduce(tail, head, R, std::vector<uint32_t>(seq, seq + n), shards);
    std::copy(t.parent.begin(), t.parent.end(), parent);
    std::copy(t.pst.begin(), t.pst.end(), pst);
  })
}

int or_merge(const uint32_t *pa, const uint32_t *wa, const uint32_t *pb, const uint32_t *wb,
             uint64_t n, uint32_t *po, uint32_t *wo) {
  OR_TRY({
    Tree a{{pa, pa + n}, {wa, wa + n}}, b{{pb, pb + n}, {wb, wb + n}};
    Tree t = mergeTrees(a, b);
    std::copy(t.parent.begin(), t.parent.end(), po);
    std::copy(t.pst.begin(), t.pst.end(), wo);
  })
}

// out[9] = width, roots, vheight, eheight, verts, edges, halo, core, fill
int or_facts(const uint32_t *parent, const uint32_t *pst, uint64_t n, uint64_t *out) {
  OR_TRY({
    Tree t{{parent, parent + n}, {pst, pst + n}};
    Facts f = getFacts(t);
    uint64_t v[9] = {f.width, f.root_cnt, f.vert_height, f.edge_height, f.vert_cnt,
                     f.edge_cnt, f.halo_id, f.core_id, f.fill};
    std::memcpy(out, v, sizeof v);
  })
}

// Persistent kid table (one per loaded tree, as in partition_tree).
void *or_kids_create(const uint32_t *parent, uint64_t n) {
  return new std::vector<std::vector<uint32_t>>(makeKids(std::vector<uint32_t>(parent, parent + n)));
}
void or_kids_free(void *k) { delete (std::vector<std::vector<uint32_t>> *)k; }

// parts_out: vid-indexed, capacity cap (>= max(seq)+1).  info[3] = created (max part+1),
// max_component, packing nodes.  seq has seq_n entries (the tree n).
int or_partition(const uint32_t *parent, const uint32_t *pst, uint64_t n, const uint32_t *seq, uint64_t seq_n,
                 void *kids, int16_t k, double balance, int vtx, int pstw, int16_t *parts_out,
                 uint64_t cap, uint64_t *vs_out, int64_t *info) {
  OR_TRY({
    Tree t{{parent, parent + n}, {pst, pst + n}};
    std::vector<uint32_t> s(seq, seq + seq_n);
    auto &kt = *(std::vector<std::vector<uint32_t>> *)kids;
    PartitionResult r = partitionTree(s, t, kt, k, balance, vtx != 0, pstw != 0);
    if (r.parts.size() > cap) throw std::length_error("parts capacity");
    std::copy(r.parts.begin(), r.parts.end(), parts_out);
    *vs_out = r.parts.size();
    info[0] = r.parts.empty() ? 0 : *std::max_element(r.parts.begin(), r.parts.end()) + 1;
    info[1] = (int64_t)r.max_component;
    info[2] = r.packing_nodes;
  })
}

// out[11] = edges_cut, vcom_vol, max_vertex_bal, ecv_hash, max_hash_bal, ecv_down,
//           max_down_bal, ecv_up, max_up_bal, getEdges, getNodes
int or_evaluate(const uint32_t *tail, const uint32_t *head, uint64_t R, const uint32_t *seq,
                uint64_t n, const int16_t *parts, uint64_t vs, uint64_t *out) {
  OR_TRY({
    LlamaGraph g(tail, head, R);
    EvalResult r = evaluate(g, std::vector<part_t>(parts, parts + vs),
                            std::vector<uint32_t>(seq, seq + n), true);
    uint64_t v[11] = {r.edges_cut, r.vcom_vol, r.max_vertex_bal, r.ecv_hash, r.max_hash_bal,
                      r.ecv_down, r.max_down_bal, r.ecv_up, r.max_up_bal, r.edges, r.nodes};
    std::memcpy(out, v, sizeof v);
  })
}

// Text renderings of the reference's stdout lines (byte-exact format strings).
int or_facts_text(const uint32_t *parent, const uint32_t *pst, uint64_t n, char *buf, uint64_t cap) {
  OR_TRY({
    Tree t{{parent, parent + n}, {pst, pst + n}};
    std::string s = factsText(getFacts(t));
    snprintf(buf, cap, "%s", s.c_str());
  })
}
int or_eval_text(const uint64_t *v, int16_t num_parts, char *buf, uint64_t cap) {
  OR_TRY({
    EvalResult r;
    r.edges_cut = v[0]; r.vcom_vol = v[1]; r.max_vertex_bal = v[2]; r.ecv_hash = v[3];
    r.max_hash_bal = v[4]; r.ecv_down = v[5]; r.max_down_bal = v[6]; r.ecv_up = v[7];
    r.max_up_bal = v[8]; r.edges = v[9]; r.nodes = v[10];
    std::string s = evalText(r, num_parts, true);
    snprintf(buf, cap, "%s", s.c_str());
  })
}
}
