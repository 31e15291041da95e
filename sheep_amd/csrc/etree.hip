// etree.hip — map step (relabel + pst + per-shard elimination tree) and the reduce
// step (pairwise tree merge), both on one GPU kernel family.
//
// Reference: JTree::insert (jtree.cpp:66-110) runs Liu's algorithm sequentially: for
// X in order, every earlier neighbour's union-find representative gets parent X
// (jnode.h:158-162, unionfind.h:82-102); later neighbours count into pst_weight.
// JNodeTable::merge (jnode.cpp:174-201) re-runs Liu over the union of two parent
// edge sets.
//
// MI355X formulation (no sequential sweep).  With vertices numbered by sequence
// position, parent(x) = min{ v > x : v adjacent to C_x } where C_x is x's component
// in G[0..x].  We compute it by divide and conquer over the position range, all
// subproblems of one level at once:
//   subproblem [l,r), split mid:  light = both ends < mid,  cross = lo < mid <= hi.
//   * union-find over the light edges (priority linking), then each component's
//     maximum = its "top" t;
//   * for every cross edge (a,b): t = top(a); m_t = min b  (atomicMin)  -> parent(t) = m_t;
//   * contract: (a,b) -> (m_t, b); drop it when b == m_t; dedup contracted pairs.
//   After the level every live edge lies inside one half; recurse.
// Every vertex gets its parent at the one level where it is the top of a light
// component with a cross edge; vertices never assigned are roots.  The result is the
// unique elimination tree of (edge multiset, order) — identical to Liu's.  Level
// ranges are dyadic in a monotone spread of [0,n) onto [0,2^L) so halves are balanced.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"

namespace sheep {
namespace {

constexpr uint64_t DEAD = ~0ull;

__device__ __forceinline__ uint32_t spread(uint32_t x, uint32_t clo) { return x + __umulhi(x, clo); }

// ---- per-level state: level-tagged words -------------------------------------------
// uf, top, mt and claim are rebuilt at every D&C level.  For n < 2^27 - 1 a word carries
// the level that wrote it in its top 5 bits (Tg): a word of another level reads as the
// reset value (uf / top: the vertex itself, mt / claim: none), so no pass restores the
// arrays between levels (the dense reset wrote 16 B per vertex per level: 9 GB of the
// RMAT-26 step).  Larger trees keep untagged words and the per-level reset.
//   uf, top, claim: tag = level + 1 (top's atomicMax: older words are smaller);
//   mt: tag = 31 - level (atomicMin: older words are larger; the reset value ~0 is larger
//       still, and at level 0, where it carries the current tag, its value is >= n).
constexpr int TAG_SHIFT = 27;
constexpr uint32_t VAL_MASK = (1u << TAG_SHIFT) - 1;
constexpr uint64_t TAG_MAX_N = VAL_MASK;   // n < 2^27 - 1: every position is < VAL_MASK

struct Tg {
  uint32_t cur, mcur;   // (level + 1) << 27, (31 - level) << 27
  bool on;
  __device__ __forceinline__ uint32_t get(uint32_t w, uint32_t self) const {   // uf / top
    return !on ? w : (w & ~VAL_MASK) == cur ? (w & VAL_MASK) : self;
  }
  __device__ __forceinline__ uint32_t enc(uint32_t v) const { return on ? (cur | v) : v; }
  __device__ __forceinline__ uint32_t claim_get(uint32_t w) const {
    return !on ? w : (w & ~VAL_MASK) == cur ? (w & VAL_MASK) : INVALID;
  }
  __device__ __forceinline__ uint32_t m_enc(uint32_t v) const { return on ? (mcur | v) : v; }
  __device__ __forceinline__ uint32_t m_get(uint32_t w) const {
    return !on ? w : ((w & ~VAL_MASK) == mcur && (w & VAL_MASK) != VAL_MASK) ? (w & VAL_MASK) : INVALID;
  }
};
__host__ __device__ inline Tg make_tag(int lvl, bool on) {
  return Tg{(uint32_t)(lvl + 1) << TAG_SHIFT, (uint32_t)(31 - lvl) << TAG_SHIFT, on};
}

// ---- union-find ---------------------------------------------------------------------
// The forest is monotone: uf[x] only ever changes from x to a smaller root (CAS hook,
// only on a current root, so no link is ever lost) or to a smaller ancestor (path
// splitting), so every value a thread can read — even a stale L1 copy — is an ancestor
// of x (a word of an older level reads as x itself, the level's start value).  Plain
// loads/stores are therefore safe while other threads hook: a stale root only makes its
// CAS fail, and the edge is simply kept for the next round.  The component's top (its
// largest id, which the etree needs) is tracked separately.
// (Linking under the larger root instead, so root = top, measured 2x slower hooking.)

// Path splitting on two chains in lockstep (both loads in flight at once).
__device__ __forceinline__ void find2(uint32_t *uf, Tg g, uint32_t &x, uint32_t &y) {
  uint32_t px = g.get(uf[x], x), py = g.get(uf[y], y);
  while (px != x || py != y) {
    if (px != x) {
      const uint32_t gg = g.get(uf[px], px);
      if (gg != px) uf[x] = g.enc(gg);
      x = px;
      px = gg;
    }
    if (py != y) {
      const uint32_t gg = g.get(uf[py], py);
      if (gg != py) uf[y] = g.enc(gg);
      y = py;
      py = gg;
    }
  }
}

// Hooks root hi under lo: succeeds only while hi is still a root (its word unchanged).
__device__ __forceinline__ bool hook(uint32_t *uf, Tg g, uint32_t hi, uint32_t lo) {
  const uint32_t w = uf[hi];
  if (g.get(w, hi) != hi) return false;
  return atomicCAS(&uf[hi], w, g.enc(lo)) == w;
}

// K independent chains in lockstep: each round issues one load per unfinished chain,
// so a thread keeps K pointer chases in flight instead of one.
// (Loads are issued for all K chains before any word is decoded — a chain that is done
// reloads its own root's word — so the K loads stay in flight together: decoding each
// word inside its chain's branch made the compiler wait for every load in turn.)
template <int K> __device__ __forceinline__ void find_many(uint32_t *uf, Tg g, uint32_t (&x)[K], const bool (&v)[K]) {
  uint32_t p[K], w[K];
#pragma unroll
  for (int k = 0; k < K; ++k) w[k] = uf[x[k]];
#pragma unroll
  for (int k = 0; k < K; ++k) p[k] = v[k] ? g.get(w[k], x[k]) : x[k];
  for (;;) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < K; ++k) any |= p[k] != x[k];
    if (!any) break;
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = uf[p[k]];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (p[k] != x[k]) {
        const uint32_t gg = g.get(w[k], p[k]);
        if (gg != p[k]) uf[x[k]] = g.enc(gg);
        x[k] = p[k];
        p[k] = gg;
      }
    }
  }
}

// ---- relabel + pst (jtree.cpp:72-91) -------------------------------------------------
// One record = one undirected pair.  Both endpoints sequenced: pst[lo]++ and a tree
// edge (lo,hi).  One endpoint sequenced, the other a slot < pos_size but absent from
// the sequence: its index stays INVALID forever -> POSTORDER for the sequenced one.
// A neighbour >= pos_size of a sequenced vertex -> index.at() throws -> error flag.
__global__ __launch_bounds__(BLOCK) void k_relabel(const sheep_xs1 *__restrict__ rec, uint64_t nrec,
                                                   const uint32_t *__restrict__ pos, uint64_t pos_size,
                                                   uint32_t *__restrict__ pst, uint64_t *__restrict__ edges,
                                                   unsigned long long *__restrict__ err) {
  // edges[i] = the relabelled tree edge of record i, or DEAD (no compaction: the first
  // etree level skips holes, and self-loops / unsequenced endpoints are rare)
  const uint64_t ntiles = (nrec + TILE - 1) / TILE;
  bool bad = false;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint64_t ev[TILE_ITEMS];
#pragma unroll
    for (int j = 0; j < TILE_ITEMS; ++j) {
      const uint64_t i = tile * TILE + (uint64_t)j * BLOCK + threadIdx.x;
      ev[j] = DEAD;
      if (i >= nrec) continue;
      const sheep_xs1 r = rec[i];
      const uint32_t t = r.tail, h = r.head;
      if (t == h) continue;
      const uint32_t pt = t < pos_size ? pos[t] : INVALID;
      const uint32_t ph = h < pos_size ? pos[h] : INVALID;
      const bool tin = pt != INVALID, hin = ph != INVALID;
      if ((tin && h >= pos_size) || (hin && t >= pos_size)) { bad = true; continue; }
      if (tin && hin) {
        const uint32_t lo = pt < ph ? pt : ph, hi = pt < ph ? ph : pt;
        ev[j] = ((uint64_t)hi << 32) | lo;   // pst[lo]: histogram of the edges' lo (hist.hip)
      } else if (tin) {
        atomicAdd(&pst[pt], 1u);
      } else if (hin) {
        atomicAdd(&pst[ph], 1u);
      }
    }
#pragma unroll
    for (int j = 0; j < TILE_ITEMS; ++j) {
      const uint64_t i = tile * TILE + (uint64_t)j * BLOCK + threadIdx.x;
      if (i < nrec) edges[i] = ev[j];
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(err, 1ull);
}

// ---- one D&C level ---------------------------------------------------------------
// Every count a level needs stays in device memory (the per-level stats row, below):
// kernels read their list lengths there and size their loops from them, the host only
// sizes grids from an upper bound.  A level is a chain of launches with no host round
// trip; kernels whose list is empty return at once.
//
// The level's input is the list (edges active at an earlier level: light ones and
// contractions) plus the bucket of edges whose first active level this is.  k_split
// streams both once and writes, in order, three dense lists: the entries that stay
// (light and right-half edges) into the NEXT list buffer, the light edges, and the cross
// edges; k_cross_apply appends the contractions after the entries that stayed.  Cross
// edges are thereby dropped from the list as they are taken, so the list never holds
// stale or dead entries for long and needs no separate compaction.
//
// stats row of level l (u64): [0] list length entering the level, [1] light edges,
// [2] cross edges, [3] entries that stayed, [4] contractions that survived, [5..7]
// unresolved light edges after hooking round 0..2, [10] edges activated from the
// level's bucket.
constexpr int ST_ROW = 16, ST_LIVE = 0, ST_NL = 1, ST_NX = 2, ST_KEPT = 3, ST_CONTR = 4, ST_HOOK = 5, ST_R0 = 10,
              ST_SCANN = 11;
// [12] the top block's MSF edges appended after the contractions, [13] the cut (the next
// split drops the list entries with spread(lo) >= cut ahead of them), [14] the tile count
// of the top block's list extraction (the dense top block, below)
constexpr int ST_EXTRA = 12, ST_CUT = 13, ST_TOPNT = 14;
// One deferred round, then the in-place finish (swept: 0 / 1 / 2 / 3 rounds = union 8.4 /
// 6.3 / 6.6 / 6.7 ms at RMAT-26; 1 also best on the Chung-Lu graph, RMAT-28 and merges):
// the first round clears the pile-up on a forming giant component's root, and what is
// left is too little to pay for more launches and packs.
constexpr int HOOK_ROUNDS = 1;
// counter sets zeroed at every level: hook rounds and the contractions (sharded appends)
constexpr int CSET_HOOK = 0, CSET_APPLY = CSET_HOOK + HOOK_ROUNDS, NCSET = CSET_APPLY + 1;
constexpr uint64_t CSET_WORDS = (uint64_t)NSHARD * SHARD_STRIDE;

// ---- first-activity buckets ---------------------------------------------------------
// An edge (lo, hi) takes part in level s only if bit s of ya = spread(lo) is 0 (light
// or cross); while ya's bits above stay 1 it sits in right halves and every level would
// just re-read it.  So the input comes grouped by its first active level f = the
// highest zero bit of ya — a range of lo (hist.hip group_edges_by_lo for a map; a
// merge's parent edges are already in lo order) — and level s activates group s: the
// list the levels stream holds only edges that have been active (and their
// contractions).

__global__ __launch_bounds__(BLOCK) void k_reset(uint32_t *__restrict__ uf, uint32_t *__restrict__ mt,
                                                 uint32_t *__restrict__ top, uint32_t *__restrict__ claim, uint64_t n,
                                                 unsigned long long *__restrict__ csets) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t t0 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t i = t0; i < n; i += stride) {
    uf[i] = (uint32_t)i;
    mt[i] = INVALID;
    top[i] = (uint32_t)i;
    claim[i] = INVALID;
  }
  for (uint64_t i = t0; i < NCSET * CSET_WORDS; i += stride) csets[i] = 0;
}

// End of a level: the counter sets back to zero.  Tagged state: parent(top(r)) = m_r for
// every root with a cross edge, from one streaming read of mt (a random store per cross
// edge in k_cross_apply cost more).  Untagged state (n >= 2^27 - 1): back to the reset
// values — entry by entry when the level's lists are short against n (only light
// endpoints, cross roots and cross hi ends were written), else densely; the choice is
// made on the device from the level's counts (no host round trip).
// Where the adoption parent(top(r)) = m_r runs for tagged state: a level with few cross
// edges against n adopts in k_cross_apply, from the edges with b == m_r (a random top read
// and parent store each, for one edge per root), instead of k_level_clean's dense pass over
// all n words of mt (~26 us at RMAT-26 even when a late level has a few thousand roots).
// Both kernels decide from the same device counts.
// (8 RMAT-26 shard maps + merge 122.4 -> 121.7 ms, C3 and C2 unchanged: profiles/r6/README.md)
__host__ __device__ inline bool sparse_adopt(uint64_t nx, uint64_t n) { return nx * 8 < n; }

struct LevelClean {   // what k_level_clean needs of the level it closes
  const uint64_t *lx;   // the level's light entries, then its cross entries (st[ST_NL] on)
  const uint32_t *xtop;
  const uint64_t *st;
  uint32_t *uf, *mt, *top, *claim;
  uint64_t n;
  bool tagged;
  int lvl;
  uint32_t *parent;
  unsigned long long *csets;
};
__device__ void level_clean(const LevelClean &lc) {
  const uint64_t *__restrict__ lbuf = lc.lx, *__restrict__ xbuf = lc.lx + lc.st[ST_NL];
  const uint32_t *__restrict__ xtop = lc.xtop;
  uint32_t *__restrict__ uf = lc.uf, *__restrict__ mt = lc.mt, *__restrict__ top = lc.top, *__restrict__ claim = lc.claim;
  uint32_t *__restrict__ parent = lc.parent;
  unsigned long long *__restrict__ csets = lc.csets;
  const uint64_t n = lc.n;
  const bool tagged = lc.tagged;
  const int lvl = lc.lvl;
  const uint64_t nl = lc.st[ST_NL], nx = lc.st[ST_NX];
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t t0 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t i = t0; i < NCSET * CSET_WORDS; i += stride) csets[i] = 0;
  if (tagged) {   // parent(top(r)) = m_r for every root r with a cross edge (jnode.h:158-162 adopt)
    const Tg g = make_tag(lvl, true);
    if (nx == 0 || sparse_adopt(nx, n)) return;   // (adopted by k_cross_apply's edges)
    for (uint64_t i = t0; i < n; i += stride) {
      const uint32_t m = g.m_get(mt[i]);
      if (m != INVALID) parent[g.get(top[i], (uint32_t)i)] = m;
    }
    return;
  }
  if ((nl + nx) * 8 >= n) {   // a scattered 4-B store costs about a line; a dense pass 16 B per vertex
    for (uint64_t i = t0; i < n; i += stride) {
      uf[i] = (uint32_t)i;
      mt[i] = INVALID;
      top[i] = (uint32_t)i;
      claim[i] = INVALID;
    }
    return;
  }
  for (uint64_t i = t0; i < nl; i += stride) {
    const uint64_t e = lbuf[i];
    const uint32_t a = (uint32_t)e, b = (uint32_t)(e >> 32);
    uf[a] = a;
    uf[b] = b;
    top[a] = a;
    top[b] = b;
  }
  for (uint64_t i = t0; i < nx; i += stride) {
    mt[xtop[i]] = INVALID;
    claim[(uint32_t)(xbuf[i] >> 32)] = INVALID;
  }
}
// The last global level's clean (the others run at the start of the next level's
// k_split_count: one launch fewer per level).
__global__ __launch_bounds__(BLOCK) void k_level_clean(LevelClean lc) { level_clean(lc); }

constexpr int XK = 8;   // items per thread in the gather kernels (independent chains in flight)

// top[root] = the component's largest id.  Every vertex of a non-singleton light
// component is an endpoint of a light edge and its maximum is the hi end of one, so a
// max over the light edges' hi ends suffices (singletons keep top = self).
__global__ __launch_bounds__(BLOCK) void k_light_top(const uint64_t *__restrict__ lbuf, const uint64_t *__restrict__ n_l,
                                                     uint32_t *uf, uint32_t *__restrict__ top, Tg g) {
  const uint64_t nl = *n_l;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK * XK;
  const uint64_t iters = (nl + stride - 1) / stride;
  uint64_t base = (uint64_t)blockIdx.x * BLOCK * XK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, base += stride) {   // wave-uniform trip count (ballots)
    uint32_t r[XK], b[XK];
    bool live[XK];
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      const uint64_t i = base + (uint64_t)k * BLOCK;
      live[k] = i < nl;
      const uint64_t e = live[k] ? lbuf[i] : 0;
      r[k] = (uint32_t)e;
      b[k] = (uint32_t)(e >> 32);
    }
    find_many<XK>(uf, g, r, live);
    // top only grows: combine lanes sharing the first lane's root, skip useless atomics
    // (tagged words: an older level's word is smaller than any of this level's)
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      const uint64_t lm = __ballot(live[k]);
      if (!lm) continue;
      const int first = __ffsll((unsigned long long)lm) - 1;
      const uint32_t r0 = __shfl(r[k], first, 64);
      const bool same = live[k] && r[k] == r0;
      const uint32_t v = wave_max(same ? b[k] : 0u);
      if ((int)__lane_id() == first && v > g.get(top[r0], r0)) atomicMax(&top[r0], g.enc(v));
      if (live[k] && !same && b[k] > g.get(top[r[k]], r[k])) atomicMax(&top[r[k]], g.enc(b[k]));
    }
  }
}

// One hooking round over the unresolved light edges (Shiloach-Vishkin style, root =
// smallest id): both roots; equal -> resolved; else ONE attempt to hook the larger
// root under the smaller (CAS, succeeds only on a current root).  A failed attempt is
// not retried here: the edge goes to `out` for the next round.  Retrying in place made
// thousands of threads fight over a forming giant component's root (each failure =
// another round trip); rounds instead resolve such a pile-up in a few passes.
// (Batched finds of all the thread's edges before any hook left more hooks to later
// rounds: 21-22 ms against 10.8 ms at RMAT-26.)
// UP (sheep_tuning hook_up): the smaller root is hooked under the larger, so a component's
// root IS its top (its largest id) and k_light_top does not run.  Any hook direction leaves
// the same components; the forest stays a forest of ancestors (a link only ever attaches a
// root, path splitting only ever names an ancestor), so every read — stale or not — is an
// ancestor of x.  The maps keep the smaller root (a hub component's root is then the few low
// ids every hook agrees on; root = top measured 2x slower hooking there).
// BATCH (sheep_tuning hook_batch): the roots of all the thread's edges are found at once
// (2 x TILE_ITEMS chains in flight, find_many) and then hooked.  A root found this way may
// be stale by its turn — hook() then fails on the hi side and the edge goes to the next
// round, or links hi under a lo that is no longer a root, which joins the same tree — so
// the result is the same; it pays where the edges are chains (merges: one dependent load
// after another, little contention) and not where a forming hub component takes every
// hook (maps: more stale roots, more rounds).
template <bool BATCH, bool UP>
__global__ __launch_bounds__(BLOCK) void k_hook_round(const uint64_t *__restrict__ in, const uint64_t *__restrict__ n_in,
                                                      uint32_t *uf, Tg g, uint64_t *__restrict__ out,
                                                      unsigned long long *__restrict__ counter) {
  const uint64_t nin = *n_in;
  const uint64_t ntiles = (nin + TILE - 1) / TILE;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint64_t ev[TILE_ITEMS];
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < TILE_ITEMS; ++j) {
      const uint64_t i = tile * TILE + (uint64_t)j * BLOCK + threadIdx.x;
      ev[j] = i < nin ? in[i] : DEAD;
    }
    if (BATCH) {
      uint32_t r[2 * TILE_ITEMS];
      bool v[2 * TILE_ITEMS];
#pragma unroll
      for (int j = 0; j < TILE_ITEMS; ++j) {
        v[2 * j] = v[2 * j + 1] = ev[j] != DEAD;
        r[2 * j] = ev[j] != DEAD ? (uint32_t)ev[j] : 0;
        r[2 * j + 1] = ev[j] != DEAD ? (uint32_t)(ev[j] >> 32) : 0;
      }
      find_many<2 * TILE_ITEMS>(uf, g, r, v);
#pragma unroll
      for (int j = 0; j < TILE_ITEMS; ++j) {
        if (ev[j] == DEAD) continue;
        uint32_t a = r[2 * j], b = r[2 * j + 1];
        if (a == b) continue;
        const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
        if (!(UP ? hook(uf, g, lo, hi) : hook(uf, g, hi, lo))) keep |= 1u << j;
      }
    } else {
#pragma unroll
      for (int j = 0; j < TILE_ITEMS; ++j) {
        if (ev[j] == DEAD) continue;
        uint32_t a = (uint32_t)ev[j], b = (uint32_t)(ev[j] >> 32);
        find2(uf, g, a, b);
        if (a == b) continue;
        const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
        if (!(UP ? hook(uf, g, lo, hi) : hook(uf, g, hi, lo))) keep |= 1u << j;
      }
    }
    uint64_t slot = shard_reserve((uint32_t)__popc(keep), counter, tile, ntiles, 1);
#pragma unroll
    for (int j = 0; j < TILE_ITEMS; ++j)
      if (keep & (1u << j)) out[slot++] = ev[j];
  }
}

// The edges still unresolved after HOOK_ROUNDS rounds (few: the pile-ups are gone) are
// hooked in place, retrying until each one's roots agree.  Lock-free: a failed CAS
// means another hook made progress.
template <bool UP>
__global__ __launch_bounds__(BLOCK) void k_hook_finish(const uint64_t *__restrict__ src, const uint64_t *__restrict__ n_in,
                                                       const unsigned long long *__restrict__ counters, uint32_t *uf, Tg g,
                                                       uint64_t *__restrict__ n_left) {
  // the hook round's survivors straight from its shard regions (no pack launch): the
  // NSHARD counts' prefix in LDS, each entry's shard by binary search over it
  static_assert(NSHARD == WAVE, "one lane per shard counter");
  __shared__ uint64_t s_pre[NSHARD + 1];
  const uint64_t ntiles = (*n_in + TILE - 1) / TILE;
  if (threadIdx.x < WAVE) {
    const uint64_t c = counters[(uint64_t)threadIdx.x * SHARD_STRIDE];
    uint64_t inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t u = __shfl_up(inc, o, 64);
      if ((int)threadIdx.x >= o) inc += u;
    }
    s_pre[threadIdx.x + 1] = inc;
    if (threadIdx.x == 0) s_pre[0] = 0;
  }
  lds_barrier();
  const uint64_t nin = s_pre[NSHARD];
  if (blockIdx.x == 0 && threadIdx.x == 0) *n_left = nin;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nin; i += stride) {
    uint32_t lo = 0, hi = NSHARD;   // s_pre[lo] <= i < s_pre[hi]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (s_pre[mid] <= i) lo = mid; else hi = mid;
    }
    const uint64_t e = src[shard_base(ntiles, lo, 1) + (i - s_pre[lo])];
    uint32_t a = (uint32_t)e, b = (uint32_t)(e >> 32);
    for (;;) {
      find2(uf, g, a, b);
      if (a == b) break;
      const uint32_t l = a < b ? a : b, h = a < b ? b : a;
      if (UP ? hook(uf, g, l, h) : hook(uf, g, h, l)) break;
    }
  }
}

// For every cross edge (a,b): r = root of a's light component; m_r = min b (atomicMin).
__global__ __launch_bounds__(BLOCK) void k_cross_find(const uint64_t *__restrict__ lx, const uint64_t *__restrict__ st,
                                                      uint32_t *uf, uint32_t *__restrict__ mt, uint32_t *__restrict__ xtop,
                                                      Tg g) {
  const uint64_t nx = st[ST_NX];
  const uint64_t *__restrict__ xbuf = lx + st[ST_NL];   // the cross entries follow the light ones
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK * XK;
  const uint64_t iters = (nx + stride - 1) / stride;
  uint64_t base = (uint64_t)blockIdx.x * BLOCK * XK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, base += stride) {   // wave-uniform trip count (ballots)
    uint32_t t[XK], b[XK];
    bool cross[XK];
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      cross[k] = base + (uint64_t)k * BLOCK < nx;
      const uint64_t e = cross[k] ? xbuf[base + (uint64_t)k * BLOCK] : 0;
      t[k] = (uint32_t)e;
      b[k] = (uint32_t)(e >> 32);
    }
    find_many<XK>(uf, g, t, cross);
#pragma unroll
    for (int k = 0; k < XK; ++k)
      if (cross[k]) xtop[base + (uint64_t)k * BLOCK] = t[k];
    // Power-law graphs send most cross edges of a level to one giant component's top:
    // combine in the wave first (lanes sharing the first lane's top) and skip atomics a
    // plain read already shows useless (mt only decreases; a stale read is >= the true
    // value, so skipping stays exact; the tagged words compare the same way).  (Issuing
    // the other lanes' atomics without the read, as no-return atomics, cost 25x at
    // RMAT-28 and Chung-Lu, where lanes beside the first still hit hub tops.)
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      const uint64_t cm = __ballot(cross[k]);
      if (!cm) continue;
      const int first = __ffsll((unsigned long long)cm) - 1;
      const uint32_t t0 = __shfl(t[k], first, 64);
      const bool same = cross[k] && t[k] == t0;
      const uint32_t v = wave_min(same ? b[k] : INVALID);
      if ((int)__lane_id() == first && g.m_enc(v) < mt[t0]) atomicMin(&mt[t0], g.m_enc(v));
      if (cross[k] && !same && g.m_enc(b[k]) < mt[t[k]]) atomicMin(&mt[t[k]], g.m_enc(b[k]));
    }
  }
}

// k_cross_find with a workgroup-private window of mt in LDS.  The first levels' cross
// edges come from distinct, mostly singleton, low-degree left endpoints: every atomicMin
// hits its own line, and 64 lanes to 64 lines run ~17x slower than one contiguous
// wave-instruction (MI355X_MICROARCH.md, atomics).  The level's list keeps each edge group
// in lo-bucket order, so a workgroup's chunk of XW_CH edges mostly has its roots inside a
// 2^XW_BITS-position window starting at the chunk's smallest lo: their minima go to LDS
// and leave in one coalesced pass; roots outside the window take the global path.
// Used for the first XW_LEVELS levels only (RMAT-26, per level: 1.30 / 2.46 ms -> 0.77 /
// 1.16 ms; from level 2 on the light components have merged, fewer roots fall inside the
// window and the coarse chunks leave CUs idle: 1.60 -> 1.74 ms, later levels ~1.5x slower).
// A 2^14 window: 1.07 / 1.58 ms.
// (sheep_tuning cross_win_levels: how many levels, default 2)
constexpr int XW_BITS = 15, XWB = 1024, XW_ITEMS = 8;
constexpr uint32_t XW = 1u << XW_BITS;
constexpr uint64_t XW_STEP = (uint64_t)XWB * XW_ITEMS, XW_CH = XW_STEP * 8;
__global__ __launch_bounds__(XWB) void k_cross_find_win(const uint64_t *__restrict__ lx, const uint64_t *__restrict__ st,
                                                        uint32_t *uf, uint32_t *__restrict__ mt,
                                                        uint32_t *__restrict__ xtop, Tg g) {
  extern __shared__ uint32_t lmin[];
  uint32_t *const s_red = lmin + XW;   // (dynamic only: allow_full_lds admits no static LDS)
  const uint64_t nx = st[ST_NX];
  const uint64_t *__restrict__ xbuf = lx + st[ST_NL];
  // chunks of XW_STEP..XW_CH edges, so that even a short list spreads over the CUs
  // (RMAT-22's first levels: ~2M cross edges, 29 chunks of XW_CH)
  uint64_t ch = (nx / 1024 + XW_STEP - 1) / XW_STEP * XW_STEP;
  ch = ch < XW_STEP ? XW_STEP : ch > XW_CH ? XW_CH : ch;
  const uint64_t nchunks = (nx + ch - 1) / ch;
  for (uint64_t chunk = blockIdx.x; chunk < nchunks; chunk += gridDim.x) {   // uniform
    const uint64_t c0 = chunk * ch, c1 = c0 + ch < nx ? c0 + ch : nx;
    uint32_t mn = INVALID;
    for (uint64_t i = c0 + threadIdx.x; i < c1; i += XWB) {
      const uint32_t lo = (uint32_t)xbuf[i];
      mn = lo < mn ? lo : mn;
    }
    mn = wave_min(mn);
    __syncthreads();   // the previous chunk's flush is done with lmin and s_red
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = mn;
    for (uint32_t j = threadIdx.x; j < XW; j += XWB) lmin[j] = INVALID;
    __syncthreads();
    uint32_t w0 = INVALID;
    for (int w = 0; w < XWB / WAVE; ++w) w0 = s_red[w] < w0 ? s_red[w] : w0;
    for (uint64_t base = c0 + threadIdx.x; base < c0 + ch; base += XW_STEP) {   // uniform trip count
      uint32_t t[XW_ITEMS], b[XW_ITEMS];
      bool live[XW_ITEMS];
#pragma unroll
      for (int k = 0; k < XW_ITEMS; ++k) {
        const uint64_t i = base + (uint64_t)k * XWB;
        live[k] = i < c1;
        const uint64_t e = live[k] ? xbuf[i] : 0;
        t[k] = (uint32_t)e;
        b[k] = (uint32_t)(e >> 32);
      }
      find_many<XW_ITEMS>(uf, g, t, live);
      bool glob[XW_ITEMS];
#pragma unroll
      for (int k = 0; k < XW_ITEMS; ++k) {
        if (live[k]) xtop[base + (uint64_t)k * XWB] = t[k];
        const bool in = live[k] && t[k] - w0 < XW;
        if (in) atomicMin(&lmin[t[k] - w0], b[k]);
        glob[k] = live[k] && !in;
      }
#pragma unroll
      for (int k = 0; k < XW_ITEMS; ++k) {
        const uint64_t cm = __ballot(glob[k]);
        if (!cm) continue;
        const int first = __ffsll((unsigned long long)cm) - 1;
        const uint32_t t0 = __shfl(t[k], first, 64);
        const bool same = glob[k] && t[k] == t0;
        const uint32_t v = wave_min(same ? b[k] : INVALID);
        if ((int)__lane_id() == first && g.m_enc(v) < mt[t0]) atomicMin(&mt[t0], g.m_enc(v));
        if (glob[k] && !same && g.m_enc(b[k]) < mt[t[k]]) atomicMin(&mt[t[k]], g.m_enc(b[k]));
      }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < XW; j += XWB) {
      const uint32_t v = lmin[j];
      if (v == INVALID) continue;
      const uint32_t e = g.m_enc(v);
      if (e < mt[w0 + j]) atomicMin(&mt[w0 + j], e);
    }
  }
}

// Contract every cross edge (a,b) -> (m_r, b) where r = a's light component; drop it
// when b == m_r.  parent(top(r)) = m_r (jnode.h:158-162 adopt) is stored by k_level_clean
// in one pass over mt (tagged state) or here by the edges with b == m_r.  Dedup: claim[b] holds
// the m of a KEPT contraction (m, b); an edge that finds its own m_r there is a duplicate
// of it and dies.  An edge that finds no claim of this level is kept and stores its m
// with a plain store: only keepers ever store, so whatever value a later read returns —
// the last store, or another XCD's older one — names a kept edge.  (Exact: only equal
// (m_r, b) pairs die.  Lossy: edges racing on a fresh claim, or carrying a second
// distinct m, are kept without a check — the common duplicates, a giant component's many
// edges into one hub, all carry the same m.)  A compare-and-swap per first touch made
// every lane of the level's first wave of tiles queue on the hubs' words.  claim is
// n x u32, L3-resident, unlike a global hash table of the pairs.
//
// The surviving contractions are APPENDED to the next list, after the entries k_split
// kept: each 2048-edge tile reserves its survivors' slots in a sharded append (one
// atomic per tile on one of 64 counters) and k_pack moves the shard regions behind the
// kept entries, so the next level reads no dead slots (at RMAT-26 most contractions die
// as duplicates: 80% of a level's list was dead slots).  Every gather stage is issued
// for all of a thread's 8 edges before the next (xtop/xbuf, then mt, then claim).
__global__ __launch_bounds__(BLOCK) void k_cross_apply(const uint64_t *__restrict__ lx, const uint32_t *__restrict__ xtop,
                                                       const uint64_t *__restrict__ st, const uint32_t *__restrict__ mt,
                                                       const uint32_t *__restrict__ top, uint32_t *__restrict__ claim,
                                                       uint64_t *__restrict__ scratch,
                                                       unsigned long long *__restrict__ counters,
                                                       uint32_t *__restrict__ parent, Tg g, uint64_t n) {
  const uint64_t nx = st[ST_NX];
  const bool adopt_here = !g.on || sparse_adopt(nx, n);   // (uniform)
  const uint64_t *__restrict__ xbuf = lx + st[ST_NL];
  const uint64_t ntiles = (nx + TILE - 1) / TILE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint32_t r[TILE_ITEMS], b[TILE_ITEMS], m[TILE_ITEMS], cl[TILE_ITEMS];
    uint32_t keep = 0;
    // each wave takes a contiguous share of the tile, so the survivors can be appended in
    // input order (k_split_write: the next passes' gathers keep their locality)
    const uint64_t w0 = tile * TILE + (uint64_t)wave * (TILE_ITEMS * WAVE) + lane;
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; ++k) {
      const uint64_t j = w0 + (uint64_t)k * WAVE;
      const bool live = j < nx;
      r[k] = live ? xtop[j] : INVALID;
      b[k] = live ? (uint32_t)(xbuf[j] >> 32) : 0;
    }
    // every gather stage issued for all 8 edges before any word is decoded (a decode
    // inside each edge's branch serialised the loads: 2x slower at RMAT-22)
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; ++k) m[k] = mt[r[k] != INVALID ? r[k] : 0];
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; ++k) m[k] = r[k] != INVALID ? g.m_get(m[k]) : INVALID;
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; ++k) cl[k] = claim[b[k]];
    if (adopt_here) {   // untagged state, or a level with few cross edges (else k_level_clean)
#pragma unroll
      for (int k = 0; k < TILE_ITEMS; ++k)
        if (r[k] != INVALID && b[k] == m[k]) parent[g.get(top[r[k]], r[k])] = m[k];
    }
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; ++k) {
      if (r[k] == INVALID || b[k] == m[k]) continue;
      const uint32_t c = g.claim_get(cl[k]);
      if (c == m[k]) continue;   // a kept edge's (m, b): this one is its duplicate
      keep |= 1u << k;
      if (c == INVALID) claim[b[k]] = g.enc(m[k]);   // first seen this level: a plain store
    }
    uint32_t run = 0, rk[TILE_ITEMS];   // ranks in the wave's share (run: wave-uniform)
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; ++k) {
      const uint64_t q = __ballot((keep >> k) & 1);
      rk[k] = run + (uint32_t)__popcll(q & lt);
      run += (uint32_t)__popcll(q);
    }
    const uint64_t wbase = __shfl(shard_reserve(lane == 0 ? run : 0u, counters, tile, ntiles, 1), 0, 64);
#pragma unroll
    for (int k = 0; k < TILE_ITEMS; ++k)
      if (keep & (1u << k)) scratch[wbase + rk[k]] = ((uint64_t)b[k] << 32) | m[k];
  }
}

// ---- the level's split: three dense outputs --------------------------------------
// Count pass (per 2048-entry tile: entries that stay, light, cross), one scan of the
// three count rows, write pass (each tile re-read and written at its offsets).  Two
// reads per entry, but every pass streams at full occupancy; an ordered single pass
// (decoupled look-back) serialised on the chunk chain.

// Classes of an entry at level s (ya, yb = spread positions of lo, hi):
//   cross  (ya ^ yb) >> s == 1          -> the cross list (contracted by k_cross_apply)
//   light  same half, bit s of yb == 0  -> the light list, and it stays in the list
//   right  same half, bit s of yb == 1  -> stays in the list
// DEAD entries (contractions that died) are dropped.
// A range-restricted run (one part of a split merge, below) keeps, at the level where the
// subproblems become that fine, only the entries of its own subproblem: ya in [lo, hi).
struct YRange {
  uint32_t lo, hi;
  bool on;
};
__device__ __forceinline__ uint32_t classify(uint64_t e, int s, uint32_t clo, YRange yr) {
  if (e == DEAD) return 0;
  const uint32_t ya = spread((uint32_t)e, clo), yb = spread((uint32_t)(e >> 32), clo);
  if (yr.on && (ya < yr.lo || ya >= yr.hi)) return 0;
  const uint32_t d = (ya ^ yb) >> s;
  if (d == 1) return 4;                          // cross
  return ((yb >> s) & 1) == 0 ? 3 : 1;           // light (bit 1: light, bit 0: stays) / right
}

// The level's virtual input: the list (prev level's kept entries + contraction slots,
// then the top block's MSF edges when the previous level cut it), then the bucket of edges
// first active at this level (none below gcut: the groups of a cut top block).  After a
// cut, the list entries inside the top block (spread(lo) >= cut, ahead of the MSF edges)
// read as dead.
// CUT: the one level right after a cut (the level kernels are instantiated without the
// filter everywhere else: the extra test in every load cost the split ~50 % at RMAT-26).
template <bool CUT>
struct SplitIn {
  const uint64_t *list, *r0;
  uint64_t len, base, rb, m;
  uint32_t cut, clo;
  __device__ SplitIn(const uint64_t *l, const uint64_t *prev, const uint64_t *r, const uint64_t *seg, int s, int L,
                     int gcut, uint32_t c)
      : list(l), r0(r), clo(c) {
    base = prev ? prev[ST_KEPT] + prev[ST_CONTR] : 0;
    len = CUT ? base + prev[ST_EXTRA] : base;
    cut = CUT ? (uint32_t)prev[ST_CUT] : 0;
    rb = seg[s];
    m = len + (s < gcut ? 0 : seg[L + s] - rb);
  }
  __device__ __forceinline__ uint64_t operator[](uint64_t i) const {
    if (CUT && i < len) {
      const uint64_t e = list[i];
      return (i < base && e != DEAD && spread((uint32_t)e, clo) >= cut) ? DEAD : e;
    }
    return i < len ? list[i] : i < m ? r0[rb + (i - len)] : DEAD;
  }
};

// The split streams SPLIT_TILE-entry tiles (its own tiling: only its count rows depend on
// it): 16 entries per thread measured 7.2 against 7.9 ms at RMAT-26 (the kernels whose
// appends pack_shards moves stay at TILE, whose 16-item form slowed k_cross_apply).
constexpr int SPLIT_ITEMS = 16;
constexpr int SPLIT_TILE = BLOCK * SPLIT_ITEMS;

// the three class bits as three 16-bit counters
__device__ __forceinline__ uint64_t pack3(uint32_t c) {
  return (uint64_t)(c & 1) | ((uint64_t)((c >> 1) & 1) << 16) | ((uint64_t)(c >> 2) << 32);
}

template <bool CUT>
__global__ __launch_bounds__(BLOCK) void k_split_count(const uint64_t *__restrict__ list, const uint64_t *__restrict__ prev,
                                                       uint64_t *__restrict__ st, int s, uint32_t clo, YRange yr,
                                                       const uint64_t *__restrict__ r0, const uint64_t *__restrict__ seg,
                                                       int L, int gcut, uint64_t *__restrict__ cnt, LevelClean clean) {
  // the three count rows at stride ntiles (this level's), then one 0: scanned as one
  // exclusive scan of 3 ntiles + 1 entries (the length in st, read by the scan).
  // clean: the previous level's k_level_clean, run first (clean.st == nullptr: none).
  if (clean.st) level_clean(clean);
  const SplitIn<CUT> in(list, prev, r0, seg, s, L, gcut, clo);
  const uint64_t ntiles = (in.m + SPLIT_TILE - 1) / SPLIT_TILE, cstride = ntiles;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st[ST_LIVE] = in.len;
    st[ST_R0] = in.m - in.len;
    st[ST_SCANN] = 3 * ntiles + 1;
    cnt[3 * ntiles] = 0;
  }
  __shared__ uint64_t s_w[BLOCK / WAVE];
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint64_t ev[SPLIT_ITEMS];
#pragma unroll
    for (int j = 0; j < SPLIT_ITEMS; ++j) ev[j] = in[tile * SPLIT_TILE + (uint64_t)j * BLOCK + threadIdx.x];
    uint64_t c3 = 0;
#pragma unroll
    for (int j = 0; j < SPLIT_ITEMS; ++j) c3 += pack3(classify(ev[j], s, clo, yr));
    c3 = wave_sum(c3);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c3;
    lds_barrier();
    if (threadIdx.x < 3) {
      uint64_t t = 0;
      for (int w = 0; w < BLOCK / WAVE; ++w) t += s_w[w];
      cnt[threadIdx.x * cstride + tile] = (t >> (16 * threadIdx.x)) & 0xFFFF;
    }
    lds_barrier();
  }
}

// cnt: the three rows (stride ntiles, then a 0) scanned as ONE exclusive scan, so a
// row's offsets are relative to its first entry; the row totals go to st.  Each class's
// run of the tile is placed in LDS in INPUT order, then copied out by consecutive lanes
// (per-thread stores to the same positions: 16.6 against 12.2 ms).  Input order keeps a
// wave's lanes on neighbouring lo in the next passes' gathers: the thread-major order it
// replaced (a thread's 16 entries, 256 apart in the input, side by side) cost the hook
// round, the cross pass and the contractions 0.8 ms per RMAT-26 step.  Each wave takes a
// contiguous quarter of the tile and ranks it item by item with ballots (the running
// counts are wave-uniform: no LDS, no barrier); one barrier adds the waves' offsets.  (A
// rank over (item, wave) pairs, with the pairs' counts scanned in LDS: +0.28 ms.)
template <bool CUT>
__global__ __launch_bounds__(BLOCK) void k_split_write(const uint64_t *__restrict__ list, const uint64_t *__restrict__ prev,
                                                       uint64_t *__restrict__ st, int s, uint32_t clo, YRange yr,
                                                       const uint64_t *__restrict__ r0, const uint64_t *__restrict__ seg,
                                                       int L, int gcut, const uint64_t *__restrict__ cnt,
                                                       uint64_t *__restrict__ next, uint64_t *__restrict__ lx) {
  constexpr int NW = BLOCK / WAVE;
  constexpr uint32_t WCH = SPLIT_ITEMS * WAVE;   // a wave's contiguous share of the tile
  static_assert(WCH <= 1024, "10-bit ranks");
  const SplitIn<CUT> in(list, prev, r0, seg, s, L, gcut, clo);
  const uint64_t ntiles = (in.m + SPLIT_TILE - 1) / SPLIT_TILE, cstride = ntiles;
  const uint64_t b0 = cnt[0], b1 = cnt[cstride], b2 = cnt[2 * cstride], b3 = cnt[3 * cstride];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st[ST_KEPT] = b1 - b0;
    st[ST_NL] = b2 - b1;
    st[ST_NX] = b3 - b2;
  }
  __shared__ uint32_t s_w[NW][3];
  __shared__ uint64_t stg[SPLIT_TILE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t lt = lanemask_lt();
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint64_t ev[SPLIT_ITEMS];
    uint32_t cl[SPLIT_ITEMS], lr[SPLIT_ITEMS];   // class bits; the ranks in the wave's share, 3 x 10 bits
    const uint64_t w0 = tile * SPLIT_TILE + (uint64_t)wave * WCH + lane;
#pragma unroll
    for (int j = 0; j < SPLIT_ITEMS; ++j) ev[j] = in[w0 + (uint64_t)j * WAVE];
    uint32_t run0 = 0, run1 = 0, run2 = 0;   // wave-uniform
#pragma unroll
    for (int j = 0; j < SPLIT_ITEMS; ++j) {
      cl[j] = classify(ev[j], s, clo, yr);
      const uint64_t q0 = __ballot(cl[j] & 1), q1 = __ballot((cl[j] >> 1) & 1), q2 = __ballot((cl[j] >> 2) & 1);
      lr[j] = (run0 + (uint32_t)__popcll(q0 & lt)) | (run1 + (uint32_t)__popcll(q1 & lt)) << 10 |
              (run2 + (uint32_t)__popcll(q2 & lt)) << 20;
      run0 += (uint32_t)__popcll(q0);
      run1 += (uint32_t)__popcll(q1);
      run2 += (uint32_t)__popcll(q2);
    }
    if (lane == 0) {
      s_w[wave][0] = run0;
      s_w[wave][1] = run1;
      s_w[wave][2] = run2;
    }
    lds_barrier();
    uint32_t off[3] = {0, 0, 0}, tot[3] = {0, 0, 0};
#pragma unroll
    for (int w = 0; w < NW; ++w)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const uint32_t x = s_w[w][k];
        if (w < wave) off[k] += x;
        tot[k] += x;
      }
    // the stay run into `next`; the light and the cross runs into lx back to back: the one
    // scan of the three rows already places cross after light (offsets from the light row's start)
    uint64_t *const outs[3] = {next, lx, lx};
    const uint64_t obase[3] = {b0, b1, b1};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int j = 0; j < SPLIT_ITEMS; ++j)
        if ((cl[j] >> k) & 1) stg[off[k] + ((lr[j] >> (10 * k)) & 1023)] = ev[j];
      lds_barrier();
      uint64_t *const o = outs[k] + (cnt[k * cstride + tile] - obase[k]);
      for (uint32_t i = threadIdx.x; i < tot[k]; i += BLOCK) o[i] = stg[i];
      lds_barrier();   // stg (and, after the last class, s_w) is rewritten next
    }
  }
}

// ---- the last levels: Liu's algorithm per block -------------------------------------
// Below level B the subproblems are blocks of 2^B spread positions (at most as many
// vertices), independent of each other: every live edge has both ends in one block, and
// a vertex whose parent an earlier level assigned is a root of its block's elimination
// tree (it was the top of its light component, so every later neighbour it had lay in
// the other half and its edges there were contracted away).  So each block runs the
// reference's own sequential algorithm — Liu's, jtree.cpp:66-110 — on its edges sorted
// by hi: for each edge (a, v), r = find(a); if r != v, parent[r] = v and r links under v.
// ONE LANE per block, its union-find in LDS (one byte per vertex, lane l's entry x at
// x * 64 + l), so B levels of a dozen launches each become one launch.
// A block with more than FIN_HEAVY edges (a hub's block) is handed to a whole wave
// instead, which takes the edges of one hi 64 at a time.  Used for merges, whose edges
// (two parent edges per node plus contractions) spread evenly over the blocks.
constexpr int FIN_LANE_BITS = 8;   // lane-per-block: 2^8 one-byte entries x 64 lanes = 16 KB of LDS per wave
constexpr int FIN_BITS_MAX = 13;   // wave-per-block: 2^13 two-byte entries = 16 KB
constexpr uint64_t FIN_HEAVY = 256;

// (rb, re) = (seg[sg], seg[L]): the groups left, none when the top block's groups were
// replaced by its MSF (cut); at most cap entries are written (the caller checks *n_out)
__global__ void k_fin_gather(const uint64_t *__restrict__ list, const uint64_t *__restrict__ prev,
                             const uint64_t *__restrict__ r0, const uint64_t *__restrict__ seg, int sg, int L, bool cut,
                             uint64_t cap, uint64_t *__restrict__ out, uint64_t *__restrict__ n_out) {
  // out = list ++ r0[rb, re), halves swapped (lo << 32 | hi) so a sort on the low bits sorts by hi
  // (the top block is only ever cut above the finishing levels: prev carries no cut)
  const uint64_t re = seg[L], rb = cut ? re : seg[sg];
  const uint64_t len = prev ? prev[ST_KEPT] + prev[ST_CONTR] + prev[ST_EXTRA] : 0, m0 = len + (re - rb);
  const uint64_t m = m0 < cap ? m0 : cap;
  if (blockIdx.x == 0 && threadIdx.x == 0) *n_out = m0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
    const uint64_t e = i < len ? list[i] : r0[rb + (i - len)];
    out[i] = e == DEAD ? DEAD : (e << 32) | (e >> 32);
  }
}

// Block bounds and classes.  eb[b] = first sorted entry of block b (an entry's block is
// spread(hi) >> B; eb[nb] = first DEAD entry), found by binary search — live edges crowd
// into a fraction of the blocks, so boundary detection would leave single threads to
// fill long runs of empty ones.  vb[b] = first vertex of block b (vb[nb] = n), by
// boundary detection over the vertices (every block holds at least one).  Non-empty
// blocks go to the light list (one lane each) or, above FIN_HEAVY edges, the heavy list.
__global__ __launch_bounds__(BLOCK) void k_fin_bounds(const uint64_t *__restrict__ fin, const uint64_t *__restrict__ n_fin,
                                                      uint32_t clo, int B, uint64_t nb, uint64_t n,
                                                      uint64_t *__restrict__ eb, uint32_t *__restrict__ vb,
                                                      uint32_t *__restrict__ light, uint32_t *__restrict__ heavy,
                                                      unsigned long long *__restrict__ n_lh, uint64_t heavy_min) {
  const uint64_t nf = *n_fin;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t t0 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  auto lower = [&](uint64_t b) {   // first entry whose block is >= b (DEAD: block nb)
    uint64_t a = 0, z = nf;
    while (a < z) {
      const uint64_t x = (a + z) / 2;
      const uint64_t e = fin[x];
      const uint64_t eb_x = e == DEAD ? nb : spread((uint32_t)e, clo) >> B;
      if (eb_x < b) a = x + 1; else z = x;
    }
    return a;
  };
  const uint64_t iters = (nb + stride - 1) / stride;   // wave-uniform (appends below)
  for (uint64_t it = 0; it < iters; ++it) {
    const uint64_t b = t0 + it * stride;
    uint64_t e0 = 0, e1 = 0;
    if (b < nb) {
      e0 = lower(b);
      e1 = lower(b + 1);
      eb[b] = e0;
      if (b + 1 == nb) eb[nb] = e1;
    }
    const bool big = e1 - e0 > heavy_min, small = e1 > e0 && !big;
    const uint64_t sl = wave_append(small, n_lh), sh = wave_append(big, n_lh + 1);
    if (small) light[sl] = (uint32_t)b;
    if (big) heavy[sh] = (uint32_t)b;
  }
  auto vblk = [&](uint64_t x) -> uint64_t { return x >= n ? nb : spread((uint32_t)x, clo) >> B; };
  for (uint64_t x = t0; x <= n; x += stride) {
    const uint64_t lo = x ? vblk(x - 1) + 1 : 0, hi = vblk(x);
    for (uint64_t b = lo; b <= hi; ++b) vb[b] = (uint32_t)x;
  }
}

template <int B>
__global__ __launch_bounds__(WAVE) void k_fin_lanes(const uint64_t *__restrict__ fin, const uint64_t *__restrict__ eb,
                                                    const uint32_t *__restrict__ vb, const uint32_t *__restrict__ light,
                                                    const unsigned long long *__restrict__ n_light,
                                                    uint32_t *__restrict__ parent) {
  static_assert(B <= 8, "one-byte union-find entries");
  __shared__ uint8_t uf[(1 << B) * WAVE];
  const int l = threadIdx.x;
  const uint64_t j = (uint64_t)blockIdx.x * WAVE + l;
  if (j >= *n_light) return;
  const uint32_t b = light[j];
  const uint64_t e0 = eb[b], e1 = eb[b + 1];
  const uint32_t v0 = vb[b], cnt = vb[b + 1] - v0;
  for (uint32_t x = 0; x < cnt; ++x) uf[x * WAVE + l] = (uint8_t)x;
  // eight loads in flight per lane: the lanes walk distinct ranges, so each load is a miss
  for (uint64_t p = e0; p < e1; p += 8) {
    uint64_t ev[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) ev[k] = p + k < e1 ? fin[p + k] : DEAD;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (ev[k] == DEAD) break;
      const uint32_t v = (uint32_t)ev[k] - v0;
      uint32_t x = (uint32_t)(ev[k] >> 32) - v0;
      if (x >= cnt || v >= cnt) continue;   // both ends lie in the block (the D&C invariant)
      uint32_t px = uf[x * WAVE + l];
      while (px != x) {   // path halving
        const uint32_t g = uf[px * WAVE + l];
        uf[x * WAVE + l] = (uint8_t)g;
        x = g;
        px = uf[x * WAVE + l];
      }
      if (x != v) {
        parent[v0 + x] = v0 + v;
        uf[x * WAVE + l] = (uint8_t)v;
      }
    }
  }
}

template <typename U> __device__ __forceinline__ uint32_t fin_find(U *uf, uint32_t x) {
  uint32_t p = uf[x];
  while (p != x) {   // path halving (pointers only move up: safe with other lanes)
    const uint32_t g = uf[p];
    uf[x] = (U)g;
    x = g;
    p = uf[x];
  }
  return x;
}

// A heavy block (and every block when B > FIN_LANE_BITS): one wave, its edges staged
// through LDS FIN_STAGE at a time (coalesced), then taken one hi at a time, 64 edges per
// step.  Lanes with the same root store the same link; distinct roots link under v side
// by side, as Liu's loop over v's neighbours would.  Entries: one byte up to 2^8
// positions, two bytes above.
constexpr int FIN_STAGE = 1024;
template <int B>
__global__ __launch_bounds__(WAVE) void k_fin_heavy(const uint64_t *__restrict__ fin, const uint64_t *__restrict__ eb,
                                                    const uint32_t *__restrict__ vb, const uint32_t *__restrict__ heavy,
                                                    const unsigned long long *__restrict__ n_heavy,
                                                    uint32_t *__restrict__ parent) {
  using U = typename std::conditional<(B <= 8), uint8_t, uint16_t>::type;
  __shared__ U uf[1 << B];
  __shared__ uint64_t stage[FIN_STAGE];
  const int lane = threadIdx.x;
  const unsigned long long nh = *n_heavy;
  for (uint64_t h = blockIdx.x; h < nh; h += gridDim.x) {
    const uint32_t b = heavy[h];
    const uint32_t v0 = vb[b], cnt = vb[b + 1] - v0;
    const uint64_t e0 = eb[b], e1 = eb[b + 1];
    lds_barrier();   // the previous block is done with uf and stage
    for (uint32_t i = lane; i < cnt; i += WAVE) uf[i] = (U)i;
    for (uint64_t base = e0; base < e1; base += FIN_STAGE) {
      const uint32_t len = (uint32_t)(e1 - base < FIN_STAGE ? e1 - base : FIN_STAGE);
      lds_barrier();
      for (uint32_t i = lane; i < len; i += WAVE) stage[i] = fin[base + i];
      lds_barrier();
      for (uint32_t p = 0; p < len;) {
        const uint32_t v = (uint32_t)stage[p];
        const uint32_t idx = p + lane;
        const uint64_t e = idx < len ? stage[idx] : DEAD;
        const bool mine = e != DEAD && (uint32_t)e == v;
        const uint64_t mask = __ballot(mine);
        const uint32_t x = (uint32_t)(e >> 32) - v0, vv = v - v0;
        if (mine && x < cnt && vv < cnt) {
          const uint32_t r = fin_find<U>(uf, x);
          if (r != vv) {
            parent[v0 + r] = v;
            uf[r] = (U)vv;
          }
        }
        lds_barrier();   // this v's links before the next v's finds
        p += __popcll(mask);   // v's entries are a prefix of the window (sorted by hi)
      }
    }
  }
}

// The last B levels of a block as the same divide and conquer, inside ONE workgroup:
// its union-find, component tops, right-half minima and claims in LDS (B <= 13: 112 KB),
// its list in global scratch as local (lo | hi << 16) words, ping-ponged between two
// buffers over the block's own range.  Per level s: (1) hook the light edges (both ends in
// the left half: CAS on the LDS roots, root = smaller id), (2) top[root] = max hi over
// the light edges and mt[root] = min hi over the cross edges, (3) parent(top(r)) = m_r for
// every root with a cross edge, and the next list = the entries that stay plus the
// contractions (m_r, b) with b != m_r, first-seen (m, b) per b kept (the claim rule of
// k_cross_apply).  Unlike Liu's sweep (k_fin_heavy: one step per hi), the work of a level
// spreads over the workgroup, so blocks can be large enough to take the last global
// levels too.  Workgroups take blocks from a ticket (largest lists need not come first:
// the blocks are short against the grid).
constexpr int FDC_T = 1024, FDC_U = 4;
__device__ __forceinline__ uint32_t dc_find(uint32_t *uf, uint32_t x) {
  for (;;) {   // path halving (pointers only move toward the root: safe beside other threads)
    const uint32_t p = uf[x];
    if (p == x) return x;
    const uint32_t g = uf[p];
    if (g == p) return p;
    uf[x] = g;
    x = g;
  }
}
// blocks whose list fits run it from LDS: the budget keeps two workgroups per CU up to
// B = 12 (14 B of state per position) and one above
constexpr uint32_t fdc_lcap(int B) {
  return (uint32_t)(((B >= 13 ? 160 * 1024 - 1024 : 80 * 1024 - 512) - 14 * (1 << B)) / 8);
}
template <int B>
__global__ __launch_bounds__(FDC_T) void k_fin_dc(const uint64_t *__restrict__ fin, const uint64_t *__restrict__ eb,
                                                  const uint32_t *__restrict__ vb, const uint32_t *__restrict__ blocks,
                                                  const unsigned long long *__restrict__ n_blocks,
                                                  const uint32_t *__restrict__ blocks2,
                                                  const unsigned long long *__restrict__ n_blocks2, uint32_t clo,
                                                  uint32_t *__restrict__ buf, uint64_t cap,
                                                  unsigned long long *__restrict__ ticket, uint32_t *__restrict__ parent) {
  constexpr uint32_t NV = 1u << B, MASK = NV - 1;
  __shared__ uint32_t uf[NV], top[NV], mt[NV];
  __shared__ uint16_t claim[NV];
  constexpr uint32_t LCAP = fdc_lcap(B);
  // static LDS: 14 B of state per position, the two list buffers and the scalars below
  static_assert(14u * NV + 8u * LCAP + 64u <= 160u * 1024u, "k_fin_dc's LDS exceeds 160 KiB");
  __shared__ uint32_t lbuf[2][LCAP];
  __shared__ unsigned s_cnt[3];   // [0], [1]: the levels' next lists by parity; [2]: the block's load
  __shared__ unsigned s_roots;
  __shared__ uint64_t s_w;
  const unsigned long long nbk = *n_blocks, nbk2 = *n_blocks2;   // the long lists first, then the short ones
  const uint32_t lane = threadIdx.x & 63;
  for (;;) {
    if (threadIdx.x == 0) s_w = atomicAdd(ticket, 1ull);
    __syncthreads();
    const uint64_t w = s_w;
    if (w >= nbk + nbk2) break;   // (uniform)
    const uint32_t b = w < nbk ? blocks[w] : blocks2[w - nbk];
    const uint32_t v0 = vb[b], cnt = vb[b + 1] - v0;
    const uint64_t e0 = eb[b], e1 = eb[b + 1];
    const uint32_t yb0 = (uint32_t)(((uint64_t)b) << B);
    auto ly = [&](uint32_t x) { return spread(v0 + x, clo) - yb0; };   // offset inside the block
    const bool in_lds = e1 - e0 <= LCAP;   // (a level's list never outgrows its input)
    uint32_t *cur = in_lds ? lbuf[0] : buf + e0, *nxt = in_lds ? lbuf[1] : buf + cap + e0;
    uint32_t n = 0;
    bool loaded = false;
    if (!in_lds) {
      // A list past LDS (a dense block): round 0 of Borůvka first, as for the top block —
      // every position's lowest lower neighbour (mt) and a has-upper-neighbour flag (top);
      // when at most one root has an edge the block is one tree and its edges become its
      // minimum spanning forest {(minlo(x), x)} (etree(G) = etree(MSF(G))): <= cnt - 1 words.
      for (uint32_t x = threadIdx.x; x < cnt; x += FDC_T) {
        mt[x] = INVALID;
        top[x] = 0;
      }
      if (threadIdx.x == 0) s_cnt[2] = s_roots = 0;
      __syncthreads();
      const uint32_t ne = (uint32_t)(e1 - e0);
      for (uint32_t i0 = threadIdx.x; i0 < ne; i0 += FDC_U * FDC_T) {
        uint64_t ev[FDC_U];
#pragma unroll
        for (int j = 0; j < FDC_U; ++j) ev[j] = i0 + j * FDC_T < ne ? fin[e0 + i0 + j * FDC_T] : DEAD;
#pragma unroll
        for (int j = 0; j < FDC_U; ++j) {
          if (ev[j] == DEAD) continue;
          const uint32_t l = (uint32_t)(ev[j] >> 32) - v0, h = (uint32_t)ev[j] - v0;
          if (l >= cnt || h >= cnt || l >= h) continue;
          if (l < mt[h]) atomicMin(&mt[h], l);
          if (!top[l]) top[l] = 1;
        }
      }
      __syncthreads();
      for (uint32_t x0 = 0; x0 < cnt; x0 += FDC_T) {   // non-roots, and roots with an edge (wave-counted)
        const uint32_t x = x0 + threadIdx.x;
        const bool nonroot = x < cnt && mt[x] != INVALID, eroot = x < cnt && !nonroot && top[x];
        const uint64_t ma = __ballot(nonroot), mb = __ballot(eroot);
        if (lane == 0 && ma) atomicAdd(&s_cnt[2], (unsigned)__popcll(ma));
        if (lane == 0 && mb) atomicAdd(&s_roots, (unsigned)__popcll(mb));
      }
      __syncthreads();
      if (s_roots <= 1) {   // (uniform)
        if (s_cnt[2] <= LCAP) {
          cur = lbuf[0];
          nxt = lbuf[1];
        }
        __syncthreads();   // s_cnt[2] read by all
        if (threadIdx.x == 0) s_cnt[2] = 0;
        __syncthreads();
        for (uint32_t x0 = 0; x0 < cnt; x0 += FDC_T) {
          const uint32_t x = x0 + threadIdx.x;
          const bool keep = x < cnt && mt[x] != INVALID;
          const uint32_t word = keep ? mt[x] | (x << 16) : 0;
          const uint64_t km = __ballot(keep);
          uint32_t base = 0;
          if (km && lane == (uint32_t)(__ffsll((unsigned long long)km) - 1)) base = atomicAdd(&s_cnt[2], (unsigned)__popcll(km));
          base = __shfl(base, __ffsll((unsigned long long)(km ? km : 1)) - 1, 64);
          if (keep) cur[base + __popcll(km & lanemask_lt())] = word;
        }
        __syncthreads();
        n = s_cnt[2];
        loaded = true;
      }
    }
    if (!loaded) {   // the block's entries (lo << 32 | hi, swapped by k_fin_gather) as local words
      if (threadIdx.x == 0) s_cnt[2] = 0;
      __syncthreads();
      const uint32_t ne = (uint32_t)(e1 - e0);
      for (uint32_t i0 = 0; i0 < ne; i0 += FDC_T) {
        const uint32_t i = i0 + threadIdx.x;
        uint32_t word = 0;
        bool keep = false;
        if (i < ne) {
          const uint64_t e = fin[e0 + i];
          const uint32_t l = (uint32_t)(e >> 32) - v0, h = (uint32_t)e - v0;
          keep = e != DEAD && l < cnt && h < cnt && l < h;   // both ends lie in the block (the D&C invariant)
          word = l | (h << 16);
        }
        const uint64_t km = __ballot(keep);
        uint32_t base = 0;
        if (km && lane == (uint32_t)(__ffsll((unsigned long long)km) - 1)) base = atomicAdd(&s_cnt[2], (unsigned)__popcll(km));
        base = __shfl(base, __ffsll((unsigned long long)(km ? km : 1)) - 1, 64);
        if (keep) cur[base + __popcll(km & lanemask_lt())] = word;
      }
      __syncthreads();
      n = s_cnt[2];
    }
    for (int s = B - 1; s >= 0 && n; --s) {
      const int par = s & 1;
      for (uint32_t x = threadIdx.x; x < cnt; x += FDC_T) {
        uf[x] = x;
        top[x] = x;
        mt[x] = INVALID;
        claim[x] = 0xFFFF;
      }
      if (threadIdx.x == 0) s_cnt[par] = 0;
      __syncthreads();
      // the list's words FDC_U per thread in flight before any is used (a long block's
      // list is in HBM: one latency per word would serialise its passes)
      auto each = [&](auto &&f) {
        for (uint32_t i0 = threadIdx.x; i0 < n; i0 += FDC_U * FDC_T) {
          uint32_t u[FDC_U];
#pragma unroll
          for (int j = 0; j < FDC_U; ++j) u[j] = i0 + j * FDC_T < n ? cur[i0 + j * FDC_T] : 0xFFFFFFFFu;
#pragma unroll
          for (int j = 0; j < FDC_U; ++j)
            if (u[j] != 0xFFFFFFFFu) f(u[j]);
        }
      };
      each([&](uint32_t u) {   // (1) light edges
        const uint32_t l = u & 0xFFFF, h = u >> 16;
        const uint32_t ya = ly(l), yb = ly(h);
        if (((ya ^ yb) >> s) != 0 || ((yb >> s) & 1)) return;
        uint32_t a = l, c2 = h;
        for (;;) {
          a = dc_find(uf, a);
          c2 = dc_find(uf, c2);
          if (a == c2) break;
          const uint32_t lo = a < c2 ? a : c2, hi = a < c2 ? c2 : a;
          if (atomicCAS(&uf[hi], hi, lo) == hi) break;
        }
      });
      __syncthreads();
      each([&](uint32_t u) {   // (2) tops and minima
        const uint32_t l = u & 0xFFFF, h = u >> 16;
        const uint32_t ya = ly(l), yb = ly(h), d = (ya ^ yb) >> s;
        if (d == 0 && ((yb >> s) & 1)) return;   // right half: untouched
        const uint32_t r = dc_find(uf, l);
        if (d == 0) {
          if (h > top[r]) atomicMax(&top[r], h);
        } else if (h < mt[r]) {
          atomicMin(&mt[r], h);
        }
      });
      __syncthreads();
      for (uint32_t x = threadIdx.x; x < cnt; x += FDC_T)   // (3) adoption
        if (mt[x] != INVALID) parent[v0 + top[x]] = v0 + mt[x];
      for (uint32_t i0 = 0; i0 < n; i0 += FDC_U * FDC_T) {   // (3) the next list (wave-uniform trips: ballots)
        uint32_t u[FDC_U];
#pragma unroll
        for (int j = 0; j < FDC_U; ++j) {
          const uint32_t i = i0 + j * FDC_T + threadIdx.x;
          u[j] = i < n ? cur[i] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int j = 0; j < FDC_U; ++j) {
          bool keep = false;
          uint32_t word = 0;
          if (u[j] != 0xFFFFFFFFu) {
            const uint32_t l = u[j] & 0xFFFF, h = u[j] >> 16;
            const uint32_t ya = ly(l), yb = ly(h), d = (ya ^ yb) >> s;
            if (d == 0) {
              keep = true;
              word = u[j];
            } else {
              const uint32_t m = mt[dc_find(uf, l)];
              if (h != m) {
                const uint32_t cl = claim[h];
                if (cl != m) {
                  keep = true;
                  word = m | (h << 16);
                  if (cl == 0xFFFF) claim[h] = (uint16_t)m;   // first seen: a plain store (k_cross_apply's rule)
                }
              }
            }
          }
          const uint64_t km = __ballot(keep);
          uint32_t base = 0;
          if (km && lane == (uint32_t)(__ffsll((unsigned long long)km) - 1)) base = atomicAdd(&s_cnt[par], (unsigned)__popcll(km));
          base = __shfl(base, __ffsll((unsigned long long)(km ? km : 1)) - 1, 64);
          if (keep) nxt[base + __popcll(km & lanemask_lt())] = word;
        }
      }
      __syncthreads();
      n = s_cnt[par];
      uint32_t *t = cur;
      cur = nxt;
      nxt = t;
    }
    __syncthreads();   // LDS and s_w are reused by the next block
  }
}

// ---- merge input ------------------------------------------------------------------
// K trees: tree 0 at t0, tree k >= 1 at t1 + (k - 1) * stride (two separate trees, or K
// stacked ones).  Node i contributes its DISTINCT parents over the K trees as edges
// (parent << 32 | i), compacted in node order — so the edges come sorted by lo and the
// first-activity groups are ranges of them (seg from the node offsets, k_seg_at).  The
// parents are deduplicated in registers; most of the K x n slots are empty or repeats
// (RMAT-26, 8 shard trees: ~47M edges in 262M slots), which the levels no longer read.
// Or parent planes (planes != nullptr): tree k's parents at planes + k * stride (u32 each)
// with the trees' pst already summed in pst_sum — the form the multi-GPU reduce gathers
// (half the bytes of whole trees; the pst sum travels as one RCCL reduce).
struct TreeSet {
  const sheep_jnode *t0, *t1;
  uint64_t stride;
  const uint32_t *planes = nullptr, *pst_sum = nullptr;
  __device__ __forceinline__ const sheep_jnode *at(uint32_t k) const { return k == 0 ? t0 : t1 + (uint64_t)(k - 1) * stride; }
};
constexpr uint32_t MERGE_KMAX = 64;   // trees per pass (a larger K is merged in passes)

// p[k] = node i's parent in tree k, INVALID when absent or equal to an earlier tree's;
// returns the summed pst weight.  A parent that is not a later node of the tree flags bad.
template <int KM>
__device__ __forceinline__ uint32_t tree_parents(const TreeSet &ts, uint32_t K, uint64_t n, uint64_t i,
                                                 uint32_t (&p)[KM], bool &bad) {
  uint32_t w = 0;
  if (ts.planes) {
    w = ts.pst_sum[i];
#pragma unroll
    for (int k = 0; k < KM; ++k) p[k] = (uint32_t)k < K ? ts.planes[(uint64_t)k * ts.stride + i] : INVALID;
  } else {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      p[k] = INVALID;
      if ((uint32_t)k < K) {
        const sheep_jnode x = ts.at(k)[i];
        w += x.pst_weight;
        p[k] = x.parent;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    // a parent must be a later, existing node (jnode.cpp kids(current) via makeKids)
    if (p[k] != INVALID && (p[k] <= i || p[k] >= n)) {
      bad = true;
      p[k] = INVALID;
    }
#pragma unroll
    for (int j = 0; j < k; ++j)
      if (p[j] == p[k]) p[k] = INVALID;
  }
  return w;
}

template <int KM>
__global__ __launch_bounds__(BLOCK) void k_tree_count(TreeSet ts, uint32_t K, uint64_t n, uint32_t *__restrict__ cnt,
                                                      uint32_t *__restrict__ pst_out, unsigned long long *__restrict__ err) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    uint32_t p[KM];
    pst_out[i] = tree_parents<KM>(ts, K, n, i, p, bad);
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < KM; ++k) c += p[k] != INVALID;
    cnt[i] = c;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(err, 1ull);
}

template <int KM>
__global__ __launch_bounds__(BLOCK) void k_tree_write(TreeSet ts, uint32_t K, uint64_t n, const uint32_t *__restrict__ off,
                                                      uint64_t *__restrict__ edges) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    uint32_t p[KM];
    tree_parents<KM>(ts, K, n, i, p, bad);
    uint64_t o = off[i];
#pragma unroll
    for (int k = 0; k < KM; ++k)
      if (p[k] != INVALID) edges[o++] = ((uint64_t)p[k] << 32) | (uint32_t)i;
  }
}

// seg[j] = off[node[j]]: the first-activity group bounds of lo-sorted edges.
struct SegNodes { uint32_t node[64]; };
__global__ void k_seg_at(const uint32_t *__restrict__ off, SegNodes sn, int cnt, uint64_t *__restrict__ seg) {
  if ((int)threadIdx.x < cnt) seg[threadIdx.x] = off[sn.node[threadIdx.x]];
}

// a tree's parents and pst as two planes (the multi-GPU reduce's send buffers)
__global__ void k_tree_planes(const sheep_jnode *__restrict__ tree, uint64_t n, uint32_t *__restrict__ parent,
                              uint32_t *__restrict__ pst) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    const sheep_jnode j = tree[i];
    parent[i] = j.parent;
    pst[i] = j.pst_weight;
  }
}

__global__ void k_pack_tree(const uint32_t *__restrict__ parent, const uint32_t *__restrict__ pst, uint64_t n,
                            sheep_jnode *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    sheep_jnode j;
    j.parent = parent[i];
    j.pst_weight = pst[i];
    out[i] = j;
  }
}

// ---- the dense top block: its minimum spanning forest in place of its edges -----------
// After the level that splits at s = TB, the block of the 2^TB highest spread positions is
// a subproblem of its own: every live edge with lo in it lies inside it — the groups
// 0..TB-1 (exactly the edges whose lo is in the block) and the list entries (contractions)
// that landed there.  On power-law graphs it is the hub core, and the later levels spend
// most of their time re-hooking it (RMAT-26: 50.8 M of the 75.4 M live edges after s = 15
// sit in its 2^15 positions; the next largest block holds < 1 M).  The elimination tree of
// a graph is that of ANY minimum spanning forest of it under the weight hi (etree(G) =
// etree(MSF(G)): parent(x) is the first t > x at which x's component in the threshold
// graph G_t grows, and every MSF keeps the components of every G_t).  So the block's edges
// are replaced by their MSF under the total order (hi, lo) — the edge word itself — found
// by Borůvka rounds with the block's labels in LDS (u16: <= 2^15 vertices).  Dense blocks
// converge in a few rounds (RMAT-22's top 2^15: 3); every round at least halves the
// components that have an outgoing edge, so TB + 1 rounds always finish.
// the map's cut: blocks of 2^16 positions (RMAT-26 k=64, etree ms: 2^15 32.59 with the cut
// 0.55; 2^16 32.15 / 0.81; 8 shard maps 77.0 -> 76.6): sheep_tuning top_bits (default 16).
constexpr int TOP_BITS_MAX = 16;            // u16 labels: <= 65536 vertices
// the top block and the dense blocks right below it, at most top_blocks in all (RMAT-26 k=64, etree
// ms: no cut 34.5; 1 block 34.1; 4 blocks 33.8; 8 blocks 33.8 — with the 10-bit finish below)
constexpr int TOPB = 1024;                  // threads per workgroup of the top-block kernels
constexpr int TOP_WG = 256;                 // workgroups per block of the LDS edge passes (one per CU)
constexpr uint32_t TOP_HOOK_LDS = 1u << 15; // hooks: par and cid in LDS up to this many components (par alone
                                            // up to 2^16, with cid in HBM); round 0: u32 minima up to this
constexpr size_t TOP_ROUND_LDS = 144 * 1024; // a round's dynamic LDS: the labels, then the minima
constexpr uint64_t TOP_DENSE = 16;          // used when the block's groups hold >= 16 edges per vertex
constexpr uint64_t NO_EDGE = ~0ull;

struct TopState {
  uint32_t *minlo;                  // round 0: per vertex, its lowest lower neighbour (block-local id)
  unsigned *hasup;                  // round 0: per vertex a bit, set when it has an upper neighbour
  uint16_t *comp;                   // per vertex: its component's id
  unsigned long long *best;         // per component: the smallest edge word leaving it
  unsigned *scal;                   // [0] components, [1] a round saw an inter-component edge, [2] done
  uint64_t *st;                     // the cut level's stats row (ST_EXTRA: edges written so far)
  uint64_t *out;                    // the MSF edges go to out[st[KEPT] + st[CONTR] + ...] (the next list)
  uint16_t *gcid;                   // cid of a hook over more than TOP_HOOK_LDS components
  uint32_t v0, V;                   // the block's first vertex and its vertex count
};

// The block's edges: the list entries the extraction moved out (sharded append regions,
// st[ST_TOPNT] = the extraction's tile count) followed by groups [g0, g1) of r0.
struct TopEdges {
  const uint64_t *tl;
  const unsigned long long *tcnt;
  const uint64_t *r0;
  uint64_t g0, g1;
};
constexpr int TOP_NB_MAX = 9;   // the top block and up to 8 below it
// Every cut block in one launch: block b is blockIdx.y of the edge kernels and blockIdx.x of
// the one-workgroup hooks, so the blocks' passes overlap instead of queueing one behind another.
struct TopSet {
  TopState s[TOP_NB_MAX];
  TopEdges e[TOP_NB_MAX];
};

__device__ __forceinline__ void top_prefix(const TopEdges &te, uint64_t *s_pre) {
  if (threadIdx.x < WAVE) {
    uint64_t inc = te.tcnt[(uint64_t)threadIdx.x * SHARD_STRIDE];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t u = __shfl_up(inc, o, 64);
      if ((int)threadIdx.x >= o) inc += u;
    }
    s_pre[threadIdx.x + 1] = inc;
    if (threadIdx.x == 0) s_pre[0] = 0;
  }
}
__device__ __forceinline__ uint64_t top_list_at(const TopEdges &te, const uint64_t *s_pre, uint64_t ntiles, uint64_t i) {
  uint32_t a = 0, b = NSHARD;   // s_pre[a] <= i < s_pre[b]
  while (b - a > 1) {
    const uint32_t mid = (a + b) / 2;
    if (s_pre[mid] <= i) a = mid; else b = mid;
  }
  return te.tl[shard_base(ntiles, a, 1) + (i - s_pre[a])];
}

// Calls f(e) for the block's edges in [b0, b1) of its index space (the list entries, then
// the groups), `nt` threads striding.  The group part (nearly all of a dense block) is read
// TOP_U words ahead per thread: the top-block passes run one 1024-thread workgroup per CU,
// so without the unrolled loads every wave waits out one HBM latency per edge.
constexpr int TOP_U = 8;
template <typename F>
__device__ __forceinline__ void top_edges(const TopEdges &te, const uint64_t *s_pre, uint64_t ntiles, uint64_t b0,
                                          uint64_t b1, uint32_t t, uint32_t nt, F &&f) {
  const uint64_t nl = s_pre[NSHARD];
  const uint64_t le = b1 < nl ? b1 : nl;
  for (uint64_t i0 = b0 + t; i0 < le; i0 += (uint64_t)TOP_U * nt) {   // TOP_U list entries in flight
    uint64_t e[TOP_U];
#pragma unroll
    for (int j = 0; j < TOP_U; ++j) {
      const uint64_t i = i0 + (uint64_t)j * nt;
      e[j] = i < le ? top_list_at(te, s_pre, ntiles, i) : DEAD;
    }
#pragma unroll
    for (int j = 0; j < TOP_U; ++j) f(e[j]);
  }
  const uint64_t g0 = (b0 > nl ? b0 : nl) - nl, g1 = b1 > nl ? b1 - nl : 0;   // group-part range
  const uint64_t *r = te.r0 + te.g0;
  uint64_t i = g0 + t;
  for (; i + (uint64_t)(TOP_U - 1) * nt < g1; i += (uint64_t)TOP_U * nt) {
    uint64_t e[TOP_U];
#pragma unroll
    for (int j = 0; j < TOP_U; ++j) e[j] = __builtin_nontemporal_load(r + i + (uint64_t)j * nt);
#pragma unroll
    for (int j = 0; j < TOP_U; ++j) f(e[j]);
  }
  for (; i < g1; i += nt) f(r[i]);
}

// The list entries of the cut blocks, one pass: block 0 = spread(lo) >= cut0 (the top
// block), block j >= 1 = [cut0 - j 2^bits, cut0 - (j - 1) 2^bits); block j's entries go to
// region j of tl (sharded appends on counter set j).  st[ST_TOPNT] = the pass's tile count.
constexpr uint64_t TOP_CSET = (uint64_t)NSHARD * SHARD_STRIDE;
__global__ __launch_bounds__(BLOCK) void k_top_extract_multi(const uint64_t *__restrict__ list, uint64_t *__restrict__ st,
                                                             uint32_t cut0, int bits, uint32_t nb, uint32_t clo,
                                                             uint64_t *__restrict__ tl, uint64_t tcap,
                                                             unsigned long long *__restrict__ tcnt) {
  const uint64_t nl = st[ST_KEPT] + st[ST_CONTR];
  const uint64_t ntiles = (nl + TILE - 1) / TILE;
  if (blockIdx.x == 0 && threadIdx.x == 0) st[ST_TOPNT] = ntiles;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint64_t ev[TILE_ITEMS];
    uint32_t blk[TILE_ITEMS];
#pragma unroll
    for (int j = 0; j < TILE_ITEMS; ++j) {
      const uint64_t i = tile * TILE + (uint64_t)j * BLOCK + threadIdx.x;
      ev[j] = i < nl ? list[i] : DEAD;
      blk[j] = nb;
      if (ev[j] != DEAD) {
        const uint32_t y = spread((uint32_t)ev[j], clo);
        blk[j] = y >= cut0 ? 0u : 1u + ((cut0 - 1 - y) >> bits);
      }
    }
    for (uint32_t b = 0; b < nb; ++b) {   // (uniform: every thread takes part in each reserve)
      uint32_t keep = 0;
#pragma unroll
      for (int j = 0; j < TILE_ITEMS; ++j) keep |= (blk[j] == b ? 1u : 0u) << j;
      if (!__syncthreads_or(keep != 0)) continue;
      uint64_t slot = shard_reserve((uint32_t)__popc(keep), tcnt + b * TOP_CSET, tile, ntiles, 1);
#pragma unroll
      for (int j = 0; j < TILE_ITEMS; ++j)
        if (keep & (1u << j)) tl[b * tcap + slot++] = ev[j];
    }
  }
}

// cnt[b] = the extraction's entries of block b (its 64 shard counters summed)
__global__ void k_top_sum_counts(const unsigned long long *__restrict__ tcnt, uint32_t nb,
                                 unsigned long long *__restrict__ cnt) {
  const uint32_t b = blockIdx.x, k = threadIdx.x;   // one wave per block
  unsigned long long v = k < NSHARD ? tcnt[b * TOP_CSET + (uint64_t)k * SHARD_STRIDE] : 0;
  v = wave_sum(v);
  if (k == 0 && b < nb) cnt[b] = v;
}

__global__ __launch_bounds__(BLOCK) void k_top_init(TopSet t) {
  const TopState &ts = t.s[blockIdx.y];
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < ts.V; v += stride) {
    ts.minlo[v] = INVALID;
    ts.best[v] = NO_EDGE;
    if (v % 32 == 0) ts.hasup[v / 32] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x < 3) ts.scal[threadIdx.x] = 0;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) ts.st[ST_EXTRA] = 0;
}

__global__ void k_set_u64(uint64_t *p, uint64_t v) { *p = v; }

// Round 0 hooks every vertex with a lower neighbour along its smallest incident edge under
// (hi, lo): (minlo(v), v).  Any set of components may hook along their smallest outgoing
// edges (each is an MSF edge), and these picks all point down, so they form a forest; the
// vertices without a lower neighbour wait for the full rounds.  hasup marks the vertices
// with an upper neighbour: when at most one root has an edge the block is one tree and
// needs no round (k_top_hook0).  Each workgroup (one per CU, a contiguous chunk of the
// edges) keeps its minima and hasup bits in LDS and flushes them with one read-checked
// atomic per vertex (the minima only fall).
// Up to 2^15 vertices the minima are u32 (atomicMin); up to 2^16 (top_bits = 16) u16
// pairs updated by a 32-bit CAS (0xFFFF = none: a lower neighbour is at most V - 2).
__device__ __forceinline__ void lds_min_u16(uint32_t *w2, uint32_t i, uint32_t v) {
  uint32_t *w = w2 + (i >> 1);
  const uint32_t sh = (i & 1) * 16;
  uint32_t old = *w;
  while (((old >> sh) & 0xFFFFu) > v) {
    const uint32_t prev = atomicCAS(w, old, (old & ~(0xFFFFu << sh)) | (v << sh));
    if (prev == old) break;
    old = prev;
  }
}
template <bool W16>
__global__ __launch_bounds__(TOPB) void k_top_min0_lds(TopSet t, const uint64_t *__restrict__ st) {
  const TopState &ts = t.s[blockIdx.y];
  const TopEdges &te = t.e[blockIdx.y];
  extern __shared__ uint32_t lmin[];
  __shared__ unsigned lup[2 * TOP_HOOK_LDS / 32];
  __shared__ uint64_t s_pre[NSHARD + 1];
  const uint32_t V = ts.V, W = (V + 31) / 32, v0 = ts.v0, NW = W16 ? (V + 1) / 2 : V;
  for (uint32_t v = threadIdx.x; v < NW; v += TOPB) lmin[v] = INVALID;
  for (uint32_t w = threadIdx.x; w < W; w += TOPB) lup[w] = 0;
  top_prefix(te, s_pre);
  __syncthreads();
  const uint64_t total = s_pre[NSHARD] + (te.g1 - te.g0);
  const uint64_t per = (total + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = (uint64_t)blockIdx.x * per, b1 = b0 + per < total ? b0 + per : total;
  top_edges(te, s_pre, st[ST_TOPNT], b0 < b1 ? b0 : b1, b1, threadIdx.x, TOPB, [&](uint64_t e) {
    if (e == DEAD) return;
    const uint32_t l = (uint32_t)e - v0, h = (uint32_t)(e >> 32) - v0;
    if (W16) lds_min_u16(lmin, h, l);
    else if (l < lmin[h]) atomicMin(&lmin[h], l);
    const unsigned bit = 1u << (l & 31);
    if (!(lup[l >> 5] & bit)) atomicOr(&lup[l >> 5], bit);
  });
  __syncthreads();
  for (uint32_t v = threadIdx.x; v < V; v += TOPB) {
    uint32_t x = W16 ? (lmin[v >> 1] >> ((v & 1) * 16)) & 0xFFFFu : lmin[v];
    if (W16 && x == 0xFFFFu) x = INVALID;
    if (x != INVALID && x < ts.minlo[v]) atomicMin(&ts.minlo[v], x);
  }
  for (uint32_t w = threadIdx.x; w < W; w += TOPB) {
    const unsigned x = lup[w];
    if (x & ~ts.hasup[w]) atomicOr(&ts.hasup[w], x);
  }
}

// One workgroup: after par[] (u16, in LDS) holds every component's pick (itself for a
// root), the forest is pointer-jumped, the roots renumbered 0..C-1 and ts.comp rewritten
// through them.  lds: par[cap], cid[cap].
__device__ void top_relabel(const TopState &ts, uint16_t *par, uint16_t *cid, uint32_t cnt, bool first_round) {
  __shared__ unsigned s_w[TOPB / WAVE];
  for (;;) {   // pointer jumping (every pick points to a neighbour component; the picks form a forest)
    bool changed = false;
    for (uint32_t c = threadIdx.x; c < cnt; c += TOPB) {
      const uint32_t p = par[c], q = par[p];
      if (q != p) { par[c] = (uint16_t)q; changed = true; }
    }
    if (!__syncthreads_or(changed)) break;
  }
  // roots -> 0..C-1: each thread owns a contiguous run of entries
  const uint32_t per = (cnt + TOPB - 1) / TOPB, b0 = threadIdx.x * per;
  uint32_t r = 0;
  for (uint32_t k = 0; k < per && b0 + k < cnt; ++k) r += par[b0 + k] == b0 + k;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = r;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int w = 0; w < TOPB / WAVE; ++w) {
    if (w < wave) off += s_w[w];
    tot += s_w[w];
  }
  uint32_t run = off + inc - r;
  for (uint32_t k = 0; k < per && b0 + k < cnt; ++k)
    if (par[b0 + k] == b0 + k) cid[b0 + k] = (uint16_t)run++;
  __syncthreads();
  for (uint32_t v = threadIdx.x; v < ts.V; v += TOPB) {
    const uint32_t c = first_round ? v : ts.comp[v];
    ts.comp[v] = cid[par[c]];
  }
  for (uint32_t c = threadIdx.x; c < tot; c += TOPB) ts.best[c] = NO_EDGE;
  if (threadIdx.x == 0) {
    ts.scal[0] = tot;
    ts.scal[1] = 0;
  }
}

// Appends the MSF edges a workgroup recorded (s_cnt of them in its LDS list) to the list.
__device__ __forceinline__ uint32_t top_record(unsigned *s_cnt, uint64_t e, uint64_t *rec_lds, uint32_t cap) {
  const uint32_t k = atomicAdd(s_cnt, 1u);
  if (k < cap) rec_lds[k] = e;
  return k;
}

constexpr uint32_t TOP_REC = 2048;   // MSF edges staged per hook launch before a flush
// (the blocks' hooks run concurrently: each flush reserves its slots on ST_EXTRA)
__device__ void top_flush(const TopState &ts, const uint64_t *rec, unsigned n) {
  __shared__ uint64_t s_base;
  if (n == 0) return;   // (uniform)
  if (threadIdx.x == 0)
    s_base = ts.st[ST_KEPT] + ts.st[ST_CONTR] + atomicAdd((unsigned long long *)&ts.st[ST_EXTRA], (unsigned long long)n);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < n; k += TOPB) ts.out[s_base + k] = rec[k];
  __syncthreads();
}

__global__ __launch_bounds__(TOPB) void k_top_hook0(TopSet t) {
  const TopState &ts = t.s[blockIdx.x];
  extern __shared__ uint16_t lds16[];
  const bool big = ts.V > TOP_HOOK_LDS;
  uint16_t *par = lds16, *cid = big ? ts.gcid : lds16 + TOP_HOOK_LDS;
  __shared__ uint64_t rec[TOP_REC];
  __shared__ unsigned s_cnt, s_roots;
  if (threadIdx.x == 0) s_cnt = s_roots = 0;
  __syncthreads();
  for (uint32_t base = 0; base < ts.V; base += TOP_REC) {   // TOP_REC vertices (<= one edge each) a pass
    const uint32_t end = base + TOP_REC < ts.V ? base + TOP_REC : ts.V;
    for (uint32_t v = base + threadIdx.x; v < end; v += TOPB) {
      const uint32_t ml = ts.minlo[v];
      uint32_t p = v;
      if (ml != INVALID) {
        p = ml;
        top_record(&s_cnt, ((uint64_t)(ts.v0 + v) << 32) | (ts.v0 + ml), rec, TOP_REC);
      } else if (ts.hasup[v >> 5] & (1u << (v & 31))) {
        atomicAdd(&s_roots, 1u);   // a root with edges
      }
      par[v] = (uint16_t)p;
    }
    __syncthreads();
    top_flush(ts, rec, s_cnt);
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  }
  top_relabel(ts, par, cid, ts.V, true);
  // every non-root's chain of picks ends at a root with an edge: with at most one such
  // root every edge lies inside one component, and the MSF is complete
  if (threadIdx.x == 0 && s_roots <= 1) ts.scal[2] = 1;
}

// A Borůvka round over the block's edges: each component's smallest outgoing edge word.
// The labels (u16) in LDS; the minima in LDS when the components fit, flushed with one
// read-checked atomic per component and workgroup.
__global__ __launch_bounds__(TOPB) void k_top_round(TopSet t, const uint64_t *__restrict__ st) {
  const TopState &ts = t.s[blockIdx.y];
  const TopEdges &te = t.e[blockIdx.y];
  if (ts.scal[2]) return;   // done (uniform)
  extern __shared__ uint16_t lds16[];
  uint16_t *comp = lds16;
  const uint32_t voff = (ts.V + 3) & ~3u;   // the minima 8-B aligned after the labels
  unsigned long long *lbest = (unsigned long long *)(lds16 + voff);
  __shared__ uint64_t s_pre[NSHARD + 1];
  const uint32_t C = ts.scal[0], v0 = ts.v0;
  const bool in_lds = C <= (uint32_t)((TOP_ROUND_LDS - voff * sizeof(uint16_t)) / sizeof(uint64_t));
  for (uint32_t v = threadIdx.x; v < ts.V; v += TOPB) comp[v] = ts.comp[v];
  if (in_lds)
    for (uint32_t c = threadIdx.x; c < C; c += TOPB) lbest[c] = NO_EDGE;
  top_prefix(te, s_pre);
  __syncthreads();
  const uint64_t total = s_pre[NSHARD] + (te.g1 - te.g0);
  bool inter = false;
  top_edges(te, s_pre, st[ST_TOPNT], 0, total, blockIdx.x * TOPB + threadIdx.x, gridDim.x * TOPB, [&](uint64_t e) {
    if (e == DEAD) return;
    const uint32_t cl = comp[(uint32_t)e - v0], ch = comp[(uint32_t)(e >> 32) - v0];
    if (cl == ch) return;
    inter = true;
    if (in_lds) {
      if (e < lbest[cl]) atomicMin(&lbest[cl], (unsigned long long)e);
      if (e < lbest[ch]) atomicMin(&lbest[ch], (unsigned long long)e);
    } else {
      if (e < ts.best[cl]) atomicMin(&ts.best[cl], (unsigned long long)e);
      if (e < ts.best[ch]) atomicMin(&ts.best[ch], (unsigned long long)e);
    }
  });
  inter = __syncthreads_or(inter);
  if (in_lds)
    for (uint32_t c = threadIdx.x; c < C; c += TOPB) {
      const unsigned long long w = lbest[c];
      if (w != NO_EDGE && w < ts.best[c]) atomicMin(&ts.best[c], w);
    }
  if (inter && threadIdx.x == 0) atomicOr(&ts.scal[1], 1u);
}

// One workgroup per block: every component hooks to the component across its smallest
// outgoing edge (a pair that picked the same edge keeps the smaller id as the root), the
// picked edges are the MSF's, then the labels are rewritten.  A round without an
// inter-component edge ends the block's rounds.
__global__ __launch_bounds__(TOPB) void k_top_hook(TopSet t) {
  const TopState &ts = t.s[blockIdx.x];
  __shared__ unsigned s_flag;
  if (threadIdx.x == 0) s_flag = ts.scal[2] ? 2u : atomicOr(&ts.scal[1], 0u) ? 1u : 0u;
  __syncthreads();
  if (s_flag == 2) return;
  if (s_flag == 0) {
    if (threadIdx.x == 0) ts.scal[2] = 1;
    return;
  }
  extern __shared__ uint16_t lds16[];
  const uint32_t C = ts.scal[0];
  const bool big = C > TOP_HOOK_LDS;
  uint16_t *par = lds16, *cid = big ? ts.gcid : lds16 + TOP_HOOK_LDS;
  __shared__ uint64_t rec[TOP_REC];
  __shared__ unsigned s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  for (uint32_t base = 0; base < C; base += TOP_REC) {
    const uint32_t end = base + TOP_REC < C ? base + TOP_REC : C;
    for (uint32_t c = base + threadIdx.x; c < end; c += TOPB) {
      const unsigned long long w = ts.best[c];
      uint32_t p = c;
      if (w != NO_EDGE) {
        const uint32_t a = ts.comp[(uint32_t)w - ts.v0], b = ts.comp[(uint32_t)(w >> 32) - ts.v0];
        const uint32_t other = a == c ? b : a;
        if (!(ts.best[other] == w && c < other)) {
          p = other;
          top_record(&s_cnt, w, rec, TOP_REC);
        }
      }
      par[c] = (uint16_t)p;
    }
    __syncthreads();
    top_flush(ts, rec, s_cnt);
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
  }
  top_relabel(ts, par, cid, C, false);
}

// ---- the top subproblem at an early level: its MSF when round 0 leaves one tree ------
// The same identity one level band higher: after the level that splits at s = big_bits the
// top 2^big_bits positions are a subproblem of their own (groups 0..BIG_BITS-1 and the
// list entries there; RMAT-26, big_bits = 19: ~380 M edges on ~256 K vertices), and the
// levels below spend most of their time in it.  Its labels do not fit LDS, so only round 0
// runs, and it picks ANY lower neighbour per vertex (plain stores, first writer seen wins:
// in LDS for the block's top BIG_HOT positions, where power-law edges mostly end, in HBM
// below) plus a has-upper-neighbour bit.  Under the weight hi alone the edges (v, l), l < v,
// tie, and Kruskal with each v's pick first takes every pick (v is a singleton when its
// weight comes up), so the picks lie in SOME minimum spanning forest; when at most one root
// has an edge they span the block as one tree and ARE that forest — and etree(G) is the
// elimination tree of every MSF under hi, whatever the tie order (the components of each
// threshold graph G_t are every MSF's).  Otherwise nothing is cut (the 2^top_bits cut runs
// later).  (Lowest lower neighbours by read-checked atomicMin cost 6.1 ms at 2^20.)
// sheep_tuning big_bits (default 21: RMAT-26 etree 2^20 27.7, 2^21 26.9 ms; at 2^22 round 0
// leaves 15 K trees) and big_dense (default 256 group edges per vertex).
constexpr uint32_t BIG_HOT = 1u << 15;
struct BigState {
  uint32_t *minlo;                  // per vertex: a lower neighbour (block-local), the round-0 pick
  // Per vertex a BYTE (plain stores, no read-modify-write, instead of bit maps and their
  // memory-side atomicOrs; measured the same at RMAT-26).  A stale read of a byte another
  // XCD just set only costs a redundant store of the same value.
  uint8_t *hasup;                   // per vertex: it has an upper neighbour
  uint8_t *picked;                  // per vertex: minlo holds a pick (a 4x smaller read check)
  unsigned long long *cnt;          // [0] vertices with a lower neighbour, [1] roots with an edge
  uint64_t *st;                     // the cut level's stats row
  uint64_t *out;                    // the MSF goes behind the level's list (st[ST_EXTRA])
  uint32_t v0, V;
  uint32_t hot;                     // the LDS window: the block's top `hot` positions (<= BIG_HOT)
};

__global__ __launch_bounds__(BLOCK) void k_big_init(BigState b) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < b.V; v += stride) {
    b.minlo[v] = INVALID;
    b.hasup[v] = b.picked[v] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) b.cnt[threadIdx.x] = 0;
}

constexpr int BIG_U = 16;   // edges per thread in flight in k_big_min0 (one 1024-thread workgroup per CU)
constexpr uint32_t BIG_UPW = 1u << 16;   // has-upper bits kept in LDS per workgroup: a window of lo
// H16: the window is the top 2^16 positions with each pick as a u16 distance h - l (0:
// none); a hot vertex whose lower neighbours seen so far all lie 2^16 or more below takes
// the device path
template <bool H16>
__global__ __launch_bounds__(TOPB) void k_big_min0(TopEdges te, BigState b, const uint64_t *__restrict__ st) {
  extern __shared__ uint32_t lmin[];   // the hot window's picks
  uint16_t *const ld = (uint16_t *)lmin;
  __shared__ unsigned lup[BIG_UPW / 32];
  __shared__ uint64_t s_pre[NSHARD + 1];
  __shared__ uint32_t s_w0;
  const uint32_t hotn = H16 ? (1u << 16) : b.hot;
  const uint32_t V = b.V, v0 = b.v0, hot0 = V > hotn ? V - hotn : 0, HW = V - hot0;
  for (uint32_t v = threadIdx.x; v < HW; v += TOPB) {
    if (H16) ld[v] = 0;
    else lmin[v] = INVALID;
  }
  // a hot vertex's pick in LDS; false: the edge takes the device path
  auto hot_pick = [&](uint32_t l, uint32_t h) -> bool {
    if (H16) {
      if (ld[h - hot0]) return true;
      if (h - l >= (1u << 16)) return false;
      ld[h - hot0] = (uint16_t)(h - l);
      return true;
    }
    if (lmin[h - hot0] == INVALID) lmin[h - hot0] = l;
    return true;
  };
  for (uint32_t w = threadIdx.x; w < BIG_UPW / 32; w += TOPB) lup[w] = 0;
  top_prefix(te, s_pre);
  __syncthreads();
  // The list part (the entries the extraction moved out, ~42 M at RMAT-26) strided over
  // every workgroup, BIG_U entries per thread in flight; the group part in one contiguous
  // chunk per workgroup.  (One chunk of list-then-groups per workgroup left the list to
  // the first ~15 workgroups, one dependent load per entry: most of the kernel's 7 ms.)
  const uint64_t nl = s_pre[NSHARD], ntiles = st[ST_TOPNT], G = te.g1 - te.g0;
  const uint64_t per = (G + gridDim.x - 1) / gridDim.x;
  const uint64_t g0 = (uint64_t)blockIdx.x * per < G ? (uint64_t)blockIdx.x * per : G;
  const uint64_t g1 = g0 + per < G ? g0 + per : G;
  // the group part comes in lo buckets, so a chunk's lo values crowd into a narrow range:
  // their has-upper bits go to an LDS window from the chunk's first lo (others: byte stores)
  if (threadIdx.x == 0) {
    const uint64_t e = g0 < g1 ? te.r0[te.g0 + g0] : DEAD;
    s_w0 = e == DEAD ? 0u : (((uint32_t)e - v0) & ~31u);
  }
  __syncthreads();
  const uint32_t w0 = s_w0;
  uint32_t *const gmin = b.minlo;
  uint8_t *const up = b.hasup, *const pk = b.picked;
  // the group part's read checks (the picks below the window, the has-upper bytes) are all
  // issued before any store: a check that waits for the previous edge's turn serialises
  // eight latencies per step, and a stale read only costs a redundant store
  const uint64_t lstride = (uint64_t)gridDim.x * TOPB;
  for (uint64_t i0 = (uint64_t)blockIdx.x * TOPB + threadIdx.x; i0 < nl; i0 += (uint64_t)BIG_U * lstride) {
    uint64_t e[BIG_U];
#pragma unroll
    for (int j = 0; j < BIG_U; ++j) {
      const uint64_t i = i0 + (uint64_t)j * lstride;
      e[j] = i < nl ? top_list_at(te, s_pre, ntiles, i) : DEAD;
    }
#pragma unroll
    for (int j = 0; j < BIG_U; ++j) {
      if (e[j] == DEAD) continue;
      const uint32_t l = (uint32_t)e[j] - v0, h = (uint32_t)(e[j] >> 32) - v0;
      if (h >= hot0 && hot_pick(l, h)) {
      } else if (!pk[h]) {
        gmin[h] = l;
        pk[h] = 1;
      }
      if (!up[l]) up[l] = 1;
    }
  }
  const uint64_t *r = te.r0 + te.g0;
  // software-pipelined: the next BIG_U edges are loaded while this batch's read checks are
  // in flight and its picks are made
  constexpr uint64_t STEP = (uint64_t)BIG_U * TOPB;
  uint64_t en[BIG_U];
  auto load = [&](uint64_t i0) {
#pragma unroll
    for (int j = 0; j < BIG_U; ++j) {
      const uint64_t i = i0 + (uint64_t)j * TOPB;
      en[j] = i < g1 ? __builtin_nontemporal_load(r + i) : DEAD;
    }
  };
  if (g0 + threadIdx.x < g1) load(g0 + threadIdx.x);
  for (uint64_t i0 = g0 + threadIdx.x; i0 < g1; i0 += STEP) {
    uint32_t l[BIG_U], h[BIG_U], gv[BIG_U], uv[BIG_U];
#pragma unroll
    for (int j = 0; j < BIG_U; ++j) {
      const uint64_t e = en[j];
      l[j] = e == DEAD ? INVALID : (uint32_t)e - v0;
      h[j] = e == DEAD ? 0 : (uint32_t)(e >> 32) - v0;
    }
#pragma unroll
    for (int j = 0; j < BIG_U; ++j) {
      gv[j] = l[j] != INVALID && h[j] < hot0 ? pk[h[j]] : 1u;
      uv[j] = l[j] != INVALID && l[j] - w0 >= BIG_UPW ? up[l[j]] : 1u;
    }
    if (i0 + STEP < g1) load(i0 + STEP);
#pragma unroll
    for (int j = 0; j < BIG_U; ++j) {
      if (l[j] == INVALID) continue;
      if (h[j] >= hot0) {
        if (!hot_pick(l[j], h[j]) && !pk[h[j]]) {   // (H16: a far pick)
          gmin[h[j]] = l[j];
          pk[h[j]] = 1;
        }
      } else if (!gv[j]) {
        gmin[h[j]] = l[j];
        pk[h[j]] = 1;
      }
      const unsigned bit = 1u << (l[j] & 31);
      const uint32_t d = l[j] - w0;
      if (d < BIG_UPW) {
        if (!(lup[d >> 5] & bit)) atomicOr(&lup[d >> 5], bit);
      } else if (!uv[j]) {
        up[l[j]] = 1;
      }
    }
  }
  __syncthreads();
  for (uint32_t v = threadIdx.x; v < HW; v += TOPB) {
    const uint32_t x = H16 ? (ld[v] ? hot0 + v - ld[v] : INVALID) : lmin[v];
    if (x != INVALID && !pk[hot0 + v]) {
      gmin[hot0 + v] = x;
      pk[hot0 + v] = 1;
    }
  }
  for (uint32_t d = threadIdx.x; d < BIG_UPW && w0 + d < V; d += TOPB)   // the window's bits as bytes
    if (((lup[d >> 5] >> (d & 31)) & 1) && !up[w0 + d]) up[w0 + d] = 1;
}

__global__ __launch_bounds__(BLOCK) void k_big_roots(BigState b) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  uint64_t nonroot = 0, eroot = 0;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < b.V; v += stride) {
    if (b.minlo[v] != INVALID) ++nonroot;
    else if (b.hasup[v]) ++eroot;
  }
  block_atomic_add(&b.cnt[0], nonroot);
  block_atomic_add(&b.cnt[1], eroot);
}

// the MSF {(minlo(x), x)} appended behind the level's list (st[ST_EXTRA] counts them)
__global__ __launch_bounds__(BLOCK) void k_big_emit(BigState b) {
  const uint64_t base = b.st[ST_KEPT] + b.st[ST_CONTR];
  // up to 32 strided vertices per thread per reservation: one atomic on the counter per
  // workgroup call (a wave-aggregated append per wave serialised ~32 K atomics on it)
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t iters = (b.V + stride - 1) / stride;
  const uint64_t v0 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t it0 = 0; it0 < iters; it0 += 32) {   // uniform over the workgroup (block_reserve)
    const uint32_t ni = iters - it0 < 32 ? (uint32_t)(iters - it0) : 32u;
    uint32_t has = 0;
    for (uint32_t q = 0; q < ni; ++q) {
      const uint64_t v = v0 + (it0 + q) * stride;
      if (v < b.V && b.minlo[v] != INVALID) has |= 1u << q;
    }
    uint64_t slot = block_reserve((uint32_t)__popc(has), (unsigned long long *)&b.st[ST_EXTRA]);
    for (uint32_t q = 0; q < ni; ++q)
      if (has & (1u << q)) {
        const uint64_t v = v0 + (it0 + q) * stride;
        b.out[base + slot++] = ((uint64_t)(b.v0 + v) << 32) | (b.v0 + b.minlo[v]);
      }
  }
}

// Debug statistic (SHEEP_DEBUG=etree): live entries per block of 2^s spread positions
// after a level (its next list plus the groups not yet activated).
__global__ void k_dbg_blocks(const uint64_t *__restrict__ a, const uint64_t *__restrict__ st, const uint64_t *__restrict__ b,
                             uint64_t nb_edges, int s, uint32_t clo, unsigned *__restrict__ cnt, uint32_t cut) {
  const uint64_t na = st[ST_KEPT] + st[ST_CONTR];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < na + nb_edges; i += stride) {
    const uint64_t e = i < na ? a[i] : b[i - na];
    if (e == DEAD) continue;
    atomicAdd(&cnt[spread((uint32_t)e, clo) >> s], 1u);
  }
}

}  // namespace

void fill_u32(Ctx &c, uint32_t *p, uint64_t n, uint32_t v);

static const bool g_debug_etree = debug_on("etree");
// Finishing block size (log2 positions; sheep_tuning fin_map_bits / fin_merge_bits).
// Liu's sweep per block (fin_dc = 0) takes one step per hi, so 10 bits were its best for
// maps (RMAT-26 etree 32.0-32.2 ms) and 11 for merges.  The per-block D&C (k_fin_dc)
// spreads a level over a workgroup and cuts long block lists to their MSF first: RMAT-26
// etree 31.0 / 30.5 / 30.0 ms at 11 / 12 / 13 bits (13: one workgroup per CU, 112 KB of
// LDS state); 8 shard maps 76.3 -> 71.2 ms and the 8-tree merge 15.4 -> 14.1 ms at 12 bits.

// spread(x) = floor(x * c / 2^32), c = floor(2^(32+L) / n) in [2^32, 2^33), L = ceil(log2 n):
// monotone, injective on [0,n), image in [0, 2^L).  clo = c - 2^32.
void spread_params(uint64_t n, int *L_out, uint32_t *clo_out) {
  int L = 0;
  while ((1ull << L) < n) ++L;
  const unsigned __int128 cfull = (((unsigned __int128)1) << (32 + L)) / n;
  *L_out = L;
  *clo_out = (uint32_t)(cfull - (((unsigned __int128)1) << 32));
}

// A level's next list holds the entries that stayed plus the surviving contractions: each
// entry of the level's input (list + activated group) yields at most one of them (it stays,
// or it is cross and contracts, or it dies), so a list never holds more than the groups
// activated so far, m, plus the MSF edges of cut blocks (<= n: at most one per vertex).
static uint64_t list_capacity(uint64_t m, uint64_t n) { return m + n + 2 * (uint64_t)TILE; }

// Elimination tree of `m` edges ((hi<<32)|lo, lo < hi < n, DEAD holes allowed), grouped
// by first active level: seg[s] / seg[L + s] (device) delimit group s.  The edges are
// read only.
// One pass of launches per level, no host synchronisation inside the loop (see the
// stats row above); the stats come back once at the end for the timers / debug log.
// The dense blocks' edges -> their minimum spanning forests (k_top_extract_multi ..
// k_top_hook).  Block 0 is the top block [cut0, 2^L) (its list entries plus groups [g0, g1)
// of r0), block j >= 1 the 2^bits positions below block j - 1 (list entries only); the
// blocks below the top are cut while they are dense (up to nb_max - 1 of them,
// sheep_tuning top_blocks).  The MSF edges are appended to `next` behind the cut level's
// contractions (st[ST_EXTRA]); st[ST_CUT] (the lowest cut block's start) makes the next split
// drop the blocks' list entries, and the caller stops activating the top block's groups.
// One host sync for the blocks' sizes, one to skip the idle Borůvka rounds.  Returns the
// number of blocks cut.
static uint32_t top_blocks(Ctx &c, uint64_t *next, uint64_t *st, const uint64_t *r0, uint64_t g0, uint64_t g1,
                           uint32_t cut0, int bits, uint32_t nb_max, uint32_t clo, uint64_t n, uint64_t lcap) {
  // the regions are sized by the cut level's list (one sync: worst-case regions of several
  // blocks would take tens of GB at RMAT-26)
  uint64_t hrow[ST_ROW];
  HIP_CHECK(hipMemcpyAsync(hrow, st, sizeof hrow, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const uint64_t nl = hrow[ST_KEPT] + hrow[ST_CONTR];
  const uint64_t tcap = (nl + TILE - 1) / TILE * TILE + TILE;
  nb_max = std::min<uint32_t>(std::max<uint32_t>(nb_max, 1), TOP_NB_MAX);
  while (nb_max > 1 && ((uint64_t)nb_max << bits) > cut0 + (1ull << bits)) --nb_max;   // blocks must lie above 0
  {   // every block's region holds the whole list: as many blocks as half the free HBM takes
    // (top_blocks = 8 with the 11-bit finish ran out of memory at RMAT-26)
    size_t free_b = 0, total_b = 0;
    HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
    const auto it = c.ws.find("et_top_list");
    const size_t have = it == c.ws.end() ? 0 : it->second.bytes;
    while (nb_max > 1 && (size_t)nb_max * tcap * sizeof(uint64_t) * 9 / 8 > have + free_b / 2) --nb_max;
  }
  uint64_t *tl = c.get_as<uint64_t>("et_top_list", nb_max * tcap);
  unsigned long long *tcnt = c.get_as<unsigned long long>("et_top_cnt", nb_max * TOP_CSET + TOP_NB_MAX);
  unsigned long long *bcnt = tcnt + nb_max * TOP_CSET;
  HIP_CHECK(hipMemsetAsync(tcnt, 0, nb_max * TOP_CSET * sizeof(unsigned long long), c.stream));
  hipLaunchKernelGGL(k_top_extract_multi, dim3(grid_tiles(nl)), dim3(BLOCK), 0, c.stream, (const uint64_t *)next, st,
                     cut0, bits, nb_max, clo, tl, tcap, tcnt);
  LAUNCH_CHECK();
  auto first_at = [&](uint64_t y) {   // min vertex x with spread(x) >= y
    uint64_t a = 0, z = n;
    while (a < z) {
      const uint64_t x = (a + z) / 2;
      if (x + ((x * (uint64_t)clo) >> 32) >= y) z = x; else a = x + 1;
    }
    return a;
  };
  uint32_t nb = 1;
  if (nb_max > 1) {   // the blocks below the top: how many in a row are dense
    hipLaunchKernelGGL(k_top_sum_counts, dim3(nb_max), dim3(WAVE), 0, c.stream, (const unsigned long long *)tcnt, nb_max,
                       bcnt);
    LAUNCH_CHECK();
    unsigned long long hb[TOP_NB_MAX];
    HIP_CHECK(hipMemcpyAsync(hb, bcnt, nb_max * sizeof(unsigned long long), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    while (nb < nb_max) {
      const uint64_t hi_cut = cut0 - ((uint64_t)(nb - 1) << bits), lo_cut = hi_cut - (1ull << bits);
      const uint64_t V = first_at(hi_cut) - first_at(lo_cut);
      if (V < 2 || hb[nb] < TOP_DENSE * V) break;
      ++nb;
    }
  }
  const uint64_t VMAX = 1ull << bits;
  uint32_t *minlo = c.get_as<uint32_t>("et_top_minlo", nb * VMAX);
  unsigned *hasup = c.get_as<unsigned>("et_top_hasup", nb * VMAX / 32);
  uint16_t *comp = c.get_as<uint16_t>("et_top_comp", nb * VMAX);
  unsigned long long *best = c.get_as<unsigned long long>("et_top_best", nb * VMAX);
  unsigned *scal = c.get_as<unsigned>("et_top_scal", 4 * nb);
  const bool big = VMAX > TOP_HOOK_LDS;   // (top_bits = 16: the hooks keep cid in HBM)
  uint16_t *gcid = big ? c.get_as<uint16_t>("et_top_gcid", nb * VMAX) : nullptr;
  TopSet set{};
  uint32_t vmax = 0;
  for (uint32_t b = 0; b < nb; ++b) {
    const uint64_t hi_cut = b == 0 ? (1ull << 32) : cut0 - ((uint64_t)(b - 1) << bits);
    const uint64_t lo_cut = b == 0 ? cut0 : hi_cut - (1ull << bits);
    const uint64_t v0 = first_at(lo_cut), v1 = b == 0 ? n : first_at(hi_cut);
    TopState &ts = set.s[b];
    ts.minlo = minlo + b * VMAX;
    ts.hasup = hasup + b * VMAX / 32;
    ts.comp = comp + b * VMAX;
    ts.best = best + b * VMAX;
    ts.scal = scal + 4 * b;
    ts.st = st;
    ts.out = next;
    ts.gcid = big ? gcid + b * VMAX : nullptr;
    ts.v0 = (uint32_t)v0;
    ts.V = (uint32_t)(v1 - v0);
    vmax = std::max(vmax, ts.V);
    set.e[b] = TopEdges{tl + b * tcap, tcnt + b * TOP_CSET, r0, b == 0 ? g0 : 0, b == 0 ? g1 : 0};
  }
  const size_t lds2 = 2 * (size_t)TOP_HOOK_LDS * sizeof(uint16_t);   // par + cid, or par alone up to 2^16
  const size_t ldsr = TOP_ROUND_LDS;                                  // labels + minima
  const size_t ldsm = TOP_HOOK_LDS * sizeof(uint32_t);                // round 0's minima
  allow_lds((const void *)k_top_hook0, (int)lds2);
  allow_lds((const void *)k_top_hook, (int)lds2);
  allow_lds((const void *)k_top_round, (int)ldsr);
  allow_lds((const void *)k_top_min0_lds<false>, (int)ldsm);
  allow_lds((const void *)k_top_min0_lds<true>, (int)ldsm);
  hipLaunchKernelGGL(k_top_init, dim3(grid_for(vmax), nb), dim3(BLOCK), 0, c.stream, set);
  LAUNCH_CHECK();
  if (vmax <= TOP_HOOK_LDS)
    hipLaunchKernelGGL(k_top_min0_lds<false>, dim3(TOP_WG, nb), dim3(TOPB), ldsm, c.stream, set, (const uint64_t *)st);
  else   // (<= 2^TOP_BITS_MAX)
    hipLaunchKernelGGL(k_top_min0_lds<true>, dim3(TOP_WG, nb), dim3(TOPB), ldsm, c.stream, set, (const uint64_t *)st);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_top_hook0, dim3(nb), dim3(TOPB), lds2, c.stream, set);
  LAUNCH_CHECK();
  for (int r = 0; r <= TOP_BITS_MAX; ++r) {   // <= bits + 1 rounds always finish (each halves the components)
    if (r == 0 || r == 2) {   // dense blocks are mostly one tree after round 0: skip the idle launches
      unsigned h[4 * TOP_NB_MAX];
      HIP_CHECK(hipMemcpyAsync(h, scal, 4 * nb * sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
      c.sync();
      bool any = false;
      for (uint32_t b = 0; b < nb; ++b) any |= h[4 * b + 2] == 0;
      if (g_debug_etree)
        for (uint32_t b = 0; b < nb; ++b)
          fprintf(stderr, "etree top round %d block %u: components %u done %u (minima %s)\n", r, b, h[4 * b],
                  h[4 * b + 2], h[4 * b] <= (TOP_ROUND_LDS - ((set.s[b].V + 3) & ~3u) * 2) / 8 ? "lds" : "hbm");
      if (!any) break;
    }
    hipLaunchKernelGGL(k_top_round, dim3(TOP_WG, nb), dim3(TOPB), ldsr, c.stream, set, (const uint64_t *)st);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_top_hook, dim3(nb), dim3(TOPB), lds2, c.stream, set);
    LAUNCH_CHECK();
  }
  // the cut for the next split: the lowest cut block's start
  const uint64_t low = nb == 1 ? cut0 : cut0 - ((uint64_t)(nb - 1) << bits);
  hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, c.stream, st + ST_CUT, low);
  LAUNCH_CHECK();
  return nb;
}

// The top 2^bits positions after the level that splits at s = bits: round 0 of Borůvka
// (k_big_*); when it leaves one tree the block's edges become its MSF behind `next`
// (st[ST_EXTRA]) and st[ST_CUT] = cut0 drops its list entries at the next split.  One sync
// for the list length, one for the counts.  Returns whether the block was cut.
static bool big_cut(Ctx &c, uint64_t *next, uint64_t *st, const uint64_t *r0, uint64_t g0, uint64_t g1, uint32_t cut0,
                    int bits, uint32_t clo, uint64_t n) {
  uint64_t hrow[ST_ROW];
  HIP_CHECK(hipMemcpyAsync(hrow, st, sizeof hrow, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const uint64_t nl = hrow[ST_KEPT] + hrow[ST_CONTR];
  const uint64_t tcap = (nl + TILE - 1) / TILE * TILE + TILE;
  uint64_t *tl = c.get_as<uint64_t>("et_top_list", tcap);
  unsigned long long *tcnt = c.get_as<unsigned long long>("et_top_cnt", TOP_CSET + TOP_NB_MAX);
  HIP_CHECK(hipMemsetAsync(tcnt, 0, TOP_CSET * sizeof(unsigned long long), c.stream));
  hipLaunchKernelGGL(k_top_extract_multi, dim3(grid_tiles(nl)), dim3(BLOCK), 0, c.stream, (const uint64_t *)next, st, cut0,
                     bits, 1u, clo, tl, tcap, tcnt);
  LAUNCH_CHECK();
  uint64_t a = 0, z = n;   // the block's first vertex: min x with spread(x) >= cut0
  while (a < z) {
    const uint64_t x = (a + z) / 2;
    if (x + ((x * (uint64_t)clo) >> 32) >= cut0) z = x; else a = x + 1;
  }
  BigState b;
  b.v0 = (uint32_t)a;
  b.V = (uint32_t)(n - a);
  b.minlo = c.get_as<uint32_t>("et_big_minlo", b.V ? b.V : 1);
  b.hasup = c.get_as<uint8_t>("et_big_hasup", b.V ? b.V : 1);
  b.picked = c.get_as<uint8_t>("et_big_picked", b.V ? b.V : 1);
  b.cnt = c.get_as<unsigned long long>("et_big_cnt", 2);
  b.st = st;
  b.out = next;
  const TopEdges te{tl, tcnt, r0, g0, g1};
  // (big_hot_bits: a smaller window leaves LDS for two workgroups per CU)
  const int hot_bits = c.tune.big_hot_bits;
  b.hot = std::min<uint32_t>(1u << std::max(10, std::min(15, hot_bits)), BIG_HOT);
  const size_t lds = b.hot * sizeof(uint32_t);
  allow_lds((const void *)k_big_min0<false>, (int)(BIG_HOT * sizeof(uint32_t)));
  allow_lds((const void *)k_big_min0<true>, (int)(BIG_HOT * sizeof(uint32_t)));
  const bool hot16 = c.tune.big_hot16 != 0;
  hipLaunchKernelGGL(k_big_init, dim3(grid_for(b.V)), dim3(BLOCK), 0, c.stream, b);
  LAUNCH_CHECK();
  if (hot16)
    hipLaunchKernelGGL(k_big_min0<true>, dim3(TOP_WG), dim3(TOPB), BIG_HOT * sizeof(uint32_t), c.stream, te, b,
                       (const uint64_t *)st);
  else
    // (a window of at most 2^14 positions leaves LDS for two workgroups per CU: twice the grid)
    hipLaunchKernelGGL(k_big_min0<false>, dim3(b.hot <= (1u << 14) ? 2 * TOP_WG : TOP_WG), dim3(TOPB), lds, c.stream,
                       te, b, (const uint64_t *)st);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_big_roots, dim3(grid_for(b.V)), dim3(BLOCK), 0, c.stream, b);
  LAUNCH_CHECK();
  unsigned long long h[2];
  HIP_CHECK(hipMemcpyAsync(h, b.cnt, sizeof h, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (g_debug_etree)
    fprintf(stderr, "etree big cut after s %d: vertices %u group edges %lu list entries scanned %lu: non-roots %llu, "
                    "roots with an edge %llu -> %s\n", bits, b.V, (unsigned long)(g1 - g0), (unsigned long)nl, h[0], h[1],
            h[1] <= 1 ? "cut" : "kept");
  if (h[1] > 1) return false;
  hipLaunchKernelGGL(k_big_emit, dim3(grid_for(b.V)), dim3(BLOCK), 0, c.stream, b);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, c.stream, st + ST_CUT, (uint64_t)cut0);
  LAUNCH_CHECK();
  return true;
}

void etree_from_edges(Ctx &c, const uint64_t *edges, uint64_t m, uint64_t n, uint32_t *parent, const uint64_t *seg,
                      int fin_bits, int filt_lvl, uint32_t ylo, uint32_t yhi, int top_bits, int hook_mode,
                      int force_big_bits) {
  const bool hook_batch = (hook_mode & HOOK_BATCH) != 0, hook_up = (hook_mode & HOOK_UP) != 0;
  fill_u32(c, parent, n, INVALID);
  if (n < 2 || m == 0) return;
  if (m >= 0xFFFFFFFFull) throw Error(SHEEP_ERR_ARG, "too many edges for one shard");
  int L;
  uint32_t clo;
  spread_params(n, &L, &clo);

  uint32_t *uf = c.get_as<uint32_t>("et_uf", n);
  uint32_t *mt = c.get_as<uint32_t>("et_mt", n);
  uint32_t *top = c.get_as<uint32_t>("et_top", n);
  uint32_t *claim = c.get_as<uint32_t>("et_claim", n);
  // every list is bounded by m; scratch regions of sharded appends need whole tiles
  const uint64_t mcap = (m + TILE - 1) / TILE * TILE;
  const uint64_t lcap = list_capacity(m, n);
  uint32_t *xtop = c.get_as<uint32_t>("et_xtop", mcap);
  // a level's light entries and then its cross entries, back to back (light + cross <= the
  // level's input, <= the list bound)
  uint64_t *lx = c.get_as<uint64_t>("et_lx", lcap);
  // the two list buffers (level l reads one and writes the other) and the bucketed input r0
  uint64_t *lists[2] = {c.get_as<uint64_t>("et_list1", lcap), c.get_as<uint64_t>("et_list2", lcap)};
  const uint64_t *r0 = edges;
  // (lx must outlive the level: its clean runs at the next level's split)
  uint64_t *alt = c.get_as<uint64_t>("et_alt", mcap);     // shard scratch of the hook round and the contractions
  unsigned long long *csets = c.get_as<unsigned long long>("et_csets", NCSET * CSET_WORDS);
  uint64_t *stats = c.get_as<uint64_t>("et_stats", (uint64_t)(L + 1) * ST_ROW);
  HIP_CHECK(hipMemsetAsync(stats, 0, (uint64_t)(L + 1) * ST_ROW * sizeof(uint64_t), c.stream));
  auto cset = [&](int k) { return csets + (uint64_t)k * CSET_WORDS; };
  const unsigned gt = grid_tiles(m), gt2 = grid_for(lcap + m, SPLIT_TILE), gf = grid_for(m, BLOCK * XK), gn = grid_for(n);
  const int FINB = fin_bits < 0 ? 0 : fin_bits > FIN_BITS_MAX ? FIN_BITS_MAX : fin_bits;   // levels s < FINB: Liu per block (0: none)
  const int nglobal = L > FINB ? L - FINB : 0;
  const bool fin_dc = c.tune.fin_dc && FINB >= 8;   // (0: Liu's sweep per block)
  // the per-level state starts clean; tagged words need no restore between levels,
  // untagged ones are restored at each level's end (k_level_clean)
  const bool tagged = n < TAG_MAX_N;
  hipLaunchKernelGGL(k_reset, dim3(gn), dim3(BLOCK), 0, c.stream, uf, mt, top, claim, n, csets);
  LAUNCH_CHECK();
  allow_full_lds((const void *)k_cross_find_win);
  // The dense top block (maps): after the level that splits at s = top_bits, its edges are
  // replaced by their minimum spanning forest when its groups are dense.
  int top_lvl = -1, gcut = 0;
  uint64_t top_g0 = 0, top_g1 = 0;
  uint32_t top_V = 0, top_cut = 0;
  std::vector<uint64_t> hs;   // the group bounds on the host, read once for both cuts
  const bool seg_known = c.seg_host.dev == seg && c.seg_host.v.size() == 2 * (size_t)L;
  c.seg_host.dev = nullptr;
  if (seg_known && g_debug_etree) {   // the grouping's host bounds against the device's
    std::vector<uint64_t> d(2 * (size_t)L);
    HIP_CHECK(hipMemcpyAsync(d.data(), seg, d.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    if (d != c.seg_host.v) throw Error(SHEEP_ERR_HIP, "etree: host group bounds differ from the device's");
  }
  auto host_seg = [&]() {
    if (hs.empty() && seg_known) hs = c.seg_host.v;
    if (hs.empty()) {
      hs.resize(2 * (size_t)L);
      HIP_CHECK(hipMemcpyAsync(hs.data(), seg, hs.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
      c.sync();
    }
  };
  if (top_bits > FINB && top_bits <= L - 1 && top_bits <= TOP_BITS_MAX) {
    host_seg();
    top_cut = (uint32_t)((1ull << L) - (1ull << top_bits));
    uint64_t a = 0, z = n;   // the block's first vertex: min x with spread(x) >= cut
    while (a < z) {
      const uint64_t x = (a + z) / 2;
      if (x + ((x * (uint64_t)clo) >> 32) >= top_cut) z = x; else a = x + 1;
    }
    top_V = (uint32_t)(n - a);
    top_g0 = hs[top_bits - 1];
    top_g1 = hs[L];
    if (top_V >= 2 && top_g1 - top_g0 >= TOP_DENSE * top_V) {
      top_lvl = L - 1 - top_bits;
      gcut = top_bits;
    }
  }
  // the early cut of the top subproblem (sheep_tuning big_bits; 0: off), tried when dense;
  // force_big_bits (merges, sheep_tuning merge_cut_bits): tried whatever the density
  const bool forced = force_big_bits > FINB && force_big_bits <= L - 1 && filt_lvl < 0;
  const int big_bits = forced ? force_big_bits : top_bits ? c.tune.big_bits : 0;
  int big_lvl = -1;
  uint64_t big_g0 = 0, big_g1 = 0;
  uint32_t big_cut0 = 0;
  if (forced || (top_lvl >= 0 && big_bits > top_bits && big_bits <= L - 1)) {
    host_seg();
    big_cut0 = (uint32_t)((1ull << L) - (1ull << big_bits));
    uint64_t a = 0, z = n;
    while (a < z) {
      const uint64_t x = (a + z) / 2;
      if (x + ((x * (uint64_t)clo) >> 32) >= big_cut0) z = x; else a = x + 1;
    }
    big_g0 = hs[big_bits - 1];
    big_g1 = hs[L];
    // only where the block is far denser than the top block's rule asks (RMAT-26: ~740 group
    // edges per vertex at 2^19, ~540 at 2^20; a 1/8 edge shard's ~90 did not pay for the
    // cut: 8 shard maps 70.2 -> 76.9 ms)
    const uint64_t big_dense = (uint64_t)c.tune.big_dense;
    if (n - a >= 2 && (forced || big_g1 - big_g0 >= big_dense * (n - a))) big_lvl = L - 1 - big_bits;
  }
  // The cross pass's LDS window (k_cross_find_win) for the first cross_win_levels levels; a
  // map too sparse for the early cut keeps singleton roots in lo order one level longer and
  // takes one window level more (8 RMAT-26 shard maps 65.3 -> 64.4 ms; a dense map and the
  // merges lose with it: C3 +0.5 ms, 8-tree merge +0.1 ms)
  const int win_levels = std::min(8, c.tune.cross_win_levels + (top_bits > 0 && big_lvl < 0 && filt_lvl < 0 ? 1 : 0));
  int cut_lvl = -1;           // the level whose split follows a cut (its list entries dropped)
  uint32_t cut_val = 0;
  // a split reads at most the list plus a bucket: (lcap + m) entries, in SPLIT_TILE tiles
  const uint64_t cstride = (lcap + m + SPLIT_TILE - 1) / SPLIT_TILE + 1;
  uint64_t *tcnt = c.get_as<uint64_t>("et_tilecnt", 3 * cstride + 1);
  for (int lvl = 0; lvl < nglobal; ++lvl) {
    const int s = L - 1 - lvl;
    uint64_t *st = stats + (uint64_t)lvl * ST_ROW;
    const uint64_t *prev = lvl ? st - ST_ROW : nullptr;
    const Tg g = make_tag(lvl, tagged);
    uint64_t *cur = lists[lvl & 1], *next = lists[(lvl + 1) & 1];
    const YRange yr{ylo, yhi, lvl == filt_lvl};
    {
      TimedRegion tr(c, "etree_split");
      // the previous level's clean first (its counters, adoptions and resets)
      const LevelClean clean = lvl ? LevelClean{lx, xtop, prev, uf, mt, top, claim, n, tagged, lvl - 1, parent, csets}
                                   : LevelClean{};
      const bool after_cut = cut_lvl >= 0 && lvl == cut_lvl + 1;
      hipLaunchKernelGGL(after_cut ? k_split_count<true> : k_split_count<false>, dim3(gt2), dim3(BLOCK), 0, c.stream,
                         (const uint64_t *)cur, prev, st, s, clo, yr,
                         (const uint64_t *)r0, (const uint64_t *)seg, L, gcut, tcnt, clean);
      LAUNCH_CHECK();
      scan_exclusive_u64_dev(c, tcnt, tcnt, 3 * cstride + 1, st + ST_SCANN);
      hipLaunchKernelGGL(after_cut ? k_split_write<true> : k_split_write<false>, dim3(gt2), dim3(BLOCK), 0, c.stream,
                         (const uint64_t *)cur, prev, st, s, clo, yr,
                         (const uint64_t *)r0, (const uint64_t *)seg, L, gcut, (const uint64_t *)tcnt, next, lx);
      LAUNCH_CHECK();
    }
    {
      TimedRegion tr(c, "etree_union");
      static_assert(HOOK_ROUNDS == 1, "k_hook_finish reads the one round's shard regions");
      auto round = hook_up ? (hook_batch ? k_hook_round<true, true> : k_hook_round<false, true>)
                           : (hook_batch ? k_hook_round<true, false> : k_hook_round<false, false>);
      hipLaunchKernelGGL(round, dim3(gt), dim3(BLOCK), 0, c.stream, (const uint64_t *)lx, (const uint64_t *)(st + ST_NL),
                         uf, g, alt, cset(CSET_HOOK));
      LAUNCH_CHECK();
      hipLaunchKernelGGL(hook_up ? k_hook_finish<true> : k_hook_finish<false>, dim3(gf), dim3(BLOCK), 0, c.stream,
                         (const uint64_t *)alt, (const uint64_t *)(st + ST_NL), (const unsigned long long *)cset(CSET_HOOK),
                         uf, g, st + ST_HOOK);
      LAUNCH_CHECK();
      if (!hook_up) {   // (hook_up: every root is its component's top already)
        hipLaunchKernelGGL(k_light_top, dim3(gf), dim3(BLOCK), 0, c.stream, (const uint64_t *)lx,
                           (const uint64_t *)(st + ST_NL), uf, top, g);
        LAUNCH_CHECK();
      }
    }
    {
      TimedRegion tr(c, "etree_cross");
      if (lvl < win_levels)
        hipLaunchKernelGGL(k_cross_find_win, dim3(grid_for(mcap, XW_STEP, 1024)), dim3(XWB),
                           (XW + XWB / WAVE) * 4, c.stream, (const uint64_t *)lx, (const uint64_t *)st, uf,
                           mt, xtop, g);
      else
        hipLaunchKernelGGL(k_cross_find, dim3(gf), dim3(BLOCK), 0, c.stream, (const uint64_t *)lx,
                           (const uint64_t *)st, uf, mt, xtop, g);
      LAUNCH_CHECK();
    }
    {
      TimedRegion tr(c, "etree_apply");
      hipLaunchKernelGGL(k_cross_apply, dim3(gt), dim3(BLOCK), 0, c.stream, (const uint64_t *)lx,
                         (const uint32_t *)xtop, (const uint64_t *)st, (const uint32_t *)mt, (const uint32_t *)top, claim,
                         alt, cset(CSET_APPLY), parent, g, n);
      LAUNCH_CHECK();
      pack_shards<uint64_t>(c, alt, next, st + ST_NX, cset(CSET_APPLY), st + ST_CONTR, nullptr, nullptr, st + ST_KEPT);
    }
    if (lvl == big_lvl) {
      TimedRegion tr(c, "etree_top");
      if (big_cut(c, next, st, r0, big_g0, big_g1, big_cut0, big_bits, clo, n)) {
        gcut = big_bits;   // groups below are never activated; the 2^top_bits cut has nothing left to do
        top_lvl = -1;
        cut_lvl = lvl;
        cut_val = big_cut0;
      }
    }
    if (lvl == top_lvl) {
      cut_lvl = lvl;
      cut_val = top_cut;
      TimedRegion tr(c, "etree_top");
      const int top_nb = c.tune.top_blocks;
      const uint32_t nbc = top_blocks(c, next, st, r0, top_g0, top_g1, top_cut, top_bits, (uint32_t)top_nb, clo, n, lcap);
      if (g_debug_etree) {
        uint64_t h[ST_ROW];
        unsigned hs[4];
        HIP_CHECK(hipMemcpyAsync(h, st, sizeof h, hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipMemcpyAsync(hs, c.get_as<unsigned>("et_top_scal", 4), sizeof hs, hipMemcpyDeviceToHost, c.stream));
        c.sync();
        fprintf(stderr, "etree top blocks after s %d: %u block(s) cut; top: vertices %u group edges %lu; list entries "
                        "scanned %lu -> MSF edges %lu (top block: components left %u, done %u)\n", top_bits, nbc, top_V,
                (unsigned long)(top_g1 - top_g0), (unsigned long)(h[ST_KEPT] + h[ST_CONTR]), (unsigned long)h[ST_EXTRA],
                hs[0], hs[2]);
      }
    }
    if (g_debug_etree && s >= 8 && s <= 15) {   // how the live edges spread over the 2^s blocks
      uint64_t hs[2] = {0, 0};
      if (s > 0 && gcut == 0) {   // (a cut top block's groups are not live any more)
        HIP_CHECK(hipMemcpyAsync(&hs[0], seg + (s - 1), sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipMemcpyAsync(&hs[1], seg + L, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
      }
      const uint64_t nblk = (1ull << L) >> s;
      unsigned *cnt = c.get_as<unsigned>("et_dbg_blocks", nblk);
      HIP_CHECK(hipMemsetAsync(cnt, 0, nblk * sizeof(unsigned), c.stream));
      c.sync();
      hipLaunchKernelGGL(k_dbg_blocks, dim3(1024), dim3(BLOCK), 0, c.stream, (const uint64_t *)next, (const uint64_t *)st,
                         r0 + hs[0], hs[1] - hs[0], s, clo, cnt, cut_lvl >= 0 && lvl > cut_lvl ? cut_val : 0u);
      LAUNCH_CHECK();
      std::vector<unsigned> h(nblk);
      HIP_CHECK(hipMemcpyAsync(h.data(), cnt, nblk * sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
      c.sync();
      std::sort(h.begin(), h.end());
      uint64_t tot = 0, ne = 0, over[5] = {0, 0, 0, 0, 0};
      const uint64_t caps[5] = {4096, 8192, 16384, 32768, 65536};
      for (unsigned x : h) {
        tot += x;
        ne += x > 0;
        for (int k = 0; k < 5; ++k) if (x > caps[k]) over[k] += x;
      }
      fprintf(stderr, "etree blocks after s %d (2^%d positions): edges %lu blocks %lu nonempty %lu max %u p99 %u p90 %u | edges in blocks > 4K %lu 8K %lu 16K %lu 32K %lu 64K %lu\n",
              s, s, (unsigned long)tot, (unsigned long)nblk, (unsigned long)ne, h.back(), h[(size_t)(nblk * 0.99)],
              h[(size_t)(nblk * 0.9)], (unsigned long)over[0], (unsigned long)over[1], (unsigned long)over[2],
              (unsigned long)over[3], (unsigned long)over[4]);
    }
  }
  if (nglobal) {   // the last level's clean (the others ran in the next level's split)
    TimedRegion tr(c, "etree_apply");
    hipLaunchKernelGGL(k_level_clean, dim3(gf), dim3(BLOCK), 0, c.stream,
                       LevelClean{lx, xtop, stats + (uint64_t)(nglobal - 1) * ST_ROW, uf, mt, top, claim, n, tagged,
                                  nglobal - 1, parent, csets});
    LAUNCH_CHECK();
  }
  if (FINB) {
    // the last min(L, B) levels: the list plus the groups s < B, sorted by hi, then
    // Liu's algorithm per 2^B-position block
    TimedRegion tr(c, "etree_finish");
    const int sg = (L < FINB ? L : FINB) - 1;   // highest group left
    const uint64_t *prev = nglobal ? stats + (uint64_t)(nglobal - 1) * ST_ROW : nullptr;
    // The finish's input, the last level's list plus the groups left (list + groups <= m +
    // the cuts' MSF edges <= lcap), goes into the list buffer the last level read, and its
    // sort's other half into lx: both are free now, so nothing is sized from the device's
    // counts and the gather reads the list length and group bounds on the device (one host
    // round trip, for the sort's length; buffers of their own sized by the list's worst
    // case took ~48 GB at RMAT-26)
    uint64_t *fin = lists[(nglobal + 1) & 1], *fin_alt = lx;
    uint64_t *n_fin = stats + (uint64_t)L * ST_ROW;
    hipLaunchKernelGGL(k_fin_gather, dim3(grid_for(lcap)), dim3(BLOCK), 0, c.stream, (const uint64_t *)lists[nglobal & 1],
                       prev, r0, seg, sg, L, gcut > sg, lcap, fin, n_fin);
    LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(c.h_scalars + 15, n_fin, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    const uint64_t nf = c.h_scalars[15];
    if (nf > lcap) throw Error(SHEEP_ERR_HIP, "etree finish: input beyond the list buffer");
    const uint64_t cap = nf + 1;
    if (nf) {
      // L + 1 bits: hi < 2^L, and DEAD (all ones) sorts after every edge
      bool in_alt = false;
      radix_sort_keys_u64(c, fin, nf, L + 1, fin_alt, &in_alt);
      if (in_alt) std::swap(fin, fin_alt);
      const uint64_t nb = L > FINB ? 1ull << (L - FINB) : 1;
      uint64_t *eb = c.get_as<uint64_t>("et_fin_eb", nb + 1);
      uint32_t *vb = c.get_as<uint32_t>("et_fin_vb", nb + 1);
      uint32_t *light = c.get_as<uint32_t>("et_fin_light", nb), *heavy = c.get_as<uint32_t>("et_fin_heavy", nb);
      unsigned long long *n_lh = (unsigned long long *)(n_fin + 1);   // light, heavy counts (zeroed with stats)
      hipLaunchKernelGGL(k_fin_bounds, dim3(grid_for(nb > n ? nb + 1 : n + 1)), dim3(BLOCK), 0, c.stream,
                         (const uint64_t *)fin, (const uint64_t *)n_fin, clo, FINB, nb, n, eb, vb, light, heavy, n_lh,
                         fin_dc ? fdc_lcap(FINB) : FINB <= FIN_LANE_BITS ? FIN_HEAVY : 0);
      LAUNCH_CHECK();
      const unsigned gl = (unsigned)((nb + WAVE - 1) / WAVE), gh = (unsigned)(nb < 8192 ? nb : 8192);
      if (fin_dc) {   // every non-empty block, one workgroup each from a ticket: lists past LDS first
        uint32_t *dbuf = c.get_as<uint32_t>("et_fin_dc", 2 * cap);
        unsigned long long *ticket = (unsigned long long *)(n_fin + 3);   // (zeroed with stats)
        const unsigned gd = (unsigned)(nb < 1024 ? nb : 1024);
        switch (FINB) {
#define SHEEP_FIN_DC(B)                                                                                    \
  case B:                                                                                                  \
    hipLaunchKernelGGL(k_fin_dc<B>, dim3(gd), dim3(FDC_T), 0, c.stream, (const uint64_t *)fin,             \
                       (const uint64_t *)eb, (const uint32_t *)vb, (const uint32_t *)heavy,                \
                       (const unsigned long long *)(n_lh + 1), (const uint32_t *)light,                    \
                       (const unsigned long long *)n_lh, clo, dbuf, cap, ticket, parent);                  \
    LAUNCH_CHECK();                                                                                        \
    break;
          SHEEP_FIN_DC(8) SHEEP_FIN_DC(9) SHEEP_FIN_DC(10) SHEEP_FIN_DC(11) SHEEP_FIN_DC(12) SHEEP_FIN_DC(13)
#undef SHEEP_FIN_DC
          default: throw Error(SHEEP_ERR_ARG, "etree: bad finishing block size");
        }
      } else switch (FINB) {
#define SHEEP_FIN_LANES(B)                                                                                       \
    hipLaunchKernelGGL(k_fin_lanes<B>, dim3(gl), dim3(WAVE), 0, c.stream, (const uint64_t *)fin, (const uint64_t *)eb, \
                       (const uint32_t *)vb, (const uint32_t *)light, (const unsigned long long *)n_lh, parent);  \
    LAUNCH_CHECK();
#define SHEEP_FIN_HEAVY(B)                                                                                       \
    hipLaunchKernelGGL(k_fin_heavy<B>, dim3(gh), dim3(WAVE), 0, c.stream, (const uint64_t *)fin, (const uint64_t *)eb, \
                       (const uint32_t *)vb, (const uint32_t *)heavy, (const unsigned long long *)(n_lh + 1), parent); \
    LAUNCH_CHECK();
#define SHEEP_FIN_CASE(B) case B: SHEEP_FIN_LANES(B) SHEEP_FIN_HEAVY(B) break;
#define SHEEP_FIN_WAVE(B) case B: SHEEP_FIN_HEAVY(B) break;
        SHEEP_FIN_CASE(1) SHEEP_FIN_CASE(2) SHEEP_FIN_CASE(3) SHEEP_FIN_CASE(4)
        SHEEP_FIN_CASE(5) SHEEP_FIN_CASE(6) SHEEP_FIN_CASE(7) SHEEP_FIN_CASE(8)
        SHEEP_FIN_WAVE(9) SHEEP_FIN_WAVE(10) SHEEP_FIN_WAVE(11) SHEEP_FIN_WAVE(12) SHEEP_FIN_WAVE(13)
#undef SHEEP_FIN_CASE
#undef SHEEP_FIN_WAVE
#undef SHEEP_FIN_LANES
#undef SHEEP_FIN_HEAVY
        default: throw Error(SHEEP_ERR_ARG, "etree: bad finishing block size");
      }
      if (g_debug_etree) {
        std::vector<uint64_t> h(nb + 1);
        uint64_t nh = 0;
        HIP_CHECK(hipMemcpyAsync(h.data(), eb, (nb + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        HIP_CHECK(hipMemcpyAsync(&nh, n_lh + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        c.sync();
        uint64_t mx = 0, nonempty = 0;
        for (uint64_t b = 0; b < nb; ++b) {
          mx = std::max(mx, h[b + 1] - h[b]);
          nonempty += h[b + 1] > h[b];
        }
        fprintf(stderr, "etree finish B %d nf %lu live %lu blocks %lu nonempty %lu heavy %lu max-edges %lu\n", FINB,
                (unsigned long)nf, (unsigned long)h[nb], (unsigned long)nb, (unsigned long)nonempty, (unsigned long)nh,
                (unsigned long)mx);
      }
    }
  }
  if (!c.timing && !g_debug_etree) return;
  // algorithmic bytes: split reads the list and the bucket and writes the
  // three lists; hooking reads each light edge once per round it takes part in; the
  // cross pass reads the edge and writes its top; apply reads edge, top, m and claim
  // and appends the contraction
  // (the timers of the run that launched these levels: counted even if timing was switched
  // off before they were read)
  auto count = [&c, nglobal](const uint64_t *h) {
    for (int lvl = 0; lvl < nglobal; ++lvl) {
      const uint64_t *r = &h[(uint64_t)lvl * ST_ROW];
      uint64_t hooked = r[ST_NL];
      for (int k = 0; k < HOOK_ROUNDS - 1; ++k) hooked += r[ST_HOOK + k];
      c.timers["etree_split"].bytes += 8 * (r[ST_LIVE] + r[ST_R0]) + 8 * (r[ST_KEPT] + r[ST_NL] + r[ST_NX]);
      c.timers["etree_union"].bytes += 8 * hooked + 8 * r[ST_NL];
      c.timers["etree_cross"].bytes += 12 * r[ST_NX];
      c.timers["etree_apply"].bytes += 20 * r[ST_NX];
    }
  };
  const size_t sbytes = (size_t)L * ST_ROW * sizeof(uint64_t);
  if (!g_debug_etree) {   // counted when the timers are read: no round trip in a timed run
    c.defer_bytes(stats, sbytes, [count](const void *h) { count((const uint64_t *)h); });
    return;
  }
  std::vector<uint64_t> h((uint64_t)L * ST_ROW);
  HIP_CHECK(hipMemcpyAsync(h.data(), stats, sbytes, hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.timing) count(h.data());
  for (int lvl = 0; lvl < nglobal; ++lvl) {
    const uint64_t *r = &h[(uint64_t)lvl * ST_ROW];
    if (g_debug_etree)
      fprintf(stderr, "etree lvl %d s %d list %lu bucket %lu kept %lu light %lu cross %lu contractions %lu hook-left %lu %lu %lu\n",
              lvl, L - 1 - lvl, (unsigned long)r[ST_LIVE], (unsigned long)r[ST_R0], (unsigned long)r[ST_KEPT],
              (unsigned long)r[ST_NL], (unsigned long)r[ST_NX], (unsigned long)r[ST_CONTR], (unsigned long)r[ST_HOOK],
              (unsigned long)r[ST_HOOK + 1], (unsigned long)r[ST_HOOK + 2]);
  }
}

void relabel_and_tree(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                      uint64_t n, sheep_jnode *tree) {
  c.step_edges = Ctx::StepEdges();
  uint32_t *pst = c.get_as<uint32_t>("bt_pst", n ? n : 1);
  uint32_t *parent = c.get_as<uint32_t>("bt_parent", n ? n : 1);
  HIP_CHECK(hipMemsetAsync(pst, 0, n * sizeof(uint32_t), c.stream));
  // the relabelled edges die with the grouping below: their workspace is the elimination
  // tree's second list buffer (et_list2), filled only by the levels
  uint64_t *edges = c.get_as<uint64_t>("et_list2", nrec ? nrec : 1);
  unsigned long long *d = (unsigned long long *)c.d_scalars + 8;
  HIP_CHECK(hipMemsetAsync(d + 1, 0, sizeof(uint64_t), c.stream));
  uint64_t m = nrec;   // edges[i] per record, DEAD holes included (k_relabel)
  bool bucketed = false;   // (k_relabel's edges keep one slot per record: no step edges for the evaluator)
  int L = 0;
  uint32_t clo = 0;
  LoGroup lg;
  bool counted = false;
  if (n >= 2) {
    spread_params(n, &L, &clo);
    lo_group_prepare(c, n, L, clo, lg);
  }
  if (nrec) {
    TimedRegion tr(c, "relabel", 20 * nrec);   // record + 2 pos gathers
    // head-bucketed relabel (hist.hip) when the key range fits its LDS buckets; it also
    // counts the edges for the grouping below
    m = relabel_bucketed(c, rec, nrec, pos, pos_size, n, pst, edges, d + 1, n >= 2 ? &lg : nullptr, &counted);
    bucketed = m != UINT64_MAX;
    if (m == UINT64_MAX) {
      m = nrec;
      hipLaunchKernelGGL(k_relabel, dim3(grid_tiles(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, pos, pos_size, pst,
                         edges, d + 1);
      LAUNCH_CHECK();
    }
  }
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 9, d + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.h_scalars[9]) throw Error(SHEEP_ERR_RANGE, "vector::_M_range_check: neighbour vid beyond the sequence's index (jtree.cpp:75)");
  if (n >= 2 && m) {
    uint64_t *r0 = c.get_as<uint64_t>("bt_grouped", m);
    uint64_t *seg = c.get_as<uint64_t>("bt_seg", 2 * (uint64_t)L);
    {
      // pst = histogram of the edges' lo; the same passes group the edges by lo
      TimedRegion tr(c, "pst_group", 20 * m);
      const uint64_t grouped = group_edges_by_lo(c, edges, m, lg, pst, r0, seg, counted);
      if (bucketed && grouped != UINT64_MAX) {   // (read by sheep_evaluate_step until the next map)
        Ctx::StepEdges &se = c.step_edges;
        se.rec = rec;
        se.nrec = nrec;
        se.pos = pos;
        se.pos_size = pos_size;
        se.n = n;
        se.edges = r0;
        se.pst = pst;
        se.m_pairs = m;
        se.m_valid = grouped;
        se.valid = true;
      }
    }
    TimedRegion tr(c, "etree", 8 * m);
    etree_from_edges(c, r0, m, n, parent, seg, c.tune.fin_map_bits, -1, 0, 0, c.tune.top_bits,
                     (c.tune.hook_batch >= 2 ? HOOK_BATCH : 0) | (c.tune.hook_up >= 2 ? HOOK_UP : 0));
  } else {
    fill_u32(c, parent, n, INVALID);
  }
  if (n) {
    hipLaunchKernelGGL(k_pack_tree, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, parent, pst, n, tree);
    LAUNCH_CHECK();
  }
}

// The merge's edges: every node's distinct parents over the K trees, compacted in node
// (= lo) order, and their first-activity group bounds (group s = the lo range whose
// spread has its highest zero bit at s).  Returns the edge count; pst = the summed weights.
// Groups b < bmax (activated at the levels a part of a split merge runs alone) are cut to
// the part's node range [v_lo, v_hi).
static uint64_t merge_edges(Ctx &c, const TreeSet &ts, uint32_t K, uint64_t n, uint32_t *pst, uint64_t **edges_out,
                            uint64_t **seg_out, int *L_out, int bmax = 0, uint64_t v_lo = 0, uint64_t v_hi = 0) {
  int L;
  uint32_t clo;
  spread_params(n, &L, &clo);
  uint32_t *off = c.get_as<uint32_t>("mg_off", n + 1);
  unsigned long long *d = (unsigned long long *)c.d_scalars + 10;
  HIP_CHECK(hipMemsetAsync(d + 1, 0, sizeof(uint64_t), c.stream));
  const unsigned g = grid_for(n);
#define SHEEP_KM(KM) hipLaunchKernelGGL(k_tree_count<KM>, dim3(g), dim3(BLOCK), 0, c.stream, ts, K, n, off, pst, d + 1)
  if (K <= 2) SHEEP_KM(2); else if (K <= 4) SHEEP_KM(4); else if (K <= 8) SHEEP_KM(8);
  else if (K <= 16) SHEEP_KM(16); else if (K <= 32) SHEEP_KM(32); else SHEEP_KM(64);
#undef SHEEP_KM
  LAUNCH_CHECK();
  scan_exclusive_u32(c, off, off, n, off + n);
  c.h_scalars[12] = 0;   // the u32 total lands in the low half
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 11, d + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 12, off + n, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.h_scalars[11]) throw Error(SHEEP_ERR_ARG, "merge: a parent is not a later node of the tree");
  const uint64_t m = c.h_scalars[12];
  uint64_t *edges = c.get_as<uint64_t>("mg_edges", m ? m : 1);
#define SHEEP_KM(KM) hipLaunchKernelGGL(k_tree_write<KM>, dim3(g), dim3(BLOCK), 0, c.stream, ts, K, n, (const uint32_t *)off, edges)
  if (K <= 2) SHEEP_KM(2); else if (K <= 4) SHEEP_KM(4); else if (K <= 8) SHEEP_KM(8);
  else if (K <= 16) SHEEP_KM(16); else if (K <= 32) SHEEP_KM(32); else SHEEP_KM(64);
#undef SHEEP_KM
  LAUNCH_CHECK();
  // group b = lo with spread(lo) in [2^L - 2^(b+1), 2^L - 2^b)
  auto first_lo = [&](uint64_t y) {   // min lo with spread(lo) >= y
    uint64_t a = 0, z = n;
    while (a < z) {
      const uint64_t x = (a + z) / 2;
      if (x + ((x * (uint64_t)clo) >> 32) >= y) z = x; else a = x + 1;
    }
    return a;
  };
  SegNodes sn{};
  for (int b = 0; b < L; ++b) {
    uint64_t g0 = first_lo((1ull << L) - (2ull << b)), g1 = first_lo((1ull << L) - (1ull << b));
    if (b < bmax) {   // the part's share of the group: a node range, so a range of the edges
      g0 = std::min(std::max(g0, v_lo), v_hi);
      g1 = std::max(std::min(g1, v_hi), g0);
    }
    sn.node[b] = (uint32_t)g0;
    sn.node[L + b] = (uint32_t)g1;
  }
  uint64_t *seg = c.get_as<uint64_t>("mg_seg", 2 * (uint64_t)L);
  hipLaunchKernelGGL(k_seg_at, dim3(1), dim3(64), 0, c.stream, (const uint32_t *)off, sn, 2 * L, seg);
  LAUNCH_CHECK();
  *edges_out = edges;
  *seg_out = seg;
  *L_out = L;
  return m;
}

// min node x with spread(x) >= y
static uint64_t first_node(uint64_t n, uint32_t clo, uint64_t y) {
  uint64_t a = 0, z = n;
  while (a < z) {
    const uint64_t x = (a + z) / 2;
    if (x + ((x * (uint64_t)clo) >> 32) >= y) z = x; else a = x + 1;
  }
  return a;
}

// The elimination tree of the union of the K trees' parent-edge sets (JNodeTable::merge,
// jnode.cpp:174-201, for K = 2; for K > 2 the same tree as K - 1 pairwise merges in any
// order — merge is associative and commutative — i.e. mpi_merge's whole reduction,
// jnode.cpp:203-250, in one pass).
//
// Split merge (nparts = 2^l > 1): after the first l levels every live edge lies inside one
// of nparts subproblems, and each is finished independently; this call runs the first l
// levels in full and then only subproblem `part` (its share of the list, of the later
// groups and of the per-block finish).  Every node's pst and the parent of every node
// assigned in the first l levels are the full merge's; below them only the nodes of the
// part's range [*v_lo, *v_hi) are (the others keep INVALID where a later level would
// have linked them).  nparts GPUs that each run one part together hold the whole tree.
static void merge_set(Ctx &c, const TreeSet &ts, uint32_t K, uint64_t n, sheep_jnode *out, uint32_t part = 0,
                      uint32_t nparts = 1, uint64_t *v_lo = nullptr, uint64_t *v_hi = nullptr) {
  if ((uint64_t)K * n >= 0xFFFFFFFFull) throw Error(SHEEP_ERR_ARG, "merge: too many parent edges for one pass");
  uint32_t *pst = c.get_as<uint32_t>("mg_pst", n);
  uint32_t *parent = c.get_as<uint32_t>("mg_parent", n);
  uint64_t *edges = nullptr, *seg = nullptr;
  int L = 0, l = 0;
  uint32_t clo = 0;
  while ((1u << l) < nparts) ++l;
  if (nparts == 0 || (1u << l) != nparts || part >= nparts) throw Error(SHEEP_ERR_ARG, "merge: parts must be a power of two");
  uint64_t lo = 0, hi = n;
  if (n >= 2) spread_params(n, &L, &clo);
  // only as many parts as global levels (below them the per-block finish runs whole)
  const int fin_merge = c.tune.fin_merge_bits;
  const int nglobal = L > fin_merge ? L - fin_merge : 0;
  if (nparts > 1 && (l >= nglobal || L > 31)) l = 0;   // too small a tree to split: every part runs it all
  uint32_t ylo = 0, yhi = 0;
  if (l > 0) {
    ylo = (uint32_t)((uint64_t)part << (L - l));
    yhi = (uint32_t)((uint64_t)(part + 1) << (L - l));
    lo = first_node(n, clo, ylo);
    hi = first_node(n, clo, yhi);
  }
  if (v_lo) *v_lo = lo;
  if (v_hi) *v_hi = hi;
  if (n < 2) {
    // one node: no edges; the weights still add up
    merge_edges(c, ts, K, n, pst, &edges, &seg, &L);
    fill_u32(c, parent, n, INVALID);
  } else {
    TimedRegion tr(c, "merge", 8 * (uint64_t)K * n);   // the K trees
    // groups activated at levels >= l are b < L - l
    const uint64_t m = merge_edges(c, ts, K, n, pst, &edges, &seg, &L, l > 0 ? L - l : 0, lo, hi);
    etree_from_edges(c, edges, m, n, parent, seg, fin_merge, l > 0 ? l : -1, ylo, yhi, 0,
                     (c.tune.hook_batch >= 1 ? HOOK_BATCH : 0) | (c.tune.hook_up >= 1 ? HOOK_UP : 0), c.tune.merge_cut_bits);
  }
  hipLaunchKernelGGL(k_pack_tree, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, parent, pst, n, out);
  LAUNCH_CHECK();
}

void tree_planes(Ctx &c, const sheep_jnode *tree, uint64_t n, uint32_t *parent, uint32_t *pst) {
  if (!n) return;
  hipLaunchKernelGGL(k_tree_planes, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, tree, n, parent, pst);
  LAUNCH_CHECK();
}

void merge_trees_part(Ctx &c, const sheep_jnode *trees, uint32_t K, uint64_t n, uint32_t part, uint32_t nparts,
                      sheep_jnode *out, uint64_t *v_lo, uint64_t *v_hi) {
  if (K == 0) throw Error(SHEEP_ERR_ARG, "merge: no trees");
  if (K > MERGE_KMAX) throw Error(SHEEP_ERR_ARG, "split merge: more trees than one pass takes");
  if (n == 0) {
    *v_lo = *v_hi = 0;
    return;
  }
  merge_set(c, TreeSet{trees, trees + n, n}, K, n, out, part, nparts, v_lo, v_hi);
}

void merge_trees(Ctx &c, const sheep_jnode *a, const sheep_jnode *b, uint64_t n, sheep_jnode *out) {
  if (n == 0) return;
  merge_set(c, TreeSet{a, b, 0}, 2, n, out);
}

// The K-way merge from parent planes (planes[k * n + i] = node i's parent in tree k) and the
// trees' summed pst (pst_sum[i]): the same tree as merge_trees_many over the whole trees.
void merge_parent_planes(Ctx &c, const uint32_t *planes, const uint32_t *pst_sum, uint32_t K, uint64_t n,
                         sheep_jnode *out) {
  if (n == 0) return;
  if (K == 0 || K > MERGE_KMAX) throw Error(SHEEP_ERR_ARG, "merge: 1..64 parent planes per pass");
  TreeSet ts{nullptr, nullptr, n};
  ts.planes = planes;
  ts.pst_sum = pst_sum;
  merge_set(c, ts, K, n, out);
}

void merge_trees_many(Ctx &c, const sheep_jnode *trees, uint32_t K, uint64_t n, sheep_jnode *out) {
  if (n == 0) return;
  if (K == 0) throw Error(SHEEP_ERR_ARG, "merge: no trees");
  if (K == 1) {
    HIP_CHECK(hipMemcpyAsync(out, trees, n * sizeof(sheep_jnode), hipMemcpyDeviceToDevice, c.stream));
    return;
  }
  // MERGE_KMAX trees per pass; later passes merge the running result with the next ones
  uint32_t done = K < MERGE_KMAX ? K : MERGE_KMAX;
  merge_set(c, TreeSet{trees, trees + n, n}, done, n, out);
  while (done < K) {
    const uint32_t k = K - done < MERGE_KMAX - 1 ? K - done : MERGE_KMAX - 1;
    merge_set(c, TreeSet{out, trees + (uint64_t)done * n, n}, k + 1, n, out);
    done += k;
  }
}

}  // namespace sheep
