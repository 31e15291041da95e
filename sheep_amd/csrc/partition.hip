// partition.hip — Partition(seq, jnodes, k, balance, vtx, pst, pre) (partition.cpp:50-67)
// with forwardPartition (partition.cpp:86-157), and JNodeTable::Facts (jnode.cpp:256-290).
//
// forwardPartition walks ids ascending: cb[id] += w(id); if cb[id] > max it std::sorts
// the kids by cb (descending; the kid table keeps that order for the next k) and
// first-fit packs unassigned kids into bins until cb[id] <= max; then cb[parent] +=
// cb[id].  A descending pass pushes parts down and packs roots into the highest bin
// that fits.
//
// GPU formulation:
//   1. subtree sums S(v) on the GPU (Euler tour + prefix sums; tree_tour.hip);
//   2. R(v) = cb(v) when the pass reaches v.  Only H = {v : S(v) > max} (ancestor-
//      closed, R <= S) can pack, and the next packing node is the LOWEST id with
//      R > max (everything below it is final).  One GPU pass over H per packing event
//      subtracts the removed weight from the packed node and its ancestors (Euler-tour
//      interval test) and finds the next such id;
//   3. the host runs each packing with the reference's own std::sort on the node's
//      current kid order plus first-fit (the sorted segment is written back, so the
//      order persists across k like partition.cpp:104-106);
//   4. roots are packed host-side in descending id order (their final R);
//   5. the GPU pushes parts down: every node takes the part of its innermost assigned
//      ancestor-or-self (assigned = packed kids + roots), found by binary search over
//      the assigned nodes' Euler-tour intervals (laminar), then re-indexes jnid -> vid.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <vector>

#include "tree_tour.hpp"

namespace sheep {
namespace {

__global__ void k_weights(const sheep_jnode *__restrict__ tree, uint64_t n, int vtx, int pstw,
                          uint64_t *__restrict__ w, unsigned long long *__restrict__ total) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  uint64_t s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    uint64_t x = (vtx ? 1ull : 0ull) + (pstw ? (uint64_t)tree[i].pst_weight : 0ull);
    w[i] = x;
    s += x;
  }
  block_atomic_add(total, s);
}

// tour-order value array for a sum channel: val[tU[c]] = up(c), val[tD[c]] = down(c)
__global__ void k_tour_vals(const uint32_t *__restrict__ tD, const uint32_t *__restrict__ tU, uint64_t n,
                            const uint64_t *__restrict__ up, const uint64_t *__restrict__ down_or_null,
                            int mode, uint64_t *__restrict__ val) {
  // mode 0: D = 0, U = up[c];   mode 1: D = +up[c], U = -up[c];   mode 2: D = +1, U = -1
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < n; c += stride) {
    uint32_t d = tD[c];
    if (d == INVALID) continue;
    uint64_t x = mode == 2 ? 1ull : up[c];
    if (mode == 0) { val[d] = 0; val[tU[c]] = x; }
    else { val[d] = x; val[tU[c]] = (uint64_t)0 - x; }
  }
}

__global__ void k_subtree(const uint32_t *__restrict__ parent, const uint32_t *__restrict__ tD,
                          const uint32_t *__restrict__ tU, uint64_t n, const uint64_t *__restrict__ w,
                          const uint64_t *__restrict__ E, uint64_t *__restrict__ S) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < n; c += stride) {
    if (parent[c] == INVALID) { S[c] = w[c]; continue; }
    S[c] = E[tU[c]] + w[c] - E[tD[c]];
  }
}
__global__ void k_root_sums(const uint32_t *__restrict__ parent, uint64_t n, uint64_t *__restrict__ S) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < n; c += stride) {
    uint32_t p = parent[c];
    if (p != INVALID && parent[p] == INVALID) atomicAdd((unsigned long long *)&S[p], (unsigned long long)S[c]);
  }
}

// order-preserving compaction of {v : pred(v)}, pred 0: S(v) > max (H);  1: root
constexpr int P_ITEMS = 8, P_TILE = BLOCK * P_ITEMS;
__device__ __forceinline__ bool pred_of(int which, uint64_t i, const uint64_t *S, uint64_t mx, const uint32_t *parent) {
  return which == 0 ? S[i] > mx : parent[i] == INVALID;
}
__global__ void k_pred_count(int which, const uint64_t *__restrict__ S, uint64_t mx, const uint32_t *__restrict__ parent,
                             uint64_t n, uint32_t *__restrict__ bcnt) {
  __shared__ uint32_t s[BLOCK / WAVE];
  uint64_t base = (uint64_t)blockIdx.x * P_TILE;
  uint32_t c = 0;
  for (int j = 0; j < P_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    if (i < n && pred_of(which, i, S, mx, parent)) ++c;
  }
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ void k_pred_write(int which, const uint64_t *__restrict__ S, uint64_t mx, const uint32_t *__restrict__ parent,
                             uint64_t n, const uint32_t *__restrict__ boff, uint32_t *__restrict__ ids,
                             uint32_t *__restrict__ rank) {
  __shared__ uint32_t wc[BLOCK / WAVE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t base = (uint64_t)blockIdx.x * P_TILE;
  uint32_t running = boff[blockIdx.x];
  for (int j = 0; j < P_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    bool f = i < n && pred_of(which, i, S, mx, parent);
    uint64_t m = __ballot(f);
    if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = running;
    for (int w = 0; w < wave; ++w) off += wc[w];
    if (i < n && rank) rank[i] = f ? off + (uint32_t)__popcll(m & lanemask_lt()) : INVALID;
    if (f) ids[off + __popcll(m & lanemask_lt())] = (uint32_t)i;
    running += wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();
  }
}

// Tour interval of every root with kids: [tD(first kid), tU(last kid)] in the kid order
// the tour was built from.  Taken before the host replay re-sorts kid segments.
__global__ void k_root_intervals(const uint32_t *__restrict__ rk, uint64_t nrk, const uint32_t *__restrict__ koff,
                                 const uint32_t *__restrict__ kids, const uint32_t *__restrict__ tD,
                                 const uint32_t *__restrict__ tU, uint32_t *__restrict__ rst,
                                 uint32_t *__restrict__ ren) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrk; i += stride) {
    uint32_t v = rk[i];
    rst[v] = tD[kids[koff[v]]];
    ren[v] = tU[kids[koff[v + 1] - 1]];
  }
}

// interval endpoints for assigned nodes: non-root -> [tD, tU]; root with kids -> its
// tour segment; root without kids -> none (INVALID)
__global__ void k_intervals(const uint32_t *__restrict__ ids, uint64_t m, const uint32_t *__restrict__ parent,
                            const uint32_t *__restrict__ koff, const uint32_t *__restrict__ rst,
                            const uint32_t *__restrict__ ren, const uint32_t *__restrict__ tD,
                            const uint32_t *__restrict__ tU, uint32_t *__restrict__ st, uint32_t *__restrict__ en) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += stride) {
    uint32_t v = ids[i];
    if (parent[v] != INVALID) { st[i] = tD[v]; en[i] = tU[v]; }
    else if (koff[v] < koff[v + 1]) { st[i] = rst[v]; en[i] = ren[v]; }
    else { st[i] = INVALID; en[i] = INVALID; }
  }
}

__global__ void k_push_down(const uint32_t *__restrict__ parent, const uint32_t *__restrict__ tD, uint64_t n,
                            const uint32_t *__restrict__ ast, const uint32_t *__restrict__ aen,
                            const int16_t *__restrict__ apart, const uint32_t *__restrict__ aencl, uint32_t na,
                            int16_t *__restrict__ parts, unsigned long long *__restrict__ err) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < n; v += stride) {
    if (parent[v] == INVALID) continue;   // roots are scattered directly; the fringe goes next
    uint32_t p = tD[v];
    uint32_t lo = 0, hi = na;              // last interval with start <= p
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (ast[mid] <= p) lo = mid + 1; else hi = mid; }
    if (lo == 0) { atomicAdd(err, 1ull); continue; }
    uint32_t j = lo - 1;
    while (j != INVALID && aen[j] < p) j = aencl[j];
    if (j == INVALID) { atomicAdd(err, 1ull); continue; }
    parts[v] = apart[j];
  }
}

__global__ void k_scatter_parts(const uint32_t *__restrict__ ids, const int16_t *__restrict__ pv, uint64_t m,
                                int16_t *__restrict__ parts) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += stride) parts[ids[i]] = pv[i];
}

__global__ void k_fill_i16(int16_t *__restrict__ p, uint64_t n, int16_t v) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) p[i] = v;
}

// jnid -> vid over the sequence's seq_n entries (partition.cpp:62-66); cnt = {#part 0,
// #part 1, max part + 1} over the converted entries (the print counts, partition.h:135-143;
// slots left INVALID_PART count for neither).  Out-of-range vids are the caller's check
// (pos_size = max(seq) + 1).
__global__ void k_parts_to_vid(const uint32_t *__restrict__ seq, uint64_t seq_n, const int16_t *__restrict__ parts,
                               int16_t *__restrict__ pv, unsigned long long *__restrict__ cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  uint64_t c0 = 0, c1 = 0, mx = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < seq_n; i += stride) {
    const int16_t p = parts[i];
    pv[seq[i]] = p;
    c0 += p == 0;
    c1 += p == 1;
    mx = (uint64_t)(p + 1) > mx ? (uint64_t)(p + 1) : mx;
  }
  block_atomic_add(&cnt[0], c0);
  block_atomic_add(&cnt[1], c1);
  block_atomic_max(&cnt[2], mx);
}

// The same by a gather over the vid slots through pos (the sequence's inverse): pv is
// written once, in order, INVALID_PART included, and the jnid-indexed parts (2 B per node,
// L2-resident) are read at random instead of stored at random (the scatter above wrote
// ~24 B per 2-B value: 805 MB for 66 MB at RMAT-26).  A slot whose jnid is >= seq_n (a
// sequence shorter than the tree's index) is not converted, as above.
__global__ void k_parts_from_pos(const uint32_t *__restrict__ pos, uint64_t pos_size, uint64_t seq_n,
                                 const int16_t *__restrict__ parts, int16_t *__restrict__ pv,
                                 unsigned long long *__restrict__ cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK * 4;
  uint64_t c0 = 0, c1 = 0, mx = 0;
  for (uint64_t i0 = (uint64_t)blockIdx.x * BLOCK * 4 + threadIdx.x; i0 < pos_size; i0 += stride) {
    uint32_t j[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t v = i0 + (uint64_t)k * BLOCK;
      j[k] = v < pos_size ? pos[v] : INVALID;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t v = i0 + (uint64_t)k * BLOCK;
      if (v >= pos_size) continue;
      const int16_t p = j[k] < seq_n ? parts[j[k]] : SHEEP_INVALID_PART;
      pv[v] = p;
      if (j[k] >= seq_n) continue;
      c0 += p == 0;
      c1 += p == 1;
      mx = (uint64_t)(p + 1) > mx ? (uint64_t)(p + 1) : mx;
    }
  }
  block_atomic_add(&cnt[0], c0);
  block_atomic_add(&cnt[1], c1);
  block_atomic_max(&cnt[2], mx);
}

// ---- raking: exact subtree sums of the light fringe -------------------------------
// Round r finishes every node whose kids are all finished and whose accumulated weight
// acc (own weight + finished kids' sums) is <= max_component: acc is then its subtree sum
// S, it cannot pack (only S > max can), and it is added into its parent.  Elimination
// trees of power-law graphs are mostly fringe (RMAT: 66% leaves; two rounds finish ~74%
// of the nodes, a third only 3% more for its scattered atomics), so the Euler tour below
// only ranks the remaining core T'.
constexpr int RAKE_ROUNDS = 2;

// The rake state of a node is ONE u64: acc << 24 | kids not yet finished, so a finished
// kid's push is a single atomicAdd(acc_kid << 24 - 1) on its parent (no borrow: the
// count is >= 1 while the kid is unfinished).  Needs every node's kid count < 2^24 and
// the total weight < 2^40 (else the partition runs without raking: all nodes are core).
constexpr int RAKE_CNT_BITS = 24;
constexpr uint64_t RAKE_CNT_MASK = (1ull << RAKE_CNT_BITS) - 1;

// round 1's mark fused in: a leaf finishes when its weight is <= max_component.  lw[v] =
// the push a round-1 leaf makes on its parent (0 for every other node), for k_rake_pull1.
// LW: the push word as lw[v] itself (u64), or, when every finishing weight fits 32 bits
// (max_component < 2^32 - 1), as w + 1 in a u32 (0: no push) — half the bytes for
// k_rake_pull1's random gather over it.
template <typename LW>
__global__ void k_rake_init(const uint32_t *__restrict__ koff, const uint64_t *__restrict__ w, uint64_t n, uint64_t maxc,
                            bool rake, uint64_t *__restrict__ pk, uint8_t *__restrict__ fin, LW *__restrict__ lw) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < n; v += stride) {
    const uint32_t nk = koff[v + 1] - koff[v];
    const bool f = rake && nk == 0 && w[v] <= maxc;
    pk[v] = (w[v] << RAKE_CNT_BITS) | nk;
    fin[v] = f;
    if (sizeof(LW) == 8) lw[v] = f ? (w[v] << RAKE_CNT_BITS) - 1 : 0;
    else lw[v] = f ? (LW)(w[v] + 1) : 0;
  }
}
template <typename LW> __device__ __forceinline__ uint64_t lw_push(LW x) {
  if (sizeof(LW) == 8) return (uint64_t)x;
  return x ? ((uint64_t)(x - 1) << RAKE_CNT_BITS) - 1 : 0;
}
// Round 1 as a PULL over the kid table: kids[i] sits in the list of kpar[i] (lists are
// contiguous, parents ascending), so a wave sums its lanes' pushes per parent run and
// adds each run with one atomic — a few neighbouring lines per wave instead of one
// scattered atomic per leaf (66% of the nodes; ~1.1 ms of pushes at RMAT-26).
template <typename LW>
__global__ __launch_bounds__(BLOCK) void k_rake_pull1(const uint32_t *__restrict__ kids, const uint32_t *__restrict__ kpar,
                                                      uint64_t nkids, const LW *__restrict__ lw,
                                                      uint64_t *__restrict__ pk) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t iters = (nkids + stride - 1) / stride;
  const int lane = (int)__lane_id();
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, i += stride) {   // wave-uniform trip count (shuffles)
    const bool live = i < nkids;
    const uint32_t p = live ? kpar[i] : INVALID;
    uint64_t x = live ? lw_push<LW>(lw[kids[i]]) : 0;
    // inclusive segmented sum over runs of equal p (runs are contiguous lanes)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      const uint32_t q = __shfl_up(p, o, 64);
      if (lane >= o && q == p) x += y;
    }
    const uint32_t pn = __shfl_down(p, 1, 64);
    const bool last = lane == 63 || pn != p;   // the run's last lane holds its sum
    if (live && last && x) atomicAdd((unsigned long long *)&pk[p], (unsigned long long)x);
  }
}
// mark, then pull: the two phases keep a round's finished set independent of timing
__global__ void k_rake_mark(const uint64_t *__restrict__ pk, uint64_t n, uint64_t maxc, uint8_t round,
                            uint8_t *__restrict__ fin) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < n; v += stride) {
    const uint64_t x = pk[v];
    if (!fin[v] && (x & RAKE_CNT_MASK) == 0 && (x >> RAKE_CNT_BITS) <= maxc) fin[v] = round;
  }
}
// Round 2 as a pull too, after k_rake_mark: a kid marked 2 pushes its packed sum on its
// parent (a node marked 2 has no kid marked 2, so its own word is stable here), and every
// list entry's core flag (kid not finished) is written in list order — the core table's
// scan input, which k_core_flags built with a second random read of fin per kid.
__global__ __launch_bounds__(BLOCK) void k_rake_pull2(const uint32_t *__restrict__ kids, const uint32_t *__restrict__ kpar,
                                                      uint64_t nkids, const uint8_t *__restrict__ fin,
                                                      uint64_t *__restrict__ pk, uint32_t *__restrict__ flag) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t iters = (nkids + stride - 1) / stride;
  const int lane = (int)__lane_id();
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, i += stride) {   // wave-uniform trip count (shuffles)
    const bool live = i < nkids;
    const uint32_t p = live ? kpar[i] : INVALID;
    const uint32_t k = live ? kids[i] : 0;
    const uint8_t f = live ? fin[k] : 1;
    if (live) flag[i] = f == 0;
    uint64_t x = f == 2 ? ((pk[k] >> RAKE_CNT_BITS) << RAKE_CNT_BITS) - 1 : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      const uint32_t q = __shfl_up(p, o, 64);
      if (lane >= o && q == p) x += y;
    }
    const uint32_t pn = __shfl_down(p, 1, 64);
    const bool last = lane == 63 || pn != p;
    if (live && last && x) atomicAdd((unsigned long long *)&pk[p], (unsigned long long)x);
  }
}

// The core's kid table: the kid table's segments with finished kids dropped (order kept);
// finished nodes become isolated (parent INVALID, no kids) so the tour skips them.
__global__ void k_core_flags(const uint32_t *__restrict__ kids, uint64_t nk, const uint8_t *__restrict__ fin,
                             uint32_t *__restrict__ flag) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < nk; j += stride) flag[j] = fin[kids[j]] == 0;
}
__global__ void k_core_build(const uint32_t *__restrict__ kids, uint64_t nk, const uint32_t *__restrict__ koff,
                             const uint32_t *__restrict__ parent, const uint8_t *__restrict__ fin, uint64_t n,
                             const uint32_t *__restrict__ pref, uint32_t *__restrict__ ckids,
                             uint32_t *__restrict__ ckoff, uint32_t *__restrict__ cparent, uint64_t *__restrict__ pk) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t t0 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t j = t0; j < nk; j += stride) {   // the scanned core flags: entry j is core iff pref steps
    const uint32_t pj = pref[j];
    if (pref[j + 1] != pj) ckids[pj] = kids[j];
  }
  for (uint64_t v = t0; v <= n; v += stride) {
    ckoff[v] = pref[koff[v]];
    if (v < n) {
      cparent[v] = fin[v] ? INVALID : parent[v];
      pk[v] >>= RAKE_CNT_BITS;   // acc out of the packed rake words (the pulls are done)
    }
  }
}

// ---- packing events with lazily computed residuals ------------------------------------
// R(a) = cb(a) when forwardPartition's ascending pass reaches a = S(a) minus the weight
// removed by every earlier packing at a or below a.  A packing at a non-root v removes
// delta from v and its ancestors: a is hit iff tD(v) lies in a's tour interval.  The host
// keeps the events sorted by tD(v) with prefix sums of their deltas (EvTable, copied to
// the device before each scan), so R(a) = S(a) - (prefix sum over the events inside a's
// interval): two binary searches, whatever the number of events.  A packing at a root
// changes only that root, which no later candidate is (candidates have larger ids), and
// the host subtracts it from the root's final residual itself.
constexpr int EV_LDS = 4096;   // event table entries held in LDS (larger tables: global reads)

// a's tour interval in the core: [tD, tU] for a non-root, its kids' span for a core root
__device__ __forceinline__ void node_interval(uint32_t a, const uint32_t *cparent, const uint32_t *ckoff,
                                              const uint32_t *tD, const uint32_t *tU, const uint32_t *rst,
                                              const uint32_t *ren, uint32_t &lo, uint32_t &hi) {
  if (cparent[a] != INVALID) { lo = tD[a]; hi = tU[a]; }
  else if (ckoff[a] < ckoff[a + 1]) { lo = rst[a]; hi = ren[a]; }
  else { lo = INVALID; hi = INVALID; }
}

// event table: m sorted positions, prefix sums pre[0..m] (pre[i] = sum of deltas before i)
struct EvView {
  const uint32_t *pos;
  const uint64_t *pre;
  uint32_t m;
  __device__ uint32_t lower(uint32_t x) const {   // first i with pos[i] >= x
    uint32_t a = 0, b = m;
    while (a < b) { const uint32_t c = (a + b) >> 1; if (pos[c] < x) a = c + 1; else b = c; }
    return a;
  }
  __device__ uint64_t removed(uint32_t lo, uint32_t hi) const {   // deltas with lo <= pos <= hi
    if (lo == INVALID || m == 0) return 0;
    const uint32_t i = lower(lo), j = hi == INVALID ? m : lower(hi + 1);
    return j > i ? pre[j] - pre[i] : 0;
  }
  // the same for P intervals at once: branchless searches with the table-wide trip count,
  // so the 2P searches' loads of one step are in flight together (one search at a time cost
  // the persistent event kernel 7 us an event at 68 entries)
  template <int P>
  __device__ void removed_many(const uint32_t (&lo)[P], const uint32_t (&hi)[P], uint64_t (&out)[P]) const {
    uint32_t bl[P], bh[P], xh[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      bl[j] = 0;
      bh[j] = 0;
      xh[j] = hi[j] == INVALID ? INVALID : hi[j] + 1;   // (pos < INVALID: lower(INVALID) = m)
      out[j] = 0;
    }
    if (m == 0) return;
    for (uint32_t n = m; n > 1; n -= n >> 1) {
      const uint32_t half = n >> 1;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        bl[j] = pos[bl[j] + half] < lo[j] ? bl[j] + half : bl[j];
        bh[j] = pos[bh[j] + half] < xh[j] ? bh[j] + half : bh[j];
      }
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const uint32_t i = bl[j] + (pos[bl[j]] < lo[j]), k = bh[j] + (pos[bh[j]] < xh[j]);
      out[j] = lo[j] != INVALID && k > i ? pre[k] - pre[i] : 0;
    }
  }
};

// Tables of up to EV_ARG events travel as a kernel argument (device-side kernarg memory):
// reading the mapped host copy cost each event launch a PCIe round trip (2.7 us).
constexpr uint32_t EV_ARG = 128;
struct EvArg {
  uint32_t m;
  uint32_t pos[EV_ARG];
  uint64_t pre[EV_ARG + 1];
};
__device__ __forceinline__ EvView load_arg(const EvArg &arg, uint32_t *spos, uint64_t *spre) {
  for (uint32_t i = threadIdx.x; i <= arg.m; i += blockDim.x) {
    if (i < arg.m) spos[i] = arg.pos[i];
    spre[i] = arg.pre[i];
  }
  __syncthreads();
  return EvView{spos, spre, arg.m};
}

// loads the table into LDS when it fits (every thread of the block must call it)
__device__ __forceinline__ EvView load_table(const uint32_t *gpos, const uint64_t *gpre, uint32_t m, uint32_t *spos,
                                             uint64_t *spre) {
  if (m > EV_LDS) return EvView{gpos, gpre, m};
  for (uint32_t i = threadIdx.x; i <= m; i += blockDim.x) {
    if (i < m) spos[i] = gpos[i];
    spre[i] = gpre[i];
  }
  __syncthreads();
  return EvView{spos, spre, m};
}

// The event search's chunks: 512 entries reach the hit in fewer dependent rounds per
// workgroup (RMAT-26 / Chung-Lu events: 2048-entry chunks 2.2 / 4.6 ms, 512 2.0 / 3.9 ms)
constexpr int EVI = 2, EV_CH = BLOCK * EVI;
constexpr uint32_t EV_STAGE = 1u << 16;   // mapped staging area (kids)
constexpr uint32_t EV_INLINE = 4096;      // kid lists staged by the event kernel itself

__device__ __forceinline__ void stage_kids(const EvView &ev, uint32_t beg, uint32_t lim, uint32_t j0, uint32_t stride,
                                           const uint32_t *kids, const uint64_t *S, const uint32_t *cparent,
                                           const uint32_t *tD, const uint32_t *tU, uint32_t *kid_out, uint64_t *r_out) {
  for (uint32_t j = j0; j < lim; j += stride) {
    const uint32_t kid = kids[beg + j];
    uint64_t r = S[kid];
    if (cparent[kid] != INVALID) r -= ev.removed(tD[kid], tU[kid]);   // fringe kids never had a packing below
    kid_out[j] = kid;
    r_out[j] = r;
  }
}

// One event's search by every workgroup: chunks of the heavy set in index order, from the
// last packing node on, until a hit below the chunk is known; the last workgroup to
// finish (event_done) then sees every other workgroup's atomicMin in `found`.
// The search state (evprev, found, done) is only ever touched by atomic read-modify-writes,
// which every XCD sees at one coherent point: a plain or atomic LOAD is served from the
// reading XCD's own L2 and can return a value an earlier event left there (a stale hit
// below every chunk made one search end empty: seen with 512-entry chunks on C4).
struct EvShared {
  unsigned long long best[BLOCK / WAVE];
  unsigned long long word;   // one thread's atomic read, for the workgroup
  bool last;
};
// the workgroup's least hit among P candidates per thread (loaded by the caller) into `found`
// (thread 0: `dep` collects the atomic's return, which event_done's ticket waits for)
template <int P>
__device__ void event_hits(const EvView &ev, const uint32_t (&ca)[P], const uint32_t (&cs)[P], const uint32_t (&ce)[P],
                           const uint64_t (&cr)[P], uint64_t base, uint32_t vlast, uint64_t maxc,
                           unsigned long long *__restrict__ found, EvShared &sh, uint32_t &dep) {
  unsigned long long best = ~0ull;
  uint64_t rm[P];
  ev.removed_many<P>(cs, ce, rm);
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const uint32_t a = ca[j];
    if (a == INVALID || (vlast != INVALID && a <= vlast)) continue;
    const uint64_t r = cr[j] - rm[j];
    if (r > maxc) {
      const unsigned long long key = ((unsigned long long)a << 32) | (base + (uint64_t)j * BLOCK + threadIdx.x);
      best = key < best ? key : best;
    }
  }
  best = wave_min(best);
  if ((threadIdx.x & 63) == 0) sh.best[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = sh.best[0];
    for (int w = 1; w < BLOCK / WAVE; ++w) b = sh.best[w] < b ? sh.best[w] : b;
    if (b != ~0ull) dep |= (uint32_t)atomicMin(found, b);
  }
  __syncthreads();
}
// every candidate's four words loaded before any is decoded (a load behind the id check
// of the same candidate serialised two latencies per candidate: 24 us a scan)
template <int P>
__device__ __forceinline__ void event_load(const uint32_t *__restrict__ hids, const uint64_t *__restrict__ SH,
                                           const uint32_t *__restrict__ hst, const uint32_t *__restrict__ hen,
                                           uint64_t nh, uint64_t base, uint32_t (&ca)[P], uint32_t (&cs)[P],
                                           uint32_t (&ce)[P], uint64_t (&cr)[P]) {
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const uint64_t h = base + (uint64_t)j * BLOCK + threadIdx.x;
    const bool in = h < nh;
    ca[j] = in ? hids[h] : INVALID;
    cr[j] = in ? SH[h] : 0;
    cs[j] = in ? hst[h] : INVALID;
    ce[j] = in ? hen[h] : INVALID;
  }
}
// the chunks from `from` on, workgroup-strided; `check_first`: a hit may already be known
// (the first chunk of a fresh search is not checked: `found` was reset with the last event)
__device__ void event_scan(const EvView &ev, const uint32_t *__restrict__ hids, uint64_t nh,
                           const uint64_t *__restrict__ SH, const uint32_t *__restrict__ hst,
                           const uint32_t *__restrict__ hen, uint64_t maxc, uint64_t from, uint32_t vlast,
                           bool check_first, unsigned long long *__restrict__ found, EvShared &sh, uint32_t &dep) {
  for (uint64_t ch = blockIdx.x;; ch += gridDim.x) {
    const uint64_t base = from + ch * EV_CH;
    if (base >= nh) break;
    if (check_first || ch != blockIdx.x) {
      if (threadIdx.x == 0) sh.word = atomicOr(found, 0ull);
      __syncthreads();
      const unsigned long long f = sh.word;
      __syncthreads();
      if (f != ~0ull && (uint32_t)f < base) break;   // a hit below this chunk is known (uniform)
    }
    uint32_t ca[EVI], cs[EVI], ce[EVI];
    uint64_t cr[EVI];
    event_load<EVI>(hids, SH, hst, hen, nh, base, ca, cs, ce, cr);
    event_hits<EVI>(ev, ca, cs, ce, cr, base, vlast, maxc, found, sh, dep);
  }
}
// The ticket: issued only after this workgroup's atomicMins have RETURNED (`zero` is 0
// computed from their results inside asm, as in scan.hip), so the last ticket sees them all;
// a __threadfence() here wrote back the XCD's L2 in every workgroup (3.6 us an event).
__device__ bool event_done(unsigned *__restrict__ done, EvShared &sh, uint32_t dep) {
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t zero;
    asm volatile("v_and_b32 %0, 0, %1" : "=v"(zero) : "v"(dep));
    sh.last = atomicAdd(done, 1u + zero) == gridDim.x - 1;
  }
  __syncthreads();
  return sh.last;
}
// the last packing node (id << 32 | its index in the heavy set; ~0 before the first)
__device__ uint64_t event_prev(uint64_t *__restrict__ evprev, EvShared &sh) {
  if (threadIdx.x == 0) sh.word = atomicOr((unsigned long long *)evprev, 0ull);
  __syncthreads();
  const uint64_t prev = sh.word;
  __syncthreads();
  return prev;
}

// The last workgroup's part: the event staged straight into mapped host memory (hdr =
// {v, koff[v], #kids, R[v] lo, R[v] hi, tD(v) (INVALID for a root), kids staged?}, the
// node's kids in their current order with their residuals, up to EV_INLINE of them), the
// search state reset for the next event, then hdr[7] = seq raised (system scope).
__device__ void event_stage(const EvView &ev, unsigned long long *__restrict__ found, uint64_t *__restrict__ evprev,
                            unsigned *__restrict__ done, const uint32_t *__restrict__ koff,
                            const uint32_t *__restrict__ kids, const uint64_t *__restrict__ S,
                            const uint32_t *__restrict__ cparent, const uint32_t *__restrict__ ckoff,
                            const uint32_t *__restrict__ tD, const uint32_t *__restrict__ tU,
                            const uint32_t *__restrict__ rst, const uint32_t *__restrict__ ren,
                            uint32_t *__restrict__ hdr, uint32_t *__restrict__ kid_out, uint64_t *__restrict__ r_out,
                            uint32_t seq, EvShared &sh, uint64_t t_start, uint64_t t_table, uint64_t t_search) {
  if (threadIdx.x == 0) sh.word = atomicOr(found, 0ull);
  __syncthreads();
  const unsigned long long e = sh.word;
  const uint32_t v = e == ~0ull ? INVALID : (uint32_t)(e >> 32);
  if (v != INVALID) {
    const uint32_t beg = koff[v], cnt = koff[v + 1] - beg;
    if (cnt <= EV_INLINE) stage_kids(ev, beg, cnt, threadIdx.x, BLOCK, kids, S, cparent, tD, tU, kid_out, r_out);
    if (threadIdx.x == 0) {
      atomicExch((unsigned long long *)evprev, e);
      uint32_t lo, hi;
      node_interval(v, cparent, ckoff, tD, tU, rst, ren, lo, hi);
      const uint64_t r = S[v] - ev.removed(lo, hi);
      hdr[0] = v;
      hdr[1] = beg;
      hdr[2] = cnt;
      hdr[3] = (uint32_t)r;
      hdr[4] = (uint32_t)(r >> 32);
      hdr[5] = cparent[v] == INVALID ? INVALID : tD[v];
      hdr[6] = cnt <= EV_INLINE;
    }
  } else if (threadIdx.x == 0) {
    hdr[0] = INVALID;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t_stage = wall_clock64();
    hdr[8] = (uint32_t)(t_table - t_start);
    hdr[9] = (uint32_t)(t_search - t_table);
    hdr[10] = (uint32_t)(t_stage - t_search);
    atomicExch(found, ~0ull);   // the next event's search starts clean
    atomicExch(done, 0u);
    __hip_atomic_store(&hdr[7], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);   // (orders the staged words)
  }
}

// One packing event in one launch.  Every workgroup scans 512-entry chunks of the heavy
// set (event_search: an event reads about the distance to the next packing node, not the
// whole heavy set), the last one stages the event (event_stage) for the host, which polls
// hdr[7] instead of synchronising the stream.  The event table is read from kernel
// arguments or mapped host memory (the host rewrites it between events), so an event is
// ONE launch.
__global__ __launch_bounds__(BLOCK) void k_event(const uint32_t *__restrict__ hids, uint64_t nh,
                                                 const uint64_t *__restrict__ SH, const uint32_t *__restrict__ hst,
                                                 const uint32_t *__restrict__ hen, const uint32_t *__restrict__ epos,
                                                 const uint64_t *__restrict__ epre, uint32_t m, uint64_t maxc,
                                                 uint64_t *__restrict__ evprev, unsigned long long *__restrict__ found,
                                                 unsigned *__restrict__ done, const uint32_t *__restrict__ koff,
                                                 const uint32_t *__restrict__ kids, const uint64_t *__restrict__ S,
                                                 const uint32_t *__restrict__ cparent, const uint32_t *__restrict__ ckoff,
                                                 const uint32_t *__restrict__ tD, const uint32_t *__restrict__ tU,
                                                 const uint32_t *__restrict__ rst, const uint32_t *__restrict__ ren,
                                                 uint32_t *__restrict__ hdr, uint32_t *__restrict__ kid_out,
                                                 uint64_t *__restrict__ r_out, uint32_t seq, const EvArg arg) {
  __shared__ uint32_t spos[EV_LDS];
  __shared__ uint64_t spre[EV_LDS + 1];
  __shared__ EvShared sh;
  const uint64_t t_start = wall_clock64();
  const EvView ev = epos ? load_table(epos, epre, m, spos, spre) : load_arg(arg, spos, spre);
  const uint64_t t_table = wall_clock64();
  const uint64_t prev = event_prev(evprev, sh);
  uint32_t dep = 0;
  event_scan(ev, hids, nh, SH, hst, hen, maxc, prev == ~0ull ? 0 : (uint32_t)prev,
             prev == ~0ull ? INVALID : (uint32_t)(prev >> 32), false, found, sh, dep);
  if (!event_done(done, sh, dep)) return;
  event_stage(ev, found, evprev, done, koff, kids, S, cparent, ckoff, tD, tU, rst, ren, hdr, kid_out, r_out, seq, sh,
              t_start, t_table, wall_clock64());
}

// The persistent form: ONE launch runs event after event.  After staging an event the last
// workgroup publishes it (go[5..7]) to the others, which prefetch the first EVP * BLOCK
// candidates of their next search (the heavy set does not change, only the table does)
// while it waits for the host's answer in mapped memory (EvReply: the host packs the kids
// with std::sort + first-fit, as for k_event) and hands it on (go[0..4], device memory,
// read-modify-write only, like the search state).  Every workgroup then inserts the event
// into its own LDS copy of the table (double-buffered) and decodes its prefetched
// candidates.  The host answers EV_STOP when the node's kids exceed EV_INLINE
// (k_event_kids stages them after this kernel has ended) or the table would outgrow `cap`
// entries; an empty search ends the kernel; either side gives up after `timeout` ticks.
struct EvReply {
  uint32_t seq, cmd, vpos, dlo, dhi;
};
constexpr uint32_t EV_CONT = 0, EV_STOP = 1;
constexpr int EV_TIMEOUT_S = 30;   // either side of the event protocol gives up after this long
constexpr int EVP = 8, EVP_CH = BLOCK * EVP;   // prefetched candidates per thread
__device__ bool wait_word(unsigned *w, uint32_t want, uint64_t timeout) {   // (thread 0)
  const uint64_t t0 = wall_clock64();
  while (atomicOr(w, 0u) != want) {
    __builtin_amdgcn_s_sleep(4);
    if (wall_clock64() - t0 > timeout) return false;
  }
  return true;
}
__global__ __launch_bounds__(BLOCK) void k_event_loop(const uint32_t *__restrict__ hids, uint64_t nh,
                                                      const uint64_t *__restrict__ SH, const uint32_t *__restrict__ hst,
                                                      const uint32_t *__restrict__ hen, const uint32_t *__restrict__ epos,
                                                      const uint64_t *__restrict__ epre, uint32_t m, uint64_t maxc,
                                                      uint64_t *__restrict__ evprev, unsigned long long *__restrict__ found,
                                                      unsigned *__restrict__ done, const uint32_t *__restrict__ koff,
                                                      const uint32_t *__restrict__ kids, const uint64_t *__restrict__ S,
                                                      const uint32_t *__restrict__ cparent,
                                                      const uint32_t *__restrict__ ckoff, const uint32_t *__restrict__ tD,
                                                      const uint32_t *__restrict__ tU, const uint32_t *__restrict__ rst,
                                                      const uint32_t *__restrict__ ren, uint32_t *__restrict__ hdr,
                                                      uint32_t *__restrict__ kid_out, uint64_t *__restrict__ r_out,
                                                      uint32_t seq0, const EvArg arg, EvReply *reply,
                                                      unsigned *__restrict__ go, uint64_t timeout) {
  __shared__ uint32_t spos[2][EV_LDS];
  __shared__ uint64_t spre[2][EV_LDS + 1];
  __shared__ EvShared sh;
  __shared__ uint32_t cmd[4];
  int cur = 0;
  if (epos) load_table(epos, epre, m, spos[0], spre[0]);   // (m <= cap <= EV_LDS: the LDS copy)
  else load_arg(arg, spos[0], spre[0]);
  uint64_t e = event_prev(evprev, sh);
  bool was_last = false;
  for (uint32_t seq = seq0 + 1;; ++seq) {
    const uint64_t start = e == ~0ull ? 0 : (uint32_t)e;
    const uint32_t vlast = e == ~0ull ? INVALID : (uint32_t)(e >> 32);
    const uint64_t pbase = start + (uint64_t)blockIdx.x * EVP_CH;
    uint32_t ca[EVP], cs[EVP], ce[EVP];
    uint64_t cr[EVP];
    event_load<EVP>(hids, SH, hst, hen, nh, pbase, ca, cs, ce, cr);
    if (seq != seq0 + 1) {   // the previous event's answer
      if (threadIdx.x == 0) {
        uint32_t c[4] = {EV_STOP, INVALID, 0, 0};
        if (was_last) {   // from the host, handed on to the other workgroups
          const uint64_t t0 = wall_clock64();
          bool ok = true;
          while (__hip_atomic_load(&reply->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq - 1) {
            __builtin_amdgcn_s_sleep(4);
            if (wall_clock64() - t0 > timeout) { ok = false; break; }
          }
          if (ok) {
            c[0] = __hip_atomic_load(&reply->cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            c[1] = __hip_atomic_load(&reply->vpos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            c[2] = __hip_atomic_load(&reply->dlo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            c[3] = __hip_atomic_load(&reply->dhi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          uint32_t d = 0, zero;   // go[0] after the four words' atomics returned (event_done's idiom)
          for (int i = 0; i < 4; ++i) d |= atomicExch(&go[1 + i], c[i]);
          asm volatile("v_and_b32 %0, 0, %1" : "=v"(zero) : "v"(d));
          atomicExch(&go[0], seq - 1 + zero);
        } else if (wait_word(&go[0], seq - 1, 2 * timeout)) {
          for (int i = 0; i < 4; ++i) c[i] = atomicOr(&go[1 + i], 0u);
        }
        for (int i = 0; i < 4; ++i) cmd[i] = c[i];
      }
      __syncthreads();
      if (cmd[0] != EV_CONT) return;
      const uint32_t vpos = cmd[1];
      if (vpos != INVALID) {   // insert (vpos, delta) behind every entry at or below vpos
        const uint64_t d = (uint64_t)cmd[2] | ((uint64_t)cmd[3] << 32);
        const uint32_t *p0 = spos[cur];
        const uint64_t *q0 = spre[cur];
        uint32_t *p1 = spos[cur ^ 1];
        uint64_t *q1 = spre[cur ^ 1];
        uint32_t lo = 0, hi = m;   // first entry above vpos
        while (lo < hi) { const uint32_t c = (lo + hi) >> 1; if (p0[c] <= vpos) lo = c + 1; else hi = c; }
        for (uint32_t j = threadIdx.x; j <= m + 1; j += BLOCK) {
          if (j <= m) p1[j] = j < lo ? p0[j] : j == lo ? vpos : p0[j - 1];
          q1[j] = j <= lo ? q0[j] : q0[j - 1] + d;
        }
        cur ^= 1;
        ++m;
        __syncthreads();
      }
    }
    const uint64_t t_start = wall_clock64();
    const EvView ev{spos[cur], spre[cur], m};
    uint32_t dep = 0;
    event_hits<EVP>(ev, ca, cs, ce, cr, pbase, vlast, maxc, found, sh, dep);
    const uint64_t t_hits = wall_clock64();
    event_scan(ev, hids, nh, SH, hst, hen, maxc, start + (uint64_t)gridDim.x * EVP_CH, vlast, true, found, sh, dep);
    const uint64_t t_scan = wall_clock64();
    was_last = event_done(done, sh, dep);
    if (was_last) {
      if (threadIdx.x == 0) {   // (SHEEP_DEBUG=part: the last workgroup's phases)
        hdr[11] = (uint32_t)(t_hits - t_start);
        hdr[12] = (uint32_t)(t_scan - t_hits);
        hdr[13] = (uint32_t)(wall_clock64() - t_scan);
        hdr[14] = (uint32_t)start;
      }
      event_stage(ev, found, evprev, done, koff, kids, S, cparent, ckoff, tD, tU, rst, ren, hdr, kid_out, r_out, seq,
                  sh, t_start, t_start, wall_clock64());
      if (threadIdx.x == 0) {   // the event to the other workgroups (sh.word: event_stage's read of found)
        uint32_t zero;
        const uint32_t d = atomicExch(&go[6], (uint32_t)sh.word) | atomicExch(&go[7], (uint32_t)(sh.word >> 32));
        asm volatile("v_and_b32 %0, 0, %1" : "=v"(zero) : "v"(d));
        atomicExch(&go[5], seq + zero);
      }
    } else if (threadIdx.x == 0) {
      sh.word = ~0ull;
      if (wait_word(&go[5], seq, 2 * timeout)) {
        sh.word = (uint64_t)atomicOr(&go[6], 0u) | ((uint64_t)atomicOr(&go[7], 0u) << 32);
      }
    }
    __syncthreads();
    e = sh.word;
    __syncthreads();
    if (e == ~0ull) return;   // the search came back empty: the partition's events are over
  }
}

// The kids [beg_j, beg_j + cap) of the last event's node (evprev) with their residuals,
// for kid lists above EV_INLINE; the last workgroup raises hdr[7] = seq.
__global__ __launch_bounds__(BLOCK) void k_event_kids(uint64_t *__restrict__ evprev,
                                                      const uint32_t *__restrict__ epos,
                                                      const uint64_t *__restrict__ epre, uint32_t m,
                                                      const uint32_t *__restrict__ koff,
                                                      const uint32_t *__restrict__ kids, const uint64_t *__restrict__ S,
                                                      const uint32_t *__restrict__ cparent,
                                                      const uint32_t *__restrict__ tD, const uint32_t *__restrict__ tU,
                                                      uint32_t *__restrict__ hdr, uint32_t *__restrict__ kid_out,
                                                      uint64_t *__restrict__ r_out, uint32_t beg_j, uint32_t cap,
                                                      unsigned *__restrict__ done, uint32_t seq) {
  __shared__ uint32_t spos[EV_LDS];
  __shared__ uint64_t spre[EV_LDS + 1];
  __shared__ bool last;
  __shared__ unsigned long long s_word;
  if (threadIdx.x == 0) s_word = atomicOr((unsigned long long *)evprev, 0ull);
  __syncthreads();
  const uint32_t v = (uint32_t)(s_word >> 32);
  const EvView ev = load_table(epos, epre, m, spos, spre);
  const uint32_t beg = koff[v] + beg_j, cnt = koff[v + 1] - koff[v];
  const uint32_t lim = cnt - beg_j < cap ? cnt - beg_j : cap;
  stage_kids(ev, beg, lim, blockIdx.x * BLOCK + threadIdx.x, gridDim.x * BLOCK, kids, S, cparent, tD, tU, kid_out,
             r_out);
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    atomicExch(done, 0u);
    __threadfence_system();
    __hip_atomic_store(&hdr[7], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Kid orders re-sorted during the events, written back in one batch at the end
// (a node packs at most once per call, so no event reads an order another one wrote).
__global__ void k_scatter_u32(const uint32_t *__restrict__ pos, const uint32_t *__restrict__ val, uint64_t m,
                              uint32_t *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += stride) out[pos[i]] = val[i];
}

__global__ void k_gather_u64(const uint64_t *__restrict__ src, const uint32_t *__restrict__ idx, uint64_t m,
                             uint64_t *__restrict__ dst) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += stride) dst[i] = src[idx[i]];
}

// every root's final residual (after all events; a root's own packing is the host's)
__global__ void k_roots_r(const uint32_t *__restrict__ ids, uint64_t m, const uint64_t *__restrict__ S,
                          const uint32_t *__restrict__ cparent, const uint32_t *__restrict__ ckoff,
                          const uint32_t *__restrict__ tD, const uint32_t *__restrict__ tU,
                          const uint32_t *__restrict__ rst, const uint32_t *__restrict__ ren,
                          const uint32_t *__restrict__ epos, const uint64_t *__restrict__ epre, uint32_t me,
                          uint64_t *__restrict__ out) {
  __shared__ uint32_t spos[EV_LDS];
  __shared__ uint64_t spre[EV_LDS + 1];
  const EvView ev = load_table(epos, epre, me, spos, spre);
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += stride) {
    const uint32_t a = ids[i];
    uint32_t lo, hi;
    node_interval(a, cparent, ckoff, tD, tU, rst, ren, lo, hi);
    out[i] = S[a] - ev.removed(lo, hi);
  }
}

// push-down for the raked fringe: a finished node takes the part of its nearest
// ancestor-or-self that has one (an assigned kid or the core node its chain reaches;
// chains of finished ancestors are at most RAKE_ROUNDS long)
__global__ void k_push_fringe(const uint32_t *__restrict__ parent, const uint8_t *__restrict__ fin, uint64_t n,
                              int16_t *__restrict__ parts, unsigned long long *__restrict__ err, int rake_rounds) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < n; v += stride) {
    if (!fin[v] || parts[v] != SHEEP_INVALID_PART) continue;
    uint32_t u = (uint32_t)v;
    int16_t p = SHEEP_INVALID_PART;
    for (int d = 0; d <= rake_rounds + 1 && u != INVALID; ++d) {
      p = parts[u];
      if (p != SHEEP_INVALID_PART) break;
      u = parent[u];
    }
    if (p == SHEEP_INVALID_PART) atomicAdd(err, 1ull);
    else parts[v] = p;
  }
}

// ---- facts ---------------------------------------------------------------------------
__global__ void k_facts_basic(const sheep_jnode *__restrict__ tree, uint64_t n, unsigned long long *__restrict__ f) {
  // f[0] = sum pst, f[1] = max pst, f[2] = roots, f[3] = min id with pst > 2 (width > 3)
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  uint64_t s = 0, mx = 0, r = 0, halo = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    sheep_jnode j = tree[i];
    s += j.pst_weight;
    mx = j.pst_weight > mx ? j.pst_weight : mx;
    r += j.parent == INVALID;
    if (j.pst_weight > 2 && i < halo) halo = i;
  }
  s = wave_sum(s); mx = wave_max(mx); r = wave_sum(r); halo = wave_min(halo);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&f[0], (unsigned long long)s);
    atomicMax(&f[1], (unsigned long long)mx);
    atomicAdd(&f[2], (unsigned long long)r);
    atomicMin(&f[3], (unsigned long long)halo);
  }
}
// depth(c) = E1[tD] + 1;  path(c) = E2[tD] + pst(c);  per-root best path via the root
// segment index (roots with kids are chained in ascending order, their starts ascend)
__global__ void k_facts_paths(const uint32_t *__restrict__ parent, const uint32_t *__restrict__ tD, uint64_t n,
                              const uint64_t *__restrict__ E1, const uint64_t *__restrict__ E2,
                              const uint64_t *__restrict__ pst64, const uint32_t *__restrict__ rstart, uint32_t nrk,
                              unsigned long long *__restrict__ best, unsigned long long *__restrict__ maxdepth) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  uint64_t md = 0;
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < n; c += stride) {
    if (parent[c] == INVALID) continue;
    uint32_t p = tD[c];
    uint64_t depth = E1[p] + 1;
    md = depth > md ? depth : md;
    uint64_t path = E2[p] + pst64[c];
    uint32_t lo = 0, hi = nrk;
    while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (rstart[mid] <= p) lo = mid + 1; else hi = mid; }
    atomicMax(&best[lo - 1], (unsigned long long)path);
  }
  md = wave_max(md);
  if ((threadIdx.x & 63) == 0 && md) atomicMax(maxdepth, (unsigned long long)md);
}
__global__ void k_root_starts(const uint32_t *__restrict__ rk, uint64_t nrk, const uint32_t *__restrict__ koff,
                              const uint32_t *__restrict__ kids, const uint32_t *__restrict__ tD,
                              uint32_t *__restrict__ rstart) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrk; i += stride)
    rstart[i] = tD[kids[koff[rk[i]]]];
}
__global__ void k_root_eheight(const uint32_t *__restrict__ rk, uint64_t nrk, const sheep_jnode *__restrict__ tree,
                               const unsigned long long *__restrict__ best, unsigned long long *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  uint64_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrk; i += stride) {
    uint64_t e = (uint64_t)tree[rk[i]].pst_weight + best[i];
    m = e > m ? e : m;
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out, (unsigned long long)m);
}
__global__ void k_pst64(const sheep_jnode *__restrict__ tree, uint64_t n, uint64_t *__restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) out[i] = tree[i].pst_weight;
}

template <typename T> void d2h(Ctx &c, T *h, const T *d, uint64_t cnt) {
  if (cnt) HIP_CHECK(hipMemcpyAsync(h, d, cnt * sizeof(T), hipMemcpyDeviceToHost, c.stream));
}
template <typename T> void h2d(Ctx &c, T *d, const T *h, uint64_t cnt) {
  if (cnt) HIP_CHECK(hipMemcpyAsync(d, h, cnt * sizeof(T), hipMemcpyHostToDevice, c.stream));
}

// order-preserving compaction; returns count; rank optional
uint64_t compact_pred(Ctx &c, int which, const uint64_t *S, uint64_t mx, const uint32_t *parent, uint64_t n,
                      uint32_t *ids, uint32_t *rank, const char *tag) {
  uint64_t nb = (n + P_TILE - 1) / P_TILE;
  uint32_t *bcnt = c.get_as<uint32_t>(std::string("pc_bcnt_") + tag, nb);
  hipLaunchKernelGGL(k_pred_count, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, which, S, mx, parent, n, bcnt);
  LAUNCH_CHECK();
  uint32_t *tot = (uint32_t *)(c.d_scalars + 30);
  HIP_CHECK(hipMemsetAsync(c.d_scalars + 30, 0, sizeof(uint64_t), c.stream));
  scan_exclusive_u32(c, bcnt, bcnt, nb, tot);
  hipLaunchKernelGGL(k_pred_write, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, which, S, mx, parent, n, bcnt, ids,
                     rank);
  LAUNCH_CHECK();
  d2h(c, c.h_scalars + 30, c.d_scalars + 30, 1);
  c.sync();
  return (uint32_t)c.h_scalars[30];
}

}  // namespace

void fill_u32(Ctx &c, uint32_t *p, uint64_t n, uint32_t v);

void partition_tree(Ctx &c, const sheep_jnode *tree, uint64_t n, const uint32_t *seq, uint64_t seq_n, uint64_t pos_size,
                    sheep_kids *k, int16_t np, double balance, int vtx, int pstw, int16_t *parts_vid,
                    sheep_partition_info *info, const uint32_t *pos) {
  if (np <= 0) throw Error(SHEEP_ERR_ARG, "number of parts must be positive");
  if (!k || k->n != n) throw Error(SHEEP_ERR_ARG, "kid table does not belong to this tree");
  if (seq_n > n) throw Error(SHEEP_ERR_RANGE, "vector::_M_range_check: the sequence is longer than the tree (partition.cpp:65 parts.at)");
  *info = sheep_partition_info();
  if (pos_size && (!pos || n == 0)) {   // (the gather below writes every slot itself)
    hipLaunchKernelGGL(k_fill_i16, dim3(grid_for(pos_size)), dim3(BLOCK), 0, c.stream, parts_vid, pos_size,
                       SHEEP_INVALID_PART);
    LAUNCH_CHECK();
  }
  if (n == 0) { c.sync(); return; }
  TimedRegion tr_all(c, "partition", 12 * n + 2 * pos_size);   // tree + seq read, parts write

  // 1. weights and max_component (partition.cpp:54-57)
  uint64_t *w = c.get_as<uint64_t>("pt_w", n);
  unsigned long long *d = (unsigned long long *)c.d_scalars + 32;
  HIP_CHECK(hipMemsetAsync(d, 0, 4 * sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_weights, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, tree, n, vtx, pstw, w, d);
  LAUNCH_CHECK();
  d2h(c, c.h_scalars + 32, c.d_scalars + 32, 1);
  c.sync();
  const uint64_t total = c.h_scalars[32];
  const uint64_t max_component = (uint64_t)((double)(total / (uint64_t)(int64_t)np) * balance);
  info->total_weight = total;
  info->max_component = max_component;

  // 2. rake the light fringe (exact subtree sums), then the core T' as its own forest
  uint64_t *S = c.get_as<uint64_t>("pt_S", n);   // the rake's packed state, then acc, then every node's subtree sum
  uint8_t *fin = c.get_as<uint8_t>("pt_fin", n);
  const bool rake = k->max_kids <= RAKE_CNT_MASK && total < (1ull << (64 - RAKE_CNT_BITS));
  const bool lw32 = max_component < 0xFFFFFFFFull;   // every finishing leaf's w + 1 fits a u32
  void *lw = c.get(std::string("pt_lw"), n * (lw32 ? 4 : 8));
  if (lw32)
    hipLaunchKernelGGL(k_rake_init<uint32_t>, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, (const uint32_t *)k->koff,
                       (const uint64_t *)w, n, max_component, rake, S, fin, (uint32_t *)lw);
  else
    hipLaunchKernelGGL(k_rake_init<uint64_t>, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, (const uint32_t *)k->koff,
                       (const uint64_t *)w, n, max_component, rake, S, fin, (uint64_t *)lw);
  LAUNCH_CHECK();
  // two rounds (1 / 2 / 3 measured 9.37 / 8.71 / 8.62 ms of partition at RMAT-26), both
  // pulls over the kid table; the second also writes the core table's flags
  static_assert(RAKE_ROUNDS == 2, "round 1 and round 2 pulls");
  const int rake_rounds = RAKE_ROUNDS;
  uint32_t *pref = c.get_as<uint32_t>("pt_cpref", k->nkids + 1);
  if (rake) {
    if (k->nkids) {
      if (lw32)
        hipLaunchKernelGGL(k_rake_pull1<uint32_t>, dim3(grid_for(k->nkids)), dim3(BLOCK), 0, c.stream,
                           (const uint32_t *)k->kids, (const uint32_t *)k->kpar, (uint64_t)k->nkids, (const uint32_t *)lw, S);
      else
        hipLaunchKernelGGL(k_rake_pull1<uint64_t>, dim3(grid_for(k->nkids)), dim3(BLOCK), 0, c.stream,
                           (const uint32_t *)k->kids, (const uint32_t *)k->kpar, (uint64_t)k->nkids, (const uint64_t *)lw, S);
      LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_rake_mark, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, (const uint64_t *)S, n, max_component,
                       (uint8_t)2, fin);
    LAUNCH_CHECK();
    if (k->nkids) {
      hipLaunchKernelGGL(k_rake_pull2, dim3(grid_for(k->nkids)), dim3(BLOCK), 0, c.stream, (const uint32_t *)k->kids,
                         (const uint32_t *)k->kpar, (uint64_t)k->nkids, (const uint8_t *)fin, S, pref);
      LAUNCH_CHECK();
    }
  } else if (k->nkids) {   // no raking: every kid is core
    hipLaunchKernelGGL(k_core_flags, dim3(grid_for(k->nkids)), dim3(BLOCK), 0, c.stream, (const uint32_t *)k->kids,
                       k->nkids, (const uint8_t *)fin, pref);
    LAUNCH_CHECK();
  }
  sheep_kids core;
  core.ctx = &c;
  core.n = n;
  core.parent = c.get_as<uint32_t>("pt_cparent", n);
  core.koff = c.get_as<uint32_t>("pt_ckoff", n + 1);
  core.kids = c.get_as<uint32_t>("pt_ckids", k->nkids + 1);
  {
    uint32_t *tot = (uint32_t *)(c.d_scalars + 31);
    HIP_CHECK(hipMemsetAsync(pref + k->nkids, 0, sizeof(uint32_t), c.stream));
    scan_exclusive_u32(c, pref, pref, k->nkids + 1, tot);
    hipLaunchKernelGGL(k_core_build, dim3(grid_for(n + 1)), dim3(BLOCK), 0, c.stream, (const uint32_t *)k->kids,
                       k->nkids, (const uint32_t *)k->koff, (const uint32_t *)k->parent, (const uint8_t *)fin, n,
                       (const uint32_t *)pref, core.kids, core.koff, core.parent, S);
    LAUNCH_CHECK();
    d2h(c, c.h_scalars + 31, c.d_scalars + 31, 1);
    c.sync();
    core.nkids = (uint32_t)c.h_scalars[31];
  }
  Tour t;
  build_tour(c, &core, t);
  uint32_t *rst = c.get_as<uint32_t>("pt_rst", n), *ren = c.get_as<uint32_t>("pt_ren", n);
  if (t.nrk) {
    hipLaunchKernelGGL(k_root_intervals, dim3(grid_for(t.nrk)), dim3(BLOCK), 0, c.stream, t.rk, t.nrk, core.koff,
                       core.kids, t.tD, t.tU, rst, ren);
    LAUNCH_CHECK();
  }
  if (t.A) {   // core subtree sums over the tour, the raked acc as node weights
    uint64_t *val = c.get_as<uint64_t>("pt_tourval", t.A);
    hipLaunchKernelGGL(k_tour_vals, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, t.tD, t.tU, n, (const uint64_t *)S,
                       (const uint64_t *)nullptr, 0, val);
    LAUNCH_CHECK();
    scan_exclusive_u64(c, val, val, t.A, nullptr);
    uint64_t *S2 = c.get_as<uint64_t>("pt_S2", n);
    hipLaunchKernelGGL(k_subtree, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, core.parent, t.tD, t.tU, n,
                       (const uint64_t *)S, (const uint64_t *)val, S2);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_root_sums, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, core.parent, n, S2);
    LAUNCH_CHECK();
    S = S2;
  }

  // 3. packing events (partition.cpp:97-135).  Only H = {v : S(v) > max} (ancestor-
  // closed, in the core) can pack; the next packing node is the LOWEST id whose residual
  // exceeds max — every node below it already has its final cb.  The host runs each
  // packing with the reference's own std::sort on the node's current kid order and
  // first-fit (the order persists across k).
  uint32_t *hids = c.get_as<uint32_t>("pt_hids", n);
  const uint64_t nh = compact_pred(c, 0, S, max_component, core.parent, n, hids, nullptr, "h");
  info->heavy_nodes = nh;
  uint32_t *hst = c.get_as<uint32_t>("pt_hst", nh ? nh : 1), *hen = c.get_as<uint32_t>("pt_hen", nh ? nh : 1);
  if (nh) {
    hipLaunchKernelGGL(k_intervals, dim3(grid_for(nh)), dim3(BLOCK), 0, c.stream, hids, nh, core.parent, core.koff,
                       (const uint32_t *)rst, (const uint32_t *)ren, t.tD, t.tU, hst, hen);
    LAUNCH_CHECK();
  }
  uint64_t *SH = c.get_as<uint64_t>("pt_SH", nh ? nh : 1);   // S of the heavy nodes, in hids order
  if (nh) {
    hipLaunchKernelGGL(k_gather_u64, dim3(grid_for(nh)), dim3(BLOCK), 0, c.stream, (const uint64_t *)S,
                       (const uint32_t *)hids, nh, SH);
    LAUNCH_CHECK();
  }
  unsigned long long *found = (unsigned long long *)(c.d_scalars + 44);
  uint64_t *evprev = c.d_scalars + 46;
  unsigned *done_ctr = (unsigned *)(c.d_scalars + 47);
  HIP_CHECK(hipMemsetAsync(evprev, 0xFF, sizeof(uint64_t), c.stream));
  HIP_CHECK(hipMemsetAsync(done_ctr, 0, sizeof(uint64_t), c.stream));
  HIP_CHECK(hipMemsetAsync(found, 0xFF, sizeof(uint64_t), c.stream));   // k_event resets it after each event
  static const bool dbg = debug_on("part");
  double dbg_tab = 0, dbg_search = 0, dbg_stage = 0, dbg_wait = 0, dbg_host = 0;
  uint64_t dbg_kids[4] = {0, 0, 0, 0}, dbg_kids_max = 0;   // packing nodes with <= 16 / 256 / 4096 / more kids
  uint8_t *stage = (uint8_t *)c.get_pinned("pt_event", 64 + (size_t)EV_STAGE * 12);
  volatile uint32_t *hdr = (volatile uint32_t *)stage;
  uint32_t *st_kids = (uint32_t *)(stage + 64);
  uint64_t *st_r = (uint64_t *)(stage + 64 + (size_t)EV_STAGE * 4);
  uint32_t *d_hdr, *d_kids;
  uint64_t *d_r;
  HIP_CHECK(hipHostGetDevicePointer((void **)&d_hdr, stage, 0));
  HIP_CHECK(hipHostGetDevicePointer((void **)&d_kids, st_kids, 0));
  HIP_CHECK(hipHostGetDevicePointer((void **)&d_r, st_r, 0));
  // the event table (sorted tD of the non-root packings, prefix sums of their deltas),
  // written by the host into mapped memory between events; the kernels read it there
  // (into LDS) — a device copy only when it outgrows the LDS copy, and once at the end
  std::vector<std::pair<uint32_t, uint64_t>> evs;
  uint32_t *ev_pos = c.get_as<uint32_t>("pt_evpos", nh + 1);
  uint64_t *ev_pre = c.get_as<uint64_t>("pt_evpre", nh + 2);
  uint8_t *ev_stage = (uint8_t *)c.get_pinned("pt_evtable", (size_t)(nh + 2) * 12 + 16);
  uint8_t *d_ev_stage;
  HIP_CHECK(hipHostGetDevicePointer((void **)&d_ev_stage, ev_stage, 0));
  uint32_t m_ev = 0;
  const uint32_t *t_pos = (const uint32_t *)d_ev_stage;   // the table the next launch reads
  const uint64_t *t_pre = (const uint64_t *)(d_ev_stage + 8);
  *(uint64_t *)(ev_stage + 8) = 0;   // empty table: pre[0] = 0
  EvArg evarg;
  evarg.m = 0;
  evarg.pre[0] = 0;
  auto write_table = [&](bool to_device) {
    m_ev = (uint32_t)evs.size();
    if (m_ev <= EV_ARG) {
      uint64_t run = 0;
      for (uint32_t i = 0; i < m_ev; ++i) { evarg.pos[i] = evs[i].first; evarg.pre[i] = run; run += evs[i].second; }
      evarg.pre[m_ev] = run;
      evarg.m = m_ev;
    }
    const size_t pre_off = ((size_t)m_ev * 4 + 15) & ~(size_t)7;
    uint32_t *hp = (uint32_t *)ev_stage;
    uint64_t *hs = (uint64_t *)(ev_stage + pre_off);
    uint64_t run = 0;
    for (uint32_t i = 0; i < m_ev; ++i) { hp[i] = evs[i].first; hs[i] = run; run += evs[i].second; }
    hs[m_ev] = run;
    if (to_device || m_ev > (uint32_t)EV_LDS) {
      if (m_ev) HIP_CHECK(hipMemcpyAsync(ev_pos, hp, m_ev * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
      HIP_CHECK(hipMemcpyAsync(ev_pre, hs, (m_ev + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
      t_pos = ev_pos;
      t_pre = ev_pre;
    } else {
      t_pos = (const uint32_t *)d_ev_stage;
      t_pre = (const uint64_t *)(d_ev_stage + pre_off);
    }
  };
  std::vector<std::pair<uint32_t, uint64_t>> root_own;   // a root's own packing delta
  uint32_t seq_no = 0;
  // waits for the event kernels' completion flag (hdr[7]): a poll of mapped memory wakes
  // the host sooner than a stream synchronisation (which would never return while
  // k_event_loop waits for this thread's answer: the wait is bounded in time instead)
  auto wait_stage = [&](uint32_t want) {
    const auto t0 = std::chrono::steady_clock::now();
    for (long spin = 0; hdr[7] != want; ++spin)
      if ((spin & 4095) == 4095 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(EV_TIMEOUT_S))
        throw Error(SHEEP_ERR_HIP, "partition: the packing event kernel did not report");
    std::atomic_thread_fence(std::memory_order_acquire);
  };
  // the persistent event kernel (sheep_tuning event_loop > 0) and its answer word
  const uint32_t ev_cap = (uint32_t)c.tune.event_loop;
  EvReply *rep = (EvReply *)c.get_pinned("pt_reply", sizeof(EvReply));
  EvReply *d_rep;
  HIP_CHECK(hipHostGetDevicePointer((void **)&d_rep, rep, 0));
  unsigned *go = c.get_as<unsigned>("pt_go", 8);
  HIP_CHECK(hipMemsetAsync(go, 0, 8 * sizeof(unsigned), c.stream));
  __atomic_store_n(&rep->seq, 0u, __ATOMIC_RELEASE);   // (a word left by the last call could match a seq)
  bool live = false;   // k_event_loop is running: it waits for an answer after each event
  auto answer = [&](uint32_t cmd, uint32_t vpos, uint64_t d) {
    volatile EvReply *r = rep;
    r->cmd = cmd;
    r->vpos = vpos;
    r->dlo = (uint32_t)d;
    r->dhi = (uint32_t)(d >> 32);
    __atomic_store_n(&rep->seq, seq_no, __ATOMIC_RELEASE);
    if (cmd != EV_CONT) live = false;
  };
  std::vector<uint64_t> part_size;
  std::vector<uint32_t> asg_ids;
  std::vector<int16_t> asg_part;
  std::vector<uint32_t> seg, order, sorted, upl_pos, upl_ids;
  std::vector<uint64_t> segR, scb;
  std::vector<char> done;
  // 64 workgroups: an event's scan usually ends within its first round of chunks, and every
  // extra workgroup adds to the last-workgroup hand-off (RMAT-26 k=64, us per event:
  // 16 WGs 26.5, 32 19.4, 64 16.5, 128 18.1, 256 27.3, 512 48)
  const unsigned gev = nh ? (unsigned)std::min<uint64_t>((nh + EV_CH - 1) / EV_CH, 64) : 1;
  auto stage_kids_of = [&](uint32_t beg_j, uint32_t cap, uint32_t *o_kids, uint64_t *o_r) {
    ++seq_no;
    hipLaunchKernelGGL(k_event_kids, dim3(256), dim3(BLOCK), 0, c.stream, evprev, t_pos, t_pre, m_ev,
                       (const uint32_t *)k->koff, (const uint32_t *)k->kids, (const uint64_t *)S,
                       (const uint32_t *)core.parent, (const uint32_t *)t.tD, (const uint32_t *)t.tU, d_hdr, o_kids, o_r,
                       beg_j, cap, done_ctr, seq_no);
    LAUNCH_CHECK();
    info->event_launches++;
    wait_stage(seq_no);
  };
  {
    TimedRegion tr(c, "partition_events");
    hdr[7] = 0;
    try {
      for (;;) {
        if (!live) {   // k_event for this event, or k_event_loop from it on (both read the table as written now)
          write_table(false);
          const bool by_arg = m_ev <= EV_ARG;
          if (ev_cap && m_ev <= ev_cap) {
            hipLaunchKernelGGL(k_event_loop, dim3(gev), dim3(BLOCK), 0, c.stream, (const uint32_t *)hids, nh,
                               (const uint64_t *)SH, (const uint32_t *)hst, (const uint32_t *)hen,
                               by_arg ? nullptr : t_pos, by_arg ? nullptr : t_pre, m_ev, max_component, evprev, found,
                               done_ctr, (const uint32_t *)k->koff, (const uint32_t *)k->kids, (const uint64_t *)S,
                               (const uint32_t *)core.parent, (const uint32_t *)core.koff, (const uint32_t *)t.tD,
                               (const uint32_t *)t.tU, (const uint32_t *)rst, (const uint32_t *)ren, d_hdr, d_kids, d_r,
                               seq_no, evarg, d_rep, go, (uint64_t)EV_TIMEOUT_S * 100000000ull);
            live = true;
            info->event_launches++;
          } else {
            hipLaunchKernelGGL(k_event, dim3(gev), dim3(BLOCK), 0, c.stream, (const uint32_t *)hids, nh,
                               (const uint64_t *)SH, (const uint32_t *)hst, (const uint32_t *)hen,
                               by_arg ? nullptr : t_pos, by_arg ? nullptr : t_pre, m_ev, max_component, evprev, found,
                               done_ctr, (const uint32_t *)k->koff, (const uint32_t *)k->kids, (const uint64_t *)S,
                               (const uint32_t *)core.parent, (const uint32_t *)core.koff, (const uint32_t *)t.tD,
                               (const uint32_t *)t.tU, (const uint32_t *)rst, (const uint32_t *)ren, d_hdr, d_kids, d_r,
                               seq_no + 1, evarg);
            info->event_launches++;
          }
          LAUNCH_CHECK();
        }
        ++seq_no;
        const auto h0 = std::chrono::steady_clock::now();
        wait_stage(seq_no);
        const auto h1 = std::chrono::steady_clock::now();
        if (dbg) {
          dbg_tab += hdr[8] / 100.0;   // wall_clock64: 100 MHz
          dbg_search += hdr[9] / 100.0;
          dbg_stage += hdr[10] / 100.0;
          dbg_wait += std::chrono::duration<double, std::micro>(h1 - h0).count();
        }
        const uint32_t v = hdr[0];
        if (dbg && live)
          fprintf(stderr, "partition event %u: hits %.1f scan %.1f done %.1f stage %.1f us, from %u, wait %.1f us\n", seq_no,
                  hdr[11] / 100.0, hdr[12] / 100.0, hdr[13] / 100.0, hdr[10] / 100.0, hdr[14],
                  std::chrono::duration<double, std::micro>(h1 - h0).count());
        if (v == INVALID) {
          if (live) answer(EV_STOP, INVALID, 0);
          break;
        }
        info->packing_nodes++;
        const uint32_t beg = hdr[1], cnt = hdr[2], vpos = hdr[5];
        uint64_t cb = (uint64_t)hdr[3] | ((uint64_t)hdr[4] << 32);
        if (!hdr[6]) {   // more kids than the event kernel stages: k_event_kids, behind k_event_loop's end
          if (live) answer(EV_STOP, INVALID, 0);
          write_table(false);
          stage_kids_of(0, EV_STAGE, d_kids, d_r);
        }
        seg.assign(st_kids, st_kids + std::min(cnt, EV_STAGE));
        segR.assign(st_r, st_r + std::min(cnt, EV_STAGE));
        if (cnt > EV_STAGE) {   // a node with more kids than the staging area: fetch the rest
          seg.resize(cnt); segR.resize(cnt);
          uint32_t *kk = c.get_as<uint32_t>("pt_kK", cnt);
          uint64_t *kR = c.get_as<uint64_t>("pt_kR", cnt);
          stage_kids_of(EV_STAGE, cnt - EV_STAGE, kk, kR);
          c.download(seg.data() + EV_STAGE, (const uint32_t *)kk, cnt - EV_STAGE);
          c.download(segR.data() + EV_STAGE, (const uint64_t *)kR, cnt - EV_STAGE);
          c.sync();
        }
        if (dbg) {
          dbg_kids[cnt <= 16 ? 0 : cnt <= 256 ? 1 : cnt <= 4096 ? 2 : 3]++;
          dbg_kids_max = std::max<uint64_t>(dbg_kids_max, cnt);
        }
        const uint64_t cb0 = cb;
        // std::sort on the current kid order with the reference comparator (:104-106);
        // sorting positions with a comparator on their keys is the same sort.
        order.resize(cnt);
        for (uint32_t j = 0; j < cnt; ++j) order[j] = j;
        std::sort(order.begin(), order.end(), [&segR](uint32_t a, uint32_t b) { return segR[a] > segR[b]; });
        sorted.resize(cnt); scb.resize(cnt);
        for (uint32_t j = 0; j < cnt; ++j) {
          sorted[j] = seg[order[j]];
          scb[j] = segR[order[j]];
          if (j != order[j]) { upl_pos.push_back(beg + j); upl_ids.push_back(sorted[j]); }
        }
        done.assign(cnt, 0);
        do {
          for (uint32_t j = 0; cb > max_component && j < cnt; ++j) {
            if (scb[j] > max_component) throw Error(SHEEP_ERR_PACK, "forwardPartition: kid exceeds max_component");
            if (done[j]) continue;
            for (size_t p = 0; p != part_size.size(); ++p) {
              if (part_size[p] + scb[j] <= max_component) {
                cb -= scb[j];
                part_size[p] += scb[j];
                done[j] = 1;
                asg_ids.push_back(sorted[j]);
                asg_part.push_back((int16_t)p);
                break;
              }
            }
          }
          if (cb > max_component) {
            bool any = false;
            for (uint32_t j = 0; j < cnt; ++j) any |= !done[j];
            if (!any || part_size.size() >= 32767)
              throw Error(SHEEP_ERR_PACK, "forwardPartition: node weight exceeds max_component (reference loops forever)");
            part_size.push_back(0);
          }
        } while (cb > max_component);
        // the event into the table for the next scan (sorted by tD; a root keeps its own)
        if (vpos != INVALID)
          evs.insert(std::upper_bound(evs.begin(), evs.end(), std::make_pair(vpos, (uint64_t)~0ull)), {vpos, cb0 - cb});
        else
          root_own.push_back({v, cb0 - cb});
        if (live) {   // k_event_loop inserts the event into its own table copy, up to ev_cap entries
          if (vpos != INVALID && evs.size() > ev_cap) answer(EV_STOP, INVALID, 0);
          else answer(EV_CONT, vpos, cb0 - cb);
        }
        if (dbg) dbg_host += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h1).count();
      }
    } catch (...) {   // k_event_loop must not wait for an answer that never comes
      if (live) answer(EV_STOP, INVALID, 0);
      throw;
    }
  }
  if (dbg)
    fprintf(stderr, "partition events %u (us total): table %.1f search %.1f stage %.1f | host wait %.1f host pack %.1f"
            " | kids <=16 %lu <=256 %lu <=4096 %lu more %lu max %lu\n",
            (unsigned)info->packing_nodes, dbg_tab, dbg_search, dbg_stage, dbg_wait, dbg_host,
            (unsigned long)dbg_kids[0], (unsigned long)dbg_kids[1], (unsigned long)dbg_kids[2], (unsigned long)dbg_kids[3],
            (unsigned long)dbg_kids_max);
  write_table(true);   // the device copy k_roots_r reads
  if (!upl_pos.empty()) {   // persist the sorted kid orders (forwardPartition mutates kids, :104-106)
    const uint64_t mu = upl_pos.size();
    uint32_t *dp = c.get_as<uint32_t>("pt_uplpos", mu), *dv = c.get_as<uint32_t>("pt_uplids", mu);
    c.upload(dp, upl_pos.data(), mu);
    c.upload(dv, upl_ids.data(), mu);
    hipLaunchKernelGGL(k_scatter_u32, dim3(grid_for(mu)), dim3(BLOCK), 0, c.stream, (const uint32_t *)dp,
                       (const uint32_t *)dv, mu, k->kids);
    LAUNCH_CHECK();
  }
  // roots (ascending) with their final cb
  uint32_t *rids = c.get_as<uint32_t>("pt_roots", n);
  const uint64_t nroots = compact_pred(c, 1, S, 0, k->parent, n, rids, nullptr, "r");
  std::vector<uint32_t> r_ids(nroots);
  std::vector<uint64_t> r_cb(nroots);
  if (nroots) {
    uint64_t *rR = c.get_as<uint64_t>("pt_rR", nroots);
    hipLaunchKernelGGL(k_roots_r, dim3(grid_for(nroots)), dim3(BLOCK), 0, c.stream, (const uint32_t *)rids, nroots,
                       (const uint64_t *)S, (const uint32_t *)core.parent, (const uint32_t *)core.koff,
                       (const uint32_t *)t.tD, (const uint32_t *)t.tU, (const uint32_t *)rst, (const uint32_t *)ren,
                       (const uint32_t *)ev_pos, (const uint64_t *)ev_pre, m_ev, rR);
    LAUNCH_CHECK();
    c.download(r_ids.data(), (const uint32_t *)rids, nroots);
    c.download(r_cb.data(), (const uint64_t *)rR, nroots);
  }
  c.sync();   // the kid-order upload vectors die with this call
  for (const auto &ro : root_own) {   // a packed root's own removed weight
    const auto it = std::lower_bound(r_ids.begin(), r_ids.end(), ro.first);
    if (it != r_ids.end() && *it == ro.first) r_cb[it - r_ids.begin()] -= ro.second;
  }

  // 4. descending pass: roots into the highest bin that fits (:146-152)
  std::vector<int16_t> root_part(nroots);
  for (uint64_t ri = nroots; ri-- > 0;) {
    uint64_t cb = r_cb[ri];
    int16_t got = -1;
    while (got < 0) {
      for (long p = (long)part_size.size() - 1; p != -1; --p) {
        if (part_size[p] + cb <= max_component) { part_size[p] += cb; got = (int16_t)p; break; }
      }
      if (got < 0) {
        if (part_size.size() >= 32767) throw Error(SHEEP_ERR_PACK, "forwardPartition: root cannot be packed");
        part_size.push_back(0);
      }
    }
    root_part[ri] = got;
  }

  // 5. push down: assigned = packed kids + roots; core nodes through the laminar tour
  // intervals of the assigned core nodes, then the fringe up its short parent chains
  HIP_CHECK(hipMemsetAsync(c.d_scalars + 36, 0, 4 * sizeof(uint64_t), c.stream));   // push-down error, print counts
  const uint64_t na = asg_ids.size() + nroots;
  std::vector<uint32_t> all_ids(asg_ids);
  all_ids.insert(all_ids.end(), r_ids.begin(), r_ids.end());
  std::vector<int16_t> all_part(asg_part);
  all_part.insert(all_part.end(), root_part.begin(), root_part.end());
  int16_t *parts = c.get_as<int16_t>("pt_parts", n);
  unsigned long long *e = (unsigned long long *)c.d_scalars + 36;
  hipLaunchKernelGGL(k_fill_i16, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, parts, n, SHEEP_INVALID_PART);
  LAUNCH_CHECK();
  {
    uint32_t *aid = c.get_as<uint32_t>("pt_aid", na);
    int16_t *ap = c.get_as<int16_t>("pt_ap", na);
    c.upload(aid, all_ids.data(), na);
    c.upload(ap, all_part.data(), na);
    hipLaunchKernelGGL(k_scatter_parts, dim3(grid_for(na)), dim3(BLOCK), 0, c.stream, aid, ap, na, parts);
    LAUNCH_CHECK();
    uint32_t *st = c.get_as<uint32_t>("pt_ast", na), *en = c.get_as<uint32_t>("pt_aen", na);
    hipLaunchKernelGGL(k_intervals, dim3(grid_for(na)), dim3(BLOCK), 0, c.stream, aid, na, core.parent, core.koff,
                       (const uint32_t *)rst, (const uint32_t *)ren, t.tD, t.tU, st, en);
    LAUNCH_CHECK();
    std::vector<uint32_t> hs(na), he(na);
    c.download(hs.data(), st, na);
    c.download(he.data(), en, na);
    c.sync();
    std::vector<uint32_t> ord;
    ord.reserve(na);
    for (uint32_t i = 0; i < na; ++i) if (hs[i] != INVALID) ord.push_back(i);
    // outer intervals first; a root's span can equal its only core kid's interval, and
    // the root is the outer one (assigned roots follow the packed kids in all_ids)
    const uint32_t nasg = (uint32_t)asg_ids.size();
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
      if (hs[a] != hs[b]) return hs[a] < hs[b];
      if (he[a] != he[b]) return he[a] > he[b];
      return (a >= nasg) > (b >= nasg);
    });
    const uint32_t m = (uint32_t)ord.size();
    std::vector<uint32_t> sst(m), sen(m), encl(m);
    std::vector<int16_t> sp(m);
    std::vector<uint32_t> stack;
    for (uint32_t i = 0; i < m; ++i) {
      sst[i] = hs[ord[i]]; sen[i] = he[ord[i]]; sp[i] = all_part[ord[i]];
      while (!stack.empty() && sen[stack.back()] < sst[i]) stack.pop_back();
      encl[i] = stack.empty() ? INVALID : stack.back();
      stack.push_back(i);
    }
    if (m) {
      uint32_t *dst_ = c.get_as<uint32_t>("pt_sst", m), *den = c.get_as<uint32_t>("pt_sen", m);
      uint32_t *dencl = c.get_as<uint32_t>("pt_encl", m);
      int16_t *dsp = c.get_as<int16_t>("pt_sp", m);
      c.upload(dst_, sst.data(), m);
      c.upload(den, sen.data(), m);
      c.upload(dencl, encl.data(), m);
      c.upload(dsp, sp.data(), m);
      hipLaunchKernelGGL(k_push_down, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, core.parent, t.tD, n, dst_, den, dsp,
                         dencl, m, parts, e);
      LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_push_fringe, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, (const uint32_t *)k->parent,
                       (const uint8_t *)fin, n, parts, e, rake_rounds);
    LAUNCH_CHECK();   // (the uploads were staged: the vectors may die with this block)
  }
  // 6. jnid -> vid (:62-66) and print counts (partition.h:138-139)
  unsigned long long *cnt = (unsigned long long *)c.d_scalars + 37;
  if (pos && pos_size) {
    hipLaunchKernelGGL(k_parts_from_pos, dim3(grid_for(pos_size, BLOCK * 4)), dim3(BLOCK), 0, c.stream, pos, pos_size,
                       seq_n, (const int16_t *)parts, parts_vid, cnt);
    LAUNCH_CHECK();
  } else if (seq_n) {
    hipLaunchKernelGGL(k_parts_to_vid, dim3(grid_for(seq_n)), dim3(BLOCK), 0, c.stream, seq, seq_n, parts, parts_vid, cnt);
    LAUNCH_CHECK();
  }
  d2h(c, c.h_scalars + 36, c.d_scalars + 36, 4);
  c.sync();
  if (c.h_scalars[36]) throw Error(SHEEP_ERR_HIP, "partition push-down: unassigned node");
  info->first_size = c.h_scalars[37];
  info->second_size = c.h_scalars[38];
  info->created = (int32_t)c.h_scalars[39];   // max part + 1 over the vid-indexed vector
}

void tree_facts(Ctx &c, const sheep_jnode *tree, uint64_t n, sheep_facts_t *out) {
  *out = sheep_facts_t();
  out->halo_id = INVALID;
  out->core_id = INVALID;
  if (n == 0) return;
  unsigned long long *f = (unsigned long long *)c.d_scalars + 40;
  HIP_CHECK(hipMemsetAsync(f, 0, 8 * sizeof(uint64_t), c.stream));
  HIP_CHECK(hipMemsetAsync(f + 3, 0xFF, sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_facts_basic, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, tree, n, f);
  LAUNCH_CHECK();
  sheep_kids k;
  build_kids(c, tree, n, &k);
  Tour t;
  uint64_t maxdepth = 0, eheight = 0;
  try {
    build_tour(c, &k, t);
    uint64_t *pst64 = c.get_as<uint64_t>("fx_pst", n);
    hipLaunchKernelGGL(k_pst64, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, tree, n, pst64);
    LAUNCH_CHECK();
    unsigned long long *best = nullptr;
    if (t.A) {
      uint64_t *E1 = c.get_as<uint64_t>("fx_E1", t.A), *E2 = c.get_as<uint64_t>("fx_E2", t.A);
      hipLaunchKernelGGL(k_tour_vals, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, t.tD, t.tU, n,
                         (const uint64_t *)pst64, (const uint64_t *)nullptr, 2, E1);
      LAUNCH_CHECK();
      hipLaunchKernelGGL(k_tour_vals, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, t.tD, t.tU, n,
                         (const uint64_t *)pst64, (const uint64_t *)nullptr, 1, E2);
      LAUNCH_CHECK();
      scan_exclusive_u64(c, E1, E1, t.A, nullptr);
      scan_exclusive_u64(c, E2, E2, t.A, nullptr);
      uint32_t *rstart = c.get_as<uint32_t>("fx_rstart", t.nrk);
      hipLaunchKernelGGL(k_root_starts, dim3(grid_for(t.nrk)), dim3(BLOCK), 0, c.stream, t.rk, t.nrk, k.koff, k.kids,
                         t.tD, rstart);
      LAUNCH_CHECK();
      best = c.get_as<unsigned long long>("fx_best", t.nrk);
      HIP_CHECK(hipMemsetAsync(best, 0, t.nrk * sizeof(uint64_t), c.stream));
      hipLaunchKernelGGL(k_facts_paths, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, k.parent, t.tD, n,
                         (const uint64_t *)E1, (const uint64_t *)E2, (const uint64_t *)pst64, rstart,
                         (uint32_t)t.nrk, best, f + 4);
      LAUNCH_CHECK();
      hipLaunchKernelGGL(k_root_eheight, dim3(grid_for(t.nrk)), dim3(BLOCK), 0, c.stream, t.rk, t.nrk, tree,
                         (const unsigned long long *)best, f + 5);
      LAUNCH_CHECK();
    }
    HIP_CHECK(hipMemcpyAsync(c.h_scalars + 40, c.d_scalars + 40, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    maxdepth = c.h_scalars[44];
    eheight = c.h_scalars[45];
  } catch (...) {
    release_kids(&c, &k);
    throw;
  }
  release_kids(&c, &k);   // the buffers stay with the context for the next kid table
  const uint64_t sum = c.h_scalars[40], mx = c.h_scalars[41], roots = c.h_scalars[42], halo = c.h_scalars[43];
  out->vert_cnt = n;
  out->edge_cnt = sum;
  out->width = 1 + mx;
  out->fill = 0;
  out->root_cnt = roots;
  out->vert_height = maxdepth + 1;   // a root alone has vheight 1
  // kidless roots: eheight = own pst
  out->edge_height = eheight;
  out->halo_id = halo == ~0ull ? INVALID : halo;
  out->core_id = 0;
}

}  // namespace sheep
