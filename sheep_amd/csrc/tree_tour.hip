// tree_tour.hip — kid table (makeKids, jnode.h:190-204) and an Euler tour of the
// elimination forest, ranked on the GPU.
//
// The trees are extremely tall (twitter vheight ~1e7), so nothing here is level
// synchronous.  The tour is a linked list of 2(n - roots) arcs; it is ranked with a
// sparse ruling set: ~1/32 of the arcs (hash-selected) walk to the next ruler
// (independent short pointer chases, all in flight at once), the ruler list is ranked
// by pointer jumping, and every arc gets ruler prefix + local offset.  Subtree sums,
// depths and path sums then become ordinary prefix sums over tour order.
#include <cstdlib>

#include "tree_tour.hpp"

namespace sheep {
namespace {

__global__ void k_max_u32(const uint32_t *__restrict__ x, uint64_t n, unsigned long long *__restrict__ out) {
  uint32_t m = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) m = x[i] > m ? x[i] : m;
  block_atomic_max(out, m);
}

__global__ void k_kid_keys(const sheep_jnode *__restrict__ tree, uint64_t n, uint32_t *__restrict__ keys,
                           uint32_t *__restrict__ vals, uint32_t *__restrict__ parent,
                           unsigned long long *__restrict__ err) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    uint32_t p = tree[i].parent;
    if (p != INVALID && (p >= n || p <= i)) { atomicAdd(err, 1ull); p = INVALID; }
    parent[i] = p;
    keys[i] = p == INVALID ? (uint32_t)n : p;
    vals[i] = (uint32_t)i;
  }
}

// Kid counts from the parent-sorted keys: a parent's kids are one run, so run_add adds
// each run with one atomic per wave it spans (a scattered atomic per node before the
// sort cost 1.4 ms at RMAT-26).
__global__ void k_kid_counts(const uint32_t *__restrict__ keys, uint64_t n, uint32_t *__restrict__ cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t iters = (n + stride - 1) / stride;
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, i += stride) {   // wave-uniform trip count (run_add)
    const uint32_t k = i < n ? keys[i] : (uint32_t)n;
    run_add(cnt, k < n ? k : INVALID, 1u);
  }
}

__global__ void k_kidpos(const uint32_t *__restrict__ kids, uint64_t nk, uint32_t *__restrict__ kidpos) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < nk; j += stride) kidpos[kids[j]] = (uint32_t)j;
}

// roots that have kids, ascending (order-preserving compaction by block counts)
constexpr int RK_ITEMS = 8, RK_TILE = BLOCK * RK_ITEMS;
__device__ __forceinline__ bool root_with_kids(const uint32_t *parent, const uint32_t *koff, uint64_t i) {
  return parent[i] == INVALID && koff[i] < koff[i + 1];
}
__global__ void k_rk_count(const uint32_t *__restrict__ parent, const uint32_t *__restrict__ koff, uint64_t n,
                           uint32_t *__restrict__ bcnt) {
  __shared__ uint32_t s[BLOCK / WAVE];
  uint64_t base = (uint64_t)blockIdx.x * RK_TILE;
  uint32_t c = 0;
  for (int j = 0; j < RK_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    if (i < n) c += root_with_kids(parent, koff, i);
  }
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ void k_rk_write(const uint32_t *__restrict__ parent, const uint32_t *__restrict__ koff, uint64_t n,
                           const uint32_t *__restrict__ boff, uint32_t *__restrict__ rk) {
  __shared__ uint32_t wc[BLOCK / WAVE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t base = (uint64_t)blockIdx.x * RK_TILE;
  uint32_t running = boff[blockIdx.x];
  for (int j = 0; j < RK_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    bool f = i < n && root_with_kids(parent, koff, i);
    uint64_t m = __ballot(f);
    if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = running;
    for (int w = 0; w < wave; ++w) off += wc[w];
    if (f) rk[off + __popcll(m & lanemask_lt())] = (uint32_t)i;
    running += wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();
  }
}

// Arc a < n: down arc into node a;  a >= n: up arc out of node a - n.
__global__ void k_succ(const uint32_t *__restrict__ parent, uint64_t n, const uint32_t *__restrict__ koff,
                       const uint32_t *__restrict__ kids, const uint32_t *__restrict__ kidpos,
                       const uint32_t *__restrict__ rootnext, uint32_t *__restrict__ succ) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < n; c += stride) {
    uint32_t p = parent[c];
    if (p == INVALID) continue;
    succ[c] = koff[c] < koff[c + 1] ? kids[koff[c]] : (uint32_t)(n + c);
    uint32_t j = kidpos[c];
    uint32_t nx;
    if (j + 1 < koff[p + 1]) nx = kids[j + 1];
    else if (parent[p] != INVALID) nx = (uint32_t)(n + p);
    else nx = rootnext[p];
    succ[n + c] = nx;
  }
}

__global__ void k_rootnext(const uint32_t *__restrict__ rk, uint64_t nrk, const uint32_t *__restrict__ koff,
                           const uint32_t *__restrict__ kids, uint32_t *__restrict__ rootnext) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrk; i += stride)
    rootnext[rk[i]] = i + 1 < nrk ? kids[koff[rk[i + 1]]] : INVALID;
}

// (nrk: the count of roots with kids, on the device; none: no head)
__global__ void k_head(const uint32_t *__restrict__ rk, const uint32_t *__restrict__ nrk, const uint32_t *__restrict__ koff,
                       const uint32_t *__restrict__ kids, uint32_t *__restrict__ head) {
  if (threadIdx.x == 0) head[0] = *nrk ? kids[koff[rk[0]]] : INVALID;
}

__device__ __forceinline__ bool hash_ruler(uint32_t a, uint32_t mask) {
  uint32_t h = a * 0x9E3779B1u;
  h ^= h >> 15;
  h *= 0x85EBCA77u;
  h ^= h >> 13;
  return (h & mask) == 0;
}

__global__ __launch_bounds__(BLOCK) void k_pick_rulers(const uint32_t *__restrict__ parent, uint64_t n, uint32_t head,
                                                       uint32_t *__restrict__ rid, uint32_t *__restrict__ rulers,
                                                       uint64_t cap, unsigned long long *__restrict__ counter, uint32_t rmask) {
  // PR_T tiles per reservation: one atomic on the single counter per workgroup call, and
  // that counter's serialised atomics (one per 2,048-arc tile) were the kernel's bound
  constexpr int PR_T = 8;
  const uint64_t total = 2 * n;
  const uint64_t ntiles = (total + TILE - 1) / TILE, nsup = (ntiles + PR_T - 1) / PR_T;
  for (uint64_t sup = blockIdx.x; sup < nsup; sup += gridDim.x) {
    uint32_t flags[PR_T], cnt = 0;
#pragma unroll
    for (int t = 0; t < PR_T; ++t) {
      flags[t] = 0;
      const uint64_t tile = sup * PR_T + t;
#pragma unroll
      for (int j = 0; j < TILE_ITEMS; ++j) {
        const uint64_t a = tile * TILE + (uint64_t)j * BLOCK + threadIdx.x;
        if (a < total) {
          const uint32_t node = (uint32_t)(a < n ? a : a - n);
          if (parent[node] != INVALID && (a == head || hash_ruler((uint32_t)a, rmask))) flags[t] |= 1u << j;
        }
      }
      cnt += (uint32_t)__popc(flags[t]);
    }
    uint64_t slot = block_reserve(cnt, counter);
#pragma unroll
    for (int t = 0; t < PR_T; ++t)
#pragma unroll
      for (int j = 0; j < TILE_ITEMS; ++j)
        if (flags[t] & (1u << j)) {
          const uint32_t a = (uint32_t)((sup * PR_T + t) * TILE + (uint64_t)j * BLOCK + threadIdx.x);
          if (slot < cap) {   // overflow is reported by the host (counter > cap)
            rid[a] = (uint32_t)slot;
            rulers[slot] = a;
          }
          ++slot;
        }
  }
}

__global__ void k_walk(const uint32_t *__restrict__ rulers, uint64_t nr, const uint32_t *__restrict__ succ,
                       const uint32_t *__restrict__ rid, uint32_t *__restrict__ owner, uint32_t *__restrict__ loff,
                       uint32_t *__restrict__ rlen, uint32_t *__restrict__ rnext, uint32_t rmask, uint64_t arcs) {
  // launched with 64-thread workgroups (one wave: the walks are long dependent chains)
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nr; r += stride) {
    uint32_t cur = rulers[r], local = 0, nx;
    const uint32_t cap = (uint32_t)(arcs + 2);   // > any list length: guards a corrupt list
    while (local < cap) {
      owner[cur] = (uint32_t)r;
      loff[cur] = local++;
      nx = succ[cur];
      if (nx == INVALID || hash_ruler(nx, rmask)) break;
      cur = nx;
    }
    rlen[r] = local;
    rnext[r] = nx == INVALID ? INVALID : rid[nx];
  }
}

// Wyllie pointer jumping on the ruler list: suffix sums of lengths.
// (The round count is fixed on the host: ceil(log2 nr).  A per-wave "still active"
// atomic on one word cost each round ~30 us for 4K waves.)
__global__ void k_jump(const uint32_t *__restrict__ nxt_in, const uint32_t *__restrict__ suf_in, uint64_t nr,
                       uint32_t *__restrict__ nxt_out, uint32_t *__restrict__ suf_out) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; r < nr; r += stride) {
    uint32_t nx = nxt_in[r];
    if (nx == INVALID) { nxt_out[r] = INVALID; suf_out[r] = suf_in[r]; continue; }
    suf_out[r] = suf_in[r] + suf_in[nx];
    nxt_out[r] = nxt_in[nx];
  }
}

__global__ void k_tpos(const uint32_t *__restrict__ parent, uint64_t n, const uint32_t *__restrict__ owner,
                       const uint32_t *__restrict__ loff, const uint32_t *__restrict__ suf, uint32_t A,
                       uint32_t *__restrict__ tD, uint32_t *__restrict__ tU) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < n; c += stride) {
    if (parent[c] == INVALID) { tD[c] = INVALID; tU[c] = INVALID; continue; }
    uint32_t o = owner[c];
    tD[c] = A - suf[o] + loff[c];
    o = owner[n + c];
    tU[c] = A - suf[o] + loff[n + c];
  }
}

__global__ void k_gather_u32(const uint32_t *__restrict__ src, const uint32_t *__restrict__ idx, uint64_t m,
                             uint32_t *__restrict__ dst) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += stride) dst[i] = src[idx[i]];
}

}  // namespace

void fill_u32(Ctx &c, uint32_t *p, uint64_t n, uint32_t v);

void gather_u32(Ctx &c, const uint32_t *src, const uint32_t *idx, uint64_t m, uint32_t *dst) {
  if (!m) return;
  hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(m)), dim3(BLOCK), 0, c.stream, src, idx, m, dst);
  LAUNCH_CHECK();
}

// A kid table's buffers back to the context for the next table (the larger table's
// buffers are kept), or freed.  The caller has made the context's device current.
void release_kids(Ctx *c, sheep_kids *k) {
  Ctx::KidBufs *sp = c ? &c->kid_spare : nullptr;
  if (sp && k->parent && k->koff && k->kids && k->kpar && (!sp->parent || sp->cap < k->cap)) {
    if (sp->parent) {
      c->sync();
      hipFree(sp->parent); hipFree(sp->koff); hipFree(sp->kids); hipFree(sp->kpar);
    }
    *sp = {k->parent, k->koff, k->kids, k->kpar, k->cap};
  } else {
    if (c) c->sync();
    hipFree(k->parent);
    hipFree(k->koff);
    hipFree(k->kids);
    hipFree(k->kpar);
  }
  k->parent = k->koff = k->kids = k->kpar = nullptr;
}

void build_kids(Ctx &c, const sheep_jnode *tree, uint64_t n, sheep_kids *k) {
  k->ctx = &c;
  k->n = n;
  Ctx::KidBufs &sp = c.kid_spare;
  if (sp.parent && sp.cap >= n) {   // stream-ordered reuse: the old table's work is queued before ours
    k->parent = sp.parent; k->koff = sp.koff; k->kids = sp.kids; k->kpar = sp.kpar; k->cap = sp.cap;
    sp = Ctx::KidBufs();
  } else {
    HIP_CHECK(hipMalloc(&k->parent, (n + 1) * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&k->koff, (n + 2) * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&k->kids, (n + 1) * sizeof(uint32_t)));
    HIP_CHECK(hipMalloc(&k->kpar, (n + 1) * sizeof(uint32_t)));
    k->cap = n;
  }
  if (n == 0) { HIP_CHECK(hipMemsetAsync(k->koff, 0, sizeof(uint32_t), c.stream)); return; }
  TimedRegion tr(c, "kids", 8 * n + 12 * n);   // tree read; parent copy, offsets, kid ids written
  // the table's own kpar / kids serve as the sort's alternate buffers: with an odd number of
  // passes (1 or 3: up to 2^9 or 2^27 nodes) the sorted pairs end there, with no copy
  uint32_t *keys = c.get_as<uint32_t>("kid_keys", n), *vals = c.get_as<uint32_t>("kid_vals", n);
  uint32_t *kalt = k->kpar, *valt = k->kids;
  HIP_CHECK(hipMemsetAsync(k->koff, 0, (n + 1) * sizeof(uint32_t), c.stream));
  unsigned long long *d = (unsigned long long *)c.d_scalars + 16;
  HIP_CHECK(hipMemsetAsync(d, 0, 3 * sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_kid_keys, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, tree, n, keys, vals, k->parent, d);
  LAUNCH_CHECK();
  int bits = 0;
  while (bits < 32 && (n >> bits)) ++bits;
  bool in_alt = false;
  radix_sort_pairs_u32(c, keys, vals, n, bits, kalt, valt, &in_alt);   // stable: kids ascending per parent
  if (!in_alt) {   // an even number of passes: the sorted pairs are in keys / vals
    HIP_CHECK(hipMemcpyAsync(k->kids, vals, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(k->kpar, keys, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
  }
  keys = k->kpar;
  hipLaunchKernelGGL(k_kid_counts, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, (const uint32_t *)keys, n, k->koff);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(k_max_u32, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, (const uint32_t *)k->koff, n, d + 2);
  LAUNCH_CHECK();   // the largest kid count (the partition's packed rake state needs it < 2^24)
  // counts -> offsets; total = number of kids
  scan_exclusive_u32(c, k->koff, k->koff, n + 1, (uint32_t *)(d + 1));
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 16, d, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.h_scalars[16]) throw Error(SHEEP_ERR_RANGE, "tree: parent out of range or not later than its kid");
  k->nkids = (uint32_t)c.h_scalars[17];
  k->max_kids = c.h_scalars[18];
}

void build_tour(Ctx &c, sheep_kids *k, Tour &t) {
  const uint64_t n = k->n;
  t = Tour();
  if (n == 0) return;
  if (2 * n >= 0xFFFFFFFFull) throw Error(SHEEP_ERR_ARG, "tree too large for a 32-bit tour");
  uint32_t *kidpos = c.get_as<uint32_t>("tour_kidpos", n);
  hipLaunchKernelGGL(k_kidpos, dim3(grid_for(k->nkids)), dim3(BLOCK), 0, c.stream, k->kids, k->nkids, kidpos);
  LAUNCH_CHECK();
  // roots with kids, ascending
  uint64_t nb = (n + RK_TILE - 1) / RK_TILE;
  uint32_t *bcnt = c.get_as<uint32_t>("tour_bcnt", nb);
  unsigned long long *d = (unsigned long long *)c.d_scalars + 20;
  HIP_CHECK(hipMemsetAsync(d, 0, 4 * sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_rk_count, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, k->parent, k->koff, n, bcnt);
  LAUNCH_CHECK();
  scan_exclusive_u32(c, bcnt, bcnt, nb, (uint32_t *)(d + 1));
  uint32_t *rk = c.get_as<uint32_t>("tour_rk", n);
  hipLaunchKernelGGL(k_rk_write, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, k->parent, k->koff, n, bcnt, rk);
  LAUNCH_CHECK();
  // head = down arc into the first kid of the first root with kids, found before the one
  // sync that reads the count (a sync of its own cost a host round trip)
  uint32_t *dhead = (uint32_t *)(c.d_scalars + 24);
  hipLaunchKernelGGL(k_head, dim3(1), dim3(WAVE), 0, c.stream, (const uint32_t *)rk, (const uint32_t *)(d + 1),
                     (const uint32_t *)k->koff, (const uint32_t *)k->kids, dhead);
  LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 20, d, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 24, dhead, sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  t.nroots = n - k->nkids;   // every non-root is one kid
  t.nrk = (uint32_t)c.h_scalars[21];
  t.rk = rk;
  t.A = 2 * (n - t.nroots);
  t.tD = c.get_as<uint32_t>("tour_tD", n);
  t.tU = c.get_as<uint32_t>("tour_tU", n);
  if (t.A == 0) {
    fill_u32(c, t.tD, n, INVALID);
    fill_u32(c, t.tU, n, INVALID);
    return;
  }
  uint32_t *rootnext = c.get_as<uint32_t>("tour_rootnext", n);
  hipLaunchKernelGGL(k_rootnext, dim3(grid_for(t.nrk)), dim3(BLOCK), 0, c.stream, rk, t.nrk, k->koff, k->kids, rootnext);
  LAUNCH_CHECK();
  uint32_t *succ = c.get_as<uint32_t>("tour_succ", 2 * n);
  hipLaunchKernelGGL(k_succ, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, k->parent, n, k->koff, k->kids, kidpos,
                     rootnext, succ);
  LAUNCH_CHECK();
  const uint32_t head = (uint32_t)c.h_scalars[24];

  uint32_t *rid = c.get_as<uint32_t>("tour_rid", 2 * n);
  // one arc in 32 is a ruler (1/32, 1/64, 1/128 measured 8.54 / 8.71 / 8.81 ms of partition
  // at RMAT-26: shorter walks against more pointer-jumping work; round 5: 1/16 and 1/8 cut
  // the walk 0.53 -> 0.44 / 0.40 ms, partition 6.46 / 6.47 / 6.60 ms: no better)
  constexpr uint32_t rmask = 31u;
  const uint64_t rcap = 2 * n * 4 / (rmask + 1) + 1024;   // expected 2n/(rmask + 1) hash-picked rulers
  uint32_t *rulers = c.get_as<uint32_t>("tour_rulers", rcap);
  HIP_CHECK(hipMemsetAsync(d + 2, 0, sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_pick_rulers, dim3(grid_tiles(2 * n)), dim3(BLOCK), 0, c.stream, k->parent, n, head, rid,
                     rulers, rcap, d + 2, rmask);
  LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 22, d + 2, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const uint64_t nr = c.h_scalars[22];
  if (nr > rcap) throw Error(SHEEP_ERR_HIP, "tour: ruler overflow");
  uint32_t *owner = c.get_as<uint32_t>("tour_owner", 2 * n), *loff = c.get_as<uint32_t>("tour_loff", 2 * n);
  uint32_t *rlen = c.get_as<uint32_t>("tour_rlen", nr), *rnext = c.get_as<uint32_t>("tour_rnext", nr);
  uint32_t *rlen2 = c.get_as<uint32_t>("tour_rlen2", nr), *rnext2 = c.get_as<uint32_t>("tour_rnext2", nr);
  {
    TimedRegion tr(c, "tour_walk");
    hipLaunchKernelGGL(k_walk, dim3(grid_for(nr, 64)), dim3(64), 0, c.stream, rulers, nr, succ, rid, owner, loff, rlen,
                       rnext, rmask, 2 * n);
    LAUNCH_CHECK();
  }
  uint32_t *sa = rlen, *na = rnext, *sb = rlen2, *nb2 = rnext2;
  // Wyllie jumping on ONE list of nr rulers: ceil(log2 nr) rounds, no host polling
  int rounds = 0;
  while ((1ull << rounds) < nr) ++rounds;
  for (int it = 0; it < rounds; ++it) {
    hipLaunchKernelGGL(k_jump, dim3(grid_for(nr)), dim3(BLOCK), 0, c.stream, na, sa, nr, nb2, sb);
    LAUNCH_CHECK();
    std::swap(sa, sb);
    std::swap(na, nb2);
  }
  hipLaunchKernelGGL(k_tpos, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, k->parent, n, owner, loff, sa,
                     (uint32_t)t.A, t.tD, t.tU);
  LAUNCH_CHECK();
}

}  // namespace sheep
