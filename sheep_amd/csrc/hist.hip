// hist.hip — large-range histograms without global random atomics.
//
// A histogram of N keys over [0, K) done with one device atomic per key runs at the
// scattered-atomic rate (~2e10/s on MI355X: 1e9 heads of RMAT-26 took 40 ms, the pst
// histogram 33 ms).  Here the keys are bucketed by their high bits into NB "fine"
// buckets of W = 2^15 keys, so each bucket's counters fit one workgroup's LDS:
//
//   1. k_hist_count   per tile of T = 2^15 keys: LDS histogram over the NB buckets
//                     -> tile_hist[bucket][tile]                      (reads the source)
//   2. exclusive scan of tile_hist (bucket-major) -> every (bucket, tile) run's offset
//   3. k_hist_scatter per tile: the keys again (32 per thread, in registers),
//                     counting sort of (bucket, 15-bit local key) in LDS, each
//                     bucket's run written contiguously as u16
//   4. k_hist_final   one workgroup per (bucket, slice of <= 2^20 keys): LDS counters
//                     over the bucket's W keys, then added into cnt[bucket*W + i]
//
// Traffic per key: two reads of the source + 2 B written + 2 B read back, all of it
// coalesced (runs of ~T/NB u16), against one scattered RMW per key.
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "common.hpp"

namespace sheep {
namespace {

constexpr int HB = 1024;        // threads per workgroup (one workgroup per CU: LDS-bound)
constexpr int WBITS = 15;       // fine bucket width 2^15 keys
constexpr uint32_t W = 1u << WBITS;
constexpr uint32_t NO_KEY = 0xFFFFFFFFu;

// ---- key sources ----------------------------------------------------------------
// Heads of XS1 records (LLAMA degree: a self-loop's head is not counted again).
// (The caller has range-checked every id against K before building the histogram.)
struct HeadKeys {
  const sheep_xs1 *rec;
  int llama;
  __device__ __forceinline__ uint32_t operator()(uint64_t i) const {
    const sheep_xs1 r = rec[i];
    return (llama && r.tail == r.head) ? NO_KEY : r.head;
  }
};
// Both endpoints: keys [0, n) are the tails, [n, 2n) the heads (HeadKeys' rule).
struct EndpointKeys {
  const sheep_xs1 *rec;
  uint64_t n;
  int llama;
  __device__ __forceinline__ uint32_t operator()(uint64_t i) const {
    if (i < n) return rec[i].tail;
    const sheep_xs1 r = rec[i - n];
    return (llama && r.tail == r.head) ? NO_KEY : r.head;
  }
};
// Both endpoints with the tail part padded to whole tiles: keys [0, np) are the tails
// (NO_KEY past n), [np, np + n) the heads — so head tile t covers exactly the records of
// record tile t (their (bucket, tile) counts are the relabel's head layout).
struct EndpointKeysP {
  const sheep_xs1 *rec;
  uint64_t n, np;
  int llama;
  __device__ __forceinline__ uint32_t operator()(uint64_t i) const {
    if (i < np) return i < n ? rec[i].tail : NO_KEY;
    const sheep_xs1 r = rec[i - np];
    return (llama && r.tail == r.head) ? NO_KEY : r.head;
  }
};
// lo = low 32 bits of a (hi << 32 | lo) tree edge; DEAD edges carry no key.
struct EdgeLoKeys {
  const uint64_t *edges;
  __device__ __forceinline__ uint32_t operator()(uint64_t i) const {
    const uint64_t e = edges[i];
    return e == ~0ull ? NO_KEY : (uint32_t)e;
  }
};

// lo of a tree edge, shifted so that every first-activity range of the elimination tree
// (etree.hip: lo with ya = spread(lo) having its highest zero bit at s) starts on a
// bucket boundary: key = lo + padoff[f(lo)].  Grouping edges by key then yields, per
// range, a run of whole buckets.
struct EdgeLoPadded {
  const uint64_t *edges;
  const uint32_t *padoff;
  uint32_t clo, mask;
  __device__ __forceinline__ uint32_t operator()(uint64_t i) const { return key(edges[i]); }
  __device__ __forceinline__ uint32_t key(uint64_t e) const {
    if (e == ~0ull) return NO_KEY;
    const uint32_t lo = (uint32_t)e;
    const uint32_t inv = ~(lo + __umulhi(lo, clo)) & mask;
    return lo + padoff[31 - __clz(inv)];
  }
};

constexpr int KPT = 32;                 // keys per thread in the scatter pass
constexpr uint32_t TLOG = 15;           // tile = HB * KPT = 32768 keys
constexpr uint32_t TKEYS = 1u << TLOG;
static_assert(HB * KPT == (int)TKEYS, "tile shape");
constexpr int CB = 256;                 // count pass: small workgroups, high occupancy
constexpr int CPT = 8;                  // count pass keys per thread per step

template <typename Src>
__global__ __launch_bounds__(CB) void k_hist_count(Src src, uint64_t n, uint32_t nb, uint32_t *__restrict__ tile_hist,
                                                   uint64_t ntiles) {
  extern __shared__ uint32_t lds[];
  for (uint32_t b = threadIdx.x; b < nb; b += CB) lds[b] = 0;
  lds_barrier();
  const uint32_t tile = xcd_tile();
  const uint64_t base = (uint64_t)tile << TLOG;
  for (uint32_t step = 0; step < TKEYS; step += CB * CPT) {
    uint32_t k[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) {   // all loads in flight before any LDS atomic
      const uint64_t i = base + step + (uint64_t)j * CB + threadIdx.x;
      k[j] = i < n ? src(i) : NO_KEY;
    }
#pragma unroll
    for (int j = 0; j < CPT; ++j)
      if (k[j] != NO_KEY) atomicAdd(&lds[k[j] >> WBITS], 1u);
  }
  lds_barrier();
  for (uint32_t b = threadIdx.x; b < nb; b += CB) tile_hist[(uint64_t)b * ntiles + tile] = lds[b];
}

// Block-wide exclusive scan of a[0, nb) in LDS (nb <= 8 * NT, NT threads), in place;
// returns total.
template <int NT = HB>
__device__ uint32_t lds_exclusive_scan(uint32_t *a, uint32_t nb, uint32_t *wsum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t per = (nb + NT - 1) / NT, b0 = threadIdx.x * per;
  uint32_t v[8];
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    v[q] = (q < (int)per && b0 + q < nb) ? a[b0 + q] : 0;
    s += v[q];
  }
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wsum[wave] = inc;
  lds_barrier();
  uint32_t off = 0, tot = 0;
  for (int w = 0; w < NT / WAVE; ++w) {
    const uint32_t x = wsum[w];
    if (w < wave) off += x;
    tot += x;
  }
  uint32_t run = off + inc - s;
#pragma unroll
  for (int q = 0; q < 8; ++q)
    if (q < (int)per && b0 + q < nb) { a[b0 + q] = run; run += v[q]; }
  lds_barrier();
  return tot;
}

// Tile keys are held in registers (one source read); counting sort of (bucket, local)
// in LDS; runs written with consecutive lanes.  stage[] carries bucket << 16 | local.
// gb[b] = the bucket's output position for this tile minus its local start, read from the
// scanned offsets once per bucket (not once per written key).
template <typename Src>
__global__ __launch_bounds__(HB) void k_hist_scatter(Src src, uint64_t n, uint32_t nb,
                                                     const uint32_t *__restrict__ offsets, uint64_t ntiles,
                                                     uint16_t *__restrict__ out) {
  extern __shared__ uint32_t lds[];
  uint32_t *cur = lds;              // nb: counts -> starts -> running cursors
  uint32_t *gb = lds + nb;          // nb: output base of each bucket's run (global - local start)
  uint32_t *wsum = lds + 2 * nb;    // HB / WAVE
  uint32_t *stage = lds + 2 * nb + HB / WAVE;
  for (uint32_t b = threadIdx.x; b < nb; b += HB) cur[b] = 0;
  lds_barrier();
  const uint32_t tile = xcd_tile();
  const uint64_t base = (uint64_t)tile << TLOG;
  uint32_t k[KPT], rk[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint64_t i = base + (uint64_t)j * HB + threadIdx.x;
    k[j] = i < n ? src(i) : NO_KEY;
  }
  // the counting atomic's old value is the key's rank in its bucket: placing it then needs
  // a read of the bucket's start, not a second atomic
#pragma unroll
  for (int j = 0; j < KPT; ++j) rk[j] = k[j] != NO_KEY ? atomicAdd(&cur[k[j] >> WBITS], 1u) : 0u;
  lds_barrier();
  const uint32_t total = lds_exclusive_scan(cur, nb, wsum);
  for (uint32_t b = threadIdx.x; b < nb; b += HB) gb[b] = offsets[(uint64_t)b * ntiles + tile] - cur[b];
  lds_barrier();
#pragma unroll
  for (int j = 0; j < KPT; ++j)
    if (k[j] != NO_KEY) {
      const uint32_t b = k[j] >> WBITS;
      stage[cur[b] + rk[j]] = (b << 16) | (k[j] & (W - 1));
    }
  lds_barrier();
  for (uint32_t j = threadIdx.x; j < total; j += HB) {
    const uint32_t x = stage[j];
    out[gb[x >> 16] + j] = (uint16_t)(x & 0xFFFF);
  }
}

// k_hist_scatter for key ranges whose bucket counters and a whole staged tile do not fit
// LDS together (more than ~4087 buckets, vertex ids above 2^27): the tile's keys are
// counting-sorted SUB = PER * HB at a time, each bucket's run of a sub-tile written at the
// bucket's running cursor (the same (bucket, tile) regions as k_hist_scatter).
template <typename Src, int PER, int NT = HB>
__global__ __launch_bounds__(NT) void k_hist_scatter_staged(Src src, uint64_t n, uint32_t nb,
                                                            const uint32_t *__restrict__ offsets, uint64_t ntiles,
                                                            uint16_t *__restrict__ out) {
  constexpr uint32_t SUB = PER * NT;
  extern __shared__ uint32_t lds[];
  uint32_t *cur = lds, *gb = lds + nb, *wsum = lds + 2 * nb;
  uint32_t *stage = lds + 2 * nb + NT / WAVE;
  const uint64_t tile = xcd_tile();
  for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] = offsets[(uint64_t)b * ntiles + tile];
  const uint64_t base = tile << TLOG;
  for (uint32_t s0 = 0; s0 < TKEYS; s0 += SUB) {
    for (uint32_t b = threadIdx.x; b < nb; b += NT) cur[b] = 0;
    lds_barrier();
    uint32_t k[PER], rk[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t i = base + s0 + (uint64_t)j * NT + threadIdx.x;
      k[j] = i < n ? src(i) : NO_KEY;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) rk[j] = k[j] != NO_KEY ? atomicAdd(&cur[k[j] >> WBITS], 1u) : 0u;   // rank in bucket
    lds_barrier();
    const uint32_t total = lds_exclusive_scan<NT>(cur, nb, wsum);
    for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] -= cur[b];
    lds_barrier();
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (k[j] != NO_KEY) stage[cur[k[j] >> WBITS] + rk[j]] = k[j];
    lds_barrier();
    for (uint32_t j = threadIdx.x; j < total; j += NT) {
      const uint32_t key = stage[j];
      out[gb[key >> WBITS] + j] = (uint16_t)(key & (W - 1));
    }
    lds_barrier();
    for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] += b + 1 < nb ? cur[b + 1] : total;   // past the run
    lds_barrier();
  }
}

// k_hist_scatter for tree edges grouped by padded lo: besides the u16 key runs it moves
// each edge into `grouped` at the same position, so the elimination tree's input comes
// out in lo-bucket order at no extra read.  SUB = PER * HB edges at a time are
// counting-sorted by bucket in LDS and each bucket's run is written with consecutive
// lanes (the u16 key beside it); one scattered 8-B store per lane took 15.4 ms at RMAT-26
// against 9.8.
template <int PER, int NT = HB>
__global__ __launch_bounds__(NT) void k_lo_scatter_staged(EdgeLoPadded src, uint64_t n, uint32_t nb,
                                                          const uint32_t *__restrict__ offsets, uint64_t ntiles,
                                                          uint16_t *__restrict__ out, uint64_t *__restrict__ grouped) {
  constexpr uint32_t SUB = PER * NT;
  extern __shared__ uint32_t lds[];
  uint32_t *cur = lds, *gb = lds + nb, *wsum = lds + 2 * nb;
  uint64_t *stage = (uint64_t *)(lds + ((2 * nb + NT / WAVE + 1) & ~1u));
  const uint64_t tile = xcd_tile();
  for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] = offsets[(uint64_t)b * ntiles + tile];
  const uint64_t base = tile << TLOG;
  for (uint32_t s0 = 0; s0 < TKEYS; s0 += SUB) {
    for (uint32_t b = threadIdx.x; b < nb; b += NT) cur[b] = 0;
    lds_barrier();
    uint64_t e[PER];
    uint32_t k[PER], rk[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t i = base + s0 + (uint64_t)j * NT + threadIdx.x;
      e[j] = i < n ? src.edges[i] : ~0ull;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      k[j] = src.key(e[j]);
      rk[j] = k[j] != NO_KEY ? atomicAdd(&cur[k[j] >> WBITS], 1u) : 0u;   // rank in bucket
    }
    lds_barrier();
    const uint32_t total = lds_exclusive_scan<NT>(cur, nb, wsum);
    for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] -= cur[b];
    lds_barrier();
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (k[j] != NO_KEY) stage[cur[k[j] >> WBITS] + rk[j]] = e[j];
    lds_barrier();
    for (uint32_t j = threadIdx.x; j < total; j += NT) {
      const uint64_t v = stage[j];
      const uint32_t key = src.key(v), dst = gb[key >> WBITS] + j;
      grouped[dst] = v;
      out[dst] = (uint16_t)(key & (W - 1));
    }
    lds_barrier();
    for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] += b + 1 < nb ? cur[b + 1] : total;   // past the run
    lds_barrier();
  }
}

// One workgroup per chunk = (bucket, slice of its keys).  A bucket's keys can be very
// skewed (pst: a few thousand positions own most lower endpoints; one bucket took
// 21 ms alone on RMAT-26), so buckets are cut into slices of <= CHUNK keys; a bucket
// with several slices adds its counts with atomics (one per nonzero counter per
// slice), a single-slice bucket owns its range and adds plainly.
struct Chunk {
  uint64_t beg, end;
  uint32_t bucket, shared;
};
constexpr uint64_t CHUNK = 1u << 20;
// Slice length for `total` keys: CHUNK for large inputs; smaller inputs (RMAT-22: 128
// buckets of ~512K keys) are cut finer so the grid still covers the 256 CUs several
// times over (no less than 2^17 keys a slice: each slice also loads or flushes a bucket's
// 2^15 LDS words).
static uint64_t chunk_for(uint64_t total) {
  const uint64_t want = total / 1024;
  const uint64_t c = want < (1ull << 17) ? (1ull << 17) : want > CHUNK ? CHUNK : want;
  return (c + 8191) & ~8191ull;
}

constexpr int HF_U = 32;   // keys per thread in flight in k_hist_final (one workgroup per CU)
__global__ __launch_bounds__(HB) void k_hist_final(const uint16_t *__restrict__ keys, const Chunk *__restrict__ chunks,
                                                   uint64_t K, const uint32_t *__restrict__ kbase,
                                                   uint32_t *__restrict__ cnt) {
  extern __shared__ uint32_t lds[];
  const Chunk ch = chunks[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < W; i += HB) lds[i] = 0;
  lds_barrier();
  for (uint64_t i0 = ch.beg; i0 < ch.end; i0 += HF_U * HB) {
    uint32_t k[HF_U];
#pragma unroll
    for (int j = 0; j < HF_U; ++j) {
      const uint64_t i = i0 + (uint64_t)j * HB + threadIdx.x;
      k[j] = i < ch.end ? keys[i] : NO_KEY;
    }
#pragma unroll
    for (int j = 0; j < HF_U; ++j)
      if (k[j] != NO_KEY) atomicAdd(&lds[k[j]], 1u);
  }
  lds_barrier();
  // counter index of the bucket's first key (padded keys: the range's own lo offset)
  const uint64_t k0 = kbase ? kbase[ch.bucket] : (uint64_t)ch.bucket << WBITS;
  for (uint32_t i = threadIdx.x; i < W; i += HB) {
    const uint32_t v = lds[i];
    if (!v || k0 + i >= K) continue;
    if (ch.shared) atomicAdd(&cnt[k0 + i], v);
    else cnt[k0 + i] += v;   // the bucket's only workgroup owns [k0, k0 + W)
  }
}

template <typename Src>
__global__ __launch_bounds__(BLOCK) void k_count_atomic(Src src, uint64_t n, uint32_t *__restrict__ cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    const uint32_t k = src(i);
    if (k != NO_KEY) atomicAdd(&cnt[k], 1u);
  }
}

// out[b] = off[b * ntiles] (each bucket's first position), out[nb] = *total: the bucket
// starts in one contiguous block for a single small copy to the host (a strided 2-D copy
// of nb 4-B rows cost ~0.15 ms of runtime time at RMAT-26)
__global__ void k_bucket_starts(const uint32_t *__restrict__ off, uint64_t ntiles, uint32_t nb,
                                const uint32_t *__restrict__ total, uint32_t *__restrict__ out) {
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b <= nb; b += gridDim.x * blockDim.x)
    out[b] = b < nb ? off[(uint64_t)b * ntiles] : *total;
}

// Adds the histogram of src's keys over [0, K) into cnt.  With `grouped`, src is
// EdgeLoPadded, K its padded key range, kbase the counter index of each bucket's first
// key, and the edges are also written to `grouped` in bucket order; bstart_out (nb + 1
// entries, device) receives each bucket's first position there.
// Returns the number of keys bucketed (UINT64_MAX on the one-atomic-per-key path).
template <typename Src>
uint64_t histogram_add(Ctx &c, Src src, uint64_t n, uint64_t K, uint32_t *cnt, uint64_t *grouped = nullptr,
                       const uint32_t *kbase = nullptr, uint32_t *bstart_out = nullptr,
                       uint32_t *save_offsets = nullptr, std::vector<uint32_t> *save_bstart = nullptr,
                       bool counted = false) {
  if (n == 0 || K == 0) return 0;
  const uint32_t nb = (uint32_t)((K + W - 1) >> WBITS);
  const uint64_t ntiles = (n + TKEYS - 1) >> TLOG;
  const size_t lds_scatter = (2 * (size_t)nb + HB / WAVE + TKEYS) * 4;   // <= 160 KiB for nb <= 4087
  const size_t lds_scatter16 = (2 * (size_t)nb + HB / WAVE + 16 * HB) * 4;   // staged: nb <= 8192
  // the staged grouping scatter holds 2 nb counters + PER * HB staged edges: nb <= 8192
  // (lds_exclusive_scan's limit) with PER = 8, i.e. padded lo ranges up to 2^28
  const size_t lds_staged16 = ((2 * (size_t)nb + HB / WAVE + 1) & ~(size_t)1) * 4 + 16 * HB * 8;
  const size_t lds_staged8 = lds_staged16 - 8 * HB * 8;
  const bool fits = std::is_same<Src, EdgeLoPadded>::value ? (nb <= 8 * HB && lds_staged8 <= 160 * 1024)
                                                            : (nb <= 8 * HB && lds_scatter16 <= 160 * 1024);
  if (!fits || ntiles * nb >= (1ull << 32) || n >= (1ull << 32)) {
    if constexpr (std::is_same<Src, EdgeLoPadded>::value) {
      throw Error(SHEEP_ERR_ARG, "group_edges_by_lo: padded lo range above 2^28 or 2^32 edges");
    } else {   // key ranges beyond the LDS buckets: one scattered atomic per key
      hipLaunchKernelGGL(k_count_atomic<Src>, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, src, n, cnt);
      LAUNCH_CHECK();
      return UINT64_MAX;
    }
  }
  for (const void *f : {(const void *)k_hist_scatter<HeadKeys>, (const void *)k_hist_scatter<EdgeLoKeys>,
                        (const void *)k_hist_scatter<EndpointKeys>, (const void *)k_hist_scatter_staged<EndpointKeys, 16>,
                        (const void *)k_hist_scatter<EndpointKeysP>, (const void *)k_hist_scatter_staged<EndpointKeysP, 16>,
                        (const void *)k_hist_scatter_staged<HeadKeys, 16>,
                        (const void *)k_hist_scatter_staged<EdgeLoKeys, 16>, (const void *)k_hist_final,
                        (const void *)k_lo_scatter_staged<16>, (const void *)k_lo_scatter_staged<8>})
    allow_full_lds(f);
  uint32_t *tile_hist = c.get_as<uint32_t>("hist_tiles", ntiles * nb + 1);
  // (the keys live only inside a histogram pass; their workspace is the elimination tree's
  // per-cross-entry root buffer, et_xtop, which the levels fill only after the relabel)
  uint16_t *keys = c.get_as<uint16_t>("et_xtop", n);
  if (!counted) {   // (counted: degree_fused already wrote tile_hist, >= nb bucket rows)
    hipLaunchKernelGGL(k_hist_count<Src>, dim3((unsigned)ntiles), dim3(CB), nb * 4, c.stream, src, n, nb, tile_hist,
                       ntiles);
    LAUNCH_CHECK();
  }
  uint32_t *total = c.get_as<uint32_t>("hist_total", 1);
  scan_exclusive_u32(c, tile_hist, tile_hist, ntiles * nb, total);
  if (save_offsets) {   // the relabel's bucket layout (relabel_bucketed, below)
    HIP_CHECK(hipMemcpyAsync(save_offsets, tile_hist, ntiles * nb * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
    HIP_CHECK(hipMemcpyAsync(save_offsets + ntiles * nb, total, sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
  }
  if constexpr (std::is_same<Src, EdgeLoPadded>::value) {
    if (lds_staged16 <= 160 * 1024)
      hipLaunchKernelGGL(k_lo_scatter_staged<16>, dim3((unsigned)ntiles), dim3(HB), lds_staged16, c.stream, src, n, nb,
                         (const uint32_t *)tile_hist, ntiles, keys, grouped);
    else
      hipLaunchKernelGGL(k_lo_scatter_staged<8>, dim3((unsigned)ntiles), dim3(HB), lds_staged8, c.stream, src, n, nb,
                         (const uint32_t *)tile_hist, ntiles, keys, grouped);
  } else if (lds_scatter <= 160 * 1024) {
    hipLaunchKernelGGL(k_hist_scatter<Src>, dim3((unsigned)ntiles), dim3(HB), lds_scatter, c.stream, src, n, nb,
                       (const uint32_t *)tile_hist, ntiles, keys);
  } else {
    hipLaunchKernelGGL((k_hist_scatter_staged<Src, 16>), dim3((unsigned)ntiles), dim3(HB), lds_scatter16, c.stream, src, n,
                       nb, (const uint32_t *)tile_hist, ntiles, keys);
  }
  LAUNCH_CHECK();
  // bucket starts (column 0 of the bucket-major offsets) -> chunk list.  Host buffers are
  // pinned, so the chunk list's copy needs no sync of its own (the next call's first sync
  // comes before it rewrites them).
  uint32_t *bstart = (uint32_t *)c.get_pinned("hist_bstart_host", (nb + 1) * sizeof(uint32_t));
  uint32_t *bs_dev = c.get_as<uint32_t>("hist_bstart_dev", nb + 1);
  hipLaunchKernelGGL(k_bucket_starts, dim3(grid_for(nb + 1)), dim3(BLOCK), 0, c.stream, (const uint32_t *)tile_hist, ntiles,
                     nb, (const uint32_t *)total, bs_dev);
  LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(bstart, bs_dev, (nb + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (save_bstart) save_bstart->assign(bstart, bstart + nb + 1);
  const uint64_t chunk = chunk_for(bstart[nb]);
  uint64_t nch = 0;
  for (uint32_t b = 0; b < nb; ++b) nch += (bstart[b + 1] - bstart[b] + chunk - 1) / chunk;
  if (bstart_out) {
    uint32_t *bs = (uint32_t *)c.get_pinned("hist_bstart_copy", (nb + 1) * sizeof(uint32_t));
    std::copy(bstart, bstart + nb + 1, bs);
    HIP_CHECK(hipMemcpyAsync(bstart_out, bs, (nb + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
  }
  const uint64_t keys_total = bstart[nb];
  if (!nch) return keys_total;
  Chunk *chunks = (Chunk *)c.get_pinned("hist_chunks_host", nch * sizeof(Chunk));
  uint64_t j = 0;
  for (uint32_t b = 0; b < nb; ++b) {
    const uint64_t beg = bstart[b], end = bstart[b + 1];
    if (beg == end) continue;
    const uint32_t shared = end - beg > chunk;
    for (uint64_t x = beg; x < end; x += chunk) chunks[j++] = {x, x + chunk < end ? x + chunk : end, b, shared};
  }
  Chunk *dch = c.get_as<Chunk>("hist_chunks", nch);
  HIP_CHECK(hipMemcpyAsync(dch, chunks, nch * sizeof(Chunk), hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_hist_final, dim3((unsigned)nch), dim3(HB), W * 4, c.stream, (const uint16_t *)keys,
                     (const Chunk *)dch, K, kbase, cnt);
  LAUNCH_CHECK();
  return keys_total;
}



// ---- degree pass fused with the heads' bucket counts (sequence.h:65-107) --------------
// k_degree's work (tails, the FILE_DAT last record's extra head, max slot, range check)
// and k_hist_count's per-tile head bucket counts in one read of the records.  Buckets are
// laid out for the capacity (nb_cap rows); the rows beyond the max slot's stay zero, so
// the same offsets serve the true key range.
// Tails: the records come tail-sorted, so a tile's tails lie in [first tail, last tail]
// (about 2K slots at RMAT-26).  When that span fits TSPAN LDS counters, each wave adds
// its tail RUNS there (one LDS atomic per run) and the tile flushes the counters with
// full-wave atomics: ~span/64 global atomic instructions per tile instead of one per
// wave-load of records (run_add), whose issue rate bound the pass (4.5 ms at RMAT-26:
// one atomic wave-instruction per ~50 ns per CU, MI355X_MICROARCH.md).  A tail outside
// the span (an unsorted stretch) takes a global atomic of its own.
constexpr uint32_t TSPAN = 4096;
constexpr int DPT = 8;   // degree pass records per thread per step (4 / 16: 4.06 / 4.59 ms against 3.95 at RMAT-26)

__global__ __launch_bounds__(CB) void k_degree_fused(const sheep_xs1 *__restrict__ rec, uint64_t n, int mode,
                                                     uint32_t *__restrict__ deg, uint64_t cap, uint32_t nb,
                                                     uint32_t *__restrict__ tile_hist, uint64_t ntiles,
                                                     unsigned long long *__restrict__ d_max,
                                                     unsigned long long *__restrict__ d_err) {
  extern __shared__ uint32_t lds[];
  uint32_t *tcnt = lds + nb;   // TSPAN tail counters after the nb head buckets
  const uint32_t tile = xcd_tile();
  const uint64_t base = (uint64_t)tile << TLOG;
  const uint64_t last = (base + TKEYS < n ? base + TKEYS : n) - 1;
  const uint32_t t0 = rec[base].tail, t1 = rec[last].tail;
  const bool span = t1 >= t0 && t1 - t0 < TSPAN;   // uniform over the workgroup
  for (uint32_t b = threadIdx.x; b < nb; b += CB) lds[b] = 0;
  if (span)
    for (uint32_t b = threadIdx.x; b <= t1 - t0; b += CB) tcnt[b] = 0;
  lds_barrier();
  const int lane = (int)__lane_id();
  uint32_t lmax = 0;
  bool bad = false;
  for (uint32_t step = 0; step < TKEYS; step += CB * DPT) {
    sheep_xs1 r[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {   // all loads in flight first
      const uint64_t i = base + step + (uint64_t)j * CB + threadIdx.x;
      if (i < n) r[j] = rec[i];
    }
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const uint64_t i = base + step + (uint64_t)j * CB + threadIdx.x;
      uint32_t kt = INVALID, kh = INVALID, inc = 1;
      if (i < n) {
        const uint32_t t = r[j].tail, h = r[j].head;
        if (t >= cap || h >= cap) {
          bad = true;
        } else {
          inc = (mode == SHEEP_DEGREE_FILE_DAT && i == n - 1) ? 2u : 1u;
          kt = t;
          kh = (mode == SHEEP_DEGREE_LLAMA && t == h) ? INVALID : h;   // LLAMA: self-loop stored once
          const uint32_t m = (t > h ? t : h) + 1;
          lmax = m > lmax ? m : lmax;
        }
      }
      if (span) {
        // runs of equal tails among the wave's consecutive lanes: the run's first lane adds
        // its length (the FILE_DAT last record's second count goes to the global counter)
        const uint32_t prev = __shfl_up(kt, 1, 64);
        const bool start = kt != INVALID && (lane == 0 || prev != kt);
        const uint64_t starts = __ballot(start);
        const uint64_t valid = __ballot(kt != INVALID);
        if (start) {
          const uint64_t above = lane == 63 ? 0ull : (starts & ~((2ull << lane) - 1));
          const uint64_t vend = lane == 63 ? 0ull : (~valid & ~((2ull << lane) - 1));
          const uint64_t stop = above | vend;
          const int next = stop ? __ffsll((long long)stop) - 1 : 64;
          const uint32_t len = (uint32_t)(next - lane);
          if (kt >= t0 && kt <= t1) atomicAdd(&tcnt[kt - t0], len);   // the tile's zeroed counters
          else atomicAdd(&deg[kt], len);
        }
        if (inc == 2) atomicAdd(&deg[kt], 1u);
      } else {
        run_add(deg, kt, inc);   // every lane of the wave takes part (uniform loop)
      }
      if (inc == 2 && kh != INVALID) atomicAdd(&deg[kh], 1u);
      if (kh != INVALID) atomicAdd(&lds[kh >> WBITS], 1u);
    }
  }
  lds_barrier();
  for (uint32_t b = threadIdx.x; b < nb; b += CB) tile_hist[(uint64_t)b * ntiles + tile] = lds[b];
  if (span)
    for (uint32_t b = threadIdx.x; b <= t1 - t0; b += CB)
      if (tcnt[b]) atomicAdd(&deg[t0 + b], tcnt[b]);
  block_atomic_max(d_max, lmax);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(d_err, 1ull);
}

// ---- degree pass for records in any order (sequence.h:65-107) --------------------------
// Tails are not in runs, so both endpoints go through the bucketed histogram; this pass
// makes its whole count step in ONE read of the records: per record tile, the range check,
// the max slot, the FILE_DAT last record's extra counts (global atomics, as k_degree) and
// the tails' and heads' bucket counts (two LDS histograms) — written as the count rows of
// EndpointKeysP's tail tile t and head tile NT + t (bucket-major, 2 NT tiles per bucket).
__global__ __launch_bounds__(CB) void k_degree_endpoints(const sheep_xs1 *__restrict__ rec, uint64_t n, int mode,
                                                         uint32_t *__restrict__ deg, uint64_t cap, uint32_t nb,
                                                         uint32_t *__restrict__ tile_hist, uint64_t nt,
                                                         unsigned long long *__restrict__ d_max,
                                                         unsigned long long *__restrict__ d_err) {
  extern __shared__ uint32_t lds[];
  uint32_t *tc = lds, *hc = lds + nb;
  const uint32_t tile = xcd_tile();
  const uint64_t base = (uint64_t)tile << TLOG;
  for (uint32_t b = threadIdx.x; b < 2 * nb; b += CB) lds[b] = 0;
  lds_barrier();
  uint32_t lmax = 0;
  bool bad = false;
  for (uint32_t step = 0; step < TKEYS; step += CB * DPT) {
    sheep_xs1 r[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const uint64_t i = base + step + (uint64_t)j * CB + threadIdx.x;
      if (i < n) r[j] = rec[i];
    }
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const uint64_t i = base + step + (uint64_t)j * CB + threadIdx.x;
      if (i >= n) continue;
      const uint32_t t = r[j].tail, h = r[j].head;
      if (t >= cap || h >= cap) { bad = true; continue; }
      const bool loop_once = mode == SHEEP_DEGREE_LLAMA && t == h;   // LLAMA: a self-loop stored once
      if (mode == SHEEP_DEGREE_FILE_DAT && i == n - 1) {   // the XS1 reader's repeated last record
        atomicAdd(&deg[t], 1u);
        if (!loop_once) atomicAdd(&deg[h], 1u);
      }
      const uint32_t m = (t > h ? t : h) + 1;
      lmax = m > lmax ? m : lmax;
      atomicAdd(&tc[t >> WBITS], 1u);
      if (!loop_once) atomicAdd(&hc[h >> WBITS], 1u);
    }
  }
  lds_barrier();
  for (uint32_t b = threadIdx.x; b < nb; b += CB) {
    tile_hist[(uint64_t)b * 2 * nt + tile] = tc[b];
    tile_hist[(uint64_t)b * 2 * nt + nt + tile] = hc[b];
  }
  block_atomic_max(d_max, lmax);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(d_err, 1ull);
}

// head layout = the head columns of the endpoint counts: out[b * nt + t] = in[b * 2nt + nt + t]
__global__ void k_head_cols(const uint32_t *__restrict__ in, uint64_t nt, uint32_t nb, uint32_t *__restrict__ out) {
  const uint64_t total = (uint64_t)nb * nt, stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint64_t b = i / nt, t = i - b * nt;
    out[i] = in[b * 2 * nt + nt + t];
  }
}

// ---- head-bucketed relabel (jtree.cpp:72-91) -----------------------------------------
// k_relabel's pos[head] gather is random over the whole 4-B-per-slot index (268 MB at
// RMAT-26): each 4-B load moves a full line.  Here the records are first scattered into
// the heads' 2^15-slot buckets -- carrying pos[tail], a near-sequential gather since
// records come tail-sorted -- with the same tiles and bucket-major offsets as the degree
// pass's head histogram (whose scanned offsets are reused), and then one workgroup per
// bucket slice holds the bucket's 128 KiB of pos in LDS and relabels from there.
//   pass A k_relabel_scatter: 12 B record + pos[tail] in, 8 B (ptail << 32 | head) out
//   pass B k_relabel_gather:  8 B in, 8 B tree edge out, pos read once per slice
// Edges come out in head-bucket order; every later stage is order-independent (the pst
// histogram groups them by lo, the elimination tree is unique for the edge multiset).
constexpr uint32_t PT_OOR = 0xFFFFFFFEu;   // tail >= pos_size (only an error if the head is sequenced)
constexpr uint64_t NO_PAIR = ~0ull;

// the relabel's keys: heads < pos_size of non-self-loop records (LLAMA HeadKeys when
// pos_size equals the degree pass's key range)
struct RelabelKeys {
  const sheep_xs1 *rec;
  uint64_t pos_size;
  __device__ __forceinline__ uint32_t operator()(uint64_t i) const {
    const sheep_xs1 r = rec[i];
    return (r.tail == r.head || r.head >= pos_size) ? NO_KEY : r.head;
  }
};

// One tile of TKEYS records per workgroup, staged SUB = PER * HB at a time (u64 payloads:
// a whole tile does not fit LDS).  gb[b] walks the tile's region of bucket b; every write
// is bounded by the output's capacity and a region not filled exactly raises flags[1]
// (stale offsets: the host recounts; a stale run's writes stay in bounds and are
// discarded) — one random LDS read per record fewer than a per-region bound.  flags[0]: a
// sequenced endpoint's neighbour >= pos_size.
template <int PER, int NT = HB, bool PL = false>   // PL: the staged pairs as two u32 planes
__global__ __launch_bounds__(NT) void k_relabel_scatter(const sheep_xs1 *__restrict__ rec, uint64_t n,
                                                        const uint32_t *__restrict__ pos, uint64_t pos_size, uint32_t nb,
                                                        const uint32_t *__restrict__ offsets, uint64_t ntiles,
                                                        uint64_t *__restrict__ out, unsigned long long *__restrict__ flags) {
  constexpr uint32_t SUB = PER * NT;
  extern __shared__ uint32_t lds[];
  uint32_t *cur = lds, *gb = lds + nb, *wsum = lds + 2 * nb;
  uint64_t *stage = (uint64_t *)(lds + ((2 * nb + NT / WAVE + 1) & ~1u));
  uint32_t *const slo = (uint32_t *)stage, *const shi = slo + SUB;
  const uint64_t tile = xcd_tile();
  const uint32_t cap = offsets[(uint64_t)nb * ntiles];   // the scanned total: the output's length
  for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] = offsets[(uint64_t)b * ntiles + tile];
  bool bad = false, lost = false;
  const uint64_t base = tile << TLOG;
  for (uint32_t s0 = 0; s0 < TKEYS; s0 += SUB) {
    for (uint32_t b = threadIdx.x; b < nb; b += NT) cur[b] = 0;
    lds_barrier();
    uint64_t x[PER];
    uint32_t pt[PER], hd[PER], rk[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {   // all record loads, then all pos[tail] loads in flight
      const uint32_t in_tile = s0 + (uint32_t)j * NT + threadIdx.x;   // (SUB need not divide the tile)
      const uint64_t i = base + in_tile;
      hd[j] = INVALID;
      pt[j] = INVALID;
      if (i < n && in_tile < TKEYS) {
        const uint32_t t = rec[i].tail, h = rec[i].head;
        if (t != h) { hd[j] = h; pt[j] = t; }
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      x[j] = NO_PAIR;
      if (hd[j] == INVALID && pt[j] == INVALID) continue;
      const uint32_t t = pt[j], h = hd[j];
      const uint32_t ptm = t < pos_size ? pos[t] : PT_OOR;
      if (h >= pos_size) {
        if (ptm < PT_OOR) bad = true;   // index.at(head) throws (jtree.cpp:75)
        continue;
      }
      x[j] = ((uint64_t)ptm << 32) | h;
      rk[j] = atomicAdd(&cur[h >> WBITS], 1u);   // the pair's rank in its bucket
    }
    lds_barrier();
    const uint32_t total = lds_exclusive_scan<NT>(cur, nb, wsum);
    for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] -= cur[b];   // region cursor - local start
    lds_barrier();
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (x[j] != NO_PAIR) {
        const uint32_t at = cur[(uint32_t)x[j] >> WBITS] + rk[j];
        if (PL) {
          slo[at] = (uint32_t)x[j];
          shi[at] = (uint32_t)(x[j] >> 32);
        } else {
          stage[at] = x[j];
        }
      }
    lds_barrier();
    for (uint32_t j = threadIdx.x; j < total; j += NT) {
      const uint64_t v = PL ? ((uint64_t)shi[j] << 32) | slo[j] : stage[j];
      const uint32_t b = (uint32_t)v >> WBITS, dst = gb[b] + j;
      if (dst < cap) out[dst] = v;
      else lost = true;
    }
    lds_barrier();
    for (uint32_t b = threadIdx.x; b < nb; b += NT) gb[b] += b + 1 < nb ? cur[b + 1] : total;   // past this sub-tile's run
    lds_barrier();
  }
  for (uint32_t b = threadIdx.x; b < nb; b += NT)
    if (gb[b] != offsets[(uint64_t)b * ntiles + tile + 1]) lost = true;   // the region's end
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(&flags[0], 1ull);
  if (__any(lost) && (threadIdx.x & 63) == 0) atomicAdd(&flags[1], 1ull);
}

// One workgroup per (bucket, slice of <= CHUNK pairs): the bucket's pos slice in LDS.
// Same outcomes as k_relabel: both endpoints sequenced -> tree edge (hi << 32 | lo);
// one sequenced, the other an unsequenced slot -> POSTORDER pst for the sequenced one.
// COUNT: also the edges' (padded-lo bucket, 32K-edge tile) counts of the grouping's
// count pass (k_hist_count<EdgeLoPadded> over the same edges, which then does not run):
// the chunk is walked one output tile at a time with the tile's counts in LDS after the
// pos slice, flushed with one atomicAdd per non-zero bucket (a tile can span two chunks).
constexpr int RG_U = 32;   // pairs per thread in flight (one 1024-thread workgroup per CU: the pos slice fills LDS)
template <bool COUNT>
__global__ __launch_bounds__(HB) void k_relabel_gather(const uint64_t *__restrict__ pairs, const Chunk *__restrict__ chunks,
                                                       const uint32_t *__restrict__ pos, uint64_t pos_size,
                                                       uint32_t *__restrict__ pst, uint64_t *__restrict__ edges,
                                                       unsigned long long *__restrict__ flags, EdgeLoPadded lk,
                                                       uint32_t lnb, uint32_t *__restrict__ tile_hist, uint64_t ntiles,
                                                       uint64_t n_tree) {
  extern __shared__ uint32_t lds[];
  uint32_t *const lcnt = lds + W;
  const Chunk ch = chunks[blockIdx.x];
  const uint64_t v0 = (uint64_t)ch.bucket << WBITS;
  for (uint32_t i = threadIdx.x; i < W; i += HB) lds[i] = v0 + i < pos_size ? pos[v0 + i] : INVALID;
  bool bad = false;
  for (uint64_t t0 = ch.beg; t0 < ch.end;) {
    const uint64_t t1 = COUNT ? ((t0 >> TLOG) + 1) << TLOG : ch.end;   // this output tile's part of the chunk
    const uint64_t s1 = t1 < ch.end ? t1 : ch.end;
    if (COUNT)
      for (uint32_t b = threadIdx.x; b < lnb; b += HB) lcnt[b] = 0;
    lds_barrier();
    for (uint64_t i0 = t0; i0 < s1; i0 += RG_U * HB) {
      uint64_t x[RG_U];
#pragma unroll
      for (int j = 0; j < RG_U; ++j) {
        const uint64_t i = i0 + (uint64_t)j * HB + threadIdx.x;
        x[j] = i >= s1 ? NO_PAIR : pairs[i];
      }
#pragma unroll
      for (int j = 0; j < RG_U; ++j) {
        const uint64_t i = i0 + (uint64_t)j * HB + threadIdx.x;
        if (i >= s1) continue;
        const uint32_t ptm = (uint32_t)(x[j] >> 32), ph = lds[(uint32_t)x[j] & (W - 1)];
        uint64_t e = ~0ull;   // DEAD
        // (ptm is a position < n_tree, INVALID or PT_OOR; anything else is a stale region
        // of a run the host discards, kept in bounds)
        if (ph != INVALID) {
          if (ptm == PT_OOR) bad = true;                       // index.at(tail) throws
          else if (ptm < n_tree) e = ptm < ph ? ((uint64_t)ph << 32) | ptm : ((uint64_t)ptm << 32) | ph;
          else if (ptm == INVALID) atomicAdd(&pst[ph], 1u);
        } else if (ptm < n_tree) {
          atomicAdd(&pst[ptm], 1u);
        }
        edges[i] = e;
        if (COUNT && e != ~0ull) atomicAdd(&lcnt[lk.key(e) >> WBITS], 1u);
      }
    }
    if (COUNT) {
      lds_barrier();
      const uint64_t tile = t0 >> TLOG;
      for (uint32_t b = threadIdx.x; b < lnb; b += HB)
        if (lcnt[b]) atomicAdd(&tile_hist[(uint64_t)b * ntiles + tile], lcnt[b]);
      lds_barrier();   // lcnt is cleared for the next tile
    }
    t0 = s1;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(&flags[0], 1ull);
}

// seg[i] = position of bucket sb[i] in the grouped array (sb: bucket indices)
__global__ void k_seg_from_buckets(const uint32_t *__restrict__ bstart, const uint64_t *__restrict__ sb, int L,
                                   uint64_t *__restrict__ seg) {
  for (int i = threadIdx.x; i < 2 * L; i += blockDim.x) seg[i] = bstart[sb[i]];
}

}  // namespace

bool degree_fused(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap,
                  unsigned long long *d_max, unsigned long long *d_err) {
  const uint64_t nb = (cap + W - 1) >> WBITS, ntiles = (nrec + TKEYS - 1) >> TLOG;
  if (nrec == 0 || nb == 0 || nb > 8192 || nrec >= (1ull << 32) || ntiles * nb + 1 >= (1ull << 32)) return false;
  uint32_t *tile_hist = c.get_as<uint32_t>("hist_tiles", ntiles * nb + 1);
  hipLaunchKernelGGL(k_degree_fused, dim3((unsigned)ntiles), dim3(CB), (nb + TSPAN) * 4, c.stream, rec, nrec, mode, deg, cap,
                     (uint32_t)nb, tile_hist, ntiles, d_max, d_err);
  LAUNCH_CHECK();
  return true;
}

void histogram_heads(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int llama, uint64_t K, uint32_t *cnt, bool counted) {
  Ctx::HeadLayout &hl = c.layout_for(rec, nrec);
  const uint64_t nb = (K + W - 1) >> WBITS, ntiles = (nrec + TKEYS - 1) >> TLOG;
  if (!llama || nb == 0 || nb > 8192 || ntiles * nb + 1 >= (1ull << 32)) {
    histogram_add(c, HeadKeys{rec, llama}, nrec, K, cnt, nullptr, nullptr, nullptr, nullptr, nullptr, counted);
    return;
  }
  uint32_t *save = c.get_as<uint32_t>(Ctx::layout_buf(hl.slot), ntiles * nb + 1);
  histogram_add(c, HeadKeys{rec, llama}, nrec, K, cnt, nullptr, nullptr, nullptr, save, &hl.bstart, counted);
  hl.rec = rec;
  hl.nrec = nrec;
  hl.K = K;
  hl.valid = hl.bstart.size() == nb + 1;
}

bool degree_endpoints(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap,
                      unsigned long long *d_max, unsigned long long *d_err) {
  const uint64_t nb = (cap + W - 1) >> WBITS, nt = (nrec + TKEYS - 1) >> TLOG;
  if (nrec == 0 || nb == 0 || nb > 8192 || nrec >= (1ull << 31) || 2 * nt * nb + 1 >= (1ull << 32)) return false;
  uint32_t *tile_hist = c.get_as<uint32_t>("hist_tiles", 2 * nt * nb + 1);
  hipLaunchKernelGGL(k_degree_endpoints, dim3((unsigned)nt), dim3(CB), 2 * nb * 4, c.stream, rec, nrec, mode, deg, cap,
                     (uint32_t)nb, tile_hist, nt, d_max, d_err);
  LAUNCH_CHECK();
  return true;
}

void histogram_endpoints(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int llama, uint64_t K, uint32_t *cnt,
                         bool counted) {
  Ctx::HeadLayout &hl = c.layout_for(rec, nrec);
  if (!counted) {   // the relabel counts its own head layout
    histogram_add(c, EndpointKeys{rec, nrec, llama}, 2 * nrec, K, cnt);
    return;
  }
  // degree_endpoints wrote the count rows (capacity buckets, 2 nt tiles each); the rows past
  // K's buckets are zero, so the scan over K's buckets serves.  The head columns, scanned on
  // their own, are the relabel's head layout (LLAMA heads: a self-loop not counted; every
  // head is below K) — no recount of the records there.
  const uint64_t nt = (nrec + TKEYS - 1) >> TLOG, nb = (K + W - 1) >> WBITS;
  if (llama && nb && nb <= 8192 && nt * nb + 1 < (1ull << 32)) {
    const uint32_t *tile_hist = c.get_as<uint32_t>("hist_tiles", 2 * nt * nb + 1);
    uint32_t *off = c.get_as<uint32_t>(Ctx::layout_buf(hl.slot), nt * nb + 1);
    hipLaunchKernelGGL(k_head_cols, dim3(grid_for(nt * nb)), dim3(BLOCK), 0, c.stream, tile_hist, nt, (uint32_t)nb, off);
    LAUNCH_CHECK();
    scan_exclusive_u32(c, off, off, nt * nb, off + nt * nb);
    uint32_t *bs_dev = c.get_as<uint32_t>("hist_bstart_dev", nb + 1);
    hipLaunchKernelGGL(k_bucket_starts, dim3(grid_for(nb + 1)), dim3(BLOCK), 0, c.stream, (const uint32_t *)off, nt,
                       (uint32_t)nb, (const uint32_t *)(off + nt * nb), bs_dev);
    LAUNCH_CHECK();
    hl.bstart.assign(nb + 1, 0);
    HIP_CHECK(hipMemcpyAsync(hl.bstart.data(), bs_dev, (nb + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    hl.rec = rec;
    hl.nrec = nrec;
    hl.K = K;
    hl.valid = true;
  }
  histogram_add(c, EndpointKeysP{rec, nrec, nt * TKEYS, llama}, nt * TKEYS + nrec, K, cnt, nullptr, nullptr, nullptr,
                nullptr, nullptr, true);
}

void fill_u32(Ctx &c, uint32_t *p, uint64_t n, uint32_t v);   // sequence.hip

uint64_t relabel_bucketed(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                          uint64_t n_tree, uint32_t *pst, uint64_t *edges, unsigned long long *err, const LoGroup *lg,
                          bool *counted) {
  if (counted) *counted = false;
  const uint64_t nb = (pos_size + W - 1) >> WBITS, ntiles = (nrec + TKEYS - 1) >> TLOG;
  if (nrec == 0 || nb == 0 || nb > 8192 || nrec >= (1ull << 32) || ntiles * nb + 1 >= (1ull << 32)) return UINT64_MAX;
  for (const void *f : {(const void *)k_relabel_scatter<8>, (const void *)k_relabel_scatter<4>,
                        (const void *)k_relabel_scatter<8, 512>, (const void *)k_relabel_scatter<8, 512, true>,
                        (const void *)k_relabel_scatter<12, 512, true>, (const void *)k_relabel_scatter<15, 512, true>,
                        (const void *)k_relabel_scatter<4, 512, true>,
                        (const void *)k_relabel_gather<false>, (const void *)k_relabel_gather<true>})
    allow_full_lds(f);
  Ctx::HeadLayout *found = c.find_layout(rec, nrec);
  Ctx::HeadLayout *hlp = found;
  unsigned long long *flags = c.get_as<unsigned long long>("rl_flags", 2);
  auto recount = [&]() -> uint32_t * {   // the relabel's own (bucket, tile) offsets
    hlp = &c.layout_for(rec, nrec);
    Ctx::HeadLayout &hl = *hlp;
    uint32_t *off = c.get_as<uint32_t>(Ctx::layout_buf(hl.slot), ntiles * nb + 1);
    hipLaunchKernelGGL(k_hist_count<RelabelKeys>, dim3((unsigned)ntiles), dim3(CB), nb * 4, c.stream,
                       RelabelKeys{rec, pos_size}, nrec, (uint32_t)nb, off, ntiles);
    LAUNCH_CHECK();
    scan_exclusive_u32(c, off, off, ntiles * nb, off + ntiles * nb);
    hl.bstart.assign(nb + 1, 0);
    uint32_t *bs_dev = c.get_as<uint32_t>("hist_bstart_dev", nb + 1);
    hipLaunchKernelGGL(k_bucket_starts, dim3(grid_for(nb + 1)), dim3(BLOCK), 0, c.stream, (const uint32_t *)off, ntiles,
                       (uint32_t)nb, (const uint32_t *)(off + ntiles * nb), bs_dev);
    LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(hl.bstart.data(), bs_dev, (nb + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    hl.rec = rec;
    hl.nrec = nrec;
    hl.K = pos_size;
    hl.valid = true;
    return off;
  };
  // The degree pass's layout serves whenever it has this many buckets: its key range K (the
  // records' largest slot + 1) may sit below pos_size (a shard's records, the sequence of
  // all shards), but no head reaches past K, so the buckets and their counts are the same.
  // (A layout that does not match the records is caught by the scatter's region check.)
  // A layout with fewer buckets (a shard of tail-sorted records: its largest slot sits below
  // the sequence's) serves too: the buckets past it are empty, so its offsets are copied
  // and the missing rows filled with the total (bst: the bucket starts this call uses).
  const bool cached = found && found->K <= pos_size && found->bstart.size() >= 2 && found->bstart.size() <= nb + 1;
  std::vector<uint32_t> bst;
  uint32_t *off;
  if (cached && found->bstart.size() == nb + 1) {
    off = c.get_as<uint32_t>(Ctx::layout_buf(found->slot), ntiles * nb + 1);
    bst = found->bstart;
  } else if (cached) {
    const uint64_t nbc = found->bstart.size() - 1;
    const uint32_t tot = found->bstart[nbc];
    const uint32_t *src = c.get_as<uint32_t>(Ctx::layout_buf(found->slot), ntiles * nbc + 1);
    off = c.get_as<uint32_t>("head_offsets_ext", ntiles * nb + 1);
    HIP_CHECK(hipMemcpyAsync(off, src, ntiles * nbc * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
    fill_u32(c, off + ntiles * nbc, ntiles * (nb - nbc) + 1, tot);
    bst = found->bstart;
    bst.resize(nb + 1, tot);
  } else {
    off = recount();
    bst = hlp->bstart;
  }
  Ctx::HeadLayout &hl = *hlp;
  (void)hl;
  const uint64_t total = bst[nb];
  // (the pairs die with the gather: their workspace is the elimination tree's first list
  // buffer, et_list1, which the levels fill only after the relabel)
  uint64_t *pairs = c.get_as<uint64_t>("et_list1", total ? total : 1);
  const size_t fixed = ((2 * nb + HB / WAVE + 1) & ~1ull) * 4;
  auto scatter = [&]() {
    HIP_CHECK(hipMemsetAsync(flags, 0, 2 * sizeof(unsigned long long), c.stream));
    // Two 512-thread workgroups per CU, 4K-record sub-tiles (81 VGPRs keep a 1024-thread
    // workgroup alone on its CU, idle at every barrier): RMAT-26 9.18 -> 8.92 ms.  Up to
    // 4096 buckets (vertex ids below 2^27), the scan's limit for 512 threads.
    {
      constexpr int NT = 512;
      // the staged pairs as two u32 planes (RMAT-26 relabel 13.56 / 13.85 ms against 14.56 /
      // 13.80 with one u64 array, two runs each: within box noise, not worse); relabel_per
      // records per thread per sub-tile (longer runs per bucket region, fewer flushes)
      const bool planes = c.tune.relabel_planes != 0;
      const int P = planes ? c.tune.relabel_per : 8;
      const size_t fx = ((2 * nb + NT / WAVE + 1) & ~1ull) * 4, lds = fx + (size_t)P * NT * 8;
      if (nb <= 8 * (uint64_t)NT && lds <= 160 * 1024) {
        if (planes && P == 15)
          hipLaunchKernelGGL((k_relabel_scatter<15, NT, true>), dim3((unsigned)ntiles), dim3(NT), lds, c.stream, rec,
                             nrec, pos, pos_size, (uint32_t)nb, (const uint32_t *)off, ntiles, pairs, flags);
        else if (planes && P == 4)
          hipLaunchKernelGGL((k_relabel_scatter<4, NT, true>), dim3((unsigned)ntiles), dim3(NT), lds, c.stream, rec,
                             nrec, pos, pos_size, (uint32_t)nb, (const uint32_t *)off, ntiles, pairs, flags);
        else if (planes && P == 12)
          hipLaunchKernelGGL((k_relabel_scatter<12, NT, true>), dim3((unsigned)ntiles), dim3(NT), lds, c.stream, rec,
                             nrec, pos, pos_size, (uint32_t)nb, (const uint32_t *)off, ntiles, pairs, flags);
        else if (planes)
          hipLaunchKernelGGL((k_relabel_scatter<8, NT, true>), dim3((unsigned)ntiles), dim3(NT), lds, c.stream, rec,
                             nrec, pos, pos_size, (uint32_t)nb, (const uint32_t *)off, ntiles, pairs, flags);
        else
          hipLaunchKernelGGL((k_relabel_scatter<8, NT>), dim3((unsigned)ntiles), dim3(NT), lds, c.stream, rec, nrec, pos,
                             pos_size, (uint32_t)nb, (const uint32_t *)off, ntiles, pairs, flags);
        LAUNCH_CHECK();
        HIP_CHECK(hipMemcpyAsync(c.h_scalars + 12, flags, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
        return;
      }
    }
    // one 1024-thread workgroup per CU: 8K-record sub-tiles (4K / 16K measured 15.8 / 15.3
    // ms against 14.3 at RMAT-26); 4K when the bucket cursors take more LDS
    const int per = fixed + 8 * HB * 8 <= 160 * 1024 ? 8 : 4;
    if (fixed + (size_t)per * HB * 8 > 160 * 1024) throw Error(SHEEP_ERR_ARG, "relabel: bucket layout exceeds LDS");
    const size_t lds = fixed + (size_t)per * HB * 8;
    const dim3 g((unsigned)ntiles), b(HB);
    const uint32_t nb32 = (uint32_t)nb;
    const uint32_t *o = off;
    if (per == 8)
      hipLaunchKernelGGL(k_relabel_scatter<8>, g, b, lds, c.stream, rec, nrec, pos, pos_size, nb32, o, ntiles, pairs, flags);
    else
      hipLaunchKernelGGL(k_relabel_scatter<4>, g, b, lds, c.stream, rec, nrec, pos, pos_size, nb32, o, ntiles, pairs, flags);
    LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(c.h_scalars + 12, flags, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  };
  // Pass B is launched right behind pass A on the layout's chunk list (pinned host memory,
  // built from the bucket starts), and ONE sync then checks pass A's flags: a stale layout
  // (the same record buffer refilled) is recounted and both passes run again; the first
  // run's writes stay in bounds (the gather checks every tail position against n) and its
  // pst / error counts are cleared.
  const uint64_t ntiles_e_max = (total + TKEYS - 1) >> TLOG;
  auto gather = [&]() -> bool {
    const uint64_t m = bst[nb];
    const uint64_t chunk = chunk_for(m);
    uint64_t nch = 0;
    for (uint32_t b = 0; b < nb; ++b) nch += (bst[b + 1] - bst[b] + chunk - 1) / chunk;
    // the grouping's count pass fused in when its bucket counters fit beside the pos slice
    const uint64_t ntiles_e = (m + TKEYS - 1) >> TLOG;
    const bool count = lg && m && lg->nb && ((size_t)W + lg->nb) * 4 <= 160 * 1024 &&
                       ntiles_e * lg->nb + 1 < (1ull << 32) && m < (1ull << 32);
    uint32_t *tile_hist = nullptr;
    if (count) {
      tile_hist = c.get_as<uint32_t>("hist_tiles", std::max(ntiles_e, ntiles_e_max) * lg->nb + 1);
      HIP_CHECK(hipMemsetAsync(tile_hist, 0, ntiles_e * lg->nb * sizeof(uint32_t), c.stream));
    }
    if (!nch) return count;
    Chunk *hch = (Chunk *)c.get_pinned("rl_chunks_host", nch * sizeof(Chunk));
    uint64_t j = 0;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint64_t beg = bst[b], end = bst[b + 1];
      for (uint64_t x = beg; x < end; x += chunk) hch[j++] = {x, x + chunk < end ? x + chunk : end, b, 0};
    }
    Chunk *dch = c.get_as<Chunk>("rl_chunks", nch);
    HIP_CHECK(hipMemcpyAsync(dch, hch, nch * sizeof(Chunk), hipMemcpyHostToDevice, c.stream));
    const EdgeLoPadded lk{edges, lg ? lg->d_pad : nullptr, lg ? lg->clo : 0, lg ? lg->mask : 0};
    if (count)
      hipLaunchKernelGGL(k_relabel_gather<true>, dim3((unsigned)nch), dim3(HB), (W + lg->nb) * 4, c.stream,
                         (const uint64_t *)pairs, (const Chunk *)dch, pos, pos_size, pst, edges, err, lk, lg->nb,
                         tile_hist, ntiles_e, n_tree);
    else
      hipLaunchKernelGGL(k_relabel_gather<false>, dim3((unsigned)nch), dim3(HB), W * 4, c.stream,
                         (const uint64_t *)pairs, (const Chunk *)dch, pos, pos_size, pst, edges, err, lk, 0u,
                         (uint32_t *)nullptr, (uint64_t)0, n_tree);
    LAUNCH_CHECK();
    return count;
  };
  scatter();
  bool count = gather();
  c.sync();
  if (c.h_scalars[13]) {   // offsets did not match these records: recount, run both passes again
    if (!cached) throw Error(SHEEP_ERR_HIP, "relabel: bucket layout inconsistent with its own count");
    HIP_CHECK(hipMemsetAsync(err, 0, sizeof(unsigned long long), c.stream));
    if (n_tree) HIP_CHECK(hipMemsetAsync(pst, 0, n_tree * sizeof(uint32_t), c.stream));
    off = recount();
    bst = hl.bstart;
    if (bst[nb] > total) pairs = c.get_as<uint64_t>("et_list1", bst[nb]);
    scatter();
    count = gather();
    c.sync();
    if (c.h_scalars[13]) throw Error(SHEEP_ERR_HIP, "relabel: bucket layout inconsistent with its own count");
  }
  const uint64_t m = bst[nb];
  if (c.h_scalars[12]) HIP_CHECK(hipMemsetAsync(err, 0xFF, 1, c.stream));   // range error (reported by the caller)
  if (counted) *counted = count;
  return m;
}

void histogram_edge_lo(Ctx &c, const uint64_t *edges, uint64_t m, uint64_t K, uint32_t *cnt) {
  histogram_add(c, EdgeLoKeys{edges}, m, K, cnt);
}

// pst[lo] += edges with that lo, and the edges grouped for the elimination tree: r0 holds
// them in padded-lo bucket order and seg[s] / seg[L + s] delimit the edges whose first
// active level is s ("first-activity buckets").
void lo_group_prepare(Ctx &c, uint64_t n, int L, uint32_t clo, LoGroup &g) {
  // lo range of level s: ya = spread(lo) in [2^L - 2^(s+1), 2^L - 2^s)
  auto first_lo = [&](uint64_t y) {
    uint64_t a = 0, b = n;
    while (a < b) {
      const uint64_t x = (a + b) / 2;
      if (x + ((x * (uint64_t)clo) >> 32) >= y) b = x; else a = x + 1;
    }
    return a;
  };
  g.L = L;
  g.clo = clo;
  g.mask = (uint32_t)((1ull << L) - 1);
  g.padoff.assign(32, 0);
  g.pstart.assign(L, 0);
  g.plen.assign(L, 0);
  uint64_t run = 0;
  for (int s = L - 1; s >= 0; --s) {   // ranges in increasing lo
    const uint64_t beg = first_lo((1ull << L) - (2ull << s)), end = first_lo((1ull << L) - (1ull << s));
    const uint64_t len = end > beg ? end - beg : 0;
    g.pstart[s] = run;
    g.plen[s] = (len + W - 1) / W * W;
    g.padoff[s] = (uint32_t)(run - beg);
    run += g.plen[s];
  }
  g.K = run ? run : W;
  if (g.K >= (1ull << 32)) throw Error(SHEEP_ERR_ARG, "group_edges_by_lo: key range too large");
  g.nb = (uint32_t)(g.K / W);
  g.kbase.assign(g.nb, 0);
  for (int s = 0; s < L; ++s)
    for (uint64_t b = g.pstart[s] / W; b < (g.pstart[s] + g.plen[s]) / W; ++b) g.kbase[b] = (uint32_t)(b * W - g.padoff[s]);
  g.d_pad = c.get_as<uint32_t>("grp_padoff", 32);
  g.d_kbase = c.get_as<uint32_t>("grp_kbase", g.nb);
  HIP_CHECK(hipMemcpyAsync(g.d_pad, g.padoff.data(), 32 * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
  HIP_CHECK(hipMemcpyAsync(g.d_kbase, g.kbase.data(), g.nb * sizeof(uint32_t), hipMemcpyHostToDevice, c.stream));
  c.sync();   // the layout's host vectors are the copies' sources
}

uint64_t group_edges_by_lo(Ctx &c, const uint64_t *edges, uint64_t m, const LoGroup &g, uint32_t *pst, uint64_t *r0,
                           uint64_t *seg, bool counted) {
  const int L = g.L;
  uint32_t *d_bstart = c.get_as<uint32_t>("grp_bstart", g.nb + 1);
  HIP_CHECK(hipMemsetAsync(d_bstart, 0, (g.nb + 1) * sizeof(uint32_t), c.stream));
  std::vector<uint32_t> bs;   // the bucket starts on the host (histogram_add has them after its sync)
  const uint64_t grouped = histogram_add(c, EdgeLoPadded{edges, g.d_pad, g.clo, g.mask}, m, g.K, pst, r0, g.d_kbase,
                                         d_bstart, nullptr, &bs, counted);
  // (pinned: no sync for the copy; histogram_add's sync above ordered any earlier use)
  uint64_t *hseg = (uint64_t *)c.get_pinned("grp_segb_host", 2 * (size_t)L * sizeof(uint64_t));
  for (int s = 0; s < L; ++s) { hseg[s] = g.pstart[s] / W; hseg[L + s] = (g.pstart[s] + g.plen[s]) / W; }
  // the same bounds for the host (the elimination tree's cut decisions read them: no copy back)
  c.seg_host.dev = nullptr;
  if (bs.size() == (size_t)g.nb + 1) {
    c.seg_host.v.resize(2 * (size_t)L);
    for (int i = 0; i < 2 * L; ++i) c.seg_host.v[i] = hseg[i] <= g.nb ? bs[hseg[i]] : 0;
    c.seg_host.dev = seg;
  }
  uint64_t *d_sb = c.get_as<uint64_t>("grp_segb", 2 * (size_t)L);
  HIP_CHECK(hipMemcpyAsync(d_sb, hseg, 2 * (size_t)L * sizeof(uint64_t), hipMemcpyHostToDevice, c.stream));
  hipLaunchKernelGGL(k_seg_from_buckets, dim3(1), dim3(64), 0, c.stream, (const uint32_t *)d_bstart,
                     (const uint64_t *)d_sb, L, seg);
  LAUNCH_CHECK();
  return grouped;
}

}  // namespace sheep
