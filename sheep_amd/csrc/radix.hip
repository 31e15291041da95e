// radix.hip — stable LSD radix sort (digits of up to 9 bits) for the degree sequence
// (key = degree, value = vid), the kid table (key = parent, value = id) and the RMAT
// generator's dedup (64-bit keys).
//
// Per pass: (1) per-tile digit histogram, (2) exclusive scan of the digit-major
// histogram, (3) per-tile stable ranking with wave ballots (64-lane peer masks),
// LDS staging into tile-sorted order, then contiguous-run stores.
#include "common.hpp"

namespace sheep {
namespace {

constexpr int R_ITEMS = 16;
constexpr int R_TILE = BLOCK * R_ITEMS;   // 4096 keys per workgroup
// A sort of `bits` key bits takes ceil(bits / 9) passes of near-equal digits (25-bit kid
// keys: 9 + 8 + 8 instead of 8 + 8 + 8 + 1; each pass reads and writes every pair).
constexpr int MAX_DBITS = 9;

// 64-lane mask of the valid lanes whose digit equals mine.
template <int DB> __device__ __forceinline__ uint64_t digit_peers(bool valid, uint32_t d) {
  uint64_t peers = __ballot(valid);
#pragma unroll
  for (int b = 0; b < DB; ++b) {
    bool bit = (d >> b) & 1;
    uint64_t bb = __ballot(bit);
    peers &= bit ? bb : ~bb;
  }
  return peers;
}

template <typename K, int DB>
__global__ __launch_bounds__(BLOCK) void k_hist(const K *__restrict__ keys, uint64_t n, int shift,
                                                uint32_t ntiles, uint32_t *__restrict__ hist) {
  constexpr int RADIX = 1 << DB;
  __shared__ uint32_t h[RADIX];
  for (int d = threadIdx.x; d < RADIX; d += BLOCK) h[d] = 0;
  lds_barrier();
  uint64_t base = (uint64_t)blockIdx.x * R_TILE;
  for (int j = 0; j < R_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    bool valid = i < n;
    uint32_t d = valid ? (uint32_t)((keys[i] >> shift) & (RADIX - 1)) : 0;
    uint64_t peers = digit_peers<DB>(valid, d);
    if (valid && (peers & lanemask_lt()) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
  }
  lds_barrier();
  for (int d = threadIdx.x; d < RADIX; d += BLOCK) hist[(uint64_t)d * ntiles + blockIdx.x] = h[d];
}

// Per tile: every wave ranks a contiguous quarter of it (index order = wave, then item,
// then lane), counting its digits in its own LDS row as it goes — LDS operations of one
// wave execute in order, so an item sees the counts of the wave's earlier items without a
// barrier; one barrier then turns the rows into per-wave digit offsets.  (Ranking the tile
// item by item across the waves took three workgroup barriers per item.)
template <typename K, bool VALS, int DB>
__global__ __launch_bounds__(BLOCK) void k_scatter(const K *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                   K *__restrict__ kout, uint32_t *__restrict__ vout,
                                                   uint64_t n, int shift, uint32_t ntiles,
                                                   const uint32_t *__restrict__ offsets) {
  constexpr int RADIX = 1 << DB, DPT = RADIX > BLOCK ? RADIX / BLOCK : 1;   // digits per thread
  constexpr int NW = BLOCK / WAVE, WCH = WAVE * R_ITEMS;                    // waves, keys per wave
  __shared__ uint32_t run[RADIX];
  __shared__ uint32_t wcnt[NW][RADIX];   // a wave's digit counts, then its digit offsets in the tile
  __shared__ uint32_t dstart[RADIX];
  __shared__ uint32_t wtot[NW];
  __shared__ K skeys[R_TILE];
  __shared__ uint32_t svals[VALS ? R_TILE : 1];

  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int d = t; d < RADIX; d += BLOCK)
    for (int w = 0; w < NW; ++w) wcnt[w][d] = 0;
  lds_barrier();

  const uint64_t tbase = (uint64_t)blockIdx.x * R_TILE, base = tbase + (uint64_t)wave * WCH;
  K key[R_ITEMS];
  uint32_t val[R_ITEMS];
  uint32_t rank[R_ITEMS];
#pragma unroll
  for (int j = 0; j < R_ITEMS; ++j) {   // every load in flight before the ranking
    const uint64_t i = base + (uint64_t)j * WAVE + lane;
    key[j] = i < n ? kin[i] : K(0);
    if (VALS) val[j] = i < n ? vin[i] : 0u;
  }
  uint32_t *const mine = wcnt[wave];
  for (int j = 0; j < R_ITEMS; ++j) {
    const bool valid = base + (uint64_t)j * WAVE + lane < n;
    const uint32_t d = (uint32_t)((key[j] >> shift) & (RADIX - 1));
    const uint64_t peers = digit_peers<DB>(valid, d);
    const uint32_t lrank = (uint32_t)__popcll(peers & lanemask_lt());
    const uint32_t before = valid ? mine[d] : 0u;
    rank[j] = before + lrank;
    if (valid && lrank == 0) mine[d] = before + (uint32_t)__popcll(peers);
  }
  lds_barrier();
  for (int d = t; d < RADIX; d += BLOCK) {   // per digit: the waves' offsets (exclusive, wave order), total
    uint32_t s = 0;
    for (int w = 0; w < NW; ++w) {
      const uint32_t x = wcnt[w][d];
      wcnt[w][d] = s;
      s += x;
    }
    run[d] = s;
  }
  lds_barrier();
  // tile-local digit starts: exclusive scan of run[] (thread t owns digits t*DPT .. +DPT)
  uint32_t v = 0;
  if (t * DPT < RADIX)
    for (int q = 0; q < DPT; ++q) v += run[t * DPT + q];
  uint32_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) wtot[wave] = inc;
  lds_barrier();
  uint32_t woff = 0;
  for (int w = 0; w < wave; ++w) woff += wtot[w];
  if (t * DPT < RADIX) {
    uint32_t x = woff + inc - v;
    for (int q = 0; q < DPT; ++q) { dstart[t * DPT + q] = x; x += run[t * DPT + q]; }
  }
  lds_barrier();
  for (int j = 0; j < R_ITEMS; ++j) {
    if (base + (uint64_t)j * WAVE + lane < n) {
      const uint32_t d = (uint32_t)((key[j] >> shift) & (RADIX - 1));
      const uint32_t lp = dstart[d] + mine[d] + rank[j];
      skeys[lp] = key[j];
      if (VALS) svals[lp] = val[j];
    }
  }
  lds_barrier();
  uint32_t cnt = (uint32_t)((n - tbase) < (uint64_t)R_TILE ? (n - tbase) : (uint64_t)R_TILE);
  for (uint32_t idx = t; idx < cnt; idx += BLOCK) {
    K k = skeys[idx];
    uint32_t d = (uint32_t)((k >> shift) & (RADIX - 1));
    uint64_t g = (uint64_t)offsets[(uint64_t)d * ntiles + blockIdx.x] + (idx - dstart[d]);
    kout[g] = k;
    if (VALS) vout[g] = svals[idx];
  }
}

template <typename K, bool VALS, int DB>
void radix_pass(Ctx &c, const K *src, const uint32_t *vs, K *dst, uint32_t *vd, uint64_t n, int shift, uint32_t ntiles,
                uint32_t *hist) {
  hipLaunchKernelGGL((k_hist<K, DB>), dim3(ntiles), dim3(BLOCK), 0, c.stream, src, n, shift, ntiles, hist);
  LAUNCH_CHECK();
  scan_exclusive_u32(c, hist, hist, ((uint64_t)1 << DB) * ntiles, nullptr);
  hipLaunchKernelGGL((k_scatter<K, VALS, DB>), dim3(ntiles), dim3(BLOCK), 0, c.stream, src, vs, dst, vd, n, shift, ntiles,
                     (const uint32_t *)hist);
  LAUNCH_CHECK();
}

template <typename K, bool VALS>
void radix_sort_impl(Ctx &c, K *keys, uint32_t *vals, uint64_t n, int end_bit, K *kalt, uint32_t *valt, bool *in_alt) {
  if (in_alt) *in_alt = false;
  if (n <= 1 || end_bit <= 0) return;
  if (n >= 0xFFFFFFFFull) throw Error(SHEEP_ERR_ARG, "radix sort: n >= 2^32");
  uint32_t ntiles = (uint32_t)((n + R_TILE - 1) / R_TILE);
  uint32_t *hist = c.get_as<uint32_t>("radix_hist", ((uint64_t)1 << MAX_DBITS) * ntiles);
  K *src = keys, *dst = kalt;
  uint32_t *vs = vals, *vd = valt;
  const int passes = (end_bit + MAX_DBITS - 1) / MAX_DBITS;
  for (int p = 0, shift = 0; p < passes; ++p) {
    const int db = (end_bit - shift + (passes - p) - 1) / (passes - p);   // near-equal digits, widest first
    switch (db) {
#define SHEEP_RADIX_PASS(B) \
      case B: radix_pass<K, VALS, B>(c, src, vs, dst, vd, n, shift, ntiles, hist); break;
      SHEEP_RADIX_PASS(1) SHEEP_RADIX_PASS(2) SHEEP_RADIX_PASS(3) SHEEP_RADIX_PASS(4) SHEEP_RADIX_PASS(5)
      SHEEP_RADIX_PASS(6) SHEEP_RADIX_PASS(7) SHEEP_RADIX_PASS(8) SHEEP_RADIX_PASS(9)
#undef SHEEP_RADIX_PASS
      default: throw Error(SHEEP_ERR_ARG, "radix sort: bad digit width");
    }
    shift += db;
    std::swap(src, dst);
    std::swap(vs, vd);
  }
  if (src != keys && in_alt) {   // the caller reads the alternate buffers
    *in_alt = true;
  } else if (src != keys) {
    HIP_CHECK(hipMemcpyAsync(keys, src, n * sizeof(K), hipMemcpyDeviceToDevice, c.stream));
    if (VALS) HIP_CHECK(hipMemcpyAsync(vals, vs, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
  }
}

}  // namespace

void radix_sort_pairs_u32(Ctx &c, uint32_t *keys, uint32_t *vals, uint64_t n, int end_bit,
                          uint32_t *keys_alt, uint32_t *vals_alt, bool *in_alt) {
  radix_sort_impl<uint32_t, true>(c, keys, vals, n, end_bit, keys_alt, vals_alt, in_alt);
}
void radix_sort_keys_u64(Ctx &c, uint64_t *keys, uint64_t n, int end_bit, uint64_t *keys_alt, bool *in_alt) {
  radix_sort_impl<uint64_t, false>(c, keys, nullptr, n, end_bit, keys_alt, nullptr, in_alt);
}

}  // namespace sheep
