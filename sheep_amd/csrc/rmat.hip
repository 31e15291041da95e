// rmat.hip — synthetic .dat records in HBM (bench/test input; not the measured path).
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"
#include "rmat.hpp"

namespace sheep {
namespace {

// self-loops get the all-ones key of the 2*scale-bit key space (a self-loop pair, so
// never a real key) and sort last
__host__ __device__ inline uint64_t dead_key(int scale) { return (1ull << (2 * scale)) - 1; }

// The keys of edges [0, M) whose tail (the larger endpoint) lies in [t0, t1), appended in
// tile order (one atomic per workgroup tile); self-loops only with t0 == 0.  A graph with
// 2^32 or more edge draws (RMAT-28) is generated one tail range at a time, each range
// sorted and deduplicated on its own (every key of a range sorts before the next range's).
template <typename Gen>
__global__ __launch_bounds__(BLOCK) void k_gen_keys(Gen g, uint64_t M, uint64_t t0, uint64_t t1,
                                                    uint64_t *__restrict__ keys, unsigned long long *__restrict__ count) {
  const uint64_t ntiles = (M + TILE - 1) / TILE;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint64_t k[TILE_ITEMS];
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < TILE_ITEMS; ++j) {
      const uint64_t i = tile * TILE + (uint64_t)j * BLOCK + threadIdx.x;
      if (i >= M) continue;
      uint32_t u, v;
      g.edge(i, u, v);
      const uint64_t t = u > v ? u : v;
      k[j] = u == v ? dead_key(g.bits()) : rmat_key(u, v, g.bits());
      if (u == v ? t0 == 0 : (t >= t0 && t < t1)) keep |= 1u << j;
    }
    uint64_t slot = block_reserve((uint32_t)__popc(keep), count);
#pragma unroll
    for (int j = 0; j < TILE_ITEMS; ++j)
      if (keep & (1u << j)) keys[slot++] = k[j];
  }
}

struct RmatGen {
  RmatParams p;
  __device__ void edge(uint64_t i, uint32_t &u, uint32_t &v) const { rmat_edge(i, p, u, v); }
  __device__ int bits() const { return p.scale; }
};

// Chung-Lu power law over V vertices: each edge draws both endpoints independently with
// probability ~ (x + x0)^-alpha, alpha = 1 / (gamma - 1) (expected degree ~ rank^-alpha,
// a degree exponent gamma), by the inverse of the continuous CDF; labels permuted by the
// same Feistel bijection (cycle-walked into [0, V)).
struct PowerGen {
  RmatParams p;      // seed, Feistel keys; p.scale = key bits (ceil log2 V)
  uint64_t V;
  double x0, e1, a0, span;   // e1 = 1 - alpha; a0 = x0^e1; span = a0 - (V + x0)^e1
  __device__ uint32_t draw(uint64_t r) const {
    const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
    double x = pow(a0 - u * span, 1.0 / e1) - x0;
    uint64_t i = x < 0 ? 0 : (uint64_t)x;
    if (i >= V) i = V - 1;
    uint32_t y = (uint32_t)i;
    do { y = rmat_permute(y, p); } while ((uint64_t)y >= V);
    return y;
  }
  __device__ void edge(uint64_t i, uint32_t &u, uint32_t &v) const {
    u = draw(mix64(p.seed ^ (2 * i) * 0xD1B54A32D192ED03ull));
    v = draw(mix64(p.seed ^ (2 * i + 1) * 0xD1B54A32D192ED03ull));
  }
  __device__ int bits() const { return p.scale; }
};

constexpr int U_ITEMS = 8;
constexpr int U_TILE = BLOCK * U_ITEMS;

__device__ __forceinline__ bool is_first(const uint64_t *keys, uint64_t i, uint64_t dead) {
  uint64_t k = keys[i];
  return k != dead && (i == 0 || keys[i - 1] != k);
}

__global__ __launch_bounds__(BLOCK) void k_unique_count(const uint64_t *__restrict__ keys, uint64_t M, uint64_t dead,
                                                        uint32_t *__restrict__ bcnt) {
  __shared__ uint32_t s[BLOCK / WAVE];
  uint64_t base = (uint64_t)blockIdx.x * U_TILE;
  uint32_t c = 0;
  for (int j = 0; j < U_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    if (i < M && is_first(keys, i, dead)) ++c;
  }
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(BLOCK) void k_unique_write(const uint64_t *__restrict__ keys, uint64_t M, int scale,
                                                        const uint32_t *__restrict__ boff, sheep_xs1 *__restrict__ out) {
  __shared__ uint32_t wc[BLOCK / WAVE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t base = (uint64_t)blockIdx.x * U_TILE;
  uint64_t running = boff[blockIdx.x];
  const uint64_t hmask = (1ull << scale) - 1;
  for (int j = 0; j < U_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    bool f = i < M && is_first(keys, i, dead_key(scale));
    uint64_t m = __ballot(f);
    if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint64_t off = running;
    for (int w = 0; w < wave; ++w) off += wc[w];
    if (f) {
      uint64_t k = keys[i];
      sheep_xs1 r;
      r.tail = (uint32_t)(k >> scale);
      r.head = (uint32_t)(k & hmask);
      r.weight = 1.0f;
      out[off + __popcll(m & lanemask_lt())] = r;
    }
    running += wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();
  }
}

}  // namespace

// Edge draws -> keys (tail << bits | head) per tail range -> sort -> unique -> records.
template <typename Gen>
static uint64_t generate(Ctx &c, const Gen &g, int bits, uint64_t nverts, uint64_t M, sheep_xs1 *out, uint64_t cap) {
  if (cap < M) throw Error(SHEEP_ERR_ARG, "generator: output capacity < edge draws");
  // tail ranges small enough for one sort (< 2^31 keys each; RMAT tails skew high: the
  // ranges split the upper half finer)
  std::vector<uint64_t> cuts = {0, nverts};
  if (M >= (1ull << 31)) {
    const uint64_t h = nverts / 2, q = nverts / 4;
    cuts = {0, h, h + q / 2, h + q, h + q + q / 2, nverts};
  }
  const uint64_t kcap = M < (1ull << 31) ? M : (M * 9) / 20;   // largest range: < 0.45 M draws
  uint64_t *keys = c.get_as<uint64_t>("rmat_keys", kcap);
  uint64_t *alt = c.get_as<uint64_t>("rmat_alt", kcap);
  unsigned long long *cnt = (unsigned long long *)(c.d_scalars + 13);
  uint64_t written = 0;
  for (size_t r = 0; r + 1 < cuts.size(); ++r) {
    HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(uint64_t), c.stream));
    hipLaunchKernelGGL(k_gen_keys<Gen>, dim3(grid_tiles(M)), dim3(BLOCK), 0, c.stream, g, M, cuts[r], cuts[r + 1], keys,
                       cnt);
    LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(c.h_scalars + 13, cnt, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    const uint64_t nk = c.h_scalars[13];
    if (nk > kcap) throw Error(SHEEP_ERR_HIP, "generator: a tail range overflowed its key buffer");
    if (nk == 0) continue;
    radix_sort_keys_u64(c, keys, nk, 2 * bits, alt);
    const uint64_t nb = (nk + U_TILE - 1) / U_TILE;
    uint32_t *bcnt = c.get_as<uint32_t>("rmat_bcnt", nb);
    hipLaunchKernelGGL(k_unique_count, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, (const uint64_t *)keys, nk,
                       dead_key(bits), bcnt);
    LAUNCH_CHECK();
    uint32_t *total = (uint32_t *)(c.d_scalars + 12);
    HIP_CHECK(hipMemsetAsync(c.d_scalars + 12, 0, sizeof(uint64_t), c.stream));
    scan_exclusive_u32(c, bcnt, bcnt, nb, total);
    hipLaunchKernelGGL(k_unique_write, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, (const uint64_t *)keys, nk, bits,
                       (const uint32_t *)bcnt, out + written);
    LAUNCH_CHECK();
    HIP_CHECK(hipMemcpyAsync(c.h_scalars + 12, c.d_scalars + 12, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    written += (uint32_t)c.h_scalars[12];
  }
  // free the generator's scratch: it is large and only needed once
  for (const char *nm : {"rmat_keys", "rmat_alt"}) {
    auto it = c.ws.find(nm);
    if (it != c.ws.end()) { HIP_CHECK(hipFree(it->second.p)); c.ws.erase(it); }
  }
  return written;
}

uint64_t rmat_generate(Ctx &c, int scale, int ef, uint64_t seed, sheep_xs1 *out, uint64_t cap) {
  if (scale < 1 || scale > 30 || ef < 1) throw Error(SHEEP_ERR_ARG, "rmat: bad scale/edgefactor");
  const uint64_t M = (uint64_t)ef << scale;
  if (cap < M) throw Error(SHEEP_ERR_ARG, "rmat: output capacity < ef << scale");
  return generate(c, RmatGen{rmat_params(scale, seed)}, scale, 1ull << scale, M, out, cap);
}

uint64_t powerlaw_generate(Ctx &c, uint64_t V, uint64_t M, double gamma, uint64_t seed, sheep_xs1 *out, uint64_t cap) {
  if (V < 2 || V > (1ull << 30) || M < 1 || !(gamma > 1.0)) throw Error(SHEEP_ERR_ARG, "powerlaw: bad arguments");
  int bits = 1;
  while ((1ull << bits) < V) ++bits;
  PowerGen g;
  g.p = rmat_params(bits, seed);
  g.V = V;
  const double alpha = 1.0 / (gamma - 1.0);
  g.e1 = 1.0 - alpha;
  // x0 sets the largest expected degree: the top vertex takes 0.1% of the 2M endpoint
  // draws (~3M adjacency entries at twitter scale, the order of twitter-2010's largest
  // hub), solved by bisection on the continuous CDF
  auto cdf1 = [&](double x0) {   // probability mass of [0, 1) under (x + x0)^-alpha on [0, V)
    const double a = std::pow(x0, g.e1), b = std::pow(x0 + 1.0, g.e1), z = std::pow((double)V + x0, g.e1);
    return (a - b) / (a - z);
  };
  double lo = 1e-3, hi = 1e9;
  for (int it = 0; it < 200; ++it) {
    const double mid = std::sqrt(lo * hi);
    if (cdf1(mid) > 0.001) lo = mid; else hi = mid;
  }
  g.x0 = lo;
  g.a0 = std::pow(g.x0, g.e1);
  g.span = g.a0 - std::pow((double)V + g.x0, g.e1);
  return generate(c, g, bits, V, M, out, cap);
}

uint64_t rmat_generate_host(int scale, int ef, uint64_t seed, sheep_xs1 *out, uint64_t cap) {
  if (scale < 1 || scale > 30 || ef < 1) throw Error(SHEEP_ERR_ARG, "rmat: bad scale/edgefactor");
  const uint64_t M = (uint64_t)ef << scale;
  if (cap < M) throw Error(SHEEP_ERR_ARG, "rmat: output capacity < ef << scale");
  RmatParams p = rmat_params(scale, seed);
  std::vector<uint64_t> keys(M);
  for (uint64_t i = 0; i < M; ++i) {
    uint32_t u, v;
    rmat_edge(i, p, u, v);
    keys[i] = u == v ? dead_key(scale) : rmat_key(u, v, scale);
  }
  std::sort(keys.begin(), keys.end());
  uint64_t n = 0;
  const uint64_t hmask = (1ull << scale) - 1;
  for (uint64_t i = 0; i < M; ++i) {
    if (keys[i] == dead_key(scale) || (i && keys[i - 1] == keys[i])) continue;
    out[n].tail = (uint32_t)(keys[i] >> scale);
    out[n].head = (uint32_t)(keys[i] & hmask);
    out[n].weight = 1.0f;
    ++n;
  }
  return n;
}

}  // namespace sheep
