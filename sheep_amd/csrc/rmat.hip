// rmat.hip — synthetic .dat records in HBM (bench/test input; not the measured path).
#include <algorithm>
#include <vector>

#include "common.hpp"
#include "rmat.hpp"

namespace sheep {
namespace {

// self-loops get the all-ones key of the 2*scale-bit key space (a self-loop pair, so
// never a real key) and sort last
__host__ __device__ inline uint64_t dead_key(int scale) { return (1ull << (2 * scale)) - 1; }

__global__ __launch_bounds__(BLOCK) void k_rmat_keys(RmatParams p, uint64_t M, uint64_t *__restrict__ keys) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < M; i += stride) {
    uint32_t u, v;
    rmat_edge(i, p, u, v);
    keys[i] = u == v ? dead_key(p.scale) : rmat_key(u, v, p.scale);
  }
}

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

uint64_t rmat_generate(Ctx &c, int scale, int ef, uint64_t seed, sheep_xs1 *out, uint64_t cap) {
  if (scale < 1 || scale > 30 || ef < 1) throw Error(SHEEP_ERR_ARG, "rmat: bad scale/edgefactor");
  const uint64_t M = (uint64_t)ef << scale;
  if (cap < M) throw Error(SHEEP_ERR_ARG, "rmat: output capacity < ef << scale");
  RmatParams p = rmat_params(scale, seed);
  uint64_t *keys = c.get_as<uint64_t>("rmat_keys", M);
  uint64_t *alt = c.get_as<uint64_t>("rmat_alt", M);
  hipLaunchKernelGGL(k_rmat_keys, dim3(grid_for(M)), dim3(BLOCK), 0, c.stream, p, M, keys);
  LAUNCH_CHECK();
  radix_sort_keys_u64(c, keys, M, 2 * scale, alt);
  uint64_t nb = (M + U_TILE - 1) / U_TILE;
  uint32_t *bcnt = c.get_as<uint32_t>("rmat_bcnt", nb);
  hipLaunchKernelGGL(k_unique_count, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, (const uint64_t *)keys, M, dead_key(scale), bcnt);
  LAUNCH_CHECK();
  uint32_t *total = (uint32_t *)(c.d_scalars + 12);
  HIP_CHECK(hipMemsetAsync(c.d_scalars + 12, 0, sizeof(uint64_t), c.stream));
  scan_exclusive_u32(c, bcnt, bcnt, nb, total);
  hipLaunchKernelGGL(k_unique_write, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, (const uint64_t *)keys, M, scale,
                     (const uint32_t *)bcnt, out);
  LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 12, c.d_scalars + 12, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  // free the generator's scratch: it is large and only needed once
  for (const char *nm : {"rmat_keys", "rmat_alt"}) {
    auto it = c.ws.find(nm);
    if (it != c.ws.end()) { HIP_CHECK(hipFree(it->second.p)); c.ws.erase(it); }
  }
  return (uint32_t)c.h_scalars[12];
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
