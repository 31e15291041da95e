// scan.hip — device-wide exclusive prefix sums (reduce -> scan block sums -> apply).
// Tiles of 256 threads x 8 items staged through LDS; coalesced (striped) global
// loads/stores, blocked per-thread sums, wave shuffles for the block scan.
#include "common.hpp"

namespace sheep {
namespace {

constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;

template <typename T> __device__ __forceinline__ T block_exclusive_scan(T v, T *lds_wave, T &block_total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) lds_wave[wave] = inc;
  lds_barrier();
  T wave_off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / WAVE; ++w) {
    T s = lds_wave[w];
    if (w < wave) wave_off += s;
    tot += s;
  }
  block_total = tot;
  return wave_off + inc - v;
}

// n_dev (optional): the length is read on the device (at most n; the grid is sized for n).
// fold (one-level scans, gridDim <= SCAN_TILE): the block sums go out by atomic exchange
// and the LAST block to finish (a ticket, reset by that block) scans them in place, so
// the scan is two launches instead of three.  Sums and ticket are read-modify-write
// atomics, performed coherently however the blocks spread over the XCDs.
// The ticket's ordering below holds on gfx950 (and gfx942) because agent-scope RMW atomics
// complete at the coherence point; the HIP/LLVM memory model alone gives no such order.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "k_reduce's last-block ticket assumes gfx950/gfx942 RMW atomics complete at the coherence point"
#endif
template <typename T>
__global__ __launch_bounds__(BLOCK) void k_reduce(const T *__restrict__ in, uint64_t n, T *__restrict__ sums,
                                                  const uint64_t *__restrict__ n_dev, unsigned *__restrict__ ticket) {
  __shared__ T lds[BLOCK / WAVE];
  __shared__ bool s_last;
  if (n_dev && *n_dev < n) n = *n_dev;
  uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  T s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    if (i < n) s += in[i];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = s;
  lds_barrier();
  if (!ticket) {
    if (threadIdx.x == 0) {
      T t = 0;
      for (int w = 0; w < BLOCK / WAVE; ++w) t += lds[w];
      sums[blockIdx.x] = t;
    }
    return;
  }
  if (threadIdx.x == 0) {
    T t = 0;
    for (int w = 0; w < BLOCK / WAVE; ++w) t += lds[w];
    // The block sum, then the ticket: both read-modify-write atomics, performed at the
    // coherence point, and the ticket add is issued only after the sum's atomic has
    // RETURNED — `zero` is 0 computed from its result inside asm, so the compiler must wait
    // for the result and cannot fold the dependency away.  The last block reads the sums
    // with atomics too, after its own ticket add returned.  (A __threadfence() or a release
    // ticket add orders the same at agent scope but writes back the XCD's L2 in every
    // block: the etree's level scans took +4 ms per RMAT-26 step with it.)
    const T old = atomicExch(&sums[blockIdx.x], t);
    uint32_t zero;
    asm volatile("v_and_b32 %0, 0, %1" : "=v"(zero) : "v"((uint32_t)old));
    s_last = atomicAdd(ticket, 1u + zero) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) atomicExch(ticket, 0u);   // ready for the next scan
  // exclusive scan of the gridDim.x sums, SCAN_ITEMS per thread
  const uint32_t nb = gridDim.x, b0 = threadIdx.x * SCAN_ITEMS;
  T v[SCAN_ITEMS], tsum = 0;
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q) {
    v[q] = b0 + q < nb ? atomicAdd(&sums[b0 + q], T(0)) : T(0);
    tsum += v[q];
  }
  T total;
  T run = block_exclusive_scan(tsum, lds, total);
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q)
    if (b0 + q < nb) { sums[b0 + q] = run; run += v[q]; }
}

template <typename T>
__global__ __launch_bounds__(BLOCK) void k_apply(const T *__restrict__ in, T *__restrict__ out, uint64_t n,
                                                 const T *__restrict__ block_off, T *__restrict__ total,
                                                 const uint64_t *__restrict__ n_dev) {
  __shared__ T tile[SCAN_TILE];
  if (n_dev && *n_dev < n) n = *n_dev;   // blocks past it see zeros; the last still writes the total
  __shared__ T lds_wave[BLOCK / WAVE];
  uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    tile[j * BLOCK + threadIdx.x] = i < n ? in[i] : T(0);
  }
  lds_barrier();
  T local[SCAN_ITEMS];
  T s = 0;
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) { local[j] = tile[threadIdx.x * SCAN_ITEMS + j]; s += local[j]; }
  T block_total;
  T ex = block_exclusive_scan(s, lds_wave, block_total);
  T off = block_off ? block_off[blockIdx.x] : T(0);
  ex += off;
  lds_barrier();
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) { tile[threadIdx.x * SCAN_ITEMS + j] = ex; ex += local[j]; }
  lds_barrier();
#pragma unroll
  for (int j = 0; j < SCAN_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    if (i < n) out[i] = tile[j * BLOCK + threadIdx.x];
  }
  if (total && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *total = off + block_total;
}

template <typename T>
void scan_rec(Ctx &c, const T *in, T *out, uint64_t n, T *total_dev, int depth, const uint64_t *n_dev = nullptr) {
  if (n == 0) {
    if (total_dev) HIP_CHECK(hipMemsetAsync(total_dev, 0, sizeof(T), c.stream));
    return;
  }
  uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb > 0x7FFFFFFFull) throw Error(SHEEP_ERR_ARG, "scan too large");
  T *sums = nullptr;
  if (nb > 1) {
    sums = c.get_as<T>("scan_sums_" + std::to_string(depth) + (sizeof(T) == 8 ? "_64" : "_32"), nb);
    if (nb <= (uint64_t)SCAN_TILE) {   // one level: the last block scans the sums
      unsigned *ticket = (unsigned *)(c.d_scalars + Ctx::SCAN_TICKET);
      hipLaunchKernelGGL(k_reduce<T>, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, in, n, sums, n_dev, ticket);
      LAUNCH_CHECK();
    } else {
      hipLaunchKernelGGL(k_reduce<T>, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, in, n, sums, n_dev,
                         (unsigned *)nullptr);
      LAUNCH_CHECK();
      scan_rec<T>(c, sums, sums, nb, nullptr, depth + 1);
    }
  }
  hipLaunchKernelGGL(k_apply<T>, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, in, out, n,
                     (const T *)sums, total_dev, n_dev);
  LAUNCH_CHECK();
}

}  // namespace

void scan_exclusive_u32(Ctx &c, const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total_dev) {
  scan_rec<uint32_t>(c, in, out, n, total_dev, 0);
}
void scan_exclusive_u64(Ctx &c, const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total_dev) {
  scan_rec<uint64_t>(c, in, out, n, total_dev, 0);
}
void scan_exclusive_u64_dev(Ctx &c, const uint64_t *in, uint64_t *out, uint64_t n_max, const uint64_t *n_dev) {
  scan_rec<uint64_t>(c, in, out, n_max, nullptr, 0, n_dev);
}

}  // namespace sheep
