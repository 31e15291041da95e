// append.hip — packing of sharded appends (see common.hpp "sharded appends").
//
// Counts stay on the device: the producer's input length is read from device memory
// (it fixes the shard regions), the packed total is written to device memory for the
// consumers, and nothing here waits for the GPU.  A level of the elimination-tree loop
// is a chain of such launches with no host round trip.
#include "common.hpp"

namespace sheep {
namespace {

constexpr int PACK_SLICES = 32;   // workgroups per shard

// Workgroup (k, slice) copies its slice of shard k to dst[prefix_k ...].
template <typename T>
__global__ __launch_bounds__(BLOCK) void k_pack(const T *__restrict__ src, T *__restrict__ dst,
                                                const uint64_t *__restrict__ n_in,
                                                const unsigned long long *__restrict__ counters,
                                                uint64_t *__restrict__ total_out, const uint64_t *__restrict__ cond,
                                                unsigned long long *__restrict__ zero_after,
                                                const uint64_t *__restrict__ dst_off) {
  if (cond && *cond == 0) return;
  __shared__ uint64_t s_prefix, s_count;
  const uint32_t k = blockIdx.x / PACK_SLICES, slice = blockIdx.x % PACK_SLICES;
  const uint64_t ntiles = (*n_in + TILE - 1) / TILE;
  if (threadIdx.x < WAVE) {
    uint64_t c = threadIdx.x < (unsigned)k ? counters[(uint64_t)threadIdx.x * SHARD_STRIDE] : 0;
    c = wave_sum(c);
    if (threadIdx.x == 0) {
      s_prefix = c;
      s_count = counters[(uint64_t)k * SHARD_STRIDE];
      if (k == NSHARD - 1 && slice == 0) *total_out = c + s_count;
    }
  }
  if (zero_after && blockIdx.x == 0 && threadIdx.x < NSHARD) zero_after[(uint64_t)threadIdx.x * SHARD_STRIDE] = 0;
  lds_barrier();
  const uint64_t cnt = s_count, per = (cnt + PACK_SLICES - 1) / PACK_SLICES;
  const uint64_t beg = (uint64_t)slice * per, end = beg + per < cnt ? beg + per : cnt;
  const T *s = src + shard_base(ntiles, k, 1);
  T *d = dst + (dst_off ? *dst_off : 0) + s_prefix;
  for (uint64_t i = beg + threadIdx.x; i < end; i += BLOCK) d[i] = s[i];
}

}  // namespace

unsigned long long *shard_counters(Ctx &c, const char *tag) {
  unsigned long long *p = c.get_as<unsigned long long>(std::string("shardcnt_") + tag, NSHARD * SHARD_STRIDE);
  HIP_CHECK(hipMemsetAsync(p, 0, NSHARD * SHARD_STRIDE * sizeof(uint64_t), c.stream));
  return p;
}

template <typename T>
void pack_shards(Ctx &c, const T *src, T *dst, const uint64_t *n_in, const unsigned long long *counters,
                 uint64_t *total_out, const uint64_t *cond, unsigned long long *zero_after, const uint64_t *dst_off) {
  hipLaunchKernelGGL(k_pack<T>, dim3(NSHARD * PACK_SLICES), dim3(BLOCK), 0, c.stream, src, dst, n_in, counters,
                     total_out, cond, zero_after, dst_off);
  LAUNCH_CHECK();
}

template void pack_shards<uint32_t>(Ctx &, const uint32_t *, uint32_t *, const uint64_t *,
                                    const unsigned long long *, uint64_t *, const uint64_t *, unsigned long long *,
                                    const uint64_t *);
template void pack_shards<uint64_t>(Ctx &, const uint64_t *, uint64_t *, const uint64_t *,
                                    const unsigned long long *, uint64_t *, const uint64_t *, unsigned long long *,
                                    const uint64_t *);

}  // namespace sheep
