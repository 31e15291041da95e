// append.hip — packing of sharded appends (see common.hpp "sharded appends").
#include "common.hpp"

namespace sheep {
namespace {

constexpr int PACK_SLICES = 32;   // workgroups per shard

// Workgroup (k, slice) copies its slice of shard k to dst[prefix_k ...].
template <typename T>
__global__ __launch_bounds__(BLOCK) void k_pack(const T *__restrict__ src, T *__restrict__ dst, uint64_t ntiles,
                                                uint32_t per_item, const unsigned long long *__restrict__ counters) {
  __shared__ uint64_t s_prefix, s_count;
  const uint32_t k = blockIdx.x / PACK_SLICES, slice = blockIdx.x % PACK_SLICES;
  if (threadIdx.x < WAVE) {
    uint64_t c = threadIdx.x < (unsigned)k ? counters[(uint64_t)threadIdx.x * SHARD_STRIDE] : 0;
    c = wave_sum(c);
    if (threadIdx.x == 0) {
      s_prefix = c;
      s_count = counters[(uint64_t)k * SHARD_STRIDE];
    }
  }
  __syncthreads();
  const uint64_t cnt = s_count, per = (cnt + PACK_SLICES - 1) / PACK_SLICES;
  const uint64_t beg = (uint64_t)slice * per, end = beg + per < cnt ? beg + per : cnt;
  const T *s = src + shard_base(ntiles, k, per_item);
  T *d = dst + s_prefix;
  for (uint64_t i = beg + threadIdx.x; i < end; i += BLOCK) d[i] = s[i];
}

}  // namespace

unsigned long long *shard_counters(Ctx &c, const char *tag) {
  unsigned long long *p = c.get_as<unsigned long long>(std::string("shardcnt_") + tag, NSHARD * SHARD_STRIDE);
  HIP_CHECK(hipMemsetAsync(p, 0, NSHARD * SHARD_STRIDE * sizeof(uint64_t), c.stream));
  return p;
}

template <typename T>
uint64_t pack_shards(Ctx &c, const T *src, T *dst, uint64_t ntiles, uint32_t per_item,
                     const unsigned long long *counters) {
  std::vector<uint64_t> h(NSHARD * SHARD_STRIDE);
  HIP_CHECK(hipMemcpyAsync(h.data(), counters, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  hipLaunchKernelGGL(k_pack<T>, dim3(NSHARD * PACK_SLICES), dim3(BLOCK), 0, c.stream, src, dst, ntiles, per_item,
                     counters);
  LAUNCH_CHECK();
  c.sync();
  uint64_t total = 0;
  for (int k = 0; k < NSHARD; ++k) total += h[(uint64_t)k * SHARD_STRIDE];
  return total;
}

template uint64_t pack_shards<uint32_t>(Ctx &, const uint32_t *, uint32_t *, uint64_t, uint32_t,
                                        const unsigned long long *);
template uint64_t pack_shards<uint64_t>(Ctx &, const uint64_t *, uint64_t *, uint64_t, uint32_t,
                                        const unsigned long long *);

}  // namespace sheep
