// common.hpp — shared host/device plumbing for libsheep_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "sheep_hip.h"

namespace sheep {

constexpr uint32_t INVALID = 0xFFFFFFFFu;
constexpr int WAVE = 64;     // CDNA wavefront
constexpr int BLOCK = 256;   // 4 waves per workgroup

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw ::sheep::Error(_e == hipErrorOutOfMemory ? SHEEP_ERR_ALLOC : SHEEP_ERR_HIP,   \
                           std::string(#expr) + ": " + hipGetErrorString(_e));            \
  } while (0)

// SHEEP_DEBUG=launches (debugging): every launch is followed by a device-wide wait and a
// stderr line naming its source line, so a kernel that never finishes names itself.
bool trace_launches();
void trace_launch(const char *file, int line);
#define LAUNCH_CHECK()                                                   \
  do {                                                                   \
    HIP_CHECK(hipGetLastError());                                        \
    if (::sheep::trace_launches()) ::sheep::trace_launch(__FILE__, __LINE__); \
  } while (0)

// Grid for a grid-stride streaming kernel: enough workgroups to fill 256 CUs x 8.
inline unsigned grid_for(uint64_t items, unsigned per_block = BLOCK, unsigned cap = 256 * 8) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g == 0) g = 1;
  return (unsigned)(g < cap ? g : cap);
}

// Raises a kernel's dynamic-LDS limit to the gfx950 CU's 160 KiB, once per (kernel,
// device): the attribute belongs to the device that is current when it is set.
// allow_lds: the same for a kernel that also has static LDS (the limit is then the dynamic
// part it launches with: static + dynamic <= 160 KiB).
// The size granted so far is kept per (kernel, device): a later, larger request raises it.
inline void allow_lds(const void *kernel, int bytes) {
  static std::mutex m;
  static std::map<std::pair<const void *, int>, int> granted;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(m);
  int &have = granted[{kernel, dev}];
  if (bytes > have) {
    HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    have = bytes;
  }
}
inline void allow_full_lds(const void *kernel) { allow_lds(kernel, 160 * 1024); }

// The one debug variable the library reads: SHEEP_DEBUG=flag[,flag...] with flags
// "launches" (sync + time every launch), "etree" (level / block statistics to stderr),
// "part" (partition event timings to stderr).
inline bool debug_on(const char *flag) {
  static const std::string v = getenv("SHEEP_DEBUG") ? std::string(",") + getenv("SHEEP_DEBUG") + "," : "";
  return !v.empty() && v.find(std::string(",") + flag + ",") != std::string::npos;
}

// The algorithm variants' defaults (include/sheep_hip.h sheep_tuning; measured).
inline sheep_tuning default_tuning() {
  sheep_tuning t;
  t.fin_map_bits = 13;     // RMAT-26 etree 31.0 / 30.5 / 30.0 ms at 11 / 12 / 13 bits
  t.fin_merge_bits = 12;   // 8-tree merge 15.4 -> 14.1 ms at 12 bits
  t.fin_dc = 1;
  t.top_bits = 16;         // RMAT-26 etree: 2^15 32.59, 2^16 32.15 ms
  t.top_blocks = 4;        // no cut 34.5; 1 block 34.1; 4 blocks 33.8; 8 blocks 33.8
  t.big_bits = 21;         // RMAT-26 etree: 2^20 27.7, 2^21 26.9 ms; 2^22 leaves 15 K trees
  t.big_dense = 256;       // a 1/8 edge shard's ~90 group edges per vertex did not pay
  t.big_hot_bits = 15;
  t.big_hot16 = 0;
  t.relabel_planes = 1;
  t.relabel_per = 8;
  t.cross_win_levels = 2;   // RMAT-26: level 0/1 1.30/2.46 -> 0.77/1.16 ms; level 2 1.60 -> 1.74 ms
  t.hook_batch = 0;        // merges 14.0 -> 18.0 ms, maps no better (RMAT-26, 8 shards)
  t.hook_up = 0;
  t.merge_cut_bits = 0;
  t.event_loop = 4096;
  return t;
}

// Per-context state: device, stream, grow-only named workspaces, pinned scalars, timers.
struct Ctx {
  int device = 0;
  sheep_tuning tune = default_tuning();
  hipStream_t stream = nullptr;
  bool own_stream = false;

  struct Buf { void *p = nullptr; size_t bytes = 0; };
  std::map<std::string, Buf> ws;
  std::map<std::string, Buf> pinned;   // host memory the kernels write directly (mapped)

  uint64_t *h_scalars = nullptr;   // pinned host mirror
  uint64_t *d_scalars = nullptr;   // device scalars (counters / flags)
  static constexpr int NSCALARS = 72;
  static constexpr int SCAN_TICKET = 64;   // d_scalars word of the scans' last-block ticket (zero between scans)

  // Bucket layouts of the last degree_count head histograms (LLAMA mode), one per record
  // buffer (up to NLAYOUT, round robin: the shards of one rank's step each keep theirs):
  // the scanned (bucket, tile) offsets live in ws[layout_buf(slot)]; relabel_bucketed
  // reuses them when it sees the same records (and verifies every region's count in-kernel).
  struct HeadLayout { const void *rec = nullptr; uint64_t nrec = 0, K = 0; std::vector<uint32_t> bstart; bool valid = false; int slot = 0; };
  static constexpr int NLAYOUT = 8;
  HeadLayout layouts[NLAYOUT];
  int layout_next = 0;
  static std::string layout_buf(int slot) { return slot ? "head_offsets" + std::to_string(slot) : "head_offsets"; }
  HeadLayout *find_layout(const void *rec, uint64_t nrec) {
    for (auto &l : layouts)
      if (l.valid && l.rec == rec && l.nrec == nrec) return &l;
    return nullptr;
  }
  // the slot for this record buffer: its own, else the next one round robin (invalidated)
  HeadLayout &layout_for(const void *rec, uint64_t nrec) {
    for (int i = 0; i < NLAYOUT; ++i)
      if (layouts[i].rec == rec && layouts[i].nrec == nrec) {
        layouts[i].valid = false;
        layouts[i].bstart.clear();
        layouts[i].slot = i;
        return layouts[i];
      }
    const int i = layout_next;
    layout_next = (layout_next + 1) % NLAYOUT;
    layouts[i] = HeadLayout();
    layouts[i].slot = i;
    return layouts[i];
  }
  // the degree pass's sortedness probe of the last record buffer (sequence.hip)
  struct SortedProbe { const void *rec = nullptr; uint64_t nrec = 0; bool sorted = true; };
  SortedProbe sorted_probe;
  // The last destroyed kid table's buffers, taken by the next sheep_kids_create: a
  // partition per tree would otherwise pay three hipMalloc / hipFree pairs of n words
  // (hipFree waits for the device), ~1 ms of idle GPU per step at RMAT-26.
  struct KidBufs { uint32_t *parent = nullptr, *koff = nullptr, *kids = nullptr, *kpar = nullptr; uint64_t cap = 0; };
  KidBufs kid_spare;
  // The last map's position-space edges, grouped by lo in the workspace bt_grouped
  // (sheep_evaluate_step reads them): m_pairs edges came out of the relabel (DEAD ones
  // included), m_valid of them are grouped.  Valid until the next map or sheep_ctx_trim.
  struct StepEdges {
    const void *rec = nullptr;
    const uint32_t *pos = nullptr;
    const uint64_t *edges = nullptr;
    const uint32_t *pst = nullptr;   // per jnid: edges with that lo (bt_pst; DEAD edges add to it too)
    uint64_t nrec = 0, pos_size = 0, n = 0, m_pairs = 0, m_valid = 0;
    bool valid = false;
  };
  StepEdges step_edges;
  // The first-activity group bounds the last grouping wrote to `dev`, on the host (taken,
  // once, by the elimination tree that reads them next)
  struct SegHost { const uint64_t *dev = nullptr; std::vector<uint64_t> v; };
  SegHost seg_host;

  bool timing = false;
  struct Timer { std::vector<std::pair<hipEvent_t, hipEvent_t>> pending; double ms = 0; uint64_t launches = 0; uint64_t bytes = 0; };
  std::map<std::string, Timer> timers;
  std::vector<hipEvent_t> event_pool;
  // Byte counts that need device-side results (the etree's per-level list sizes): the
  // results are copied into a pinned buffer on the stream and counted when the timers are
  // collected, so a timed run pays no host round trip for them.
  struct Deferred { void *host; size_t bytes; std::function<void(const void *)> count; };
  std::vector<Deferred> deferred;
  std::vector<std::pair<void *, size_t>> deferred_pool;
  void defer_bytes(const void *dev, size_t bytes, std::function<void(const void *)> count) {
    void *h = nullptr;
    for (size_t i = 0; i < deferred_pool.size(); ++i)
      if (deferred_pool[i].second >= bytes) {
        h = deferred_pool[i].first;
        bytes = deferred_pool[i].second;
        deferred_pool.erase(deferred_pool.begin() + (long)i);
        break;
      }
    if (!h) {
      if (deferred.size() >= 256) collect_timers();   // (bounded: a long timed run without reads)
      for (size_t i = 0; !h && i < deferred_pool.size(); ++i)
        if (deferred_pool[i].second >= bytes) {
          h = deferred_pool[i].first;
          bytes = deferred_pool[i].second;
          deferred_pool.erase(deferred_pool.begin() + (long)i);
        }
      if (!h) HIP_CHECK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    }
    HIP_CHECK(hipMemcpyAsync(h, dev, bytes, hipMemcpyDeviceToHost, stream));
    deferred.push_back({h, bytes, std::move(count)});
  }

  void *get(const std::string &name, size_t bytes) {
    Buf &b = ws[name];
    if (b.bytes < bytes) {
      if (b.p) HIP_CHECK(hipFree(b.p));
      b.p = nullptr;
      size_t want = bytes + bytes / 8 + 256;
      HIP_CHECK(hipMalloc(&b.p, want));
      b.bytes = want;
    }
    return b.p;
  }
  template <typename T> T *get_as(const std::string &name, size_t count) {
    return (T *)get(name, count * sizeof(T));
  }
  // Host buffer a kernel can store into: results small enough to stage arrive with the
  // one stream sync that has to happen anyway, instead of a copy per array.
  void *get_pinned(const std::string &name, size_t bytes) {
    Buf &b = pinned[name];
    if (b.bytes < bytes) {
      if (b.p) HIP_CHECK(hipHostFree(b.p));
      b.p = nullptr;
      HIP_CHECK(hipHostMalloc(&b.p, bytes, hipHostMallocMapped));
      b.bytes = bytes;
    }
    return b.p;
  }
  // Pinned staging for copies of pageable host vectors: a copy from or to pageable memory
  // is synchronous (each one a host round trip, 30-50 us of idle GPU); staged, it is queued
  // like any other copy.  Downloads land in their vectors at the next sync().
  struct Stage { char *p = nullptr; size_t cap = 0, used = 0; };
  Stage stage;
  std::vector<char *> stage_old;
  std::vector<std::function<void()>> after_sync;
  void *stage_alloc(size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    if (stage.used + bytes > stage.cap) {
      if (stage.p) stage_old.push_back(stage.p);   // still read by queued copies: freed at sync()
      const size_t cap = std::max(bytes, std::max(2 * stage.cap, (size_t)1 << 20));
      HIP_CHECK(hipHostMalloc((void **)&stage.p, cap, hipHostMallocDefault));
      stage.cap = cap;
      stage.used = 0;
    }
    void *r = stage.p + stage.used;
    stage.used += bytes;
    return r;
  }
  template <typename T> void download(T *h, const T *d, uint64_t cnt) {
    if (!cnt) return;
    T *s = (T *)stage_alloc(cnt * sizeof(T));
    HIP_CHECK(hipMemcpyAsync(s, d, cnt * sizeof(T), hipMemcpyDeviceToHost, stream));
    after_sync.push_back([h, s, cnt]() { memcpy(h, s, cnt * sizeof(T)); });
  }
  template <typename T> void upload(T *d, const T *h, uint64_t cnt) {
    if (!cnt) return;
    T *s = (T *)stage_alloc(cnt * sizeof(T));
    memcpy(s, h, cnt * sizeof(T));
    HIP_CHECK(hipMemcpyAsync(d, s, cnt * sizeof(T), hipMemcpyHostToDevice, stream));
  }
  void sync() {
    const hipError_t e = hipStreamSynchronize(stream);
    if (e != hipSuccess) after_sync.clear();   // (the vectors they fill may not outlive the error)
    HIP_CHECK(e);
    for (auto &f : after_sync) f();
    after_sync.clear();
    stage.used = 0;
    for (char *p : stage_old) HIP_CHECK(hipHostFree(p));
    stage_old.clear();
  }
  // algorithmic bytes learned only after the launches (device-side counts)
  void add_bytes(const char *name, uint64_t bytes) { if (timing) timers[name].bytes += bytes; }

  // Timing events only (TimedRegion): without the system-scope fence a record is a bare
  // timestamp — a default event's record writes back and invalidates the caches, which
  // showed as a ~10 us idle gap at every region boundary and cold caches after it.
  hipEvent_t ev() {
    if (!event_pool.empty()) { hipEvent_t e = event_pool.back(); event_pool.pop_back(); return e; }
    hipEvent_t e; HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence)); return e;
  }
  void collect_timers() {
    if (!deferred.empty()) {
      sync();
      for (auto &d : deferred) {
        d.count(d.host);
        deferred_pool.push_back({d.host, d.bytes});
      }
      deferred.clear();
    }
    for (auto &kv : timers) {
      for (auto &p : kv.second.pending) {
        float ms = 0;
        HIP_CHECK(hipEventSynchronize(p.second));
        HIP_CHECK(hipEventElapsedTime(&ms, p.first, p.second));
        kv.second.ms += ms;
        kv.second.launches++;
        event_pool.push_back(p.first);
        event_pool.push_back(p.second);
      }
      kv.second.pending.clear();
    }
  }
};

}  // namespace sheep

// The C ABI's opaque context handle (include/sheep_hip.h).
struct sheep_ctx {
  sheep::Ctx c;
};

namespace sheep {

// Brackets one instrumented launch with HIP events on the context stream.  `bytes` is
// the launch's ALGORITHMIC traffic, summed per timer name.
struct TimedRegion {
  Ctx &c; const char *name; hipEvent_t a = nullptr, b = nullptr;
  TimedRegion(Ctx &ctx, const char *n, uint64_t bytes = 0) : c(ctx), name(n) {
    if (c.timing) {
      c.timers[name].bytes += bytes;
      a = c.ev(); b = c.ev(); HIP_CHECK(hipEventRecord(a, c.stream));
    }
  }
  ~TimedRegion() {
    if (c.timing) {
      if (hipEventRecord(b, c.stream) == hipSuccess) c.timers[name].pending.push_back({a, b});
    }
  }
};

// ---------------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------------
__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup release/acquire
// over all of memory, so it first waits for every global load and store the wave has in
// flight (vmcnt(0)): a streaming kernel's prefetches and write-backs drain at each of its
// barriers.  For kernels whose threads exchange data through LDS only (the bucket sorts,
// scans, the level splits); a kernel that reads global memory another thread of its
// workgroup wrote keeps __syncthreads().
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  unsigned l = __lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// +1 at c[key] for every live lane of the wave: one atomic per distinct key while the keys
// repeat across the lanes (histograms of parts or of hub ids), one per lane once a key
// turns out rare.  Every lane of the wave calls it (uniform control flow).
template <typename C> __device__ __forceinline__ void wave_count(C *c, uint32_t key, bool live) {
  uint64_t todo = __ballot(live);
  while (todo) {   // (uniform)
    const int leader = __ffsll((long long)todo) - 1;
    const uint32_t k = __shfl(key, leader, 64);
    const uint64_t same = __ballot(live && key == k) & todo;
    const uint32_t cnt = (uint32_t)__popcll(same);
    if (cnt < 8) {   // rare: every lane left adds its own
      if ((todo >> __lane_id()) & 1) atomicAdd(&c[key], (C)1);
      break;
    }
    if ((int)__lane_id() == leader) atomicAdd(&c[k], (C)cnt);
    todo &= ~same;
  }
}

// Adds w into cnt[key] for every lane whose key != INVALID, with one atomic per run of
// equal keys in consecutive lanes (records sorted by tail, as generated and as many
// edge lists are stored, make tail runs long; a hub's endpoints collapse too).
__device__ __forceinline__ void run_add(uint32_t *cnt, uint32_t key, uint32_t w) {
  const int lane = (int)__lane_id();
  const uint32_t prev = __shfl_up(key, 1, 64);
  const bool start = key != INVALID && (lane == 0 || prev != key);
  const uint64_t starts = __ballot(start);
  const uint32_t rid = (uint32_t)__popcll(starts & ((lane == 63) ? ~0ull : ((2ull << lane) - 1)));
  uint32_t v = key != INVALID ? w : 0;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_down(v, o, 64);
    const uint32_t ro = __shfl_down(rid, o, 64);
    const uint32_t ko = __shfl_down(key, o, 64);
    if (lane + o < 64 && ro == rid && ko == key) v += u;
  }
  if (start && v) atomicAdd(&cnt[key], v);
}

template <typename T> __device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T> __device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o, 64); v = w > v ? w : v; }
  return v;
}
template <typename T> __device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o, 64); v = w < v ? w : v; }
  return v;
}

// One atomic per workgroup for a value every thread contributes (every thread of the
// workgroup calls; blockDim.x a multiple of 64, <= 1024).  Per-wave atomics on one word
// serialise a launch of ~1e5 workgroups (k_compact_count: 1.5 ms for 1.3e5 of them).
// Both always issue their one atomic: a load-before-atomic check could be served a stale
// line from another XCD's L2 (coherence across XCDs).
__device__ __forceinline__ uint64_t block_reduce_u64(uint64_t v, bool is_max) {
  __shared__ uint64_t s_red[16];
  v = is_max ? wave_max(v) : wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  lds_barrier();
  uint64_t r = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = is_max ? (s_red[w] > r ? s_red[w] : r) : r + s_red[w];
  lds_barrier();   // s_red is reused by the next call
  return r;          // meaningful in thread 0
}
__device__ __forceinline__ void block_atomic_max(unsigned long long *dst, uint64_t v) {
  const uint64_t m = block_reduce_u64(v, true);
  if (threadIdx.x == 0 && m) atomicMax(dst, (unsigned long long)m);
}
__device__ __forceinline__ void block_atomic_add(unsigned long long *dst, uint64_t v) {
  const uint64_t m = block_reduce_u64(v, false);
  if (threadIdx.x == 0 && m) atomicAdd(dst, (unsigned long long)m);
}

// The tile of this workgroup in a grid of one workgroup per tile.  Workgroups are dealt
// round-robin over the 8 XCDs (b and b + 8 share one), so this gives XCD x a contiguous
// run of tiles: the tiles running at once on one XCD then share the lines of their
// (bucket, tile) counter columns in that XCD's L2.  A bijection on [0, gridDim.x).
__device__ __forceinline__ uint32_t xcd_tile() {
  const uint32_t g = gridDim.x, b = blockIdx.x, x = b & 7, q = g >> 3, r = g & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}

// Workgroup-aggregated append: reserves `cnt` consecutive slots for every thread with
// ONE device atomic per workgroup call (a single hot counter takes ~0.1 G atomics/s, so
// per-wave appends serialise a streaming kernel).  Every thread of the workgroup must
// call it (it synchronises the workgroup); returns the thread's first slot.  Slots are
// handed out in thread order within the call.
__device__ __forceinline__ uint64_t block_reserve(uint32_t cnt, unsigned long long *counter) {
  __shared__ uint32_t s_w[BLOCK / WAVE];
  __shared__ unsigned long long s_base;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) s_w[wave] = inc;
  lds_barrier();
  uint32_t woff = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / WAVE; ++w) {
    uint32_t x = s_w[w];
    if (w < wave) woff += x;
    tot += x;
  }
  if (threadIdx.x == 0) s_base = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
  lds_barrier();
  const uint64_t first = s_base + woff + inc - cnt;
  lds_barrier();   // s_w / s_base are reused by the next call
  return first;
}

// Tiles for streaming kernels that append: BLOCK threads x TILE_ITEMS items, items
// strided by BLOCK so each load instruction is coalesced.
constexpr int TILE_ITEMS = 8;
constexpr int TILE = BLOCK * TILE_ITEMS;
inline unsigned grid_tiles(uint64_t items, unsigned cap = 256 * 8) {
  uint64_t t = (items + TILE - 1) / TILE;
  if (t == 0) t = 1;
  return (unsigned)(t < cap ? t : cap);
}

// ---- sharded appends ------------------------------------------------------------------
// Even one returning atomic per 2048-item tile saturates a single counter (~0.1 G/s):
// a streaming pass over 1e9 edges would wait ~5 ms on it.  Tile t instead appends to
// shard t % NSHARD (its own counter on its own 128-B line) inside the shard's region
// of the output; shard k's region holds exactly the tiles t = k (mod NSHARD), so it
// cannot overflow.  pack_shards() then moves the regions together (stable per shard).
constexpr int NSHARD = 64;
constexpr int SHARD_STRIDE = 16;   // u64 counters 128 B apart
__host__ __device__ inline uint64_t shard_base(uint64_t ntiles, uint32_t k, uint32_t per_item) {
  const uint64_t q = ntiles / NSHARD, r = ntiles % NSHARD;
  return (uint64_t)TILE * per_item * (k * q + (k < r ? k : r));
}
__device__ __forceinline__ uint64_t shard_reserve(uint32_t cnt, unsigned long long *counters, uint64_t tile,
                                                  uint64_t ntiles, uint32_t per_item) {
  const uint32_t k = (uint32_t)(tile % NSHARD);
  return shard_base(ntiles, k, per_item) + block_reserve(cnt, counters + (uint64_t)k * SHARD_STRIDE);
}

// Wave-aggregated append: every lane with `pred` gets a unique slot in [0, *counter).
__device__ __forceinline__ uint64_t wave_append(bool pred, unsigned long long *counter) {
  uint64_t mask = __ballot(pred);
  uint64_t base = 0;
  if (mask == 0) return 0;
  int leader = __ffsll((unsigned long long)mask) - 1;
  if ((int)__lane_id() == leader) base = atomicAdd(counter, (unsigned long long)__popcll(mask));
  base = __shfl(base, leader, 64);
  return base + __popcll(mask & lanemask_lt());
}

}  // namespace sheep

// Host entry points shared between translation units.
namespace sheep {
void set_error(const char *msg);
// scan.hip
void scan_exclusive_u32(Ctx &c, const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *total_dev);
void scan_exclusive_u64(Ctx &c, const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *total_dev);
// the first *n_dev (<= n_max) entries, the length read on the device (launch sized for n_max)
void scan_exclusive_u64_dev(Ctx &c, const uint64_t *in, uint64_t *out, uint64_t n_max, const uint64_t *n_dev);
// radix.hip — stable LSD sort of (key, value) pairs on bits [0, end_bit); results end
// in (keys, vals); alt buffers are scratch of the same size.  With in_alt, a result left
// in the alt buffers (an odd number of passes) stays there and *in_alt says so (no copy).
void radix_sort_pairs_u32(Ctx &c, uint32_t *keys, uint32_t *vals, uint64_t n, int end_bit,
                          uint32_t *keys_alt, uint32_t *vals_alt, bool *in_alt = nullptr);
void radix_sort_keys_u64(Ctx &c, uint64_t *keys, uint64_t n, int end_bit, uint64_t *keys_alt,
                         bool *in_alt = nullptr);
// hist.hip — cnt[key] += occurrences, keys bucketed through LDS (no scattered atomics)
void histogram_heads(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int llama, uint64_t K, uint32_t *cnt,
                     bool counted = false);
// both endpoints (every tail, and the heads as above) for records in no particular order
void histogram_endpoints(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int llama, uint64_t K, uint32_t *cnt,
                         bool counted = false);
// records in any order: the degree pass with both endpoints' bucket counts (hist.hip)
bool degree_endpoints(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap,
                      unsigned long long *d_max, unsigned long long *d_err);
// the degree pass fused with the heads' bucket counts; false (nothing launched) when the
// capacity does not fit the bucket layout
bool degree_fused(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap,
                  unsigned long long *d_max, unsigned long long *d_err);
// relabel (jtree.cpp:72-91) in head-bucket order; returns the number of edges written, or
// UINT64_MAX when the key range / record count does not fit the bucket layout.
// The padded-lo bucket layout of the first-activity grouping (group_edges_by_lo): host
// copy + the device padding offsets / bucket bases.
struct LoGroup {
  int L = 0;
  uint32_t clo = 0, mask = 0, nb = 0;
  uint64_t K = 0;
  std::vector<uint32_t> padoff, kbase;
  std::vector<uint64_t> pstart, plen;
  uint32_t *d_pad = nullptr, *d_kbase = nullptr;
};
void lo_group_prepare(Ctx &c, uint64_t n, int L, uint32_t clo, LoGroup &g);
// relabel (jtree.cpp:72-91) in head-bucket order; returns the number of edges written, or
// UINT64_MAX when the key range / record count does not fit the bucket layout.  With lg,
// the gather also writes the edges' (padded-lo bucket, tile) counts for the grouping
// (*counted = true), so group_edges_by_lo skips its count pass.
// n_tree = the sequence's length (pst entries).
uint64_t relabel_bucketed(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                          uint64_t n_tree, uint32_t *pst, uint64_t *edges, unsigned long long *err,
                          const LoGroup *lg = nullptr, bool *counted = nullptr);
void histogram_edge_lo(Ctx &c, const uint64_t *edges, uint64_t m, uint64_t K, uint32_t *cnt);
uint64_t group_edges_by_lo(Ctx &c, const uint64_t *edges, uint64_t m, const LoGroup &g, uint32_t *pst, uint64_t *r0,
                           uint64_t *seg, bool counted);
// etree.hip
// filt_lvl >= 0: at that level only entries with spread(lo) in [ylo, yhi) are kept (one
// subproblem of a split merge; the caller cuts the later groups to it).  top_bits > 0: the
// block of the 2^top_bits highest positions is replaced by its minimum spanning forest when
// dense (maps; etree.hip "the dense top block").
// hook_mode: HOOK_BATCH — the hook rounds find all of a thread's edges' roots at once
// (merges: chains of tree edges, little contention) instead of one edge after another (maps:
// hub pile-ups); HOOK_UP — the smaller root is hooked under the larger (root = top).
void etree_from_edges(Ctx &c, const uint64_t *edges, uint64_t m, uint64_t n, uint32_t *parent, const uint64_t *seg,
                      int fin_bits, int filt_lvl = -1, uint32_t ylo = 0, uint32_t yhi = 0, int top_bits = 0,
                      int hook_mode = 0, int force_big_bits = 0);
constexpr int HOOK_BATCH = 1, HOOK_UP = 2;
void spread_params(uint64_t n, int *L, uint32_t *clo);
// append.hip — sharded appends: counters (NSHARD * SHARD_STRIDE u64, zeroed).  The pack
// step moves the shard regions of a producer that streamed *n_in items together in dst
// and writes the total to *total_out (device; must not alias n_in).  With cond, it runs
// only if *cond != 0, and then also zeroes the counter set zero_after.  With dst_off the
// packed items start at dst + *dst_off (a device count).  No host sync.
unsigned long long *shard_counters(Ctx &c, const char *tag);
template <typename T>
void pack_shards(Ctx &c, const T *src, T *dst, const uint64_t *n_in, const unsigned long long *counters,
                 uint64_t *total_out, const uint64_t *cond = nullptr, unsigned long long *zero_after = nullptr,
                 const uint64_t *dst_off = nullptr);
}  // namespace sheep
