// sequence.hip — degree counting and the (degree, vid) degree sequence.
//
//   k_degree            sequence.h:70-78 (mpiSequence local degrees = LLAMA out_degree:
//                       self-loop once, graph_wrapper.h:87-89) and sequence.h:99-107
//                       (fileSequence: +1 per endpoint per record; XS1 last record twice)
//   k_compact_*         sequence.h:80-83 (slots with degree != 0, ascending vid)
//   radix_sort_pairs    sequence.h:85-91 (sort by degree; stable, so ties keep vid order)
//   k_scatter_pos       jtree.h:113,142-143 (vid -> jnid index; INVALID elsewhere)
//
// Layout in HBM: records are the 12-byte XS1 AoS exactly as on disk; degree/pos are
// dense u32 arrays over vertex slots; seq is a dense u32 array over jnids.
#include <cstdlib>

#include "common.hpp"

namespace sheep {
namespace {

// tails: add the tails here (run-combined atomics: records stored tail-sorted); otherwise
// the tails go through the LDS-bucketed histogram with the heads and only the FILE_DAT
// last record's extra tail count is added here.
__global__ __launch_bounds__(BLOCK) void k_degree(const sheep_xs1 *__restrict__ rec, uint64_t nrec, int mode,
                                                  uint32_t *__restrict__ deg, uint64_t cap,
                                                  unsigned long long *__restrict__ d_max,
                                                  unsigned long long *__restrict__ d_err, bool tails) {
  uint32_t lmax = 0;
  bool bad = false;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t iters = (nrec + stride - 1) / stride;
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, i += stride) {   // wave-uniform trip count
    uint32_t kt = INVALID, kh = INVALID, inc = 1;
    if (i < nrec) {
      const sheep_xs1 r = rec[i];
      const uint32_t t = r.tail, h = r.head;
      if (t >= cap || h >= cap) {
        bad = true;
      } else {
        inc = (mode == SHEEP_DEGREE_FILE_DAT && i == nrec - 1) ? 2u : 1u;
        kt = t;
        kh = (mode == SHEEP_DEGREE_LLAMA && t == h) ? INVALID : h;   // LLAMA: self-loop stored once
        const uint32_t m = (t > h ? t : h) + 1;
        lmax = m > lmax ? m : lmax;
      }
    }
    // tails here (runs: records are usually stored sorted by tail); heads go through
    // the LDS-bucketed histogram (hist.hip), except the FILE_DAT last record's extra
    if (tails) run_add(deg, kt, inc);
    else if (inc == 2) atomicAdd(&deg[kt], 1u);
    if (inc == 2 && kh != INVALID) atomicAdd(&deg[kh], 1u);
  }
  block_atomic_max(d_max, lmax);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(d_err, 1ull);
}

// Sortedness probe: descents tail[i + 1] < tail[i] at `samples` evenly spaced i.
__global__ __launch_bounds__(BLOCK) void k_tail_descents(const sheep_xs1 *__restrict__ rec, uint64_t nrec, uint64_t step,
                                                         uint64_t samples, unsigned long long *__restrict__ cnt) {
  const uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint64_t i = j * step;
  const bool d = j < samples && i + 1 < nrec && rec[i + 1].tail < rec[i].tail;
  block_atomic_add(cnt, d ? 1 : 0);
}

constexpr int C_ITEMS = 8;
constexpr int C_TILE = BLOCK * C_ITEMS;

__global__ __launch_bounds__(BLOCK) void k_compact_count(const uint32_t *__restrict__ deg, uint64_t vs,
                                                         uint32_t *__restrict__ block_cnt,
                                                         unsigned long long *__restrict__ d_maxdeg) {
  // tiles strided over a capped grid, the maximum reduced over all of a workgroup's tiles:
  // one atomicMax per tile (32 K at RMAT-26, all on one word) was the kernel's bound
  __shared__ uint32_t s[BLOCK / WAVE];
  const uint64_t ntiles = (vs + C_TILE - 1) / C_TILE;
  uint32_t mx = 0;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t base = tile * C_TILE;
    uint32_t cnt = 0;
#pragma unroll
    for (int j = 0; j < C_ITEMS; ++j) {
      const uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
      if (i < vs) { const uint32_t d = deg[i]; cnt += d != 0; mx = d > mx ? d : mx; }
    }
    cnt = wave_sum(cnt);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) block_cnt[tile] = s[0] + s[1] + s[2] + s[3];
    __syncthreads();   // s is rewritten by the next tile
  }
  block_atomic_max(d_maxdeg, mx);
}

// Order-preserving compaction: (key = degree, value = vid) for every non-zero slot.
__global__ __launch_bounds__(BLOCK) void k_compact_write(const uint32_t *__restrict__ deg, uint64_t vs,
                                                         const uint32_t *__restrict__ block_off,
                                                         uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  __shared__ uint32_t wcount[BLOCK / WAVE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t base = (uint64_t)blockIdx.x * C_TILE;
  uint32_t running = block_off[blockIdx.x];
  for (int j = 0; j < C_ITEMS; ++j) {
    uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    uint32_t d = i < vs ? deg[i] : 0;
    uint64_t m = __ballot(d != 0);
    if (lane == 0) wcount[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = running;
    for (int w = 0; w < wave; ++w) off += wcount[w];
    if (d != 0) {
      uint32_t o = off + (uint32_t)__popcll(m & lanemask_lt());
      keys[o] = d;
      vals[o] = (uint32_t)i;
    }
    running += wcount[0] + wcount[1] + wcount[2] + wcount[3];
    __syncthreads();
  }
}

__global__ void k_fill_u32(uint32_t *p, uint64_t n, uint32_t v) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) p[i] = v;
}

__global__ void k_scatter_pos(const uint32_t *__restrict__ seq, uint64_t n, uint32_t *__restrict__ pos) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) pos[seq[i]] = (uint32_t)i;
}

// readSequence path: arbitrary vids; detect out-of-range and duplicates.
__global__ void k_scatter_pos_checked(const uint32_t *__restrict__ seq, uint64_t n, uint32_t *__restrict__ pos,
                                      uint64_t pos_size, unsigned long long *__restrict__ d_err) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) {
    uint32_t v = seq[i];
    if (v >= pos_size) { atomicAdd(d_err, 1ull); continue; }
    if (atomicExch(&pos[v], (uint32_t)i) != INVALID) atomicAdd(d_err, 1ull);
  }
}

}  // namespace

void fill_u32(Ctx &c, uint32_t *p, uint64_t n, uint32_t v) {
  if (!n) return;
  hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, p, n, v);
  LAUNCH_CHECK();
}

// Records stored sorted by tail (as generated, as hep-th and most edge lists are) put a
// tail's records in one run, so the degree pass adds each run with one atomic.  In a
// generic order every record's tail is its own scattered atomic (RMAT-26 shuffled: 44 ms),
// so then the tails are bucketed in LDS together with the heads instead.
static bool tails_sorted(Ctx &c, const sheep_xs1 *rec, uint64_t nrec) {
  constexpr uint64_t SAMPLES = 1 << 16;
  if (nrec < 2 * SAMPLES) return true;   // small inputs: the atomics cost nothing
  // the answer is kept per record buffer: either path counts correctly, so a buffer
  // refilled in another order only costs speed, and a repeated call skips the probe's sync
  if (c.sorted_probe.rec == rec && c.sorted_probe.nrec == nrec) return c.sorted_probe.sorted;
  unsigned long long *d = (unsigned long long *)c.d_scalars + 2;
  HIP_CHECK(hipMemsetAsync(d, 0, sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_tail_descents, dim3((unsigned)(SAMPLES / BLOCK)), dim3(BLOCK), 0, c.stream, rec, nrec,
                     (nrec - 1) / SAMPLES, SAMPLES, d);
  LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 2, d, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  c.sorted_probe = {rec, nrec, c.h_scalars[2] * 50 < SAMPLES};   // fewer than 2% descents
  return c.sorted_probe.sorted;
}

void degree_count(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap,
                  uint64_t *max_slot) {
  if (mode < 0 || mode > 2) throw Error(SHEEP_ERR_ARG, "bad degree mode");
  unsigned long long *d = (unsigned long long *)c.d_scalars;
  const bool sorted = !nrec || nrec >= (1ull << 31) || tails_sorted(c, rec, nrec);
  HIP_CHECK(hipMemsetAsync(d, 0, 2 * sizeof(uint64_t), c.stream));
  bool counted = false;   // heads' (bucket, tile) counts made by the same pass (hist.hip)
  if (nrec) {
    TimedRegion tr(c, "degree", 12 * nrec);   // one read of the 12-B records
    counted = sorted ? degree_fused(c, rec, nrec, mode, deg, cap, d, d + 1)
                     : degree_endpoints(c, rec, nrec, mode, deg, cap, d, d + 1);
    if (!counted) {
      hipLaunchKernelGGL(k_degree, dim3(grid_for(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, mode, deg, cap, d, d + 1,
                         sorted);
      LAUNCH_CHECK();
    }
  }
  HIP_CHECK(hipMemcpyAsync(c.h_scalars, d, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.h_scalars[1]) throw Error(SHEEP_ERR_RANGE, "degree count: vertex id >= degree capacity");
  *max_slot = c.h_scalars[0];
  if (nrec) {
    TimedRegion tr(c, "degree_heads", 12 * nrec);
    if (sorted) histogram_heads(c, rec, nrec, mode == SHEEP_DEGREE_LLAMA, *max_slot, deg, counted);
    else histogram_endpoints(c, rec, nrec, mode == SHEEP_DEGREE_LLAMA, *max_slot, deg, counted);
  }
}

uint64_t sequence_from_degrees(Ctx &c, const uint32_t *deg, uint64_t vs, uint32_t *seq, uint32_t *pos) {
  TimedRegion tr(c, "sequence", 8 * vs);   // degree read + pos write
  fill_u32(c, pos, vs, INVALID);
  if (vs == 0) return 0;
  uint64_t nb = (vs + C_TILE - 1) / C_TILE;
  uint32_t *bcnt = c.get_as<uint32_t>("seq_bcnt", nb + 1);
  unsigned long long *d = (unsigned long long *)c.d_scalars;
  HIP_CHECK(hipMemsetAsync(d, 0, 2 * sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_compact_count, dim3(grid_for(nb, 1)), dim3(BLOCK), 0, c.stream, deg, vs, bcnt, d);
  LAUNCH_CHECK();
  scan_exclusive_u32(c, bcnt, bcnt, nb, (uint32_t *)(c.d_scalars + 1));
  HIP_CHECK(hipMemcpyAsync(c.h_scalars, d, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  uint64_t maxdeg = c.h_scalars[0];
  uint64_t n = (uint32_t)c.h_scalars[1];
  if (n == 0) return 0;
  uint32_t *keys = c.get_as<uint32_t>("seq_keys", n), *kalt = c.get_as<uint32_t>("seq_kalt", n);
  uint32_t *valt = c.get_as<uint32_t>("seq_valt", n);
  hipLaunchKernelGGL(k_compact_write, dim3((unsigned)nb), dim3(BLOCK), 0, c.stream, deg, vs, bcnt, keys, seq);
  LAUNCH_CHECK();
  int bits = 0;
  while (bits < 32 && (maxdeg >> bits)) ++bits;
  bool in_alt = false;
  radix_sort_pairs_u32(c, keys, seq, n, bits, kalt, valt, &in_alt);
  if (in_alt)   // the sorted vids are in valt: only they go back (the degree keys are not needed)
    HIP_CHECK(hipMemcpyAsync(seq, valt, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, c.stream));
  hipLaunchKernelGGL(k_scatter_pos, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, seq, n, pos);
  LAUNCH_CHECK();
  return n;
}

void positions(Ctx &c, const uint32_t *seq, uint64_t n, uint32_t *pos, uint64_t pos_size) {
  fill_u32(c, pos, pos_size, INVALID);
  unsigned long long *d = (unsigned long long *)c.d_scalars;
  HIP_CHECK(hipMemsetAsync(d, 0, sizeof(uint64_t), c.stream));
  if (n) {
    hipLaunchKernelGGL(k_scatter_pos_checked, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, seq, n, pos, pos_size, d);
    LAUNCH_CHECK();
  }
  HIP_CHECK(hipMemcpyAsync(c.h_scalars, d, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.h_scalars[0]) throw Error(SHEEP_ERR_ARG, "sequence has duplicate or out-of-range vids");
}

}  // namespace sheep
