// evaluate.hip — Partition::evaluate(graph) (partition.cpp:428-473) and
// Partition::evaluate(graph, seq) (partition.cpp:475-521) over the records in HBM.
//
// The reference walks every node X and its LLAMA adjacency (a record (u,v) gives the
// entries u->v and v->u; a self-loop gives one entry), inserting an "owner" part per
// entry into an unordered_set.  Per record the owners are symmetric:
//   ECV(down): part of the endpoint earlier in the sequence (both entries)
//   ECV(up)  : part of the later endpoint
//   ECV(hash): part of the endpoint with the smaller cormen hash (s odd -> bijective)
//   Vcom vol : the other endpoint's part (plus X's own part, added per node)
// so one pass over the records ORs owner bits into per-vertex part bitsets and a second
// pass over vertex slots pops the bits.  Balances and edges-cut are per-block LDS
// histograms.
//
// Layout (HBM): one row of RW = 1 + M * W64 u64 words per vertex slot v.  Word 0 is
// pp = pos << 16 | part (the two per-vertex gathers a record needs, in one 8-B load);
// then M bit arrays (the requested ones, in the order down, up, hash, vcom), each
// W64 = ceil(nparts / 64) words: row[v][1 + a * W64 + w].
//
// Traffic: a record's tail side is near-sequential when records come tail-sorted (runs
// of equal tails are OR-combined in the wave first).  Its head side is random over a
// 0.5-1 GB array at RMAT-26, far above the Infinity Cache: with pp and the bits in
// separate arrays it cost two random lines per record (37.8 ms at RMAT-26); in one row
// the bit word shares the line the pp gather already brought in (k <= 64, one array: a
// 16-B row, one 16-B load).  The atomicOr is issued only when the bit is still clear —
// power-law heads saturate their bitsets after a few records.
//
// The sharded form (one call per edge shard, bitsets OR-combined and accumulators
// summed across shards, then one node pass) is the distributed evaluator of SURVEY
// §8(e) step 6.
#include "common.hpp"

namespace sheep {
namespace {

__device__ __forceinline__ uint32_t cormen_hash(uint32_t k) { return k * 2654435769u; }

constexpr int LDS_PARTS = 2048;
constexpr uint64_t NO_PP = ~0ull;

// accumulator row: scalars then the three record-side balance histograms
constexpr int AC_CUT = 0, AC_BAD = 1, AC_LOOPS = 2, AC_RECS = 3, AC_SCAL = 8;

// row heads (identical for every shard, so the OR-combine of states keeps them)
__global__ void k_pp(const uint32_t *__restrict__ pos, const int16_t *__restrict__ parts, uint64_t vs, uint32_t RW,
                     uint64_t *__restrict__ rows) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < vs; v += stride) {
    const uint32_t p = pos[v];
    const int16_t q = parts[v];
    rows[v * RW] = (p == INVALID || q < 0) ? NO_PP : ((uint64_t)p << 16) | (uint16_t)q;
  }
}

// OR of `m` over the run of consecutive lanes sharing `key` (INVALID: no key), delivered
// to the run's first lane (returns 0 elsewhere).
__device__ __forceinline__ uint64_t run_or(uint32_t key, uint64_t m) {
  const int lane = (int)__lane_id();
  const uint32_t prev = __shfl_up(key, 1, 64);
  const bool start = key != INVALID && (lane == 0 || prev != key);
  const uint64_t starts = __ballot(start);
  const uint32_t rid = (uint32_t)__popcll(starts & ((lane == 63) ? ~0ull : ((2ull << lane) - 1)));
  uint64_t v = key != INVALID ? m : 0;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_down(v, o, 64);
    const uint32_t ro = __shfl_down(rid, o, 64);
    const uint32_t ko = __shfl_down(key, o, 64);
    if (lane + o < 64 && ro == rid && ko == key) v |= u;
  }
  return start ? v : 0;
}

__device__ __forceinline__ void or_bits(unsigned long long *bits, uint64_t idx, uint64_t m) {
  if (!m) return;
  if ((bits[idx] & m) != m) atomicOr(&bits[idx], (unsigned long long)m);
}

template <bool ROW16>   // ROW16: one bit array of one word (RW == 2), loaded with the head's pp
__global__ __launch_bounds__(BLOCK) void k_eval_records(const sheep_xs1 *__restrict__ rec, uint64_t nrec,
                                                        uint64_t pos_size, int what, int M, uint32_t W64, int nparts,
                                                        unsigned long long *__restrict__ rows,
                                                        unsigned long long *__restrict__ acc) {
  const uint32_t RW = 1 + (uint32_t)M * W64;
  unsigned long long *const bal = acc + AC_SCAL;   // [0,n) down, [n,2n) up, [2n,3n) hash
  __shared__ uint32_t lbal[3][LDS_PARTS];
  const bool lds = nparts <= LDS_PARTS;
  if (lds)
    for (int i = threadIdx.x; i < 3 * LDS_PARTS; i += BLOCK) (&lbal[0][0])[i] = 0;
  __syncthreads();
  // bit-array index of each metric (-1: not requested)
  const int ad = (what & 2) ? 0 : -1;
  const int au = (what & 4) ? ((what & 2) ? 1 : 0) : -1;
  const int ah = (what & 1) ? M - 2 : -1, av = (what & 1) ? M - 1 : -1;
  uint64_t cut = 0, bad = 0, loops = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t iters = (nrec + stride - 1) / stride;
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, i += stride) {   // wave-uniform trip count (run_or)
    uint32_t t = INVALID, h = INVALID;
    int tp = 0, hp = 0;
    bool live = false;
    uint32_t pt = 0, ph = 0;
    uint64_t hw = 0;   // ROW16: the head's bit word, read with its pp
    if (i < nrec) {
      const sheep_xs1 r = rec[i];
      if (r.tail >= pos_size || r.head >= pos_size) {
        ++bad;
      } else {
        const uint64_t a = rows[(uint64_t)r.tail * RW];
        uint64_t b;
        if (ROW16) {
          const ulonglong2 hr = *reinterpret_cast<const ulonglong2 *>(rows + (uint64_t)r.head * 2);
          b = hr.x;
          hw = hr.y;
        } else {
          b = rows[(uint64_t)r.head * RW];
        }
        if (a == NO_PP || b == NO_PP) {
          ++bad;
        } else {
          t = r.tail;
          h = r.head;
          pt = (uint32_t)(a >> 16);
          ph = (uint32_t)(b >> 16);
          tp = (int)(uint16_t)a;
          hp = (int)(uint16_t)b;
          live = true;
        }
      }
    }
    const bool loop = live && t == h;
    loops += loop;
    // owner parts (a self-loop's entry X->X owns X's part in every metric)
    const int pd = loop ? tp : (pt < ph ? tp : hp), pu = loop ? tp : (pt < ph ? hp : tp);
    const int po = loop ? tp : (cormen_hash(t) < cormen_hash(h) ? tp : hp);
    if (live && !loop) {
      if (ad >= 0) { if (lds) atomicAdd(&lbal[0][pd], 1u); else atomicAdd(&bal[pd], 1ull); }
      if (au >= 0) { if (lds) atomicAdd(&lbal[1][pu], 1u); else atomicAdd(&bal[nparts + pu], 1ull); }
      if (ah >= 0) {
        if (lds) atomicAdd(&lbal[2][po], 1u); else atomicAdd(&bal[2 * nparts + po], 1ull);
        cut += tp != hp;
      }
    }
    // the tail side: runs of equal tails combined in the wave (single-word bitsets)
    const int own_t[4] = {pd, pu, po, hp};   // down, up, hash, vcom owner seen from t
    const int own_h[4] = {pd, pu, po, tp};
    const int arr[4] = {ad, au, ah, av};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (arr[q] < 0) continue;   // uniform
      if (W64 == 1) {
        const uint64_t m = run_or(live ? t : INVALID, live ? 1ull << own_t[q] : 0);
        if (m) or_bits(rows, (uint64_t)t * RW + 1 + arr[q], m);
      } else if (live) {
        or_bits(rows, (uint64_t)t * RW + 1 + arr[q] * W64 + (own_t[q] >> 6), 1ull << (own_t[q] & 63));
      }
      if (live && !loop) {
        if (ROW16) {
          const uint64_t m = 1ull << own_h[q];
          if ((hw & m) != m) atomicOr(&rows[(uint64_t)h * 2 + 1], (unsigned long long)m);
        } else {
          or_bits(rows, (uint64_t)h * RW + 1 + arr[q] * W64 + (own_h[q] >> 6), 1ull << (own_h[q] & 63));
        }
      }
    }
  }
  block_atomic_add(&acc[AC_CUT], cut);
  block_atomic_add(&acc[AC_BAD], bad);
  block_atomic_add(&acc[AC_LOOPS], loops);
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&acc[AC_RECS], (unsigned long long)nrec);
  __syncthreads();
  if (lds)
    for (int x = threadIdx.x; x < 3 * nparts; x += BLOCK) {
      const uint32_t v = lbal[x / nparts][x % nparts];
      if (v) atomicAdd(&bal[x], (unsigned long long)v);
    }
}

// dst |= src over the bit words, dst += src over the accumulators (shard combine)
__global__ void k_eval_combine(unsigned long long *__restrict__ dst, const unsigned long long *__restrict__ src,
                               uint64_t words, unsigned long long *__restrict__ adst,
                               const unsigned long long *__restrict__ asrc, uint64_t awords) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < words; i += stride) dst[i] |= src[i];
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < awords; i += stride) adst[i] += asrc[i];
}

// Per vertex slot: a node is a slot whose first bit array is non-empty (every record
// sets a bit in every requested array at both endpoints).  out = {ecv down, up, hash,
// vcom, nodes}; vbal = vertex balance histogram.
__global__ __launch_bounds__(BLOCK) void k_eval_nodes(uint64_t vs, const int16_t *__restrict__ parts, int what, int M,
                                                      uint32_t W64, int nparts,
                                                      const unsigned long long *__restrict__ rows,
                                                      unsigned long long *__restrict__ vbal,
                                                      unsigned long long *__restrict__ out) {
  __shared__ uint32_t lv[LDS_PARTS];
  const bool lds = nparts <= LDS_PARTS;
  if (lds)
    for (int i = threadIdx.x; i < LDS_PARTS; i += BLOCK) lv[i] = 0;
  __syncthreads();
  const int ad = (what & 2) ? 0 : -1;
  const int au = (what & 4) ? ((what & 2) ? 1 : 0) : -1;
  const int ah = (what & 1) ? M - 2 : -1, av = (what & 1) ? M - 1 : -1;
  uint64_t s[4] = {0, 0, 0, 0}, nodes = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < vs; v += stride) {
    const unsigned long long *b = rows + v * (1 + (uint64_t)M * W64) + 1;
    bool node = false;
    for (uint32_t w = 0; w < W64; ++w) node |= b[w] != 0;
    if (!node) continue;
    ++nodes;
    const int p = parts[v];
    const int arr[4] = {ad, au, ah, av};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (arr[q] < 0) continue;
      uint32_t cnt = 0;
      for (uint32_t w = 0; w < W64; ++w) {
        uint64_t x = b[arr[q] * W64 + w];
        if (q == 3 && p >= 0 && (uint32_t)(p >> 6) == w) x |= 1ull << (p & 63);   // Vcom: own part
        cnt += __popcll(x);
      }
      s[q] += cnt - 1;
    }
    if (av >= 0 && p >= 0 && p < nparts) {
      if (lds) atomicAdd(&lv[p], 1u); else atomicAdd(&vbal[p], 1ull);
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) block_atomic_add(&out[q], s[q]);
  block_atomic_add(&out[4], nodes);
  __syncthreads();
  if (lds)
    for (int x = threadIdx.x; x < nparts; x += BLOCK)
      if (lv[x]) atomicAdd(&vbal[x], (unsigned long long)lv[x]);
}

__global__ void k_max_part(const int16_t *__restrict__ parts, uint64_t vs, unsigned long long *__restrict__ out) {
  int m = -1;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < vs; i += stride) m = parts[i] > m ? parts[i] : m;
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0 && m >= 0) atomicMax(out, (unsigned long long)m);
}

int eval_arrays(int what) { return ((what & 2) ? 1 : 0) + ((what & 4) ? 1 : 0) + ((what & 1) ? 2 : 0); }

}  // namespace

// Layout of the evaluator state for `what` (0 = all) and nparts parts (max part + 1).
void eval_sizes(int what, int nparts, uint64_t pos_size, uint64_t *bits_words, uint64_t *acc_words) {
  if (what == 0) what = 7;
  if (what & ~7) throw Error(SHEEP_ERR_ARG, "evaluate: unknown metric bits");
  if (nparts < 1) nparts = 1;
  const uint64_t W64 = ((uint64_t)nparts + 63) / 64;
  *bits_words = pos_size * (1 + (uint64_t)eval_arrays(what) * W64);
  *acc_words = AC_SCAL + 3 * (uint64_t)nparts;
}

int eval_num_parts(Ctx &c, const int16_t *parts, uint64_t pos_size) {
  unsigned long long *d = (unsigned long long *)c.d_scalars + 55;
  HIP_CHECK(hipMemsetAsync(d, 0, sizeof(uint64_t), c.stream));
  if (pos_size) {
    hipLaunchKernelGGL(k_max_part, dim3(grid_for(pos_size)), dim3(BLOCK), 0, c.stream, parts, pos_size, d);
    LAUNCH_CHECK();
  }
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 55, d, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  return (int)c.h_scalars[55] + 1;   // max part + 1 (partition.cpp:433-435)
}

// One shard's records: owner bits ORed into bits, counts added into acc (both zeroed by
// the caller before the first shard).  Asynchronous.
void eval_shard(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                const int16_t *parts, int what, int nparts, uint64_t *bits, uint64_t *acc) {
  if (what == 0) what = 7;
  const int M = eval_arrays(what);
  const uint32_t W64 = (uint32_t)((nparts + 63) / 64);
  if (!nrec) return;
  if (pos_size == 0) {   // every record is out of range
    hipLaunchKernelGGL(k_eval_records<false>, dim3(grid_for(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, (uint64_t)0,
                       what, M, W64, nparts, (unsigned long long *)bits, (unsigned long long *)acc);
    LAUNCH_CHECK();
    return;
  }
  const uint32_t RW = 1 + (uint32_t)M * W64;
  hipLaunchKernelGGL(k_pp, dim3(grid_for(pos_size)), dim3(BLOCK), 0, c.stream, pos, parts, pos_size, RW, bits);
  LAUNCH_CHECK();
  auto kern = RW == 2 ? k_eval_records<true> : k_eval_records<false>;
  hipLaunchKernelGGL(kern, dim3(grid_for(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, pos_size, what, M, W64, nparts,
                     (unsigned long long *)bits, (unsigned long long *)acc);
  LAUNCH_CHECK();
}

void eval_combine(Ctx &c, uint64_t *bits, const uint64_t *bits_src, uint64_t words, uint64_t *acc,
                  const uint64_t *acc_src, uint64_t acc_words) {
  const uint64_t mx = words > acc_words ? words : acc_words;
  if (!mx) return;
  hipLaunchKernelGGL(k_eval_combine, dim3(grid_for(mx)), dim3(BLOCK), 0, c.stream, (unsigned long long *)bits,
                     (const unsigned long long *)bits_src, words, (unsigned long long *)acc,
                     (const unsigned long long *)acc_src, acc_words);
  LAUNCH_CHECK();
}

// The node pass over the (combined) state and the result; synchronises.
void eval_finish(Ctx &c, const uint64_t *bits, const uint64_t *acc, uint64_t pos_size, const int16_t *parts, int what,
                 int nparts, sheep_eval *out) {
  *out = sheep_eval();
  if (what == 0) what = 7;
  const int M = eval_arrays(what);
  const uint32_t W64 = (uint32_t)((nparts + 63) / 64);
  unsigned long long *vbal = c.get_as<unsigned long long>("ev_vbal", (uint64_t)nparts);
  unsigned long long *res = (unsigned long long *)c.d_scalars + 48;   // ecv down, up, hash, vcom, nodes
  HIP_CHECK(hipMemsetAsync(vbal, 0, (uint64_t)nparts * sizeof(uint64_t), c.stream));
  HIP_CHECK(hipMemsetAsync(res, 0, 5 * sizeof(uint64_t), c.stream));
  if (pos_size) {
    hipLaunchKernelGGL(k_eval_nodes, dim3(grid_for(pos_size)), dim3(BLOCK), 0, c.stream, pos_size, parts, what, M, W64,
                       nparts, (const unsigned long long *)bits, vbal, res);
    LAUNCH_CHECK();
  }
  const uint64_t aw = AC_SCAL + 3 * (uint64_t)nparts;
  std::vector<uint64_t> ha(aw), hv(nparts);
  HIP_CHECK(hipMemcpyAsync(ha.data(), acc, aw * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(hv.data(), vbal, (uint64_t)nparts * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 48, res, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (ha[AC_BAD]) throw Error(SHEEP_ERR_RANGE, "evaluate: a vertex is unsequenced or unassigned");
  auto mx = [&](const uint64_t *h) { uint64_t m = 0; for (int p = 0; p < nparts; ++p) m = h[p] > m ? h[p] : m; return m; };
  const uint64_t *bal = ha.data() + AC_SCAL;
  out->nodes = c.h_scalars[52];
  // adjacency entries = 2 per record, 1 per self-loop (LLAMA stores a self-loop once)
  out->edges = (2 * ha[AC_RECS] - ha[AC_LOOPS]) / 2;
  if (what & 2) { out->ecv_down = c.h_scalars[48]; out->max_down_bal = mx(bal); }
  if (what & 4) { out->ecv_up = c.h_scalars[49]; out->max_up_bal = mx(bal + nparts); }
  if (what & 1) {
    out->ecv_hash = c.h_scalars[50];
    out->vcom_vol = c.h_scalars[51];
    out->edges_cut = ha[AC_CUT];
    out->max_hash_bal = mx(bal + 2 * (uint64_t)nparts);
    out->max_vertex_bal = mx(hv.data());
  }
}

// `what` bitmask: 1 = evaluate(graph) metrics, 2 = ECV(down), 4 = ECV(up); 0 = all.
// Metrics outside the mask come back 0.
void evaluate(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
              const int16_t *parts, int what, sheep_eval *out) {
  uint64_t words = 0, aw = 0;
  eval_sizes(what, 1, pos_size, &words, &aw);   // validates `what`
  const int nparts = eval_num_parts(c, parts, pos_size);
  eval_sizes(what, nparts, pos_size, &words, &aw);
  uint64_t *bits = c.get_as<uint64_t>("ev_bits", words ? words : 1);
  uint64_t *acc = c.get_as<uint64_t>("ev_acc", aw);
  HIP_CHECK(hipMemsetAsync(bits, 0, words * sizeof(uint64_t), c.stream));
  HIP_CHECK(hipMemsetAsync(acc, 0, aw * sizeof(uint64_t), c.stream));
  {
    // B_eval: record read + 2 pos + 2 part gathers, bitset write + read
    // (2 B per slot per 8 parts, per bit array)
    TimedRegion tr(c, "evaluate", 28 * nrec + 2 * (words - pos_size) * 8);
    eval_shard(c, rec, nrec, pos, pos_size, parts, what, nparts, bits, acc);
    eval_finish(c, bits, acc, pos_size, parts, what, nparts, out);
  }
}

namespace {

// ---- the same counts from the map's position-space edges --------------------------------
// A map (relabel_and_tree) leaves every non-loop record as a tree edge (hi << 32 | lo) of
// positions, grouped by lo, in HBM (Ctx::step_edges).  In position space both evaluators'
// owners come from the jnid-indexed parts pj (2 B per node: cache-resident) and, for the
// hash owner, seq (the vids): down = part(lo), up = part(hi), hash = the part of the
// endpoint with the smaller cormen hash, Vcom = the other endpoint's part.  The lo side's
// bit words lie in the group's 2^15-position window; the hi side's are random over a
// row array of n * M * W64 words (262 MB for one metric at RMAT-26, 1.07 GB for the record
// evaluator's vid-indexed 16-B rows).  A vertex's OWN part enters two sets without any
// per-edge bit: ECV(down) at lo iff the vertex is the lo end of an edge (pst > 0: the map's
// lo histogram), ECV(up) at hi through a byte flag (a plain store, no atomic) — the per-edge
// read-and-atomicOr of the lo's own down bit cost 7 of the 17.6 ms at RMAT-26, its lines
// shared by the eight XCDs.  Self-loops are no edges: when the records hold any
// (nrec != the relabel's pair count) one pass over the records adds each loop vertex's own
// part to its sets and counts them; an endpoint without a position or a part is the
// reference's pos.at() throw, as in k_eval_records.
__global__ void k_parts_jnid(const uint32_t *__restrict__ seq, uint64_t n, const int16_t *__restrict__ parts_vid,
                             const uint32_t *__restrict__ pos, uint64_t pos_size, int16_t *__restrict__ pj,
                             unsigned long long *__restrict__ bad) {
  // pj[x] = the part of seq[x] (-1: none; an error only where x turns out to be an edge
  // endpoint, as in k_eval_records).  pos[seq[x]] == x checks that seq is the sequence the
  // map's index (and so its edges) came from.
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  bool b = false;
  for (uint64_t x = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; x < n; x += stride) {
    const uint32_t v = seq[x];
    const bool in = v < pos_size;
    b |= !in || pos[v] != (uint32_t)x;
    pj[x] = in ? parts_vid[v] : (int16_t)-1;
  }
  if (__any(b) && (threadIdx.x & 63) == 0) atomicAdd(bad, 1ull);
}

__global__ __launch_bounds__(BLOCK) void k_eval_edges(const uint64_t *__restrict__ edges, uint64_t m,
                                                      const int16_t *__restrict__ pj, const uint32_t *__restrict__ seq,
                                                      int what, int M, uint32_t W64, int nparts,
                                                      unsigned long long *__restrict__ bits,
                                                      uint8_t *__restrict__ up_own,
                                                      unsigned long long *__restrict__ acc) {
  const uint32_t RW = (uint32_t)M * W64;
  unsigned long long *const bal = acc + AC_SCAL;
  __shared__ uint32_t lbal[3][LDS_PARTS];
  const bool lds = nparts <= LDS_PARTS;
  if (lds)
    for (int i = threadIdx.x; i < 3 * LDS_PARTS; i += BLOCK) (&lbal[0][0])[i] = 0;
  __syncthreads();
  const int ad = (what & 2) ? 0 : -1;
  const int au = (what & 4) ? ((what & 2) ? 1 : 0) : -1;
  const int ah = (what & 1) ? M - 2 : -1, av = (what & 1) ? M - 1 : -1;
  const bool need_hi = (what & 5) != 0;   // up, hash and Vcom read the hi end's part
  uint64_t cut = 0, nopart = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const uint64_t iters = (m + stride - 1) / stride;
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  for (uint64_t it = 0; it < iters; ++it, i += stride) {   // wave-uniform trip count (wave_count)
    const bool in = i < m;
    const uint64_t e = in ? __builtin_nontemporal_load(&edges[i]) : 0ull;   // (streamed once: caches kept for the rows)
    const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
    const int pl = in ? pj[lo] : 0, ph = in && need_hi ? pj[hi] : 0;
    // an endpoint without a part (-1) is the reference's throw: counted, never an index (a
    // hi end's part is read here only when a metric needs it; the node pass checks the rest)
    const bool live = in && pl >= 0 && ph >= 0;
    nopart += in && !live;
    int po = 0;
    if ((what & 1) && live) {
      po = cormen_hash(seq[lo]) < cormen_hash(seq[hi]) ? pl : ph;
      cut += pl != ph;
    }
    // (per wave: the lanes mostly share a part; lds is uniform)
    if (ad >= 0) { if (lds) wave_count(lbal[0], (uint32_t)pl, live); else wave_count(bal, (uint32_t)pl, live); }
    if (au >= 0) { if (lds) wave_count(lbal[1], (uint32_t)ph, live); else wave_count(bal + nparts, (uint32_t)ph, live); }
    if (ah >= 0) { if (lds) wave_count(lbal[2], (uint32_t)po, live); else wave_count(bal + 2 * nparts, (uint32_t)po, live); }
    if (!live) continue;
    const int own_lo[4] = {pl, ph, po, ph};   // down, up, hash, Vcom owner seen from lo
    const int own_hi[4] = {pl, ph, po, pl};   // ... and from hi
    const int arr[4] = {ad, au, ah, av};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (arr[q] < 0) continue;   // uniform
      if (q != 0)   // (down at lo: lo's own part, from pst in the node pass)
        or_bits(bits, (uint64_t)lo * RW + arr[q] * W64 + (own_lo[q] >> 6), 1ull << (own_lo[q] & 63));
      if (q != 1)   // (up at hi: hi's own part, flagged below)
        or_bits(bits, (uint64_t)hi * RW + arr[q] * W64 + (own_hi[q] >> 6), 1ull << (own_hi[q] & 63));
    }
    if (au >= 0) up_own[hi] = 1;
  }
  block_atomic_add(&acc[AC_CUT], cut);
  block_atomic_add(&acc[AC_BAD], nopart);
  __syncthreads();
  if (lds)
    for (int x = threadIdx.x; x < 3 * nparts; x += BLOCK) {
      const uint32_t v = lbal[x / nparts][x % nparts];
      if (v) atomicAdd(&bal[x], (unsigned long long)v);
    }
}

// self-loops (own part into every requested set of the vertex) and the records the edges
// do not account for: loops counted, an endpoint without a position is bad
__global__ __launch_bounds__(BLOCK) void k_eval_loops(const sheep_xs1 *__restrict__ rec, uint64_t nrec,
                                                      const uint32_t *__restrict__ pos, uint64_t pos_size,
                                                      const int16_t *__restrict__ pj, int what, int M, uint32_t W64,
                                                      unsigned long long *__restrict__ bits,
                                                      unsigned long long *__restrict__ acc) {
  const uint32_t RW = (uint32_t)M * W64;
  uint64_t loops = 0, bad = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrec; i += stride) {
    const sheep_xs1 r = rec[i];
    const uint32_t pt = r.tail < pos_size ? pos[r.tail] : INVALID, ph = r.head < pos_size ? pos[r.head] : INVALID;
    if (pt == INVALID || ph == INVALID) { ++bad; continue; }
    if (r.tail != r.head) continue;
    ++loops;
    const int p = pj[pt];
    if (p < 0) { ++bad; continue; }
    for (int a = 0; a < M; ++a) or_bits(bits, (uint64_t)pt * RW + a * W64 + (p >> 6), 1ull << (p & 63));
  }
  block_atomic_add(&acc[AC_LOOPS], loops);
  block_atomic_add(&acc[AC_BAD], bad);
}

// per jnid: as k_eval_nodes over the jnid rows (no pp word), parts by jnid
__global__ __launch_bounds__(BLOCK) void k_eval_nodes_j(uint64_t n, const int16_t *__restrict__ pj, int what, int M,
                                                        uint32_t W64, int nparts,
                                                        const unsigned long long *__restrict__ bits,
                                                        const uint32_t *__restrict__ pst,
                                                        const uint8_t *__restrict__ up_own,
                                                        unsigned long long *__restrict__ vbal,
                                                        unsigned long long *__restrict__ out,
                                                        unsigned long long *__restrict__ acc) {
  __shared__ uint32_t lv[LDS_PARTS];
  const bool lds = nparts <= LDS_PARTS;
  if (lds)
    for (int i = threadIdx.x; i < LDS_PARTS; i += BLOCK) lv[i] = 0;
  __syncthreads();
  const int ad = (what & 2) ? 0 : -1;
  const int au = (what & 4) ? ((what & 2) ? 1 : 0) : -1;
  const int ah = (what & 1) ? M - 2 : -1, av = (what & 1) ? M - 1 : -1;
  uint64_t s[4] = {0, 0, 0, 0}, nodes = 0, nopart = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t x = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; x < n; x += stride) {
    const unsigned long long *b = bits + x * (uint64_t)M * W64;
    const int p = pj[x];
    // the own-part entries the edge pass left out: down (x is some edge's lo), up (flag)
    const bool own[4] = {ad >= 0 && pst[x] != 0, au >= 0 && up_own[x] != 0, false, true};
    bool node = own[ad >= 0 ? 0 : 1];   // (the first array: an own entry alone makes a node)
    for (uint32_t w = 0; w < W64; ++w) node |= b[w] != 0;
    if (!node) continue;
    if (p < 0) { ++nopart; continue; }   // an endpoint without a part (the edge pass skipped it)
    ++nodes;
    const int arr[4] = {ad, au, ah, av};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (arr[q] < 0) continue;
      uint32_t cnt = 0;
      for (uint32_t w = 0; w < W64; ++w) {
        uint64_t v = b[arr[q] * W64 + w];
        if (own[q] && (uint32_t)(p >> 6) == w) v |= 1ull << (p & 63);   // Vcom: always; down / up: as flagged
        cnt += __popcll(v);
      }
      s[q] += cnt - 1;
    }
    if (av >= 0 && p < nparts) {
      if (lds) atomicAdd(&lv[p], 1u); else atomicAdd(&vbal[p], 1ull);
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) block_atomic_add(&out[q], s[q]);
  block_atomic_add(&out[4], nodes);
  block_atomic_add(&acc[AC_BAD], nopart);
  __syncthreads();
  if (lds)
    for (int x = threadIdx.x; x < nparts; x += BLOCK)
      if (lv[x]) atomicAdd(&vbal[x], (unsigned long long)lv[x]);
}

}  // namespace

// sheep_evaluate's counts from the edges the context's last map left (Ctx::step_edges):
// the records, sequence and index must be the ones that map ran on.
void evaluate_step(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *seq, uint64_t n, const uint32_t *pos,
                   uint64_t pos_size, const int16_t *parts, int what, sheep_eval *out) {
  const Ctx::StepEdges se = c.step_edges;
  if (!se.valid || se.rec != rec || se.nrec != nrec || se.pos != pos || se.pos_size != pos_size || se.n != n)
    throw Error(SHEEP_ERR_ARG, "evaluate_step: the context's last map did not run on these records and this sequence");
  uint64_t words = 0, aw = 0;
  eval_sizes(what, 1, pos_size, &words, &aw);   // validates `what`
  if (what == 0) what = 7;
  const int nparts = eval_num_parts(c, parts, pos_size);
  const int M = eval_arrays(what);
  const uint32_t W64 = (uint32_t)((nparts + 63) / 64);
  aw = AC_SCAL + 3 * (uint64_t)nparts;
  words = n * (uint64_t)M * W64;
  uint64_t *bits = c.get_as<uint64_t>("ev_bits", words ? words : 1);
  uint64_t *acc = c.get_as<uint64_t>("ev_acc", aw);
  int16_t *pj = c.get_as<int16_t>("ev_pj", n ? n : 1);
  uint8_t *up_own = c.get_as<uint8_t>("ev_upown", n ? n : 1);
  unsigned long long *vbal = c.get_as<unsigned long long>("ev_vbal", (uint64_t)nparts);
  unsigned long long *res = (unsigned long long *)c.d_scalars + 48;   // ecv down, up, hash, vcom, nodes
  unsigned long long *pbad = (unsigned long long *)c.d_scalars + 53;
  *out = sheep_eval();
  {
    // B_eval as sheep_evaluate's (the evaluation's algorithmic bytes)
    TimedRegion tr(c, "evaluate", 28 * nrec + 2 * (uint64_t)M * W64 * 8 * pos_size);
    HIP_CHECK(hipMemsetAsync(bits, 0, words * sizeof(uint64_t), c.stream));
    HIP_CHECK(hipMemsetAsync(acc, 0, aw * sizeof(uint64_t), c.stream));
    HIP_CHECK(hipMemsetAsync(vbal, 0, (uint64_t)nparts * sizeof(uint64_t), c.stream));
    HIP_CHECK(hipMemsetAsync(res, 0, 6 * sizeof(uint64_t), c.stream));
    if (what & 4) HIP_CHECK(hipMemsetAsync(up_own, 0, n, c.stream));
    if (n) {
      hipLaunchKernelGGL(k_parts_jnid, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, seq, n, parts, pos, pos_size, pj,
                         pbad);
      LAUNCH_CHECK();
    }
    if (se.m_valid) {
      hipLaunchKernelGGL(k_eval_edges, dim3(grid_for(se.m_valid)), dim3(BLOCK), 0, c.stream, se.edges, se.m_valid,
                         (const int16_t *)pj, seq, what, M, W64, nparts, (unsigned long long *)bits, up_own,
                         (unsigned long long *)acc);
      LAUNCH_CHECK();
    }
    if (se.m_pairs != nrec) {   // self-loops or endpoints past the index: the records say which
      hipLaunchKernelGGL(k_eval_loops, dim3(grid_for(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, pos, pos_size,
                         (const int16_t *)pj, what, M, W64, (unsigned long long *)bits, (unsigned long long *)acc);
      LAUNCH_CHECK();
    }
    if (n) {
      hipLaunchKernelGGL(k_eval_nodes_j, dim3(grid_for(n)), dim3(BLOCK), 0, c.stream, n, (const int16_t *)pj, what, M,
                         W64, nparts, (const unsigned long long *)bits, se.pst, (const uint8_t *)up_own, vbal, res,
                         (unsigned long long *)acc);
      LAUNCH_CHECK();
    }
    std::vector<uint64_t> ha(aw), hv(nparts);
    HIP_CHECK(hipMemcpyAsync(ha.data(), acc, aw * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(hv.data(), vbal, (uint64_t)nparts * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    HIP_CHECK(hipMemcpyAsync(c.h_scalars + 48, res, 6 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
    c.sync();
    // another sequence than the map's index came from
    if (c.h_scalars[53])
      throw Error(SHEEP_ERR_ARG, "evaluate_step: seq is not the sequence whose index the context's last map used");
    // a DEAD edge (an endpoint without a position), an endpoint without a part, or a bad record
    if (se.m_valid != se.m_pairs || ha[AC_BAD])
      throw Error(SHEEP_ERR_RANGE, "evaluate: a vertex is unsequenced or unassigned");
    auto mx = [&](const uint64_t *h) { uint64_t m = 0; for (int p = 0; p < nparts; ++p) m = h[p] > m ? h[p] : m; return m; };
    const uint64_t *bal = ha.data() + AC_SCAL;
    out->nodes = c.h_scalars[52];
    out->edges = (2 * nrec - ha[AC_LOOPS]) / 2;
    if (what & 2) { out->ecv_down = c.h_scalars[48]; out->max_down_bal = mx(bal); }
    if (what & 4) { out->ecv_up = c.h_scalars[49]; out->max_up_bal = mx(bal + nparts); }
    if (what & 1) {
      out->ecv_hash = c.h_scalars[50];
      out->vcom_vol = c.h_scalars[51];
      out->edges_cut = ha[AC_CUT];
      out->max_hash_bal = mx(bal + 2 * (uint64_t)nparts);
      out->max_vertex_bal = mx(hv.data());
    }
  }
}

}  // namespace sheep

// ---- partition files (partition.cpp:588-670 writePartitionedGraph) -----------------------
namespace sheep {
namespace {

// The part an edge is written to: the part of its earlier-positioned endpoint
// (X_pos < Y_pos ? X_part : Y_part; a self-loop takes its vertex's part).  An endpoint
// outside the sequence or without a part is the reference's pos.at() throw / assert.
__global__ __launch_bounds__(BLOCK) void k_edge_parts(const sheep_xs1 *__restrict__ rec, uint64_t nrec,
                                                      const uint32_t *__restrict__ pos, uint64_t pos_size,
                                                      const int16_t *__restrict__ parts, int16_t *__restrict__ out,
                                                      unsigned long long *__restrict__ err) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  bool bad = false;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrec; i += stride) {
    const sheep_xs1 r = rec[i];
    int16_t p = SHEEP_INVALID_PART;
    if (r.tail < pos_size && r.head < pos_size) {
      const uint32_t xp = pos[r.tail], yp = pos[r.head];
      const int16_t xq = parts[r.tail], yq = parts[r.head];
      if (xp != INVALID && yp != INVALID && xq != SHEEP_INVALID_PART && yq != SHEEP_INVALID_PART) p = xp < yp ? xq : yq;
    }
    bad |= p == SHEEP_INVALID_PART;
    out[i] = p;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicAdd(err, 1ull);
}

}  // namespace

void edge_parts(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                const int16_t *parts_vid, int16_t *out) {
  if (!nrec) return;
  unsigned long long *err = (unsigned long long *)c.d_scalars + 58;
  HIP_CHECK(hipMemsetAsync(err, 0, sizeof(uint64_t), c.stream));
  hipLaunchKernelGGL(k_edge_parts, dim3(grid_for(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, pos, pos_size, parts_vid,
                     out, err);
  LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 58, err, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.h_scalars[58]) throw Error(SHEEP_ERR_RANGE, "vector::_M_range_check: an edge endpoint has no position or part (partition.cpp:657-664)");
}

}  // namespace sheep
