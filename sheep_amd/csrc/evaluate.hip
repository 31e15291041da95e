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
// so one pass over the records ORs owner bits into per-vertex part bitsets
// (k bits per vertex, word-interleaved per vertex), and a second pass over vertex
// slots pops the bits.  Balances and edges-cut are per-block LDS histograms.
#include "common.hpp"

namespace sheep {
namespace {

__device__ __forceinline__ uint32_t cormen_hash(uint32_t k) { return k * 2654435769u; }

constexpr int LDS_PARTS = 2048;

__device__ __forceinline__ void set_bit(uint32_t *bits, uint32_t W, uint32_t v, int p) {
  atomicOr(&bits[(uint64_t)v * W + (p >> 5)], 1u << (p & 31));
}

__global__ __launch_bounds__(BLOCK) void k_eval_records(const sheep_xs1 *__restrict__ rec, uint64_t nrec,
                                                        const uint32_t *__restrict__ pos, uint64_t pos_size,
                                                        const int16_t *__restrict__ parts, int what, uint32_t W,
                                                        int nparts, uint32_t *__restrict__ bdown,
                                                        uint32_t *__restrict__ bup, uint32_t *__restrict__ bhash,
                                                        uint32_t *__restrict__ bvc, unsigned long long *__restrict__ bal,
                                                        unsigned long long *__restrict__ scal,
                                                        unsigned long long *__restrict__ selfl) {
  // bal: [0,nparts) down, [nparts,2n) up, [2n,3n) hash
  __shared__ uint32_t lbal[3][LDS_PARTS];
  const bool lds = nparts <= LDS_PARTS;
  if (lds)
    for (int i = threadIdx.x; i < 3 * LDS_PARTS; i += BLOCK) (&lbal[0][0])[i] = 0;
  __syncthreads();
  uint64_t cut = 0, bad = 0, sl = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nrec; i += stride) {
    sheep_xs1 r = rec[i];
    uint32_t t = r.tail, h = r.head;
    if (t >= pos_size || h >= pos_size) { ++bad; continue; }
    int tp = parts[t], hp = parts[h];
    uint32_t pt = pos[t], ph = pos[h];
    if (tp < 0 || hp < 0 || pt == INVALID || ph == INVALID) { ++bad; continue; }
    if (t == h) {
      ++sl;
      if (what & 2) set_bit(bdown, W, t, tp);
      if (what & 4) set_bit(bup, W, t, tp);
      if (what & 1) { set_bit(bhash, W, t, tp); set_bit(bvc, W, t, tp); }
      continue;
    }
    const int pdown = pt < ph ? tp : hp, pup = pt < ph ? hp : tp;
    if (what & 2) {
      set_bit(bdown, W, t, pdown); set_bit(bdown, W, h, pdown);
      if (lds) atomicAdd(&lbal[0][pdown], 1u); else atomicAdd(&bal[pdown], 1ull);
    }
    if (what & 4) {
      set_bit(bup, W, t, pup); set_bit(bup, W, h, pup);
      if (lds) atomicAdd(&lbal[1][pup], 1u); else atomicAdd(&bal[nparts + pup], 1ull);
    }
    if (what & 1) {
      const int ph_ = cormen_hash(t) < cormen_hash(h) ? tp : hp;
      set_bit(bhash, W, t, ph_); set_bit(bhash, W, h, ph_);
      if (lds) atomicAdd(&lbal[2][ph_], 1u); else atomicAdd(&bal[2 * nparts + ph_], 1ull);
      set_bit(bvc, W, t, hp); set_bit(bvc, W, h, tp);
      cut += tp != hp;
    }
  }
  cut = wave_sum(cut);
  bad = wave_sum(bad);
  sl = wave_sum(sl);
  if ((threadIdx.x & 63) == 0) {
    if (sl) atomicAdd(selfl, (unsigned long long)sl);
    if (cut) atomicAdd(&scal[0], (unsigned long long)cut);
    if (bad) atomicAdd(&scal[1], (unsigned long long)bad);
  }
  __syncthreads();
  if (lds)
    for (int i = threadIdx.x; i < 3 * nparts; i += BLOCK) {
      int a = i / nparts, p = i % nparts;
      uint32_t v = lbal[a][p];
      if (v) atomicAdd(&bal[i], (unsigned long long)v);
    }
}

// per vertex slot: nodes are the slots whose Vcom / ECV bitsets are non-empty
__global__ __launch_bounds__(BLOCK) void k_eval_nodes(uint64_t vs, const int16_t *__restrict__ parts, int what,
                                                      uint32_t W, int nparts, const uint32_t *__restrict__ bdown,
                                                      const uint32_t *__restrict__ bup,
                                                      const uint32_t *__restrict__ bhash,
                                                      const uint32_t *__restrict__ bvc,
                                                      unsigned long long *__restrict__ vbal,
                                                      unsigned long long *__restrict__ scal) {
  uint64_t sdown = 0, sup = 0, shash = 0, svc = 0, nodes = 0;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < vs; v += stride) {
    const uint32_t *any = (what & 2) ? bdown : ((what & 4) ? bup : bhash);
    uint32_t cd = 0, cu = 0, chh = 0, cv = 0;
    bool node = false;
    for (uint32_t w = 0; w < W; ++w) node |= any[v * W + w] != 0;
    if (!node) continue;
    ++nodes;
    int p = parts[v];
    for (uint32_t w = 0; w < W; ++w) {
      uint64_t o = v * W + w;
      if (what & 2) cd += __popc(bdown[o]);
      if (what & 4) cu += __popc(bup[o]);
      if (what & 1) {
        chh += __popc(bhash[o]);
        uint32_t x = bvc[o];
        if ((uint32_t)(p >> 5) == w) x |= 1u << (p & 31);
        cv += __popc(x);
      }
    }
    sdown += cd - 1; sup += cu - 1; shash += chh - 1; svc += cv - 1;
    if ((what & 1) && p >= 0 && p < nparts) atomicAdd(&vbal[p], 1ull);
  }
  sdown = wave_sum(sdown); sup = wave_sum(sup); shash = wave_sum(shash); svc = wave_sum(svc); nodes = wave_sum(nodes);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&scal[2], (unsigned long long)sdown);
    atomicAdd(&scal[3], (unsigned long long)sup);
    atomicAdd(&scal[4], (unsigned long long)shash);
    atomicAdd(&scal[5], (unsigned long long)svc);
    atomicAdd(&scal[6], (unsigned long long)nodes);
  }
}

__global__ void k_max_part(const int16_t *__restrict__ parts, uint64_t vs, unsigned long long *__restrict__ out) {
  int m = -1;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < vs; i += stride) m = parts[i] > m ? parts[i] : m;
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0 && m >= 0) atomicMax(out, (unsigned long long)m);
}

}  // namespace

// `what` bitmask: 1 = evaluate(graph) metrics, 2 = ECV(down), 4 = ECV(up).
void evaluate(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
              const int16_t *parts, int what, sheep_eval *out) {
  *out = sheep_eval();
  if (what == 0) what = 7;
  unsigned long long *scal = (unsigned long long *)c.d_scalars + 48;
  HIP_CHECK(hipMemsetAsync(scal, 0, 9 * sizeof(uint64_t), c.stream));
  if (pos_size) {
    hipLaunchKernelGGL(k_max_part, dim3(grid_for(pos_size)), dim3(BLOCK), 0, c.stream, parts, pos_size, scal + 7);
    LAUNCH_CHECK();
  }
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 55, scal + 7, sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  const int nparts = (int)c.h_scalars[55] + 1;   // max part + 1 (partition.cpp:433-435)
  const uint32_t W = (uint32_t)((nparts + 31) / 32);
  const uint64_t words = pos_size * W;
  uint32_t *bd = c.get_as<uint32_t>("ev_bdown", words ? words : 1);
  uint32_t *bu = (what & 4) ? c.get_as<uint32_t>("ev_bup", words) : bd;
  uint32_t *bh = (what & 1) ? c.get_as<uint32_t>("ev_bhash", words) : bd;
  uint32_t *bv = (what & 1) ? c.get_as<uint32_t>("ev_bvc", words) : bd;
  if (!(what & 2)) bd = (what & 4) ? bu : bh;
  for (uint32_t *b : {bd, bu, bh, bv}) HIP_CHECK(hipMemsetAsync(b, 0, words * sizeof(uint32_t), c.stream));
  unsigned long long *bal = c.get_as<unsigned long long>("ev_bal", 4 * (uint64_t)nparts);
  HIP_CHECK(hipMemsetAsync(bal, 0, 4 * (uint64_t)nparts * sizeof(uint64_t), c.stream));
  {
    // B_eval: record read + 2 pos + 2 part gathers, bitset write + read
    TimedRegion tr(c, "evaluate", 28 * nrec + 8 * words);
    if (nrec) {
      hipLaunchKernelGGL(k_eval_records, dim3(grid_for(nrec)), dim3(BLOCK), 0, c.stream, rec, nrec, pos, pos_size,
                         parts, what, W, nparts, bd, bu, bh, bv, bal, scal, scal + 8);
      LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_eval_nodes, dim3(grid_for(pos_size)), dim3(BLOCK), 0, c.stream, pos_size, parts, what, W,
                       nparts, bd, bu, bh, bv, bal + 3 * (uint64_t)nparts, scal);
    LAUNCH_CHECK();
  }
  std::vector<uint64_t> hb(4 * (uint64_t)nparts);
  HIP_CHECK(hipMemcpyAsync(hb.data(), bal, hb.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  HIP_CHECK(hipMemcpyAsync(c.h_scalars + 48, scal, 9 * sizeof(uint64_t), hipMemcpyDeviceToHost, c.stream));
  c.sync();
  if (c.h_scalars[49]) throw Error(SHEEP_ERR_RANGE, "evaluate: a vertex is unsequenced or unassigned");
  auto mx = [&](int a) { uint64_t m = 0; for (int p = 0; p < nparts; ++p) m = std::max(m, hb[(uint64_t)a * nparts + p]); return m; };
  out->edges_cut = c.h_scalars[48];
  out->ecv_down = c.h_scalars[50];
  out->ecv_up = c.h_scalars[51];
  out->ecv_hash = c.h_scalars[52];
  out->vcom_vol = c.h_scalars[53];
  out->nodes = c.h_scalars[54];
  // adjacency entries = 2 per record, 1 per self-loop (LLAMA stores a self-loop once)
  out->edges = (2 * nrec - c.h_scalars[56]) / 2;
  out->max_down_bal = mx(0);
  out->max_up_bal = mx(1);
  out->max_hash_bal = mx(2);
  out->max_vertex_bal = mx(3);
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
