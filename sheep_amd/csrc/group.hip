// group.hip — several GPUs of one node as one Sheep "world": the MI355X replacement of
// graph2tree's MPI -i / -r path (graph2tree.cpp:134-216).
//
// One process drives every device (one context and stream per rank, one host thread
// per rank for the per-shard compute).  Exchanges between distinct devices go over RCCL
// (one communicator clique from ncclCommInitAll, xGMI); a device listed more than once
// (several shards rehearsed on one GPU) exchanges by device-to-device copies instead.
//
//   reference (MPI)                               here
//   MPI_Allreduce(MAX / SUM) in mpiSequence       sheep_group_sequence: ncclAllReduce of the
//     (sequence.h:72,78)                          degree histograms, host max of max_slot
//   MPI_Reduce(mpi_merge_reduction)               sheep_group_build_tree: a gather of the
//     (jnode.cpp:203-250)                         partial trees + ONE K-way merge on rank 0,
//                                                 or binomial rounds of pairwise merges on
//                                                 disjoint device pairs (ncclSend/ncclRecv)
//   Partition::mpi_sync (partition.cpp:69-79)     sheep_group_broadcast_parts: ncclBroadcast
//   (evaluate on one rank)                        sheep_group_evaluate: per-shard bitsets,
//                                                 binomial OR-reduction, node pass on rank 0
#include <rccl/rccl.h>

#include <cstring>
#include <exception>
#include <functional>
#include <thread>
#include <vector>

#include "common.hpp"

struct sheep_group {
  std::vector<sheep_ctx *> ctx;
  std::vector<int> dev;
  std::vector<ncclComm_t> comm;   // empty: copy transport
};

namespace sheep {
void degree_count(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap, uint64_t *max_slot);
uint64_t sequence_from_degrees(Ctx &c, const uint32_t *deg, uint64_t vs, uint32_t *seq, uint32_t *pos);
void relabel_and_tree(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size, uint64_t n,
                      sheep_jnode *tree);
void merge_trees(Ctx &c, const sheep_jnode *a, const sheep_jnode *b, uint64_t n, sheep_jnode *out);
void merge_trees_many(Ctx &c, const sheep_jnode *trees, uint32_t k, uint64_t n, sheep_jnode *out);
void eval_sizes(int what, int nparts, uint64_t pos_size, uint64_t *bits_words, uint64_t *acc_words);
int eval_num_parts(Ctx &c, const int16_t *parts, uint64_t pos_size);
void eval_shard(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                const int16_t *parts, int what, int nparts, uint64_t *bits, uint64_t *acc);
void eval_combine(Ctx &c, uint64_t *bits, const uint64_t *bits_src, uint64_t words, uint64_t *acc,
                  const uint64_t *acc_src, uint64_t acc_words);
void eval_finish(Ctx &c, const uint64_t *bits, const uint64_t *acc, uint64_t pos_size, const int16_t *parts, int what,
                 int nparts, sheep_eval *out);
void set_error(const char *msg);

namespace {

#define NCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess) throw Error(SHEEP_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

__global__ void k_add_u32(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) dst[i] += src[i];
}

Ctx &C(sheep_group *g, int r) { return g->ctx[r]->c; }
int size(const sheep_group *g) { return (int)g->ctx.size(); }

// Runs f(rank) on one host thread per rank (each on its rank's device) and rethrows the
// first failure.
void per_rank(sheep_group *g, const std::function<void(int)> &f) {
  const int P = size(g);
  if (P == 1) {
    HIP_CHECK(hipSetDevice(g->dev[0]));
    f(0);
    return;
  }
  std::vector<std::exception_ptr> err(P);
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r)
    th.emplace_back([&, r]() {
      try {
        HIP_CHECK(hipSetDevice(g->dev[r]));
        f(r);
      } catch (...) {
        err[r] = std::current_exception();
      }
    });
  for (auto &t : th) t.join();
  for (auto &e : err)
    if (e) std::rethrow_exception(e);
}

void sync_all(sheep_group *g) {
  for (int r = 0; r < size(g); ++r) {
    HIP_CHECK(hipSetDevice(g->dev[r]));
    C(g, r).sync();
  }
}

// bytes from rank `from` (src on its device) to rank `to` (dst on its device)
struct Xfer { int from, to; const void *src; void *dst; size_t bytes; };

// A set of point-to-point transfers issued together (one RCCL group: every pair on its
// own xGMI link), complete on return.
void transfer(sheep_group *g, const std::vector<Xfer> &xs) {
  if (xs.empty()) return;
  if (!g->comm.empty()) {
    NCCL_CHECK(ncclGroupStart());
    for (const Xfer &x : xs) {
      NCCL_CHECK(ncclSend(x.src, x.bytes, ncclUint8, x.to, g->comm[x.from], C(g, x.from).stream));
      NCCL_CHECK(ncclRecv(x.dst, x.bytes, ncclUint8, x.from, g->comm[x.to], C(g, x.to).stream));
    }
    NCCL_CHECK(ncclGroupEnd());
    sync_all(g);
    return;
  }
  sync_all(g);   // the sources are complete before another stream copies them
  for (const Xfer &x : xs) {
    HIP_CHECK(hipSetDevice(g->dev[x.to]));
    if (g->dev[x.from] == g->dev[x.to])
      HIP_CHECK(hipMemcpyAsync(x.dst, x.src, x.bytes, hipMemcpyDeviceToDevice, C(g, x.to).stream));
    else
      HIP_CHECK(hipMemcpyPeerAsync(x.dst, g->dev[x.to], x.src, g->dev[x.from], x.bytes, C(g, x.to).stream));
  }
  sync_all(g);
}

// In-place sum of one u32 array per rank (the degree all-reduce).
void allreduce_sum_u32(sheep_group *g, uint32_t *const *buf, uint64_t count) {
  const int P = size(g);
  if (P == 1 || count == 0) return;
  if (!g->comm.empty()) {
    NCCL_CHECK(ncclGroupStart());
    for (int r = 0; r < P; ++r)
      NCCL_CHECK(ncclAllReduce(buf[r], buf[r], count, ncclUint32, ncclSum, g->comm[r], C(g, r).stream));
    NCCL_CHECK(ncclGroupEnd());
    sync_all(g);
    return;
  }
  HIP_CHECK(hipSetDevice(g->dev[0]));
  uint32_t *tmp = C(g, 0).get_as<uint32_t>("grp_reduce_tmp", count);
  for (int r = 1; r < P; ++r) {
    transfer(g, {Xfer{r, 0, buf[r], tmp, count * sizeof(uint32_t)}});
    HIP_CHECK(hipSetDevice(g->dev[0]));
    hipLaunchKernelGGL(k_add_u32, dim3(grid_for(count)), dim3(BLOCK), 0, C(g, 0).stream, buf[0], (const uint32_t *)tmp,
                       count);
    LAUNCH_CHECK();
  }
  std::vector<Xfer> xs;
  for (int r = 1; r < P; ++r) xs.push_back(Xfer{0, r, buf[0], buf[r], count * sizeof(uint32_t)});
  transfer(g, xs);
}

void broadcast(sheep_group *g, void *const *buf, size_t bytes) {
  const int P = size(g);
  if (P == 1 || bytes == 0) return;
  if (!g->comm.empty()) {
    NCCL_CHECK(ncclGroupStart());
    for (int r = 0; r < P; ++r)
      NCCL_CHECK(ncclBroadcast(buf[r], buf[r], bytes, ncclUint8, 0, g->comm[r], C(g, r).stream));
    NCCL_CHECK(ncclGroupEnd());
    sync_all(g);
    return;
  }
  std::vector<Xfer> xs;
  for (int r = 1; r < P; ++r) xs.push_back(Xfer{0, r, buf[0], buf[r], bytes});
  transfer(g, xs);
}

}  // namespace
}  // namespace sheep

using sheep::Error;

#define GAPI_BEGIN try {
#define GAPI_END                                                                        \
  }                                                                                     \
  catch (const sheep::Error &e) { sheep::set_error(e.what()); return e.code; }           \
  catch (const std::bad_alloc &) { sheep::set_error("bad_alloc"); return SHEEP_ERR_ALLOC; } \
  catch (const std::exception &e) { sheep::set_error(e.what()); return SHEEP_ERR_HIP; }  \
  return SHEEP_OK;
#define GNEED(cond, msg) \
  if (!(cond)) throw sheep::Error(SHEEP_ERR_ARG, msg)

// restores the caller's current device on return
struct DeviceRestore {
  int prev = -1;
  DeviceRestore() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
  ~DeviceRestore() { if (prev >= 0) (void)hipSetDevice(prev); }
};

extern "C" {

int sheep_group_create(const int *devices, int ndev, sheep_group **out) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(devices && ndev >= 1 && out, "bad argument");
  sheep_group *g = new sheep_group();
  try {
    bool distinct = true;
    for (int r = 0; r < ndev; ++r) {
      for (int q = 0; q < r; ++q) distinct &= devices[q] != devices[r];
      sheep_ctx *c = nullptr;
      const int rc = sheep_ctx_create(devices[r], SHEEP_OWN_STREAM, &c);
      if (rc != SHEEP_OK) throw sheep::Error(rc, sheep_last_error());
      g->ctx.push_back(c);
      g->dev.push_back(devices[r]);
    }
    if (distinct && ndev > 1) {
      g->comm.resize(ndev);
      NCCL_CHECK(ncclCommInitAll(g->comm.data(), ndev, devices));
    }
  } catch (...) {
    for (ncclComm_t c : g->comm) if (c) ncclCommDestroy(c);
    for (sheep_ctx *c : g->ctx) sheep_ctx_destroy(c);
    delete g;
    throw;
  }
  *out = g;
  GAPI_END
}

int sheep_group_destroy(sheep_group *g) {
  DeviceRestore dr;
  GAPI_BEGIN
  if (!g) return SHEEP_OK;
  for (ncclComm_t c : g->comm) ncclCommDestroy(c);
  for (sheep_ctx *c : g->ctx) sheep_ctx_destroy(c);
  delete g;
  GAPI_END
}

int sheep_group_size(const sheep_group *g) { return g ? (int)g->ctx.size() : 0; }
sheep_ctx *sheep_group_ctx(sheep_group *g, int rank) {
  return g && rank >= 0 && rank < (int)g->ctx.size() ? g->ctx[rank] : nullptr;
}
int sheep_group_uses_rccl(const sheep_group *g) { return g && !g->comm.empty(); }

int sheep_group_sequence(sheep_group *g, const sheep_xs1 *const *rec, const uint64_t *nrec, uint32_t *const *deg,
                         uint64_t cap, uint32_t *const *seq, uint32_t *const *pos, uint64_t *n_out, uint64_t *vs_out) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && rec && nrec && deg && seq && pos && n_out && vs_out, "null argument");
  const int P = sheep::size(g);
  std::vector<uint64_t> ms(P, 0), n(P, 0);
  sheep::per_rank(g, [&](int r) {   // each shard's LLAMA degrees (mpiSequence, sequence.h:76-77)
    sheep::degree_count(sheep::C(g, r), rec[r], nrec[r], SHEEP_DEGREE_LLAMA, deg[r], cap, &ms[r]);
  });
  uint64_t vs = 0;
  for (uint64_t m : ms) vs = m > vs ? m : vs;                         // MPI_Allreduce(MAX), sequence.h:72
  sheep::allreduce_sum_u32(g, deg, vs);                               // MPI_Allreduce(SUM), sequence.h:78
  sheep::per_rank(g, [&](int r) {
    n[r] = sheep::sequence_from_degrees(sheep::C(g, r), deg[r], vs, seq[r], pos[r]);
    sheep::C(g, r).sync();
  });
  *n_out = n[0];
  *vs_out = vs;
  GAPI_END
}

int sheep_group_reduce_trees(sheep_group *g, sheep_jnode *const *tree, uint64_t n, int reduce) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && tree, "null argument");
  GNEED(reduce >= 0 && reduce <= 2, "bad reduce mode");
  const int P = sheep::size(g);
  if (P == 1 || reduce == 0 || n == 0) return SHEEP_OK;
  const size_t tb = n * sizeof(sheep_jnode);
  if (reduce == 1) {   // gather + one K-way merge on rank 0 (every transfer on its own link)
    HIP_CHECK(hipSetDevice(g->dev[0]));
    sheep_jnode *stack = sheep::C(g, 0).get_as<sheep_jnode>("grp_stack", (uint64_t)P * n);
    HIP_CHECK(hipMemcpyAsync(stack, tree[0], tb, hipMemcpyDeviceToDevice, sheep::C(g, 0).stream));
    std::vector<sheep::Xfer> xs;
    for (int r = 1; r < P; ++r) xs.push_back(sheep::Xfer{r, 0, tree[r], stack + (uint64_t)r * n, tb});
    sheep::transfer(g, xs);
    HIP_CHECK(hipSetDevice(g->dev[0]));
    sheep::merge_trees_many(sheep::C(g, 0), stack, (uint32_t)P, n, tree[0]);
    sheep::C(g, 0).sync();
    return SHEEP_OK;
  }
  // binomial: at hop d, rank i with i % 2d == 0 receives from i + d (disjoint pairs) and merges
  for (int d = 1; d < P; d *= 2) {
    std::vector<sheep::Xfer> xs;
    for (int i = 0; i + d < P; i += 2 * d) {
      HIP_CHECK(hipSetDevice(g->dev[i]));
      sheep_jnode *in = sheep::C(g, i).get_as<sheep_jnode>("grp_in", n);
      xs.push_back(sheep::Xfer{i + d, i, tree[i + d], in, tb});
    }
    sheep::transfer(g, xs);
    sheep::per_rank(g, [&](int r) {
      if (r % (2 * d) != 0 || r + d >= P) return;
      sheep_jnode *in = sheep::C(g, r).get_as<sheep_jnode>("grp_in", n);
      sheep_jnode *out = sheep::C(g, r).get_as<sheep_jnode>("grp_out", n);
      sheep::merge_trees(sheep::C(g, r), tree[r], in, n, out);
      HIP_CHECK(hipMemcpyAsync(tree[r], out, tb, hipMemcpyDeviceToDevice, sheep::C(g, r).stream));
      sheep::C(g, r).sync();
    });
  }
  GAPI_END
}

int sheep_group_build_tree(sheep_group *g, const sheep_xs1 *const *rec, const uint64_t *nrec,
                           const uint32_t *const *pos, uint64_t pos_size, uint64_t n, sheep_jnode *const *tree,
                           int reduce) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && rec && nrec && pos && tree, "null argument");
  GNEED(n < 0xFFFFFFFFull, "tree too large for 32-bit node ids");
  GNEED(reduce >= 0 && reduce <= 2, "bad reduce mode");
  sheep::per_rank(g, [&](int r) {   // map: JTree on every shard (graph2tree.cpp:185-189)
    sheep::relabel_and_tree(sheep::C(g, r), rec[r], nrec[r], pos[r], pos_size, n, tree[r]);
    sheep::C(g, r).sync();
  });
  const int rc = sheep_group_reduce_trees(g, tree, n, reduce);
  if (rc != SHEEP_OK) return rc;
  GAPI_END
}

int sheep_device_count(int *out) {
  GAPI_BEGIN
  GNEED(out, "null argument");
  HIP_CHECK(hipGetDeviceCount(out));
  GAPI_END
}

int sheep_group_broadcast_parts(sheep_group *g, int16_t *const *parts, uint64_t pos_size) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && parts, "null argument");
  sheep::sync_all(g);
  sheep::broadcast(g, (void *const *)parts, pos_size * sizeof(int16_t));
  GAPI_END
}

int sheep_group_evaluate(sheep_group *g, const sheep_xs1 *const *rec, const uint64_t *nrec,
                         const uint32_t *const *pos, uint64_t pos_size, const int16_t *const *parts, int what,
                         sheep_eval *out) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && rec && nrec && pos && parts && out, "null argument");
  GNEED(!(what & ~7), "bad argument");
  const int P = sheep::size(g);
  HIP_CHECK(hipSetDevice(g->dev[0]));
  const int nparts = sheep::eval_num_parts(sheep::C(g, 0), parts[0], pos_size);
  uint64_t words = 0, aw = 0;
  sheep::eval_sizes(what, nparts, pos_size, &words, &aw);
  std::vector<uint64_t *> bits(P), acc(P), rb(P), ra(P);
  sheep::per_rank(g, [&](int r) {   // every shard's owner bits and counts
    sheep::Ctx &c = sheep::C(g, r);
    bits[r] = c.get_as<uint64_t>("grp_ev_bits", words ? words : 1);
    acc[r] = c.get_as<uint64_t>("grp_ev_acc", aw);
    rb[r] = c.get_as<uint64_t>("grp_ev_rbits", words ? words : 1);
    ra[r] = c.get_as<uint64_t>("grp_ev_racc", aw);
    HIP_CHECK(hipMemsetAsync(bits[r], 0, words * sizeof(uint64_t), c.stream));
    HIP_CHECK(hipMemsetAsync(acc[r], 0, aw * sizeof(uint64_t), c.stream));
    sheep::eval_shard(c, rec[r], nrec[r], pos[r], pos_size, parts[r], what, nparts, bits[r], acc[r]);
    c.sync();
  });
  for (int d = 1; d < P; d *= 2) {   // binomial OR / sum reduction to rank 0
    std::vector<sheep::Xfer> xs;
    for (int i = 0; i + d < P; i += 2 * d) {
      xs.push_back(sheep::Xfer{i + d, i, bits[i + d], rb[i], words * sizeof(uint64_t)});
      xs.push_back(sheep::Xfer{i + d, i, acc[i + d], ra[i], aw * sizeof(uint64_t)});
    }
    sheep::transfer(g, xs);
    sheep::per_rank(g, [&](int r) {
      if (r % (2 * d) != 0 || r + d >= P) return;
      sheep::eval_combine(sheep::C(g, r), bits[r], rb[r], words, acc[r], ra[r], aw);
      sheep::C(g, r).sync();
    });
  }
  HIP_CHECK(hipSetDevice(g->dev[0]));
  sheep::eval_finish(sheep::C(g, 0), bits[0], acc[0], pos_size, parts[0], what, nparts, out);
  GAPI_END
}

}  // extern "C"
