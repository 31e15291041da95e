// group.hip — several GPUs of one node as one Sheep "world": the MI355X replacement of
// graph2tree's MPI -i / -r path (graph2tree.cpp:134-216).
//
// A world has `world` ranks; rank r owns edge shard r on one device.  Two ways to run it:
//   * one process drives every rank (sheep_group_create): a context and stream per rank,
//     one host thread per rank for the per-shard compute;
//   * one process per rank (sheep_group_join): `mpiexec -n W graph2tree ... -ir`, or one
//     rank per torch.distributed process in bench.py.  The processes meet over TCP
//     (mesh.hpp), which carries the RCCL bootstrap, barriers and host scalars.
// The algorithm is written once, over the ranks this process holds ("local" ranks):
// every exchange below names global ranks and does only its local side.
//
// Transports (the same for both ways, chosen when the world is formed):
//   RCCL   — every rank on a distinct device: ncclSend/ncclRecv, ncclAllReduce and
//            ncclBroadcast over xGMI (ncclCommInitAll in one process, ncclCommInitRank
//            with rank 0's unique id across processes);
//   copy   — one process, a device listed more than once: device-to-device copies;
//   host   — one process per rank, devices repeated (a one-GPU rehearsal of W ranks):
//            device -> host -> TCP -> host -> device.
//
//   reference (MPI)                               here
//   MPI_Allreduce(MAX / SUM) in mpiSequence       sheep_group_sequence: all-reduce of the
//     (sequence.h:72,78)                          degree histograms, max of max_slot
//   MPI_Reduce(mpi_merge_reduction)               sheep_group_build_tree: a gather of the
//     (jnode.cpp:203-250)                         partial trees + ONE K-way merge on rank 0,
//                                                 or binomial rounds of pairwise merges on
//                                                 disjoint rank pairs
//   Partition::mpi_sync (partition.cpp:69-79)     sheep_group_broadcast_parts
//   (evaluate on one rank)                        sheep_group_evaluate: per-shard bitsets,
//                                                 binomial OR-reduction, node pass on rank 0
//
// Failure path (what MPI's default error handler gives graph2tree -ir: a dead or stalled
// rank ends the job instead of wedging it).  A joined world opens its communicator
// NON-BLOCKING (ncclConfig_t.blocking = 0) and never waits inside RCCL: after every group
// of RCCL calls it polls ncclCommGetAsyncError and the ranks' streams against a deadline of
// SHEEP_JOIN_TIMEOUT seconds (default 300); the TCP links poll their sockets against the
// same deadline (mesh.hpp).  On an error or an expired deadline the collective aborts the
// communicators (ncclCommAbort), prints ONE line per local rank to stderr — rank, device bus
// id, collective, bytes, cause — and returns SHEEP_ERR_HIP through the C ABI; the world is
// then unusable (every later collective fails at once), and the drivers exit non-zero.
// sheep_group_abort does the same on request (a driver whose own control plane saw a rank
// die).
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

#include "common.hpp"
#include "mesh.hpp"

struct sheep_group {
  std::vector<sheep_ctx *> ctx;   // the local ranks' contexts
  std::vector<int> dev;           // their devices
  std::vector<int> rank;          // their global ranks
  int world = 0;
  std::vector<ncclComm_t> comm;   // per local rank when RCCL carries the data
  std::unique_ptr<sheep::Mesh> mesh;   // one process per rank
  int timeout_s = 300;            // SHEEP_JOIN_TIMEOUT: the deadline of every wait on other ranks
  bool failed = false;            // a collective failed or timed out: the communicators are aborted
  std::string failure;
};

namespace sheep {
void degree_count(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap, uint64_t *max_slot);
uint64_t sequence_from_degrees(Ctx &c, const uint32_t *deg, uint64_t vs, uint32_t *seq, uint32_t *pos);
void relabel_and_tree(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size, uint64_t n,
                      sheep_jnode *tree);
void merge_trees(Ctx &c, const sheep_jnode *a, const sheep_jnode *b, uint64_t n, sheep_jnode *out);
void merge_trees_many(Ctx &c, const sheep_jnode *trees, uint32_t k, uint64_t n, sheep_jnode *out);
void merge_parent_planes(Ctx &c, const uint32_t *planes, const uint32_t *pst_sum, uint32_t K, uint64_t n,
                         sheep_jnode *out);
void tree_planes(Ctx &c, const sheep_jnode *tree, uint64_t n, uint32_t *parent, uint32_t *pst);
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

// (ncclInProgress: a non-blocking communicator accepted the call; rccl_wait completes it)
#define NCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess && _r != ncclInProgress)                                        \
      throw Error(SHEEP_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r));     \
  } while (0)

int join_timeout() {
  // (a run-time setting, not a debug knob: how long the ranks wait for each other)
  const char *v = getenv("SHEEP_JOIN_TIMEOUT");
  const int t = v ? atoi(v) : 300;
  return t > 0 ? t : 300;
}

std::string bus_id(int device) {
  char b[64] = {0};
  if (hipDeviceGetPCIBusId(b, sizeof b, device) != hipSuccess) return "dev" + std::to_string(device);
  return b;
}

// Ends the world: one stderr line per local rank, every communicator aborted (its queued
// and running RCCL kernels stop), later collectives refused.
void fail_world(sheep_group *g, const char *what, size_t bytes, const std::string &why) {
  if (g->failed) return;
  g->failed = true;
  g->failure = std::string(what) + ": " + why;
  for (size_t i = 0; i < g->rank.size(); ++i)
    fprintf(stderr, "sheep: rank %d of %d (bus %s): %s of %zu bytes failed: %s\n", g->rank[i], g->world,
            bus_id(g->dev[i]).c_str(), what, bytes, why.c_str());
  fflush(stderr);
  for (ncclComm_t &c : g->comm)
    if (c) {
      (void)ncclCommAbort(c);
      c = nullptr;
    }
}

// Runs one collective; any failure inside it ends the world (above) and is rethrown.
template <typename F> void collective(sheep_group *g, const char *what, size_t bytes, F &&f) {
  if (g->failed) throw Error(SHEEP_ERR_HIP, std::string(what) + ": the world failed before (" + g->failure + ")");
  try {
    f();
  } catch (const std::exception &e) {
    fail_world(g, what, bytes, e.what());
    throw;
  }
}

__global__ void k_add_u32(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += stride) dst[i] += src[i];
}

Ctx &C(sheep_group *g, int li) { return g->ctx[li]->c; }
int nlocal(const sheep_group *g) { return (int)g->ctx.size(); }
// local index of global rank r, -1 when another process holds it
int local_of(const sheep_group *g, int r) {
  if (!g->mesh) return r;
  return r == g->rank[0] ? 0 : -1;
}
bool host_transport(const sheep_group *g) { return g->mesh && g->comm.empty(); }

// Runs f(local index) on one host thread per local rank (each on its rank's device) and
// rethrows the first failure.
void per_rank(sheep_group *g, const std::function<void(int)> &f) {
  const int L = nlocal(g);
  if (L == 1) {
    HIP_CHECK(hipSetDevice(g->dev[0]));
    f(0);
    return;
  }
  std::vector<std::exception_ptr> err(L);
  std::vector<std::thread> th;
  for (int i = 0; i < L; ++i)
    th.emplace_back([&, i]() {
      try {
        HIP_CHECK(hipSetDevice(g->dev[i]));
        f(i);
      } catch (...) {
        err[i] = std::current_exception();
      }
    });
  for (auto &t : th) t.join();
  for (auto &e : err)
    if (e) std::rethrow_exception(e);
}

void sync_all(sheep_group *g) {
  for (int i = 0; i < nlocal(g); ++i) {
    HIP_CHECK(hipSetDevice(g->dev[i]));
    C(g, i).sync();
  }
}

// Completes the RCCL calls just grouped: polls every local communicator's async state and
// stream until all are done, an error shows, or the deadline passes (no blocking wait
// inside RCCL or HIP, so a peer that never posts its side cannot wedge this rank).
void rccl_wait(sheep_group *g) {
  using Clock = std::chrono::steady_clock;
  const auto t0 = Clock::now(), until = t0 + std::chrono::seconds(g->timeout_s);
  for (;;) {
    bool done = true;
    for (int i = 0; i < nlocal(g); ++i) {
      ncclResult_t st = ncclSuccess;
      NCCL_CHECK(ncclCommGetAsyncError(g->comm[i], &st));
      if (st == ncclInProgress) { done = false; continue; }
      if (st != ncclSuccess) throw Error(SHEEP_ERR_HIP, std::string("RCCL: ") + ncclGetErrorString(st));
      HIP_CHECK(hipSetDevice(g->dev[i]));
      const hipError_t q = hipStreamQuery(C(g, i).stream);
      if (q == hipErrorNotReady) { done = false; continue; }
      HIP_CHECK(q);
    }
    if (done) break;
    const auto now = Clock::now();
    if (now > until) throw Error(SHEEP_ERR_HIP, "timed out after " + std::to_string(g->timeout_s) + " s (SHEEP_JOIN_TIMEOUT)");
    if (now - t0 > std::chrono::milliseconds(2)) std::this_thread::sleep_for(std::chrono::microseconds(50));
    else std::this_thread::yield();
  }
  sync_all(g);   // (complete: runs the contexts' after-sync work)
}

// bytes from rank `from` to rank `to` (global ranks): `src` is meaningful where `from` is
// local, `dst` where `to` is local.
struct Xfer { int from, to; const void *src; void *dst; size_t bytes; };

// Host transport: device -> host -> socket; sends on a helper thread, receives here.
void host_transfer(sheep_group *g, const std::vector<Xfer> &xs) {
  const int me = g->rank[0];
  std::vector<const Xfer *> out, in;
  for (const Xfer &x : xs) {
    if (x.from == me && x.to != me) out.push_back(&x);
    if (x.to == me && x.from != me) in.push_back(&x);
  }
  Ctx &c = C(g, 0);
  HIP_CHECK(hipSetDevice(g->dev[0]));
  c.sync();
  std::exception_ptr serr;
  std::thread sender([&]() {
    try {
      HIP_CHECK(hipSetDevice(g->dev[0]));
      std::vector<char> buf;
      for (const Xfer *x : out) {
        buf.resize(x->bytes);
        HIP_CHECK(hipMemcpy(buf.data(), x->src, x->bytes, hipMemcpyDeviceToHost));
        g->mesh->send(x->to, buf.data(), x->bytes);
      }
    } catch (...) {
      serr = std::current_exception();
    }
  });
  std::exception_ptr rerr;
  try {
    std::vector<char> buf;
    for (const Xfer *x : in) {
      buf.resize(x->bytes);
      g->mesh->recv(x->from, buf.data(), x->bytes);
      HIP_CHECK(hipMemcpy(x->dst, buf.data(), x->bytes, hipMemcpyHostToDevice));
    }
  } catch (...) {
    rerr = std::current_exception();
  }
  sender.join();
  for (const Xfer &x : xs)   // a transfer within this process (never issued today)
    if (x.from == me && x.to == me)
      HIP_CHECK(hipMemcpyAsync(x.dst, x.src, x.bytes, hipMemcpyDeviceToDevice, c.stream));
  if (serr) std::rethrow_exception(serr);
  if (rerr) std::rethrow_exception(rerr);
  c.sync();
}

// A set of point-to-point transfers issued together (one RCCL group: every pair on its
// own xGMI link), complete on return.  Every rank calls it with the same list.
void transfer_now(sheep_group *g, const std::vector<Xfer> &xs) {
  if (!g->comm.empty()) {
    sync_all(g);   // the sources are complete (they may come from other streams)
    NCCL_CHECK(ncclGroupStart());
    for (const Xfer &x : xs) {
      const int lf = local_of(g, x.from), lt = local_of(g, x.to);
      if (lf >= 0) NCCL_CHECK(ncclSend(x.src, x.bytes, ncclUint8, x.to, g->comm[lf], C(g, lf).stream));
      if (lt >= 0) NCCL_CHECK(ncclRecv(x.dst, x.bytes, ncclUint8, x.from, g->comm[lt], C(g, lt).stream));
    }
    NCCL_CHECK(ncclGroupEnd());
    rccl_wait(g);
    return;
  }
  if (host_transport(g)) {
    host_transfer(g, xs);
    return;
  }
  sync_all(g);   // copy transport: the sources are complete before another stream copies them
  for (const Xfer &x : xs) {
    HIP_CHECK(hipSetDevice(g->dev[x.to]));
    if (g->dev[x.from] == g->dev[x.to])
      HIP_CHECK(hipMemcpyAsync(x.dst, x.src, x.bytes, hipMemcpyDeviceToDevice, C(g, x.to).stream));
    else
      HIP_CHECK(hipMemcpyPeerAsync(x.dst, g->dev[x.to], x.src, g->dev[x.from], x.bytes, C(g, x.to).stream));
  }
  sync_all(g);
}

void transfer(sheep_group *g, const std::vector<Xfer> &xs, const char *what = "send/recv") {
  if (xs.empty()) return;
  size_t bytes = 0;
  for (const Xfer &x : xs) bytes += x.bytes;
  collective(g, what, bytes, [&]() { transfer_now(g, xs); });
}

// In-place sum of one u32 array per rank (the degree all-reduce); buf[li] per local rank.
void allreduce_sum_u32(sheep_group *g, uint32_t *const *buf, uint64_t count) {
  const int P = g->world;
  if (count == 0) return;
  if (!g->comm.empty()) {   // (also a world of one that asked for RCCL: the identity, through RCCL)
    collective(g, "all-reduce(sum) of degrees", count * sizeof(uint32_t), [&]() {
      sync_all(g);
      NCCL_CHECK(ncclGroupStart());
      for (int i = 0; i < nlocal(g); ++i)
        NCCL_CHECK(ncclAllReduce(buf[i], buf[i], count, ncclUint32, ncclSum, g->comm[i], C(g, i).stream));
      NCCL_CHECK(ncclGroupEnd());
      rccl_wait(g);
    });
    return;
  }
  if (P == 1) return;
  // reduce to rank 0, one rank at a time into a scratch array, then broadcast
  const int l0 = local_of(g, 0);
  uint32_t *tmp = nullptr;
  if (l0 >= 0) {
    HIP_CHECK(hipSetDevice(g->dev[l0]));
    tmp = C(g, l0).get_as<uint32_t>("grp_reduce_tmp", count);
  }
  for (int r = 1; r < P; ++r) {
    const int lr = local_of(g, r);
    transfer(g, {Xfer{r, 0, lr >= 0 ? buf[lr] : nullptr, tmp, count * sizeof(uint32_t)}}, "all-reduce(sum) of degrees");
    if (l0 >= 0) {
      HIP_CHECK(hipSetDevice(g->dev[l0]));
      hipLaunchKernelGGL(k_add_u32, dim3(grid_for(count)), dim3(BLOCK), 0, C(g, l0).stream, buf[l0],
                         (const uint32_t *)tmp, count);
      LAUNCH_CHECK();
    }
  }
  std::vector<Xfer> xs;
  for (int r = 1; r < P; ++r) {
    const int lr = local_of(g, r);
    xs.push_back(Xfer{0, r, l0 >= 0 ? buf[l0] : nullptr, lr >= 0 ? buf[lr] : nullptr, count * sizeof(uint32_t)});
  }
  transfer(g, xs, "all-reduce(sum) of degrees");
}

// Sum of one u32 array per rank into rank 0's (in place there); buf[li] per local rank.
void reduce_sum_u32_to0(sheep_group *g, uint32_t *const *buf, uint64_t count, const char *what) {
  const int P = g->world;
  if (count == 0) return;
  if (!g->comm.empty()) {
    collective(g, what, count * sizeof(uint32_t), [&]() {
      sync_all(g);
      NCCL_CHECK(ncclGroupStart());
      for (int i = 0; i < nlocal(g); ++i)
        NCCL_CHECK(ncclReduce(buf[i], buf[i], count, ncclUint32, ncclSum, 0, g->comm[i], C(g, i).stream));
      NCCL_CHECK(ncclGroupEnd());
      rccl_wait(g);
    });
    return;
  }
  if (P == 1) return;
  const int l0 = local_of(g, 0);
  uint32_t *tmp = nullptr;
  if (l0 >= 0) {
    HIP_CHECK(hipSetDevice(g->dev[l0]));
    tmp = C(g, l0).get_as<uint32_t>("grp_reduce_tmp", count);
  }
  for (int r = 1; r < P; ++r) {
    const int lr = local_of(g, r);
    transfer(g, {Xfer{r, 0, lr >= 0 ? buf[lr] : nullptr, tmp, count * sizeof(uint32_t)}}, what);
    if (l0 >= 0) {
      HIP_CHECK(hipSetDevice(g->dev[l0]));
      hipLaunchKernelGGL(k_add_u32, dim3(grid_for(count)), dim3(BLOCK), 0, C(g, l0).stream, buf[l0],
                         (const uint32_t *)tmp, count);
      LAUNCH_CHECK();
    }
  }
}

// rank 0's bytes to every rank; buf[li] per local rank
void broadcast(sheep_group *g, void *const *buf, size_t bytes, const char *what) {
  const int P = g->world;
  if (bytes == 0) return;
  if (!g->comm.empty()) {
    collective(g, what, bytes, [&]() {
      sync_all(g);
      NCCL_CHECK(ncclGroupStart());
      for (int i = 0; i < nlocal(g); ++i)
        NCCL_CHECK(ncclBroadcast(buf[i], buf[i], bytes, ncclUint8, 0, g->comm[i], C(g, i).stream));
      NCCL_CHECK(ncclGroupEnd());
      rccl_wait(g);
    });
    return;
  }
  if (P == 1) return;
  const int l0 = local_of(g, 0);
  std::vector<Xfer> xs;
  for (int r = 1; r < P; ++r) {
    const int lr = local_of(g, r);
    xs.push_back(Xfer{0, r, l0 >= 0 ? buf[l0] : nullptr, lr >= 0 ? buf[lr] : nullptr, bytes});
  }
  transfer(g, xs, what);
}

uint64_t allreduce_max(sheep_group *g, const std::vector<uint64_t> &local, const char *what) {
  uint64_t m = 0;
  for (uint64_t v : local) m = v > m ? v : m;
  if (g->mesh) collective(g, what, sizeof m, [&]() { m = g->mesh->allreduce_max(m); });
  return m;
}

void mesh_bcast(sheep_group *g, void *buf, size_t bytes, const char *what) {
  if (g->mesh) collective(g, what, bytes, [&]() { g->mesh->bcast(buf, bytes); });
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

static void group_free(sheep_group *g) {
  for (ncclComm_t c : g->comm) if (c) ncclCommDestroy(c);   // (aborted ones are null)
  for (sheep_ctx *c : g->ctx) sheep_ctx_destroy(c);
  delete g;
}

extern "C" {

int sheep_group_create(const int *devices, int ndev, sheep_group **out) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(devices && ndev >= 1 && out, "bad argument");
  sheep_group *g = new sheep_group();
  try {
    bool distinct = true;
    g->world = ndev;
    g->timeout_s = sheep::join_timeout();
    for (int r = 0; r < ndev; ++r) {
      for (int q = 0; q < r; ++q) distinct &= devices[q] != devices[r];
      sheep_ctx *c = nullptr;
      const int rc = sheep_ctx_create(devices[r], SHEEP_OWN_STREAM, &c);
      if (rc != SHEEP_OK) throw sheep::Error(rc, sheep_last_error());
      g->ctx.push_back(c);
      g->dev.push_back(devices[r]);
      g->rank.push_back(r);
    }
    if (distinct && ndev > 1) {
      g->comm.resize(ndev);
      NCCL_CHECK(ncclCommInitAll(g->comm.data(), ndev, devices));
    }
  } catch (...) {
    group_free(g);
    throw;
  }
  *out = g;
  GAPI_END
}

int sheep_group_join(int device, int rank, int world, const char *host, int port, int link, sheep_group **out) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(out && host && world >= 1 && rank >= 0 && rank < world && port > 0 && port < 65536, "bad argument");
  GNEED(link >= SHEEP_LINK_AUTO && link <= SHEEP_LINK_HOST, "bad link");
  sheep_group *g = new sheep_group();
  try {
    g->world = world;
    sheep_ctx *c = nullptr;
    const int rc = sheep_ctx_create(device, SHEEP_OWN_STREAM, &c);
    if (rc != SHEEP_OK) throw sheep::Error(rc, sheep_last_error());
    g->ctx.push_back(c);
    g->dev.push_back(device);
    g->rank.push_back(rank);
    g->timeout_s = sheep::join_timeout();
    g->mesh.reset(new sheep::Mesh(rank, world, host, port, sheep::bus_id(device), g->timeout_s));
    bool distinct = true;
    const auto &bus = g->mesh->bus_ids();
    for (int r = 0; r < world; ++r)
      for (int q = 0; q < r; ++q) distinct &= bus[q] != bus[r];
    if (link == SHEEP_LINK_RCCL && !distinct)
      throw sheep::Error(SHEEP_ERR_ARG, "RCCL needs every rank on its own device (two ranks share one)");
    // RCCL when asked for (a world of one included: every collective and a self send/recv
    // then run through RCCL, the one-GPU check of this transport) or, by default, when
    // every rank has a device of its own
    if (link == SHEEP_LINK_RCCL || (world > 1 && link == SHEEP_LINK_AUTO && distinct)) {
      ncclUniqueId id;
      if (rank == 0) NCCL_CHECK(ncclGetUniqueId(&id));
      sheep::mesh_bcast(g, &id, sizeof id, "RCCL bootstrap");
      HIP_CHECK(hipSetDevice(device));
      g->comm.resize(1);
      // non-blocking: the init runs in the background while this rank polls it against the
      // deadline (a rank that never arrives would otherwise hold ncclCommInitRank forever)
      sheep::collective(g, "ncclCommInitRank", 0, [&]() {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        NCCL_CHECK(ncclCommInitRankConfig(&g->comm[0], world, id, rank, &cfg));
        const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(g->timeout_s);
        for (;;) {
          ncclResult_t st = ncclInProgress;
          NCCL_CHECK(ncclCommGetAsyncError(g->comm[0], &st));
          if (st == ncclSuccess) break;
          if (st != ncclInProgress) throw sheep::Error(SHEEP_ERR_HIP, std::string("RCCL: ") + ncclGetErrorString(st));
          if (std::chrono::steady_clock::now() > until)
            throw sheep::Error(SHEEP_ERR_HIP, "timed out after " + std::to_string(g->timeout_s) + " s (SHEEP_JOIN_TIMEOUT)");
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
      });
    }
  } catch (...) {
    group_free(g);
    throw;
  }
  *out = g;
  GAPI_END
}

int sheep_group_destroy(sheep_group *g) {
  DeviceRestore dr;
  GAPI_BEGIN
  if (!g) return SHEEP_OK;
  group_free(g);
  GAPI_END
}

int sheep_group_size(const sheep_group *g) { return g ? g->world : 0; }
int sheep_group_local_count(const sheep_group *g) { return g ? (int)g->ctx.size() : 0; }
int sheep_group_rank(const sheep_group *g, int local) {
  return g && local >= 0 && local < (int)g->rank.size() ? g->rank[local] : -1;
}
sheep_ctx *sheep_group_ctx(sheep_group *g, int local) {
  return g && local >= 0 && local < (int)g->ctx.size() ? g->ctx[local] : nullptr;
}
int sheep_group_uses_rccl(const sheep_group *g) { return g && !g->comm.empty(); }

int sheep_group_barrier(sheep_group *g) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g, "null argument");
  sheep::collective(g, "barrier", 0, [&]() {
    sheep::sync_all(g);
    if (g->mesh) g->mesh->barrier();
  });
  GAPI_END
}

int sheep_group_allreduce_max_u64(sheep_group *g, uint64_t *v) {
  GAPI_BEGIN
  GNEED(g && v, "null argument");
  *v = sheep::allreduce_max(g, {*v}, "all-reduce(max)");
  GAPI_END
}

int sheep_group_abort(sheep_group *g, const char *reason) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g, "null argument");
  sheep::fail_world(g, "abort", 0, reason && *reason ? reason : "requested by the caller");
  GAPI_END
}

int sheep_group_failed(const sheep_group *g) { return g && g->failed ? 1 : 0; }

int sheep_group_set_tuning(sheep_group *g, const sheep_tuning *t) {
  GAPI_BEGIN
  GNEED(g, "null argument");
  for (sheep_ctx *c : g->ctx) {
    const int rc = sheep_ctx_set_tuning(c, t);
    if (rc != SHEEP_OK) return rc;
  }
  GAPI_END
}

int sheep_group_sequence(sheep_group *g, const sheep_xs1 *const *rec, const uint64_t *nrec, uint32_t *const *deg,
                         uint64_t cap, uint32_t *const *seq, uint32_t *const *pos, uint64_t *n_out, uint64_t *vs_out) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && rec && nrec && deg && seq && pos && n_out && vs_out, "null argument");
  const int L = sheep::nlocal(g);
  std::vector<uint64_t> ms(L, 0), n(L, 0);
  sheep::per_rank(g, [&](int i) {   // each shard's LLAMA degrees (mpiSequence, sequence.h:76-77)
    sheep::degree_count(sheep::C(g, i), rec[i], nrec[i], SHEEP_DEGREE_LLAMA, deg[i], cap, &ms[i]);
  });
  const uint64_t vs = sheep::allreduce_max(g, ms, "all-reduce(max) of max_slot");   // MPI_Allreduce(MAX), sequence.h:72
  sheep::allreduce_sum_u32(g, deg, vs);                              // MPI_Allreduce(SUM), sequence.h:78
  sheep::per_rank(g, [&](int i) {
    n[i] = sheep::sequence_from_degrees(sheep::C(g, i), deg[i], vs, seq[i], pos[i]);
    sheep::C(g, i).sync();
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
  const int P = g->world;
  // (a world of one over RCCL still runs the K-way path: its RCCL reduce and the parent-plane
  // merge, the one-GPU check of them; the merged tree of one tree is that tree)
  if ((P == 1 && g->comm.empty()) || reduce == 0 || n == 0) return SHEEP_OK;
  GNEED(reduce != 1 || P <= 64, "K-way reduce: at most 64 ranks (one merge pass)");
  const size_t tb = n * sizeof(sheep_jnode);
  const int l0 = sheep::local_of(g, 0);
  if (reduce == 1) {
    // gather + one K-way merge on rank 0.  Only the parents travel (n x 4 B per rank, every
    // transfer on its own link): the merge needs each tree's parents and the SUM of their pst
    // weights, which is one RCCL reduce to rank 0 instead of P - 1 more planes.
    const int L = sheep::nlocal(g);
    std::vector<uint32_t *> par(L), pst(L);
    uint32_t *planes = nullptr;
    sheep::per_rank(g, [&](int i) {
      sheep::Ctx &c = sheep::C(g, i);
      pst[i] = c.get_as<uint32_t>("grp_pst", n);
      if (i == l0) {   // rank 0's own parents straight into plane 0 of the stack
        planes = c.get_as<uint32_t>("grp_planes", (uint64_t)P * n);
        par[i] = planes;
      } else {
        par[i] = c.get_as<uint32_t>("grp_par", n);
      }
      sheep::tree_planes(c, tree[i], n, par[i], pst[i]);
      c.sync();
    });
    std::vector<sheep::Xfer> xs;
    for (int r = 1; r < P; ++r) {
      const int lr = sheep::local_of(g, r);
      xs.push_back(sheep::Xfer{r, 0, lr >= 0 ? par[lr] : nullptr, planes ? planes + (uint64_t)r * n : nullptr,
                               n * sizeof(uint32_t)});
    }
    {
      // the gather (and the pst reduce) as a timed region of every local rank's context
      // ("gather": send on the others, receive on rank 0; the host link's copies fall inside
      // the events too)
      std::vector<std::unique_ptr<sheep::TimedRegion>> tr;
      for (int i = 0; i < L; ++i) {
        HIP_CHECK(hipSetDevice(g->dev[i]));
        tr.emplace_back(new sheep::TimedRegion(sheep::C(g, i), "gather", tb / 2 + n * sizeof(uint32_t)));
      }
      sheep::transfer(g, xs, "gather of partial trees' parents");
      sheep::reduce_sum_u32_to0(g, pst.data(), n, "reduce of partial trees' pst");
      for (int i = 0; i < L; ++i) {
        HIP_CHECK(hipSetDevice(g->dev[i]));
        tr[i].reset();
      }
    }
    if (l0 >= 0) {
      HIP_CHECK(hipSetDevice(g->dev[l0]));
      sheep::merge_parent_planes(sheep::C(g, l0), planes, pst[l0], (uint32_t)P, n, tree[l0]);
      sheep::C(g, l0).sync();
    }
    return SHEEP_OK;
  }
  // binomial: at hop d, rank i with i % 2d == 0 receives from i + d (disjoint pairs) and merges
  for (int d = 1; d < P; d *= 2) {
    std::vector<sheep::Xfer> xs;
    for (int i = 0; i + d < P; i += 2 * d) {
      const int li = sheep::local_of(g, i), ls = sheep::local_of(g, i + d);
      sheep_jnode *in = nullptr;
      if (li >= 0) {
        HIP_CHECK(hipSetDevice(g->dev[li]));
        in = sheep::C(g, li).get_as<sheep_jnode>("grp_in", n);
      }
      xs.push_back(sheep::Xfer{i + d, i, ls >= 0 ? tree[ls] : nullptr, in, tb});
    }
    sheep::transfer(g, xs, "binomial hop of partial trees");
    sheep::per_rank(g, [&](int li) {
      const int r = g->rank[li];
      if (r % (2 * d) != 0 || r + d >= P) return;
      sheep_jnode *in = sheep::C(g, li).get_as<sheep_jnode>("grp_in", n);
      sheep_jnode *out = sheep::C(g, li).get_as<sheep_jnode>("grp_out", n);
      sheep::merge_trees(sheep::C(g, li), tree[li], in, n, out);
      HIP_CHECK(hipMemcpyAsync(tree[li], out, tb, hipMemcpyDeviceToDevice, sheep::C(g, li).stream));
      sheep::C(g, li).sync();
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
  sheep::per_rank(g, [&](int i) {   // map: JTree on every shard (graph2tree.cpp:185-189)
    sheep::relabel_and_tree(sheep::C(g, i), rec[i], nrec[i], pos[i], pos_size, n, tree[i]);
    sheep::C(g, i).sync();
  });
  const int rc = sheep_group_reduce_trees(g, tree, n, reduce);
  if (rc != SHEEP_OK) return rc;
  GAPI_END
}

int sheep_group_transfer(sheep_group *g, int from, int to, const void *src, void *dst, uint64_t bytes) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && from >= 0 && from < g->world && to >= 0 && to < g->world, "bad argument");
  const int lf = sheep::local_of(g, from), lt = sheep::local_of(g, to);
  GNEED((lf < 0 || src) && (lt < 0 || dst), "null buffer on a local rank");
  sheep::transfer(g, {sheep::Xfer{from, to, src, dst, (size_t)bytes}}, "send/recv");
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
  sheep::broadcast(g, (void *const *)parts, pos_size * sizeof(int16_t), "broadcast of parts");
  GAPI_END
}

int sheep_group_evaluate(sheep_group *g, const sheep_xs1 *const *rec, const uint64_t *nrec,
                         const uint32_t *const *pos, uint64_t pos_size, const int16_t *const *parts, int what,
                         sheep_eval *out) {
  DeviceRestore dr;
  GAPI_BEGIN
  GNEED(g && rec && nrec && pos && parts && out, "null argument");
  GNEED(!(what & ~7), "bad argument");
  const int P = g->world;
  const int l0 = sheep::local_of(g, 0);
  uint64_t np = 0;
  if (l0 >= 0) {
    HIP_CHECK(hipSetDevice(g->dev[l0]));
    np = (uint64_t)sheep::eval_num_parts(sheep::C(g, l0), parts[l0], pos_size);
  }
  sheep::mesh_bcast(g, &np, sizeof np, "broadcast of the part count");
  const int nparts = (int)np;
  uint64_t words = 0, aw = 0;
  sheep::eval_sizes(what, nparts, pos_size, &words, &aw);
  const int L = sheep::nlocal(g);
  std::vector<uint64_t *> bits(L), acc(L), rb(L), ra(L);
  sheep::per_rank(g, [&](int i) {   // every shard's owner bits and counts
    sheep::Ctx &c = sheep::C(g, i);
    bits[i] = c.get_as<uint64_t>("grp_ev_bits", words ? words : 1);
    acc[i] = c.get_as<uint64_t>("grp_ev_acc", aw);
    rb[i] = c.get_as<uint64_t>("grp_ev_rbits", words ? words : 1);
    ra[i] = c.get_as<uint64_t>("grp_ev_racc", aw);
    HIP_CHECK(hipMemsetAsync(bits[i], 0, words * sizeof(uint64_t), c.stream));
    HIP_CHECK(hipMemsetAsync(acc[i], 0, aw * sizeof(uint64_t), c.stream));
    sheep::eval_shard(c, rec[i], nrec[i], pos[i], pos_size, parts[i], what, nparts, bits[i], acc[i]);
    c.sync();
  });
  for (int d = 1; d < P; d *= 2) {   // binomial OR / sum reduction to rank 0
    std::vector<sheep::Xfer> xs;
    for (int i = 0; i + d < P; i += 2 * d) {
      const int li = sheep::local_of(g, i), ls = sheep::local_of(g, i + d);
      xs.push_back(sheep::Xfer{i + d, i, ls >= 0 ? bits[ls] : nullptr, li >= 0 ? rb[li] : nullptr,
                               words * sizeof(uint64_t)});
      xs.push_back(sheep::Xfer{i + d, i, ls >= 0 ? acc[ls] : nullptr, li >= 0 ? ra[li] : nullptr,
                               aw * sizeof(uint64_t)});
    }
    sheep::transfer(g, xs, "evaluator state reduction");
    sheep::per_rank(g, [&](int li) {
      const int r = g->rank[li];
      if (r % (2 * d) != 0 || r + d >= P) return;
      sheep::eval_combine(sheep::C(g, li), bits[li], rb[li], words, acc[li], ra[li], aw);
      sheep::C(g, li).sync();
    });
  }
  *out = sheep_eval();
  if (l0 >= 0) {
    HIP_CHECK(hipSetDevice(g->dev[l0]));
    sheep::eval_finish(sheep::C(g, l0), bits[l0], acc[l0], pos_size, parts[l0], what, nparts, out);
  }
  GAPI_END
}

}  // extern "C"
