// capi.hip — the extern "C" boundary of libsheep_hip.so (declared in include/sheep_hip.h).
// Exceptions never cross it: every entry point maps sheep::Error / std::exception to a
// status code and a thread-local message.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>

#include "common.hpp"
#include "tree_tour.hpp"

namespace sheep {
static thread_local std::string g_last_error;
void set_error(const char *msg) { g_last_error = msg; }
bool trace_launches() {
  static const bool on = debug_on("launches");
  return on;
}
void trace_launch(const char *file, int line) {
  const auto t0 = std::chrono::steady_clock::now();
  const hipError_t e = hipDeviceSynchronize();
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  fprintf(stderr, "sheep launch %s:%d %.1f us%s\n", file, line, us, e == hipSuccess ? "" : " FAILED");
}

void degree_count(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap, uint64_t *max_slot);
uint64_t sequence_from_degrees(Ctx &c, const uint32_t *deg, uint64_t vs, uint32_t *seq, uint32_t *pos);
void positions(Ctx &c, const uint32_t *seq, uint64_t n, uint32_t *pos, uint64_t pos_size);
void relabel_and_tree(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size, uint64_t n,
                      sheep_jnode *tree);
void merge_trees(Ctx &c, const sheep_jnode *a, const sheep_jnode *b, uint64_t n, sheep_jnode *out);
void merge_trees_many(Ctx &c, const sheep_jnode *trees, uint32_t k, uint64_t n, sheep_jnode *out);
void merge_trees_part(Ctx &c, const sheep_jnode *trees, uint32_t k, uint64_t n, uint32_t part, uint32_t nparts,
                      sheep_jnode *out, uint64_t *v_lo, uint64_t *v_hi);
void partition_tree(Ctx &c, const sheep_jnode *tree, uint64_t n, const uint32_t *seq, uint64_t seq_n, uint64_t pos_size,
                    sheep_kids *k, int16_t np, double balance, int vtx, int pstw, int16_t *parts_vid,
                    sheep_partition_info *info, const uint32_t *pos = nullptr);
void evaluate(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
              const int16_t *parts, int what, sheep_eval *out);
void evaluate_step(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *seq, uint64_t n, const uint32_t *pos,
                   uint64_t pos_size, const int16_t *parts, int what, sheep_eval *out);
void eval_sizes(int what, int nparts, uint64_t pos_size, uint64_t *bits_words, uint64_t *acc_words);
int eval_num_parts(Ctx &c, const int16_t *parts, uint64_t pos_size);
void eval_shard(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                const int16_t *parts, int what, int nparts, uint64_t *bits, uint64_t *acc);
void eval_combine(Ctx &c, uint64_t *bits, const uint64_t *bits_src, uint64_t words, uint64_t *acc,
                  const uint64_t *acc_src, uint64_t acc_words);
void eval_finish(Ctx &c, const uint64_t *bits, const uint64_t *acc, uint64_t pos_size, const int16_t *parts, int what,
                 int nparts, sheep_eval *out);
void tree_facts(Ctx &c, const sheep_jnode *tree, uint64_t n, sheep_facts_t *out);
void edge_parts(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                const int16_t *parts_vid, int16_t *out);
void record_stats(Ctx &c, const sheep_xs1 *rec, uint64_t nrec, uint64_t *max_slot, uint64_t *loops);
uint64_t parse_net(Ctx &c, const char *text, uint64_t bytes, int skip_comments, sheep_xs1 *out, uint64_t cap);
uint64_t rmat_generate(Ctx &c, int scale, int ef, uint64_t seed, sheep_xs1 *out, uint64_t cap);
uint64_t powerlaw_generate(Ctx &c, uint64_t V, uint64_t M, double gamma, uint64_t seed, sheep_xs1 *out, uint64_t cap);
uint64_t rmat_generate_host(int scale, int ef, uint64_t seed, sheep_xs1 *out, uint64_t cap);
}  // namespace sheep

using sheep::Error;

// Every entry point that takes a context runs on that context's device (workspaces are
// allocated and kernels launched there), whatever device the calling thread has current;
// the caller's current device is restored on return.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(const sheep_ctx *x) {
    if (!x) return;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != x->c.device) HIP_CHECK(hipSetDevice(x->c.device));
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

#define API_BEGIN try {
#define API_END                                                          \
  }                                                                      \
  catch (const sheep::Error &e) { sheep::set_error(e.what()); return e.code; } \
  catch (const std::bad_alloc &e) { sheep::set_error("bad_alloc"); return SHEEP_ERR_ALLOC; } \
  catch (const std::exception &e) { sheep::set_error(e.what()); return SHEEP_ERR_HIP; } \
  return SHEEP_OK;

#define NEED(cond, msg) \
  if (!(cond)) throw sheep::Error(SHEEP_ERR_ARG, msg)

extern "C" {

const char *sheep_last_error(void) { return sheep::g_last_error.c_str(); }

int sheep_abi_version(void) { return SHEEP_ABI_VERSION; }

int sheep_ctx_create(int device, void *hip_stream, sheep_ctx **out) {
  API_BEGIN
  NEED(out, "null out");
  int ndev = 0;
  HIP_CHECK(hipGetDeviceCount(&ndev));
  NEED(device >= 0 && device < ndev, "no such HIP device");
  HIP_CHECK(hipSetDevice(device));
  sheep_ctx *x = new sheep_ctx();
  x->c.device = device;
  if (hip_stream != SHEEP_OWN_STREAM) {
    x->c.stream = (hipStream_t)hip_stream;
  } else {
    HIP_CHECK(hipStreamCreateWithFlags(&x->c.stream, hipStreamNonBlocking));
    x->c.own_stream = true;
  }
  HIP_CHECK(hipHostMalloc((void **)&x->c.h_scalars, sheep::Ctx::NSCALARS * sizeof(uint64_t), hipHostMallocDefault));
  HIP_CHECK(hipMalloc((void **)&x->c.d_scalars, sheep::Ctx::NSCALARS * sizeof(uint64_t)));
  HIP_CHECK(hipMemset(x->c.d_scalars, 0, sheep::Ctx::NSCALARS * sizeof(uint64_t)));
  *out = x;
  API_END
}

int sheep_ctx_trim(sheep_ctx *ctx) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null context");
  sheep::Ctx &c = ctx->c;
  HIP_CHECK(hipSetDevice(c.device));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  for (auto &kv : c.ws) if (kv.second.p) HIP_CHECK(hipFree(kv.second.p));
  c.ws.clear();
  for (auto &l : c.layouts) l = sheep::Ctx::HeadLayout();   // their offsets lived in the workspace
  c.layout_next = 0;
  c.step_edges = sheep::Ctx::StepEdges();     // and the last map's grouped edges
  if (c.kid_spare.parent) {
    hipFree(c.kid_spare.parent); hipFree(c.kid_spare.koff); hipFree(c.kid_spare.kids); hipFree(c.kid_spare.kpar);
  }
  c.kid_spare = sheep::Ctx::KidBufs();
  API_END
}

int sheep_ctx_destroy(sheep_ctx *ctx) {
  API_BEGIN
  DeviceGuard dg(ctx);
  if (!ctx) return SHEEP_OK;
  sheep::Ctx &c = ctx->c;
  HIP_CHECK(hipSetDevice(c.device));
  HIP_CHECK(hipStreamSynchronize(c.stream));
  for (auto &kv : c.ws) if (kv.second.p) hipFree(kv.second.p);
  if (c.kid_spare.parent) {
    hipFree(c.kid_spare.parent); hipFree(c.kid_spare.koff); hipFree(c.kid_spare.kids); hipFree(c.kid_spare.kpar);
  }
  for (auto &kv : c.pinned) if (kv.second.p) hipHostFree(kv.second.p);
  for (auto &d : c.deferred) hipHostFree(d.host);
  for (auto &d : c.deferred_pool) hipHostFree(d.first);
  if (c.stage.p) hipHostFree(c.stage.p);
  for (char *p : c.stage_old) hipHostFree(p);
  for (auto &kv : c.timers) for (auto &p : kv.second.pending) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
  for (hipEvent_t e : c.event_pool) hipEventDestroy(e);
  if (c.h_scalars) hipHostFree(c.h_scalars);
  if (c.d_scalars) hipFree(c.d_scalars);
  if (c.own_stream) hipStreamDestroy(c.stream);
  delete ctx;
  API_END
}

int sheep_ctx_sync(sheep_ctx *ctx) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null ctx");
  ctx->c.sync();
  API_END
}

void *sheep_ctx_stream(sheep_ctx *ctx) { return ctx ? (void *)ctx->c.stream : nullptr; }

int sheep_malloc(sheep_ctx *ctx, size_t bytes, void **dev_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && dev_out, "null argument");
  HIP_CHECK(hipSetDevice(ctx->c.device));
  HIP_CHECK(hipMalloc(dev_out, bytes ? bytes : 1));
  API_END
}

int sheep_free(sheep_ctx *ctx, void *dev) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null ctx");
  if (dev) HIP_CHECK(hipFree(dev));
  API_END
}

int sheep_memcpy_h2d(sheep_ctx *ctx, void *dst, const void *src, size_t bytes) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null ctx");
  if (bytes) {
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->c.stream));
    ctx->c.sync();
  }
  API_END
}

int sheep_memcpy_d2h(sheep_ctx *ctx, void *dst, const void *src, size_t bytes) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null ctx");
  if (bytes) {
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->c.stream));
    ctx->c.sync();
  }
  API_END
}

int sheep_memcpy_d2d(sheep_ctx *ctx, void *dst, const void *src, size_t bytes) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null ctx");
  if (bytes) HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->c.stream));
  API_END
}

int sheep_record_stats(sheep_ctx *ctx, const sheep_xs1 *rec, uint64_t nrec, uint64_t *max_slot_out, uint64_t *loops_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && (rec || !nrec) && max_slot_out && loops_out, "null argument");
  sheep::record_stats(ctx->c, rec, nrec, max_slot_out, loops_out);
  API_END
}

int sheep_timer_enable(sheep_ctx *ctx, int on) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null ctx");
  ctx->c.timing = on != 0;
  API_END
}

int sheep_timer_get(sheep_ctx *ctx, const char *name, double *ms, uint64_t *launches, uint64_t *alg_bytes) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && name && ms && launches, "null argument");
  ctx->c.collect_timers();
  auto it = ctx->c.timers.find(name);
  const bool none = it == ctx->c.timers.end();
  *ms = none ? 0.0 : it->second.ms;
  *launches = none ? 0 : it->second.launches;
  if (alg_bytes) *alg_bytes = none ? 0 : it->second.bytes;
  API_END
}

int sheep_timer_names(sheep_ctx *ctx, char *buf, size_t cap) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && buf && cap, "null argument");
  std::string s;
  for (auto &kv : ctx->c.timers) { if (!s.empty()) s += ','; s += kv.first; }
  NEED(s.size() < cap, "buffer too small");
  memcpy(buf, s.c_str(), s.size() + 1);
  API_END
}

int sheep_ctx_workspace(sheep_ctx *ctx, char *buf, size_t cap) {
  API_BEGIN
  NEED(ctx && buf && cap, "null argument");
  std::vector<std::pair<size_t, std::string>> v;
  for (auto &kv : ctx->c.ws) if (kv.second.p) v.push_back({kv.second.bytes, kv.first});
  std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
  std::string s;
  for (auto &x : v) s += (s.empty() ? "" : ",") + x.second + "=" + std::to_string(x.first);
  NEED(s.size() < cap, "buffer too small");
  memcpy(buf, s.c_str(), s.size() + 1);
  API_END
}

int sheep_tuning_default(sheep_tuning *out) {
  API_BEGIN
  NEED(out, "null argument");
  *out = sheep::default_tuning();
  API_END
}

// The defaults filled in for SHEEP_TUNE_DEFAULT fields, every field range-checked.
static sheep_tuning resolve_tuning(const sheep_tuning *t) {
  const sheep_tuning d = sheep::default_tuning();
  if (!t) return d;
  sheep_tuning r = *t;
#define SHEEP_TUNE(f, ok)                                                                  \
  if (r.f == SHEEP_TUNE_DEFAULT) r.f = d.f;                                                \
  else if (!(ok)) throw sheep::Error(SHEEP_ERR_ARG, "sheep_tuning: " #f " out of range");
  SHEEP_TUNE(fin_map_bits, r.fin_map_bits >= 8 && r.fin_map_bits <= 13)
  SHEEP_TUNE(fin_merge_bits, r.fin_merge_bits >= 8 && r.fin_merge_bits <= 13)
  SHEEP_TUNE(fin_dc, r.fin_dc == 0 || r.fin_dc == 1)
  SHEEP_TUNE(top_bits, r.top_bits == 0 || (r.top_bits >= 9 && r.top_bits <= 16))
  SHEEP_TUNE(top_blocks, r.top_blocks >= 1 && r.top_blocks <= 9)
  SHEEP_TUNE(big_bits, r.big_bits == 0 || (r.big_bits >= 17 && r.big_bits <= 30))
  SHEEP_TUNE(big_dense, r.big_dense >= 1)
  SHEEP_TUNE(big_hot_bits, r.big_hot_bits >= 10 && r.big_hot_bits <= 15)
  SHEEP_TUNE(big_hot16, r.big_hot16 == 0 || r.big_hot16 == 1)
  SHEEP_TUNE(relabel_planes, r.relabel_planes == 0 || r.relabel_planes == 1)
  SHEEP_TUNE(relabel_per, r.relabel_per == 4 || r.relabel_per == 8 || r.relabel_per == 12 || r.relabel_per == 15)
  SHEEP_TUNE(cross_win_levels, r.cross_win_levels >= 0 && r.cross_win_levels <= 8)
  SHEEP_TUNE(hook_batch, r.hook_batch >= 0 && r.hook_batch <= 2)
  SHEEP_TUNE(hook_up, r.hook_up >= 0 && r.hook_up <= 2)
  SHEEP_TUNE(merge_cut_bits, r.merge_cut_bits == 0 || (r.merge_cut_bits >= 14 && r.merge_cut_bits <= 30))
  SHEEP_TUNE(event_loop, r.event_loop >= 0 && r.event_loop <= 4096)
#undef SHEEP_TUNE
  return r;
}

int sheep_ctx_set_tuning(sheep_ctx *ctx, const sheep_tuning *t) {
  API_BEGIN
  NEED(ctx, "null ctx");
  ctx->c.tune = resolve_tuning(t);
  API_END
}

int sheep_ctx_get_tuning(sheep_ctx *ctx, sheep_tuning *out) {
  API_BEGIN
  NEED(ctx && out, "null argument");
  *out = ctx->c.tune;
  API_END
}

int sheep_timer_reset(sheep_ctx *ctx) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx, "null ctx");
  ctx->c.collect_timers();
  ctx->c.timers.clear();
  API_END
}

int sheep_degree_count(sheep_ctx *ctx, const sheep_xs1 *rec, uint64_t nrec, int mode, uint32_t *deg, uint64_t cap,
                       uint64_t *max_slot_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && (rec || !nrec) && deg && max_slot_out, "null argument");
  sheep::degree_count(ctx->c, rec, nrec, mode, deg, cap, max_slot_out);
  API_END
}

int sheep_sequence_from_degrees(sheep_ctx *ctx, const uint32_t *deg, uint64_t vs, uint32_t *seq, uint32_t *pos,
                                uint64_t *n_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && (deg || !vs) && n_out, "null argument");
  *n_out = sheep::sequence_from_degrees(ctx->c, deg, vs, seq, pos);
  API_END
}

int sheep_positions(sheep_ctx *ctx, const uint32_t *seq, uint64_t n, uint32_t *pos, uint64_t pos_size) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && (seq || !n) && (pos || !pos_size), "null argument");
  sheep::positions(ctx->c, seq, n, pos, pos_size);
  API_END
}

int sheep_build_tree(sheep_ctx *ctx, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                     uint64_t n, sheep_jnode *tree) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && (rec || !nrec) && (pos || !pos_size) && (tree || !n), "null argument");
  NEED(n < 0xFFFFFFFFull, "tree too large for 32-bit node ids");
  sheep::relabel_and_tree(ctx->c, rec, nrec, pos, pos_size, n, tree);
  API_END
}

int sheep_merge_trees(sheep_ctx *ctx, const sheep_jnode *a, const sheep_jnode *b, uint64_t n, sheep_jnode *out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && ((a && b && out) || !n), "null argument");
  sheep::merge_trees(ctx->c, a, b, n, out);
  API_END
}

int sheep_merge_trees_many(sheep_ctx *ctx, const sheep_jnode *trees, uint32_t k, uint64_t n, sheep_jnode *out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && ((trees && out) || !n), "null argument");
  NEED(k >= 1, "merge: no trees");
  sheep::merge_trees_many(ctx->c, trees, k, n, out);
  API_END
}

int sheep_merge_trees_part(sheep_ctx *ctx, const sheep_jnode *trees, uint32_t k, uint64_t n, uint32_t part,
                           uint32_t nparts, sheep_jnode *out, uint64_t *v_lo, uint64_t *v_hi) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && v_lo && v_hi && ((trees && out) || !n), "null argument");
  NEED(k >= 1, "merge: no trees");
  sheep::merge_trees_part(ctx->c, trees, k, n, part, nparts, out, v_lo, v_hi);
  API_END
}

int sheep_kids_create(sheep_ctx *ctx, const sheep_jnode *tree, uint64_t n, sheep_kids **out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && out && (tree || !n), "null argument");
  sheep_kids *k = new sheep_kids();
  try {
    sheep::build_kids(ctx->c, tree, n, k);
  } catch (...) {
    hipFree(k->parent); hipFree(k->koff); hipFree(k->kids); hipFree(k->kpar);
    delete k;
    throw;
  }
  *out = k;
  API_END
}

int sheep_kids_destroy(sheep_kids *k) {
  API_BEGIN
  if (!k) return SHEEP_OK;
  int prev = -1;
  if (k->ctx && hipGetDevice(&prev) == hipSuccess && prev != k->ctx->device) HIP_CHECK(hipSetDevice(k->ctx->device));
  else prev = -1;
  sheep::release_kids(k->ctx, k);
  delete k;
  if (prev >= 0) HIP_CHECK(hipSetDevice(prev));
  API_END
}

int sheep_partition(sheep_ctx *ctx, const sheep_jnode *tree, uint64_t n, const uint32_t *seq, uint64_t seq_n, uint64_t pos_size,
                    sheep_kids *kids, int16_t k, double balance, int vtx_weight, int pst_weight, int16_t *parts_vid,
                    sheep_partition_info *info) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && kids && info && (tree || !n) && (seq || !seq_n) && (parts_vid || !pos_size), "null argument");
  sheep::partition_tree(ctx->c, tree, n, seq, seq_n, pos_size, kids, k, balance, vtx_weight, pst_weight, parts_vid, info);
  API_END
}

int sheep_partition_pos(sheep_ctx *ctx, const sheep_jnode *tree, uint64_t n, const uint32_t *seq, uint64_t seq_n,
                        const uint32_t *pos, uint64_t pos_size, sheep_kids *kids, int16_t k, double balance, int vtx_weight,
                        int pst_weight, int16_t *parts_vid, sheep_partition_info *info) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && kids && info && (tree || !n) && (seq || !seq_n) && ((parts_vid && pos) || !pos_size), "null argument");
  sheep::partition_tree(ctx->c, tree, n, seq, seq_n, pos_size, kids, k, balance, vtx_weight, pst_weight, parts_vid, info,
                        pos);
  API_END
}

int sheep_evaluate(sheep_ctx *ctx, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                   const int16_t *parts_vid, int what, sheep_eval *out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && out && (rec || !nrec) && ((pos && parts_vid) || !pos_size), "null argument");
  sheep::evaluate(ctx->c, rec, nrec, pos, pos_size, parts_vid, what, out);
  API_END
}

int sheep_evaluate_step(sheep_ctx *ctx, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *seq, uint64_t seq_n,
                        const uint32_t *pos, uint64_t pos_size, const int16_t *parts_vid, int what, sheep_eval *out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && out && (rec || !nrec) && (seq || !seq_n) && ((pos && parts_vid) || !pos_size), "null argument");
  sheep::evaluate_step(ctx->c, rec, nrec, seq, seq_n, pos, pos_size, parts_vid, what, out);
  API_END
}

int sheep_eval_sizes(int what, int32_t nparts, uint64_t pos_size, uint64_t *bits_words, uint64_t *acc_words) {
  API_BEGIN
  NEED(bits_words && acc_words && nparts >= 1, "bad argument");
  sheep::eval_sizes(what, nparts, pos_size, bits_words, acc_words);
  API_END
}

int sheep_eval_num_parts(sheep_ctx *ctx, const int16_t *parts_vid, uint64_t pos_size, int32_t *nparts_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && nparts_out && (parts_vid || !pos_size), "null argument");
  *nparts_out = sheep::eval_num_parts(ctx->c, parts_vid, pos_size);
  API_END
}

int sheep_eval_shard(sheep_ctx *ctx, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                     const int16_t *parts_vid, int what, int32_t nparts, uint64_t *bits, uint64_t *acc) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && bits && acc && (rec || !nrec) && ((pos && parts_vid) || !pos_size), "null argument");
  NEED(nparts >= 1 && !(what & ~7), "bad argument");
  sheep::eval_shard(ctx->c, rec, nrec, pos, pos_size, parts_vid, what, nparts, bits, acc);
  API_END
}

int sheep_eval_combine(sheep_ctx *ctx, uint64_t *bits, const uint64_t *bits_src, uint64_t words, uint64_t *acc,
                       const uint64_t *acc_src, uint64_t acc_words) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && ((bits && bits_src) || !words) && ((acc && acc_src) || !acc_words), "null argument");
  sheep::eval_combine(ctx->c, bits, bits_src, words, acc, acc_src, acc_words);
  API_END
}

int sheep_eval_finish(sheep_ctx *ctx, const uint64_t *bits, const uint64_t *acc, uint64_t pos_size,
                      const int16_t *parts_vid, int what, int32_t nparts, sheep_eval *out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && out && acc && ((bits && parts_vid) || !pos_size), "null argument");
  NEED(nparts >= 1 && !(what & ~7), "bad argument");
  sheep::eval_finish(ctx->c, bits, acc, pos_size, parts_vid, what, nparts, out);
  API_END
}

int sheep_edge_parts(sheep_ctx *ctx, const sheep_xs1 *rec, uint64_t nrec, const uint32_t *pos, uint64_t pos_size,
                     const int16_t *parts_vid, int16_t *edge_part) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && ((rec && pos && parts_vid && edge_part) || !nrec), "null argument");
  sheep::edge_parts(ctx->c, rec, nrec, pos, pos_size, parts_vid, edge_part);
  API_END
}

int sheep_facts(sheep_ctx *ctx, const sheep_jnode *tree, uint64_t n, sheep_facts_t *out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && out && (tree || !n), "null argument");
  sheep::tree_facts(ctx->c, tree, n, out);
  API_END
}

int sheep_parse_net(sheep_ctx *ctx, const char *text, uint64_t bytes, int skip_comments, sheep_xs1 *out, uint64_t cap,
                    uint64_t *nrec_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && nrec_out && (text || !bytes) && (out || !cap), "null argument");
  *nrec_out = sheep::parse_net(ctx->c, text, bytes, skip_comments, out, cap);
  API_END
}

int sheep_rmat_generate(sheep_ctx *ctx, int scale, int ef, uint64_t seed, sheep_xs1 *out, uint64_t cap,
                        uint64_t *nrec_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && out && nrec_out, "null argument");
  *nrec_out = sheep::rmat_generate(ctx->c, scale, ef, seed, out, cap);
  API_END
}

int sheep_powerlaw_generate(sheep_ctx *ctx, uint64_t nverts, uint64_t draws, double gamma, uint64_t seed,
                            sheep_xs1 *out, uint64_t cap, uint64_t *nrec_out) {
  API_BEGIN
  DeviceGuard dg(ctx);
  NEED(ctx && out && nrec_out, "null argument");
  *nrec_out = sheep::powerlaw_generate(ctx->c, nverts, draws, gamma, seed, out, cap);
  API_END
}

int sheep_rmat_generate_host(int scale, int ef, uint64_t seed, sheep_xs1 *out, uint64_t cap, uint64_t *nrec_out) {
  API_BEGIN
  NEED(out && nrec_out, "null argument");
  *nrec_out = sheep::rmat_generate_host(scale, ef, seed, out, cap);
  API_END
}

}  // extern "C"
