// sheep.hpp — C++ façade of libsheep_hip.so with the reference's lib/ names, so the
// drop-in CLIs (sheep_amd/cli/) read like chan150/sheep's own graph2tree.cpp,
// partition_tree.cpp, merge_trees.cpp and degree_sequence.cpp.
//
//   reference (file:line)                         here
//   GraphWrapper / LLAMAGraph (graph_wrapper.h:43)  GraphWrapper   (records resident in HBM)
//   degreeSequence / mpiSequence (sequence.h:52,65) degreeSequence (LLAMA degrees, on the GPU)
//   fileSequence (sequence.h:95-128)              fileSequence   (file degrees, on the GPU)
//   readSequence / writeSequence (:153-184)       readSequence / writeSequence (host text I/O)
//   JNodeTable (jnode.h:48-297)                   JNodeTable     (host nodes + device mirror)
//   JTree (jtree.h:111-122)                       JTree          (map step on the GPU)
//   Partition (partition.h:51-188)                Partition      (forwardPartition + evaluators)
//
// Errors: the C ABI's status codes become the exceptions the reference throws in the
// same places (std::bad_alloc for I/O and allocation, std::out_of_range for .at()).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "sheep_hip.h"

namespace sheep {

typedef uint32_t vid_t;   // defs.h:76 (LLAMA build)
typedef uint32_t esize_t;
typedef uint32_t jnid_t;  // jnode.h:42
typedef int16_t part_t;   // partition.h:43
constexpr vid_t INVALID_VID = 0xFFFFFFFFu;
constexpr jnid_t INVALID_JNID = 0xFFFFFFFFu;
constexpr part_t INVALID_PART = -1;

inline void check(int rc) {
  if (rc == SHEEP_OK) return;
  const std::string msg = sheep_last_error();
  if (rc == SHEEP_ERR_ALLOC) throw std::bad_alloc();
  if (rc == SHEEP_ERR_RANGE) throw std::out_of_range(msg);
  if (rc == SHEEP_ERR_ARG) throw std::invalid_argument(msg);
  throw std::runtime_error(msg);
}

// One HIP device + a stream of its own, shared by everything in the process.
// SHEEP_DEVICE selects the device (default 0).
class Context {
 public:
  static Context &get() {
    static Context c;
    return c;
  }
  sheep_ctx *handle() const { return h_; }
  void sync() const { check(sheep_ctx_sync(h_)); }
  ~Context() { sheep_ctx_destroy(h_); }

 private:
  Context() {
    if (sheep_abi_version() != SHEEP_ABI_VERSION)   // built against another header: struct layouts differ
      throw std::runtime_error("libsheep_hip.so ABI version " + std::to_string(sheep_abi_version()) +
                               ", this build expects " + std::to_string(SHEEP_ABI_VERSION));
    const char *d = getenv("SHEEP_DEVICE");
    check(sheep_ctx_create(d ? atoi(d) : 0, SHEEP_OWN_STREAM, &h_));
  }
  sheep_ctx *h_ = nullptr;
};
inline sheep_ctx *ctx() { return Context::get().handle(); }

// Owning device buffer (move-only), on the process context's device or a given one.
template <typename T>
class DeviceArray {
 public:
  DeviceArray() = default;
  explicit DeviceArray(size_t n, sheep_ctx *c = nullptr) : n_(n), c_(c ? c : ctx()) {
    void *p = nullptr;
    check(sheep_malloc(c_, (n ? n : 1) * sizeof(T), &p));
    p_ = (T *)p;
  }
  DeviceArray(DeviceArray &&o) noexcept : p_(o.p_), n_(o.n_), c_(o.c_) { o.p_ = nullptr; o.n_ = 0; }
  DeviceArray &operator=(DeviceArray &&o) noexcept {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    std::swap(c_, o.c_);
    return *this;
  }
  DeviceArray(const DeviceArray &) = delete;
  DeviceArray &operator=(const DeviceArray &) = delete;
  ~DeviceArray() {
    if (p_) sheep_free(c_, p_);
  }
  T *get() const { return p_; }
  size_t size() const { return n_; }
  void upload(const T *h, size_t cnt) { check(sheep_memcpy_h2d(c_, p_, h, cnt * sizeof(T))); }
  void upload_at(size_t off, const T *h, size_t cnt) { check(sheep_memcpy_h2d(c_, p_ + off, h, cnt * sizeof(T))); }
  void copy_from(const T *dev, size_t cnt) { check(sheep_memcpy_d2d(c_, p_, dev, cnt * sizeof(T))); }
  sheep_ctx *context() const { return c_; }
  void download(T *h, size_t cnt) const { check(sheep_memcpy_d2h(c_, h, p_, cnt * sizeof(T))); }

 private:
  T *p_ = nullptr;
  size_t n_ = 0;
  sheep_ctx *c_ = nullptr;
};

inline bool is_dat(const char *filename) {
  const size_t l = strlen(filename);
  return l >= 4 && strcmp(".dat", filename + l - 4) == 0;
}

inline std::vector<char> readBytes(const char *filename) {
  FILE *f = fopen(filename, "rb");
  if (!f) throw std::bad_alloc();   // the reference's loaders fail with bad_alloc / abort
  fseek(f, 0, SEEK_END);
  const long bytes = ftell(f);
  fseek(f, 0, SEEK_SET);
  std::vector<char> b(bytes > 0 ? (size_t)bytes : 0);
  const size_t got = b.empty() ? 0 : fread(b.data(), 1, b.size(), f);
  fclose(f);
  b.resize(got);
  return b;
}

// A .net (SNAP text) file parsed on the GPU (sheep_parse_net): the records in HBM.
// skip_comments: the graph loader's '#' / '%' header lines (see readRecords).
inline DeviceArray<sheep_xs1> parseNet(const char *filename, bool skip_comments, uint64_t *nrec, sheep_ctx *c = nullptr) {
  const std::vector<char> text = readBytes(filename);
  DeviceArray<char> dtext(text.size(), c);
  if (!text.empty()) dtext.upload(text.data(), text.size());
  DeviceArray<sheep_xs1> rec(text.size() / 4 + 1, c);   // a record takes >= 4 bytes ("a b\n")
  check(sheep_parse_net(c ? c : ctx(), dtext.get(), text.size(), skip_comments ? 1 : 0, rec.get(), rec.size(), nrec));
  return rec;
}

// The records of part `part` of `num_parts` (1-indexed contiguous record ranges, LLAMA's
// partial load: LLAMAGraph(filename, part, num_parts), graph_wrapper.h:43-63; num_parts = 0:
// the whole file) in HBM on context c.  A .dat file is read with pread over exactly the
// part's byte range (sheep_dat_range / sheep_read_dat), in 48-MB chunks uploaded as they
// arrive: no other byte of the file is read and no whole-part host copy is kept.  A SNAP
// text file is parsed whole on the GPU (record boundaries are only known after parsing;
// skip_comments: the graph loader's '#' / '%' lines) and the part's range kept.
inline DeviceArray<sheep_xs1> loadRecords(const char *filename, size_t part, size_t num_parts, sheep_ctx *c,
                                          bool skip_comments, uint64_t *nrec) {
  if (is_dat(filename)) {
    uint64_t first = 0, count = 0;
    if (sheep_dat_range(filename, part, num_parts, &first, &count) != SHEEP_OK)
      throw std::bad_alloc();   // the reference's loaders fail with bad_alloc / abort
    DeviceArray<sheep_xs1> rec(count, c);
    const uint64_t chunk = 1ull << 22;   // records (48 MB)
    std::vector<sheep_xs1> buf((size_t)std::min(count, chunk));
    uint64_t done = 0;
    while (done < count) {
      const uint64_t want = std::min(chunk, count - done);
      uint64_t got = 0;
      if (sheep_read_dat(filename, first + done, want, buf.data(), &got) != SHEEP_OK) throw std::bad_alloc();
      if (got) rec.upload_at(done, buf.data(), got);
      done += got;
      if (got < want) break;   // (the file shrank under us)
    }
    *nrec = done;
    return rec;
  }
  uint64_t n = 0;
  DeviceArray<sheep_xs1> all = parseNet(filename, skip_comments, &n, c);
  if (num_parts == 0) {
    *nrec = n;
    return all;
  }
  if (part < 1 || part > num_parts) throw std::bad_alloc();
  const uint64_t beg = (part - 1) * n / num_parts, end = part * n / num_parts;
  DeviceArray<sheep_xs1> rec(end - beg, c);
  if (end > beg) rec.copy_from(all.get() + beg, end - beg);
  *nrec = end - beg;
  return rec;
}

// 1 + the largest vid (max_nodes) and the self-loop count of records in HBM (one device pass)
inline void recordStats(sheep_ctx *c, const sheep_xs1 *rec, uint64_t nrec, uint64_t *max_slot, uint64_t *loops) {
  check(sheep_record_stats(c, rec, nrec, max_slot, loops));
}

// The graph of one (optionally partial, `part`/`num_parts` 1-indexed, contiguous record
// ranges like LLAMA's partial load) edge file, resident in HBM.  LLAMA semantics:
// undirected doubling, a self-loop stored once, degree-0 slots are not nodes.
class GraphWrapper {
 public:
  GraphWrapper(const char *filename, size_t part = 0, size_t num_parts = 0) {
    rec_ = loadRecords(filename, part, num_parts, ctx(), true, &nrec_);
    uint64_t loops = 0;
    recordStats(ctx(), rec_.get(), nrec_, &max_nodes_, &loops);
    edges_ = (2 * nrec_ - loops) / 2;   // max_edges / 2 (graph_wrapper.h:79-81)
    dat_ = is_dat(filename);
  }
  size_t getMaxVid() const { return max_nodes_; }
  size_t getEdges() const { return edges_; }
  size_t getNodes() const;   // slots with degree != 0 (counted on the GPU)
  const sheep_xs1 *records() const { return rec_.get(); }
  uint64_t numRecords() const { return nrec_; }
  bool isDat() const { return dat_; }
  std::vector<sheep_xs1> hostRecords() const {
    std::vector<sheep_xs1> h(nrec_);
    if (nrec_) rec_.download(h.data(), nrec_);
    return h;
  }

 private:
  DeviceArray<sheep_xs1> rec_;
  uint64_t nrec_ = 0, max_nodes_ = 0, edges_ = 0;
  bool dat_ = false;
  mutable int64_t nodes_ = -1;
};

// A sequence as the GPU path uses it: seq[n] and its inverse pos[pos_size] in HBM.
struct DeviceSequence {
  DeviceArray<uint32_t> seq, pos;
  uint64_t n = 0, pos_size = 0;
  std::vector<vid_t> host() const {
    std::vector<vid_t> h(n);
    if (n) seq.download(h.data(), n);
    return h;
  }
};

inline DeviceSequence sequenceFromDegrees(DeviceArray<uint32_t> &deg, uint64_t vs) {
  DeviceSequence s;
  s.seq = DeviceArray<uint32_t>(vs);
  s.pos = DeviceArray<uint32_t>(vs);
  check(sheep_sequence_from_degrees(ctx(), deg.get(), vs, s.seq.get(), s.pos.get(), &s.n));
  s.pos_size = vs;
  return s;
}

// degreeSequence (sequence.h:52-63): ascending (LLAMA degree, vid).
inline DeviceSequence degreeSequence(const GraphWrapper &g) {
  const uint64_t cap = std::max<uint64_t>(g.getMaxVid(), 1);
  DeviceArray<uint32_t> deg(cap);
  std::vector<uint32_t> zero(cap, 0);
  deg.upload(zero.data(), cap);
  uint64_t vs = 0;
  check(sheep_degree_count(ctx(), g.records(), g.numRecords(), SHEEP_DEGREE_LLAMA, deg.get(), cap, &vs));
  return sequenceFromDegrees(deg, vs);
}

inline size_t GraphWrapper::getNodes() const {
  if (nodes_ < 0) nodes_ = (int64_t)degreeSequence(*this).n;
  return (size_t)nodes_;
}

// fileSequence (sequence.h:95-128): degrees straight from the file records (self-loop
// +2; XS1Reader hands the last record out twice, readerwriter.h:138-146).
inline std::vector<vid_t> fileSequence(const char *filename) {
  uint64_t nrec = 0, cap = 0, loops = 0;
  // SNAPReader semantics for text (no comment skipping), parsed on the GPU
  DeviceArray<sheep_xs1> rec = loadRecords(filename, 0, 0, ctx(), false, &nrec);
  recordStats(ctx(), rec.get(), nrec, &cap, &loops);
  cap = std::max<uint64_t>(cap, 1);
  DeviceArray<uint32_t> deg(cap);
  std::vector<uint32_t> zero(cap, 0);
  deg.upload(zero.data(), cap);
  uint64_t vs = 0;
  check(sheep_degree_count(ctx(), rec.get(), nrec, is_dat(filename) ? SHEEP_DEGREE_FILE_DAT : SHEEP_DEGREE_FILE_NET,
                           deg.get(), cap, &vs));
  return sequenceFromDegrees(deg, vs).host();
}

inline std::vector<vid_t> readSequence(const char *filename) {   // readTextSequence
  std::vector<vid_t> seq;
  std::ifstream stream(filename);
  vid_t X;
  while (stream >> X) seq.push_back(X);
  return seq;
}

inline void writeSequence(const std::vector<vid_t> &seq, const char *filename) {   // writeTextSequence
  FILE *f = fopen(filename, "w");
  if (!f) throw std::runtime_error(std::string("cannot write ") + filename);
  for (vid_t X : seq) fprintf(f, "%u\n", X);
  fclose(f);
}

inline DeviceSequence uploadSequence(const std::vector<vid_t> &seq) {
  DeviceSequence s;
  s.n = seq.size();
  s.pos_size = seq.empty() ? 0 : (uint64_t)*std::max_element(seq.begin(), seq.end()) + 1;   // jtree.h:113
  s.seq = DeviceArray<uint32_t>(s.n);
  if (s.n) s.seq.upload(seq.data(), s.n);
  s.pos = DeviceArray<uint32_t>(s.pos_size);
  check(sheep_positions(ctx(), s.seq.get(), s.n, s.pos.get(), s.pos_size));
  return s;
}

// TREEFAQS (jnode.cpp:256-290, print jnode.h:285-291).
struct Facts {
  sheep_facts_t f;
  void print() const {
    printf("TREEFAQS: width:%zu\troots:%zu\n", (size_t)f.width, (size_t)f.root_cnt);
    printf("\tvheight:%zu\teheight:%zu\n", (size_t)f.vert_height, (size_t)f.edge_height);
    printf("\tverts:%zu\tedges:%zu\n", (size_t)f.vert_cnt, (size_t)f.edge_cnt);
    printf("\thalo:%zu\tcore:%zu\n", (size_t)f.halo_id, (size_t)f.core_id);
    printf("\tfill:%zu\n", (size_t)f.fill);
  }
};

// JNodeTable: host nodes ([end_id] + max_id JNodes, the .tre layout) with a device
// mirror and the persistent kid table (makeKids) made on demand.
class JNodeTable {
 public:
  explicit JNodeTable(jnid_t max_jnids = 0) : nodes_(max_jnids, sheep_jnode{INVALID_JNID, 0}), end_id_(0) {}
  explicit JNodeTable(const char *filename) {   // jnode.cpp:76-102 (load)
    FILE *f = fopen(filename, "rb");
    if (!f) throw std::bad_alloc();
    fseek(f, 0, SEEK_END);
    const long bytes = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (bytes < (long)sizeof(jnid_t)) { fclose(f); throw std::bad_alloc(); }
    nodes_.resize(((size_t)bytes - sizeof(jnid_t)) / sizeof(sheep_jnode));
    bool ok = fread(&end_id_, sizeof(jnid_t), 1, f) == 1;
    ok = ok && (nodes_.empty() || fread(nodes_.data(), sizeof(sheep_jnode), nodes_.size(), f) == nodes_.size());
    fclose(f);
    if (!ok || end_id_ > nodes_.size()) throw std::bad_alloc();
  }
  JNodeTable(JNodeTable &&) = default;
  JNodeTable &operator=(JNodeTable &&) = default;
  ~JNodeTable() {
    if (kids_) sheep_kids_destroy(kids_);
  }

  jnid_t size() const { return end_id_; }
  jnid_t max_id() const { return (jnid_t)nodes_.size(); }
  jnid_t parent(jnid_t id) const { return nodes_.at(id).parent; }
  esize_t pst_weight(jnid_t id) const { return nodes_.at(id).pst_weight; }
  std::vector<sheep_jnode> &nodes() { return nodes_; }
  const std::vector<sheep_jnode> &nodes() const { return nodes_; }

  void save(const char *filename) const {   // jnode.cpp:164-168
    FILE *f = fopen(filename, "wb");
    if (!f) throw std::bad_alloc();
    fwrite(&end_id_, sizeof(jnid_t), 1, f);
    if (!nodes_.empty()) fwrite(nodes_.data(), sizeof(sheep_jnode), nodes_.size(), f);
    fclose(f);
  }

  // The first end_id nodes in HBM (uploaded once; invalidated by assignments).
  const sheep_jnode *device() const {
    if (!dev_) {
      dev_.reset(new DeviceArray<sheep_jnode>(end_id_));
      if (end_id_) dev_->upload(nodes_.data(), end_id_);
    }
    return dev_->get();
  }
  // makeKids (jnode.h:190-204): kid lists in ascending id, kept on the device; the FFD
  // sort order persists across Partition calls (partition.cpp:104-106).
  sheep_kids *kids() const {
    if (!kids_) check(sheep_kids_create(ctx(), device(), end_id_, &kids_));
    return kids_;
  }

  // Result of a device computation: n nodes, end_id = n.
  void assign_from_device(const DeviceArray<sheep_jnode> &d, jnid_t n, jnid_t max_id) {
    nodes_.assign(std::max(n, max_id), sheep_jnode{INVALID_JNID, 0});
    if (n) d.download(nodes_.data(), n);
    end_id_ = n;
    dev_.reset();
    if (kids_) { sheep_kids_destroy(kids_); kids_ = nullptr; }
  }

  // merge (jnode.cpp:174-201): Liu over the union of both parent-edge sets, pst summed.
  void merge(const JNodeTable &lhs, const JNodeTable &rhs) {
    const jnid_t n = lhs.size();
    if (rhs.size() != n) throw std::invalid_argument("merge: trees of different sizes");
    DeviceArray<sheep_jnode> out(n);
    check(sheep_merge_trees(ctx(), lhs.device(), rhs.device(), n, out.get()));
    assign_from_device(out, n, std::max<jnid_t>(max_id(), n));
  }

  Facts getFacts() const {
    Facts x;
    check(sheep_facts(ctx(), device(), end_id_, &x.f));
    return x;
  }

  // JNodeTable::print(id) (jnode.h:263-267) on the default path: no junction data, so
  // width = 1 + pst (jnode.h:258-260), and pre_weight is 0 without USE_PRE_WEIGHT
  // (defs.h:62, jnode.h:139-153).
  void print(jnid_t id) const { printNode(nodes_.at(id)); }
  static void printNode(const sheep_jnode &x) {
    printf("%6zu:w%6zu:pre%6zu:pst        ->[%4zu]\n", (size_t)1 + x.pst_weight, (size_t)0, (size_t)x.pst_weight,
           (size_t)x.parent);
  }

 private:
  std::vector<sheep_jnode> nodes_;
  jnid_t end_id_ = 0;
  mutable std::unique_ptr<DeviceArray<sheep_jnode>> dev_;
  mutable sheep_kids *kids_ = nullptr;
};

// JTree(graph, seq) (jtree.h:111-122 + jtree.cpp:66-145): the map step.
class JTree {
 public:
  JNodeTable jnodes;
  JTree(const GraphWrapper &graph, const DeviceSequence &seq) {
    DeviceArray<sheep_jnode> t(seq.n);
    check(sheep_build_tree(ctx(), graph.records(), graph.numRecords(), seq.pos.get(), seq.pos_size, seq.n, t.get()));
    jnodes.assign_from_device(t, (jnid_t)seq.n, (jnid_t)seq.n);
  }
  jnid_t size() const { return jnodes.size(); }
  // JTree::print (jtree.h:60-66): one line per jnid, "id:vid" and the node's print(id).
  // The jnid->vid map is the sequence itself (get_sequence, jtree.h:50-57: every vid of
  // the sequence holds a jnid, make_pad being the default, jtree.h:88).
  void print(const std::vector<vid_t> &seq) const { printTree(jnodes.nodes(), size(), seq); }
  static void printTree(const std::vector<sheep_jnode> &nodes, jnid_t n, const std::vector<vid_t> &seq) {
    for (jnid_t id = 0; id != n; ++id) {
      printf("%4zu:%-8zu", (size_t)id, (size_t)seq.at(id));
      JNodeTable::printNode(nodes.at(id));
    }
  }
};

// The text files of writePartitionedGraph (partition.cpp:588-670): one SNAP text file per
// part, PREFIX%04d, lines "X Y"; record i goes to part ep[i].
//   file_order = true  — partition_tree -o (:632-670): the records as the input file is
//                        read; an XS1 file repeats its last record (XS1Reader tests eof
//                        before the read that fails, readerwriter.h:50-57).
//   file_order = false — graph2tree -p -o (:588-630): the graph's node order, X ascending,
//                        its adjacency in load (record) order, only X < Y.  LLAMA's own
//                        edge-iterator order is not in the reference, so the order of lines
//                        within a file is parity-unpinned here (the line multiset is pinned).
inline void write_partition_files(const std::vector<sheep_xs1> &rec, const std::vector<int16_t> &ep, part_t max_part,
                                  uint64_t vmax, const char *prefix, bool file_order, bool is_dat) {
  const uint64_t R = rec.size();
  if (max_part >= 10000) throw std::runtime_error("writePartitionedGraph: more than 9999 parts (partition.cpp:599)");
  std::vector<FILE *> files;
  std::vector<std::string> bufs(max_part + 1);
  for (part_t p = 0; p <= max_part; ++p) {
    char name[4096];
    snprintf(name, sizeof name, "%s%04d", prefix, (int)p);
    FILE *f = fopen(name, "w");
    if (!f) {
      for (FILE *o : files) fclose(o);
      throw std::runtime_error(std::string("cannot create ") + name);
    }
    files.push_back(f);
  }
  auto put = [&](part_t p, uint32_t x, uint32_t y) {
    std::string &b = bufs.at(p);
    char line[32];
    const int len = snprintf(line, sizeof line, "%u %u\n", x, y);
    b.append(line, len);
    if (b.size() > (1u << 20)) { fwrite(b.data(), 1, b.size(), files[p]); b.clear(); }
  };
  if (file_order) {
    for (uint64_t i = 0; i < R; ++i) put(ep[i], rec[i].tail, rec[i].head);
    if (is_dat && R) put(ep[R - 1], rec[R - 1].tail, rec[R - 1].head);
  } else {
    // counting sort of the non-loop records by their smaller vid, stable in record order
    std::vector<uint64_t> start(vmax + 1, 0);
    for (uint64_t i = 0; i < R; ++i)
      if (rec[i].tail != rec[i].head) ++start[std::min(rec[i].tail, rec[i].head) + 1];
    for (uint64_t v = 0; v < vmax; ++v) start[v + 1] += start[v];
    std::vector<uint64_t> order(start[vmax]);
    for (uint64_t i = 0; i < R; ++i)
      if (rec[i].tail != rec[i].head) order[start[std::min(rec[i].tail, rec[i].head)]++] = i;
    for (uint64_t i : order) put(ep[i], std::min(rec[i].tail, rec[i].head), std::max(rec[i].tail, rec[i].head));
  }
  for (part_t p = 0; p <= max_part; ++p) {
    fwrite(bufs[p].data(), 1, bufs[p].size(), files[p]);
    fclose(files[p]);
  }
}

inline void print_ratio_line(const char *label, uint64_t v, double denom) {
  printf("%s%zu (%f%%)\n", label, (size_t)v, (double)v / denom);
}

// Partition(seq, jnodes, k, balance, vtx, pst, pre) (partition.cpp:50-67).
class Partition {
 public:
  Partition(const DeviceSequence &seq, const JNodeTable &jnodes, part_t np, double balance_factor = 1.03,
            bool vtx_weight = false, bool pst_weight = true, bool pre_weight = false)
      : num_parts_(np) {
    if (pre_weight) throw std::invalid_argument("pre_weight (-u) is outside this build's scope");
    parts_ = DeviceArray<int16_t>(seq.pos_size);
    check(sheep_partition_pos(ctx(), jnodes.device(), jnodes.size(), seq.seq.get(), seq.n, seq.pos.get(), seq.pos_size,
                              jnodes.kids(), np, balance_factor, vtx_weight, pst_weight, parts_.get(), &info_));
  }
  const sheep_partition_info &info() const { return info_; }
  const int16_t *device() const { return parts_.get(); }
  std::vector<part_t> parts() const {
    std::vector<part_t> h(parts_.size());
    if (!h.empty()) parts_.download(h.data(), h.size());
    return h;
  }

  void print() const {   // partition.h:135-143
    printf("Actually created %d partitions.\n", (int)info_.created);
    printf("First two partition sizes: %zu and %zu\n", (size_t)info_.first_size, (size_t)info_.second_size);
  }

  // evaluate(graph) (partition.cpp:428-473) then evaluate(graph, seq) (:475-521).
  void evaluate(const GraphWrapper &graph, const DeviceSequence &seq) const {
    sheep_eval e;
    check(sheep_evaluate(ctx(), graph.records(), graph.numRecords(), seq.pos.get(), seq.pos_size, parts_.get(), 0,
                         &e));
    const double E = (double)e.edges;
    const double Nk = (double)(e.nodes / (uint64_t)num_parts_), Ek = (double)(e.edges / (uint64_t)num_parts_);
    print_ratio_line("edges cut: ", e.edges_cut, E);
    print_ratio_line("Vcom. vol: ", e.vcom_vol, E);
    print_ratio_line("  balance: ", e.max_vertex_bal, Nk);
    print_ratio_line("ECV(hash): ", e.ecv_hash, E);
    print_ratio_line("  balance: ", e.max_hash_bal, Ek);
    print_ratio_line("ECV(down): ", e.ecv_down, E);
    print_ratio_line("  balance: ", e.max_down_bal, Ek);
    print_ratio_line("ECV(up)  : ", e.ecv_up, E);
    print_ratio_line("  balance: ", e.max_up_bal, Ek);
  }

  // writePartitionedGraph (partition.cpp:588-670): one SNAP text file per part,
  // PREFIX%04d, lines "X Y".  An edge goes to the part of its earlier-positioned endpoint
  // (computed on the GPU, sheep_edge_parts).
  //   file_order = true  — partition_tree -o (:632-670): the records as the input file
  //                        is read; an XS1 file repeats its last record (XS1Reader tests
  //                        eof before the read that fails, readerwriter.h:50-57).
  //   file_order = false — graph2tree -p -o (:588-630): the graph's node order, X
  //                        ascending, its adjacency in load (record) order, only X < Y.
  void writePartitionedGraph(const GraphWrapper &g, const DeviceSequence &seq, const char *prefix,
                             bool file_order) const {
    const uint64_t R = g.numRecords();
    DeviceArray<int16_t> dpart(R);
    check(sheep_edge_parts(ctx(), g.records(), R, seq.pos.get(), seq.pos_size, parts_.get(), dpart.get()));
    std::vector<int16_t> ep(R);
    if (R) dpart.download(ep.data(), R);
    const std::vector<part_t> pv = parts();
    part_t max_part = -1;
    for (part_t x : pv) max_part = std::max(max_part, x);
    write_partition_files(g.hostRecords(), ep, max_part, g.getMaxVid(), prefix, file_order, g.isDat());
  }

 private:
  DeviceArray<int16_t> parts_;
  part_t num_parts_;
  sheep_partition_info info_{};
};

}  // namespace sheep
