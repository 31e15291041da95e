// =====================================================================================
//  ref_harness.cpp — drives the REFERENCE's own lib/ code (compiled from
//  /root/reference/lib where it lies; nothing is copied) to produce golden fixtures.
//
//  TEST INFRASTRUCTURE ONLY (oracle/).  Built by oracle/ref/Makefile into oracle/_ref/.
//
//  What is reference code here: JTree (jtree.h/.cpp), JNodeTable incl. merge, Facts,
//  save/load (jnode.h/.cpp), FastUnionFind (unionfind.h), Partition incl.
//  forwardPartition, evaluate(graph), evaluate(graph, seq), print,
//  writePartitionedGraph (partition.h/.cpp), degreeSequence / fileSequence /
//  readSequence / writeSequence (sequence.h), XS1Reader / SNAPReader (readerwriter.h).
//
//  What is ours: HarnessGraph, an implementation of the reference's GraphType template
//  concept (getMaxVid/getNodes/getEdges/isNode/getDeg/getNodeItr/getEdgeItr — the
//  concept LLAMAGraph and SNAPGraph implement, graph_wrapper.h:71-162).  LLAMA itself
//  is un-vendored (README:3-8); we do NOT provide a llama.h.  `#undef USE_LLAMA` after
//  defs.h keeps graph_wrapper.h from naming it, exactly as a USE_SNAP build would.
//  HarnessGraph restates LLAMA's load semantics (undirected doubling, self-loop stored
//  once, degree-0 slots not nodes) — see DESIGN.md §Oracle for what is pinned.
// =====================================================================================
#include <cstdint>
#include <cstring>
#include "defs.h"
#undef USE_LLAMA
#include "jtree.h"
#include "partition.h"
#include "sequence.h"

#include <omp.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

class HarnessGraph {
  std::vector<uint64_t> off;
  std::vector<vid_t> adj;
  vid_t max_nodes = 0;
  size_t num_nodes = 0;

 public:
  HarnessGraph(char const *filename, size_t part = 0, size_t num_parts = 0) {
    std::vector<vid_t> t, h;
    vid_t X, Y;
    size_t base = 0;   // index of the first record held in t/h
    if (strcmp(".dat", filename + strlen(filename) - 4) == 0) {
      std::ifstream s(filename, std::ios::binary);
      xs1 rec;
      if (num_parts != 0) {   // a partial load reads only its own contiguous record range
        s.seekg(0, std::ios::end);
        const size_t R = (size_t)s.tellg() / sizeof(xs1);
        const size_t b = (part - 1) * R / num_parts, e = part * R / num_parts;
        s.seekg((std::streamoff)(b * sizeof(xs1)), std::ios::beg);
        std::vector<xs1> buf(e - b);
        s.read((char *)buf.data(), (std::streamsize)(buf.size() * sizeof(xs1)));
        for (const xs1 &x : buf) { t.push_back(x.tail); h.push_back(x.head); }
        base = b;
        part = 1;
        num_parts = 0;
      } else {
        while (s.read((char *)&rec, sizeof rec)) { t.push_back(rec.tail); h.push_back(rec.head); }
      }
    } else {
      std::ifstream s(filename);
      while ((s >> X) && (s >> Y)) { t.push_back(X); h.push_back(Y); }
    }
    (void)base;
    size_t R = t.size(), beg = 0, end = R;
    if (num_parts != 0) { beg = (part - 1) * R / num_parts; end = part * R / num_parts; }
    for (size_t i = beg; i < end; ++i) max_nodes = std::max(max_nodes, std::max(t[i], h[i]) + 1);
    off.assign((size_t)max_nodes + 2, 0);
    for (size_t i = beg; i < end; ++i) { off[t[i] + 1]++; if (t[i] != h[i]) off[h[i] + 1]++; }
    for (size_t v = 0; v <= max_nodes; ++v) off[v + 1] += off[v];
    adj.resize(off[max_nodes]);
    std::vector<uint64_t> cur(off.begin(), off.end() - 1);
    for (size_t i = beg; i < end; ++i) {
      adj[cur[t[i]]++] = h[i];
      if (t[i] != h[i]) adj[cur[h[i]]++] = t[i];
    }
    for (vid_t v = 0; v < max_nodes; ++v) if (getDeg(v) != 0) ++num_nodes;
  }
  vid_t getMaxVid() const { return max_nodes; }
  size_t getNodes() const { return num_nodes; }
  size_t getEdges() const { return adj.size() / 2; }
  bool isNode(vid_t X) const { return X < max_nodes && getDeg(X) != 0; }
  size_t getDeg(vid_t X) const { return X < max_nodes ? off[X + 1] - off[X] : 0; }

  class NodeItr {
    HarnessGraph const *g; vid_t n;
   public:
    NodeItr(HarnessGraph const *gr) : g(gr), n(0) { while (n != g->max_nodes && g->getDeg(n) == 0) ++n; }
    vid_t operator*() const { return n; }
    vid_t operator++() { do { ++n; } while (n != g->max_nodes && g->getDeg(n) == 0); return n; }
    bool isEnd() const { return n == g->max_nodes; }
  };
  class EdgeItr {
    HarnessGraph const *g; uint64_t e, end;
   public:
    EdgeItr(HarnessGraph const *gr, vid_t X) : g(gr), e(gr->off[X]), end(gr->off[X + 1]) {}
    vid_t operator*() const { return g->adj[e]; }
    vid_t operator++() { ++e; return e < end ? g->adj[e] : INVALID_VID; }
    bool isEnd() const { return e == end; }
  };
  NodeItr getNodeItr() const { return NodeItr(this); }
  EdgeItr getEdgeItr(vid_t X) const { return EdgeItr(this, X); }
};

// The GraphType concept over an all-reduced degree vector: what degreeSequence
// (sequence.h:52-63) reads (getNodes, getNodeItr, getDeg), so the reference's own sort
// (by-reference comparator) orders mpiSequence's summed degrees.
class DegreeGraph {
  std::vector<esize_t> const &deg;
  size_t nodes = 0;

 public:
  explicit DegreeGraph(std::vector<esize_t> const &d) : deg(d) {
    for (esize_t x : d) nodes += x != 0;
  }
  size_t getNodes() const { return nodes; }
  size_t getDeg(vid_t X) const { return deg[X]; }
  class NodeItr {
    DegreeGraph const *g; vid_t n;
   public:
    NodeItr(DegreeGraph const *gr) : g(gr), n(0) { while (n != g->deg.size() && g->deg[n] == 0) ++n; }
    vid_t operator*() const { return n; }
    vid_t operator++() { do { ++n; } while (n != g->deg.size() && g->deg[n] == 0); return n; }
    bool isEnd() const { return n == g->deg.size(); }
  };
  NodeItr getNodeItr() const { return NodeItr(this); }
};

static void dump_parts(Partition const &p, char const *path) {
  std::ofstream o(path, std::ios::binary | std::ios::trunc);
  o.write((char const *)p.parts.data(), p.parts.size() * sizeof(part_t));
}

static int usage() {
  fprintf(stderr,
          "ref_harness seq G OUT_SEQ                      degreeSequence (LLAMA degrees)\n"
          "ref_harness tree G SEQ|- OUT_TRE [p/k]         JTree (+ partial load), TREEFAQS\n"
          "ref_harness print G SEQ|- [p/k]                JTree (+ partial load), JTree::print (graph2tree -t)\n"
          "ref_harness part G SEQ|- TREE PARTS_PREFIX k.. partition_tree -f -g flow + parts dumps\n"
          "ref_harness write G SEQ|- TREE k PREFIX        Partition + graph-based writePartitionedGraph\n"
          "ref_harness writefile G SEQ|- TREE k PREFIX    Partition + file-based writePartitionedGraph\n"
          "ref_harness time G k                           seconds for degreeSequence + JTree + Partition(k)\n"
          "mpiexec -n P ref_harness mpi G k              graph2tree -r -p k over P MPI ranks (timed)\n"
          "mpiexec -n P ref_harness mpi_ir G k           the same with the literal -i mpiSequence (sequence.h:85)\n"
          "ref_harness snap FILE                          SNAPReader::read pairs, one \"X Y\" per line\n");
  return 1;
}

int main(int argc, char **argv) {
  if (argc < 2) return usage();
  std::string cmd = argv[1];
  if (cmd == "snap" && argc == 3) {   // readerwriter.h:78-90, the text reader of .net files
    SNAPReader r(argv[2]);
    vid_t X, Y;
    while (r.read(X, Y)) printf("%u %u\n", (unsigned)X, (unsigned)Y);
    return 0;
  }
  if (cmd == "seq" && argc == 4) {
    HarnessGraph g(argv[2]);
    writeSequence(degreeSequence(g), argv[3]);
    return 0;
  }
  if (cmd == "tree" && (argc == 5 || argc == 6)) {
    size_t part = 0, num_parts = 0;
    if (argc == 6) sscanf(argv[5], "%zu/%zu", &part, &num_parts);
    HarnessGraph g(argv[2], part, num_parts);
    std::vector<vid_t> seq = strcmp(argv[3], "-") == 0 ? degreeSequence(g) : readSequence(argv[3]);
    JTree tree(g, seq);
    tree.jnodes.save(argv[4]);
    tree.jnodes.getFacts().print();
    return 0;
  }
  if (cmd == "print" && (argc == 4 || argc == 5)) {   // graph2tree -t (graph2tree.cpp:229-230)
    size_t part = 0, num_parts = 0;
    if (argc == 5) sscanf(argv[4], "%zu/%zu", &part, &num_parts);
    HarnessGraph g(argv[2], part, num_parts);
    std::vector<vid_t> seq = strcmp(argv[3], "-") == 0 ? degreeSequence(g) : readSequence(argv[3]);
    JTree tree(g, seq);
    tree.print();   // jtree.h:60-66 -> jnode.h:263-267
    return 0;
  }
  if (cmd == "part" && argc >= 7) {
    HarnessGraph g(argv[2]);
    std::vector<vid_t> seq = strcmp(argv[3], "-") == 0 ? degreeSequence(g) : readSequence(argv[3]);
    JNodeTable jnodes(argv[4]);
    jnodes.getFacts().print();
    for (int i = 6; i < argc; ++i) {
      short const k = atoi(argv[i]);
      Partition part(seq, jnodes, k, 1.03, false, true, false);
      part.print();
      part.evaluate(g, seq);
      std::string path = std::string(argv[5]) + "k" + argv[i] + ".parts";
      dump_parts(part, path.c_str());
    }
    return 0;
  }
  if (cmd == "write" && argc == 7) {
    HarnessGraph g(argv[2]);
    std::vector<vid_t> seq = strcmp(argv[3], "-") == 0 ? degreeSequence(g) : readSequence(argv[3]);
    JNodeTable jnodes(argv[4]);
    Partition part(seq, jnodes, (short)atoi(argv[5]), 1.03, false, true, false);
    part.print();
    part.writePartitionedGraph(g, seq, argv[6]);
    return 0;
  }
  if (cmd == "writefile" && argc == 7) {   // partition_tree -g G -o PREFIX SEQ TREE k
    HarnessGraph g(argv[2]);
    std::vector<vid_t> seq = strcmp(argv[3], "-") == 0 ? degreeSequence(g) : readSequence(argv[3]);
    JNodeTable jnodes(argv[4]);
    Partition part(seq, jnodes, (short)atoi(argv[5]), 1.03, false, true, false);
    part.print();
    char const *const input = argv[2];
    part.writePartitionedGraph(input, seq, argv[6]);
    return 0;
  }
  if (cmd == "time" && argc == 4) {   // bench.py cpu_baseline: graph load untimed (inputs resident)
    HarnessGraph g(argv[2]);
    auto const t0 = std::chrono::steady_clock::now();
    std::vector<vid_t> seq = degreeSequence(g);
    JTree tree(g, seq);
    tree.jnodes.makeKids();   // graph2tree.cpp:204-206 (Partition requires kids)
    Partition part(seq, tree.jnodes, (short)atoi(argv[3]), 1.03, false, true, false);
    double const s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"seconds\": %.6f, \"records\": %zu, \"nodes\": %zu, \"parts\": %zu}\n", s,
           (size_t)g.getEdges(), seq.size(), part.parts.size());
    return 0;
  }
  // bench.py cpu_baseline: graph2tree.cpp:134-216 (-i -r -p k).  "mpi_ir" is the literal
  // -ir: the reference's own mpiSequence (sequence.h:65-93), whose sort comparator captures
  // the degree vector BY VALUE (sequence.h:85); "mpi" sorts the same all-reduced degrees
  // with degreeSequence's by-reference comparator (sequence.h:52-63).
  if ((cmd == "mpi" || cmd == "mpi_ir") && argc == 4) {
    const bool literal = cmd == "mpi_ir";
    MPI_Init(nullptr, nullptr);
    int rank = 0, size = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    HarnessGraph g(argv[2], rank + 1, size);   // this rank's edge shard (graph2tree.cpp:162), untimed
    MPI_Barrier(MPI_COMM_WORLD);
    auto const t0 = std::chrono::steady_clock::now();
    // mpiSequence (sequence.h:65-83): the degree all-reduce as the reference does it; the
    // sort is degreeSequence's (by-reference comparator) over the summed degrees -- the
    // by-value capture at sequence.h:85 copies the degree vector per comparison and does
    // not finish at these sizes
    std::vector<vid_t> seq;
    if (literal) {
      seq = mpiSequence(g);
    } else {
      vid_t max_vid = 0, local_max = g.getMaxVid();
      MPI_Allreduce(&local_max, &max_vid, 1, MPI_UINT32_T, MPI_MAX, MPI_COMM_WORLD);
      std::vector<esize_t> degree(max_vid + 1), local_degree(max_vid + 1, 0);
      for (auto nitr = g.getNodeItr(); !nitr.isEnd(); ++nitr) local_degree[*nitr] = g.getDeg(*nitr);
      MPI_Allreduce(local_degree.data(), degree.data(), max_vid, MPI_UINT32_T, MPI_SUM, MPI_COMM_WORLD);
      seq = degreeSequence(DegreeGraph(degree));
    }
    auto const t1 = std::chrono::steady_clock::now();
    JTree tree(g, seq);                                   // map (graph2tree.cpp:185-189)
    auto const t2 = std::chrono::steady_clock::now();
    tree.jnodes.mpi_merge(false);                         // reduce (graph2tree.cpp:196)
    auto const t3 = std::chrono::steady_clock::now();
    if (rank == 0) tree.jnodes.makeKids();                // graph2tree.cpp:203-210
    Partition p = rank == 0 ? Partition(seq, tree.jnodes, (short)atoi(argv[3])) : Partition();
    p.mpi_sync();
    MPI_Barrier(MPI_COMM_WORLD);
    auto const t4 = std::chrono::steady_clock::now();
    auto sec = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double>(b - a).count();
    };
    if (rank == 0) {
      // FNV-1a digests of what the flow produced (untimed): the sequence, the merged tree and
      // the parts, so runs of the two sequence forms can be compared
      auto fnv = [](const void *p, size_t bytes) {
        uint64_t h = 1469598103934665603ull;
        for (size_t i = 0; i < bytes; ++i) h = (h ^ ((const unsigned char *)p)[i]) * 1099511628211ull;
        return (unsigned long long)h;
      };
      const unsigned long long hs = fnv(seq.data(), seq.size() * sizeof(vid_t));
      std::vector<uint32_t> tw(2 * (size_t)tree.jnodes.size());
      for (jnid_t i = 0; i < tree.jnodes.size(); ++i) {
        tw[2 * (size_t)i] = tree.jnodes.parent(i);
        tw[2 * (size_t)i + 1] = tree.jnodes.pst_weight(i);
      }
      const unsigned long long ht = fnv(tw.data(), tw.size() * sizeof(uint32_t));
      const unsigned long long hp = fnv(p.parts.data(), p.parts.size() * sizeof(part_t));
      printf("{\"seconds\": %.6f, \"ranks\": %d, \"threads\": %d, \"nodes\": %zu, \"sequence\": \"%s\", "
             "\"phases\": {\"sort\": %.6f, \"map\": %.6f, \"reduce\": %.6f, \"partition\": %.6f}, "
             "\"fnv\": {\"seq\": \"%016llx\", \"tree\": \"%016llx\", \"parts\": \"%016llx\"}}\n",
             sec(t0, t4), size, omp_get_max_threads(), seq.size(), literal ? "mpiSequence" : "degreeSequence",
             sec(t0, t1), sec(t1, t2), sec(t2, t3), sec(t3, t4), hs, ht, hp);
    }
    MPI_Finalize();
    return 0;
  }
  return usage();
}
