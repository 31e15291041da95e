// graph2tree — drop-in for chan150/sheep graph2tree.cpp (same getopt string, same
// stdout lines, same .seq/.tre files) over libsheep_hip.so.
//
//   graph2tree input_graph [-s SEQ] [-o OUT] [-p K] [-l n/k] [-i] [-r] [-f] [-t] [-c] [-v]
//
// Phases (graph2tree.cpp:161-218): load the records into HBM, degree sequence (or -s
// read), map (JTree on the GPU), [reduce], [partition], [TREEFAQS].  -i / -r select the
// reference's MPI sort / reduce over a world of GPUs (sheep/world.hpp): one process per
// rank under `mpiexec -n W` (or torchrun), exactly the reference's launch, or one process
// driving the ranks of SHEEP_DEVICES — edge shards, an RCCL all-reduce of the degrees,
// per-GPU partial trees, the merge on rank 0, the parts broadcast and per-rank partition
// files, with the reference's file names (include/sheep_hip.h sheep_group_*).  With one
// rank the single-GPU path runs.  -t prints every node (JTree::print, jtree.h:60-66) on
// every rank.  Flags of the junction-tree experiments (-e -j -m -w -x) are rejected with a
// message.
#include <unistd.h>

#include <cassert>
#include <chrono>

#include "sheep/sheep.hpp"
#include "sheep/world.hpp"

using namespace sheep;

static double seconds_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t).count() / 1000.0;
}

// JTree::isValid (jtree.cpp:238-300) as far as it checks anything (the per-edge ancestor
// checks are vacuous there): index count == verts, parents later and in range.
static bool tree_valid(const std::vector<sheep_jnode> &nodes, uint64_t n, uint64_t vert_cnt) {
  bool ok = vert_cnt == n;
  for (uint64_t id = 0; ok && id != n; ++id) {
    const jnid_t p = nodes[id].parent;
    ok = p == INVALID_JNID || (p > id && p < n);
  }
  return ok;
}

// The -i / -r MPI world over several GPUs (graph2tree.cpp:134-216).  This process holds
// w.local() of the w.size() ranks (all of them without a launcher, one under mpiexec).
static int run_world(World &w, const char *graph_filename, bool use_mpi_sort, bool use_mpi_reduce,
                     size_t partitions, const char *sequence_filename, const char *output_filename, bool verbose,
                     bool do_faqs, bool do_print, bool do_validate,
                     std::chrono::steady_clock::time_point start_point) {
  const int P = w.size(), L = w.local();
  if (!use_mpi_sort && strcmp(sequence_filename, "") == 0) {
    printf("graph2tree: -r needs -i or -s SEQ (every rank must use the same sequence).\n");
    return 1;
  }
  const bool leader_here = w.rank(0) == 0;   // rank 0 prints (graph2tree.cpp:158-159)
  if (verbose) printf("Loading %s...\n", graph_filename);
  std::vector<RankState> rk(L);
  uint64_t cap = 1;   // the degree array's capacity: the same on every rank (the world's max vid + 1)
  for (int i = 0; i < L; ++i) {   // rank r loads part r+1 of P (graph2tree.cpp:137-143, 162): only its records
    const int r = w.rank(i);
    rk[i].rank = r;
    rk[i].rec = loadRecords(graph_filename, (size_t)r + 1, (size_t)P, w.ctx(i), true, &rk[i].nrec);
    uint64_t loops = 0;
    recordStats(w.ctx(i), rk[i].rec.get(), rk[i].nrec, &rk[i].max_vid, &loops);
    cap = std::max(cap, rk[i].max_vid);
  }
  check(sheep_group_allreduce_max_u64(w.handle(), &cap));
  const double load_s = seconds_since(start_point);
  if (leader_here) printf("Loaded graph in: %f seconds\n", load_s);

  std::vector<const sheep_xs1 *> recp(L);
  std::vector<uint64_t> nrec(L);
  std::vector<uint32_t *> seqp(L), posp(L), degp(L);
  for (int i = 0; i < L; ++i) { recp[i] = rk[i].rec.get(); nrec[i] = rk[i].nrec; }
  uint64_t n = 0, pos_size = 0;
  if (use_mpi_sort) {   // mpiSequence (sequence.h:65-93)
    const std::vector<uint32_t> zero(cap, 0);
    for (int i = 0; i < L; ++i) {
      rk[i].deg = DeviceArray<uint32_t>(cap, w.ctx(i));
      rk[i].deg.upload(zero.data(), cap);
      rk[i].seq = DeviceArray<uint32_t>(cap, w.ctx(i));
      rk[i].pos = DeviceArray<uint32_t>(cap, w.ctx(i));
      degp[i] = rk[i].deg.get(); seqp[i] = rk[i].seq.get(); posp[i] = rk[i].pos.get();
    }
    check(sheep_group_sequence(w.handle(), recp.data(), nrec.data(), degp.data(), cap, seqp.data(), posp.data(), &n,
                               &pos_size));
    if (leader_here && strcmp(sequence_filename, "") != 0) {   // rank 0 writes it (graph2tree.cpp:177-178)
      std::vector<vid_t> h(n);
      if (n) rk[0].seq.download(h.data(), n);
      writeSequence(h, sequence_filename);
    }
  } else {   // readSequence on every rank
    const std::vector<vid_t> h = readSequence(sequence_filename);
    n = h.size();
    pos_size = h.empty() ? 0 : (uint64_t)*std::max_element(h.begin(), h.end()) + 1;
    for (int i = 0; i < L; ++i) {
      rk[i].seq = DeviceArray<uint32_t>(n, w.ctx(i));
      if (n) rk[i].seq.upload(h.data(), n);
      rk[i].pos = DeviceArray<uint32_t>(pos_size, w.ctx(i));
      check(sheep_positions(w.ctx(i), rk[i].seq.get(), n, rk[i].pos.get(), pos_size));
      posp[i] = rk[i].pos.get();
    }
  }
  const double sort_s = seconds_since(start_point) - load_s;
  if (leader_here && (use_mpi_sort || strcmp(sequence_filename, "") == 0)) printf("Sorted in: %f seconds\n", sort_s);

  std::vector<sheep_jnode *> treep(L);
  for (int i = 0; i < L; ++i) { rk[i].tree = DeviceArray<sheep_jnode>(n, w.ctx(i)); treep[i] = rk[i].tree.get(); }
  std::vector<const uint32_t *> cposp(posp.begin(), posp.end());
  check(sheep_group_build_tree(w.handle(), recp.data(), nrec.data(), cposp.data(), pos_size, n, treep.data(), 0));
  const double map_s = seconds_since(start_point) - sort_s - load_s;
  if (leader_here) printf("Mapped in: %f seconds\n", map_s);
  if (use_mpi_reduce) {   // mpi_merge (jnode.cpp:213-250): gather + one K-way merge on rank 0
    check(sheep_group_reduce_trees(w.handle(), treep.data(), n, 1));
    const double reduce_s = seconds_since(start_point) - map_s - sort_s - load_s;
    if (leader_here) printf("Reduced in: %f seconds\n", reduce_s);
  }

  // graph2tree.cpp:144-156: -i alone maps rank r into OUTPUTrr r0.tre (its partition files
  // too), -r -p writes PREFIX-wRRRR-pPPPP
  auto rank_output = [&](int r) {
    char buf[4096];
    if (!use_mpi_reduce) snprintf(buf, sizeof buf, "%s%02dr0.tre", output_filename, r);
    else if (partitions != 0) snprintf(buf, sizeof buf, "%s-w%04d-p", output_filename, r);
    else snprintf(buf, sizeof buf, "%s", output_filename);
    return std::string(buf);
  };
  if (partitions != 0) {   // graph2tree.cpp:203-213
    std::vector<int16_t *> partp(L);
    for (int i = 0; i < L; ++i) { rk[i].parts = DeviceArray<int16_t>(pos_size, w.ctx(i)); partp[i] = rk[i].parts.get(); }
    sheep_partition_info info{};
    // with -r rank 0 partitions the merged tree and mpi_sync broadcasts it; without, every
    // rank partitions its own partial tree
    for (int i = 0; i < L; ++i) {
      if (use_mpi_reduce && rk[i].rank != 0) continue;
      sheep_kids *kids = nullptr;
      check(sheep_kids_create(w.ctx(i), rk[i].tree.get(), n, &kids));
      sheep_partition_info inf{};
      const int rc = sheep_partition_pos(w.ctx(i), rk[i].tree.get(), n, rk[i].seq.get(), n, rk[i].pos.get(), pos_size,
                                         kids, (int16_t)partitions, 1.03, 0, 1, rk[i].parts.get(), &inf);
      sheep_kids_destroy(kids);
      check(rc);
      if (rk[i].rank == 0) info = inf;
    }
    if (use_mpi_reduce) check(sheep_group_broadcast_parts(w.handle(), partp.data(), pos_size));   // p.mpi_sync()
    if (strcmp(output_filename, "") != 0) {   // every rank writes its shard's files
      for (int i = 0; i < L; ++i) {
        std::vector<int16_t> pv(pos_size);
        if (pos_size) rk[i].parts.download(pv.data(), pos_size);
        part_t max_part = -1;
        for (part_t x : pv) max_part = std::max(max_part, x);
        DeviceArray<int16_t> ep(nrec[i], w.ctx(i));
        check(sheep_edge_parts(w.ctx(i), rk[i].rec.get(), nrec[i], rk[i].pos.get(), pos_size, rk[i].parts.get(),
                               ep.get()));
        std::vector<int16_t> eh(nrec[i]);
        if (nrec[i]) ep.download(eh.data(), nrec[i]);
        std::vector<sheep_xs1> host(nrec[i]);   // (the writer's records: read back only to write them)
        if (nrec[i]) rk[i].rec.download(host.data(), nrec[i]);
        write_partition_files(host, eh, max_part, rk[i].max_vid, rank_output(rk[i].rank).c_str(), false, false);
      }
    } else if (leader_here) {
      printf("Actually created %d partitions.\n", (int)info.created);
      printf("First two partition sizes: %zu and %zu\n", (size_t)info.first_size, (size_t)info.second_size);
    }
  } else if (strcmp(output_filename, "") != 0) {
    for (int i = 0; i < L; ++i) {
      if (use_mpi_reduce && rk[i].rank != 0) continue;   // rank 0 saves the merged tree (:217-218)
      JNodeTable t;
      t.assign_from_device(rk[i].tree, (jnid_t)n, (jnid_t)n);
      t.save(rank_output(rk[i].rank).c_str());
    }
  }
  w.barrier();   // MPI_Finalize
  if (verbose) printf("Built in: %f seconds\n", seconds_since(start_point));
  // graph2tree.cpp:227-236 are not leader-gated: every rank prints its own tree's facts,
  // nodes and check (rank 0's tree is the merged one with -r, the others' their shard's);
  // a process holding several ranks prints them one rank after another
  if (do_faqs || do_print || do_validate) {
    std::vector<vid_t> seq_host;
    if (do_print) {
      seq_host.resize(n);
      if (n) rk[0].seq.download(seq_host.data(), n);
    }
    for (int i = 0; i < L; ++i) {
      Facts f;
      check(sheep_facts(w.ctx(i), rk[i].tree.get(), n, &f.f));
      if (do_faqs) f.print();
      std::vector<sheep_jnode> h;
      if (do_print || do_validate) {
        h.resize(n);
        if (n) rk[i].tree.download(h.data(), n);
      }
      if (do_print) JTree::printTree(h, (jnid_t)n, seq_host);
      if (do_validate) printf(tree_valid(h, n, f.f.vert_cnt) ? "Tree is valid.\n" : "ERROR: Tree is not valid.\n");
    }
  }
  if (verbose) printf("Finished in: %f seconds\n", seconds_since(start_point));
  return 0;
}

int main(int argc, char *argv[]) {
  bool use_mpi_sort = false, use_mpi_reduce = false;
  size_t part = 0, num_parts = 0, partitions = 0;
  const char *sequence_filename = "";
  const char *output_filename = "";
  bool verbose = false, do_faqs = false, do_print = false, do_validate = false;

  opterr = 0;
  int opt;
  while ((opt = getopt(argc, argv, "irl:p:s:o:vkejm:w:xfdtc")) != -1) {
    switch (opt) {
      case 'i': use_mpi_sort = !use_mpi_sort; break;
      case 'r': use_mpi_reduce = !use_mpi_reduce; break;
      case 'l':
        part = atoll(strtok(optarg, "/"));
        num_parts = atoll(strtok(nullptr, "/"));
        break;
      case 'p': partitions = atoll(optarg); break;
      case 's': sequence_filename = optarg; break;
      case 'o': output_filename = optarg; break;
      case 'v': verbose = !verbose; break;
      case 'k': break;   // make_kids: the kid table is always built on demand
      case 'd': break;
      case 'f': do_faqs = !do_faqs; break;
      case 't': do_print = !do_print; break;
      case 'c': do_validate = !do_validate; break;
      case 'e': case 'j': case 'm': case 'w': case 'x':
        printf("Option -%c (junction-tree / width experiments) is not supported by this build.\n", opt);
        return 1;
      case '?':
        if (optopt == 's' || optopt == 'o')
          printf("Option -%c requires a string.\n", optopt);
        else if (optopt == 'm' || optopt == 'w')
          printf("Option -%c requires a long long.\n", optopt);
        else
          printf("Unknown option character '\\x%x'.\n", optopt);
        return 1;
      default: abort();
    }
  }
  if (optind >= argc) {
    printf("USAGE: graph2tree input_graph [options ...]\n");
    return 1;
  }
  const char *const graph_filename = argv[optind];
  auto start_point = std::chrono::steady_clock::now();

  if (use_mpi_sort || use_mpi_reduce) {
    try {
      std::unique_ptr<World> w = World::from_env();
      if (w->size() > 1)
        return run_world(*w, graph_filename, use_mpi_sort, use_mpi_reduce, partitions, sequence_filename,
                         output_filename, verbose, do_faqs, do_print, do_validate, start_point);
    } catch (const std::out_of_range &e) {
      fprintf(stderr, "terminate called after throwing an instance of 'std::out_of_range'\n  what():  %s\n", e.what());
      return 134;
    } catch (const std::exception &e) {
      fprintf(stderr, "graph2tree: %s\n", e.what());
      return 1;
    }
  }
  std::string out_name = output_filename;
  if (use_mpi_sort || use_mpi_reduce) {   // one rank: rank 0 of a size-1 world (graph2tree.cpp:134-157)
    part = 1;
    num_parts = 1;
    char buf[64];
    if (!use_mpi_reduce && out_name != "") {
      snprintf(buf, sizeof buf, "%02dr0.tre", 0);
      out_name += buf;
    } else if (use_mpi_reduce && partitions != 0 && out_name != "") {
      snprintf(buf, sizeof buf, "-w%04d-p", 0);
      out_name += buf;
    }
  }
  const bool mpi = use_mpi_sort || use_mpi_reduce;
  const bool is_leader = (mpi && part == 1) || (!mpi && strcmp(sequence_filename, "") == 0);

  try {
    if (verbose) printf("Loading %s...\n", graph_filename);
    GraphWrapper graph(graph_filename, part, num_parts);
    if (verbose) printf("Nodes:%zu Edges:%zu\n", graph.getNodes(), graph.getEdges());
    const double load_s = seconds_since(start_point);
    if (is_leader) printf("Loaded graph in: %f seconds\n", load_s);

    DeviceSequence seq = (!use_mpi_sort && strcmp(sequence_filename, "") != 0)
                             ? uploadSequence(readSequence(sequence_filename))
                             : degreeSequence(graph);
    if (use_mpi_sort && part == 1 && strcmp(sequence_filename, "") != 0) writeSequence(seq.host(), sequence_filename);
    const double sort_s = seconds_since(start_point) - load_s;
    if (is_leader && (use_mpi_sort || strcmp(sequence_filename, "") == 0)) printf("Sorted in: %f seconds\n", sort_s);

    JTree tree(graph, seq);
    Context::get().sync();
    const double map_s = seconds_since(start_point) - sort_s - load_s;
    if (is_leader) printf("Mapped in: %f seconds\n", map_s);

    if (use_mpi_reduce) {   // a single shard: the reduction is the identity
      const double reduce_s = seconds_since(start_point) - map_s - sort_s - load_s;
      if (is_leader) printf("Reduced in: %f seconds\n", reduce_s);
    }

    if (partitions != 0) {
      Partition p(seq, tree.jnodes, (part_t)partitions);
      if (out_name != "") {
        p.writePartitionedGraph(graph, seq, out_name.c_str(), false);   // graph2tree.cpp:212-213
      } else if (is_leader) {
        p.print();
      }
    } else if (out_name != "") {
      tree.jnodes.save(out_name.c_str());   // graph2tree.cpp:185-189 / 217-218: [end_id][JNodes]
    }

    if (verbose) printf("Built in: %f seconds\n", seconds_since(start_point));
    if (do_faqs) tree.jnodes.getFacts().print();
    if (do_print) tree.print(seq.host());   // graph2tree.cpp:229-230
    if (do_validate) {
      const Facts f = tree.jnodes.getFacts();
      printf(tree_valid(tree.jnodes.nodes(), tree.size(), f.f.vert_cnt) && f.f.vert_cnt == seq.n
                 ? "Tree is valid.\n" : "ERROR: Tree is not valid.\n");
    }
    if (verbose) printf("Finished in: %f seconds\n", seconds_since(start_point));
  } catch (const std::out_of_range &e) {
    fprintf(stderr, "terminate called after throwing an instance of 'std::out_of_range'\n  what():  %s\n", e.what());
    return 134;
  } catch (const std::bad_alloc &) {
    fprintf(stderr, "terminate called after throwing an instance of 'std::bad_alloc'\n");
    return 134;
  } catch (const std::exception &e) {
    fprintf(stderr, "graph2tree: %s\n", e.what());
    return 1;
  }
  return 0;
}
