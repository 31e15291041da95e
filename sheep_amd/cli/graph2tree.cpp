// graph2tree — drop-in for chan150/sheep graph2tree.cpp (same getopt string, same
// stdout lines, same .seq/.tre files) over libsheep_hip.so.
//
//   graph2tree input_graph [-s SEQ] [-o OUT] [-p K] [-l n/k] [-i] [-r] [-f] [-c] [-v]
//
// Phases (graph2tree.cpp:161-218): load the records into HBM, degree sequence (or -s
// read), map (JTree on the GPU), [reduce], [partition], [TREEFAQS].  -i / -r select the
// reference's MPI sort / reduce; here a single process drives one GPU, so they only
// keep their file-naming and printing behaviour (the multi-GPU edge-shard path is
// bench.py's torch.distributed + RCCL driver).  Flags of the
// junction-tree experiments (-e -j -m -w -x) and -t are rejected with a message.
#include <unistd.h>

#include <cassert>
#include <chrono>

#include "sheep/sheep.hpp"

using namespace sheep;

static double seconds_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t).count() / 1000.0;
}

int main(int argc, char *argv[]) {
  bool use_mpi_sort = false, use_mpi_reduce = false;
  size_t part = 0, num_parts = 0, partitions = 0;
  const char *sequence_filename = "";
  const char *output_filename = "";
  bool verbose = false, do_faqs = false, do_validate = false;

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
      case 'c': do_validate = !do_validate; break;
      case 'e': case 'j': case 'm': case 'w': case 'x': case 't':
        printf("Option -%c (junction-tree / width / print experiments) is not supported by this build.\n", opt);
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
    if (do_validate) {
      // JTree::isValid (jtree.cpp:238-300): index count == verts, parents later & in range
      const Facts f = tree.jnodes.getFacts();
      bool ok = f.f.vert_cnt == seq.n;
      for (jnid_t id = 0; ok && id != tree.size(); ++id) {
        const jnid_t p = tree.jnodes.parent(id);
        ok = p == INVALID_JNID || (p > id && p < tree.size());
      }
      printf(ok ? "Tree is valid.\n" : "ERROR: Tree is not valid.\n");
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
