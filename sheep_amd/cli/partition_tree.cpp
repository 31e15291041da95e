// partition_tree — drop-in for chan150/sheep partition_tree.cpp (getopt "vfb:xdug:o:",
// same stdout lines) over libsheep_hip.so.
//
//   partition_tree [-v -f -b BAL -x -d -u -g GRAPH -o PREFIX] SEQ TREE K [K ...]
//
// Modes (partition_tree.cpp:114-163): simple (no -g: print per k), partition + evaluate
// (-g: both evaluators per k, SEQ "-" = degree sequence), partition + files (-g -o:
// one k, SEQ "-" = file sequence, one SNAP file per part in input-record order).
// One kid table serves every k, so the FFD sort order persists across k exactly like
// the reference's in-place std::sort (partition.cpp:104-106).
#include <unistd.h>

#include <chrono>

#include "sheep/sheep.hpp"

using namespace sheep;

static double seconds_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t).count() / 1000.0;
}

int main(int argc, char *argv[]) {
  bool verbose = true, do_faqs = false;
  double balance_factor = 1.03;
  bool vtx_weight = false, pst_weight = false, pre_weight = false;
  const char *graph_filename = "";
  const char *output_filename = "";

  opterr = 0;
  int opt;
  while ((opt = getopt(argc, argv, "vfb:xdug:o:")) != -1) {
    switch (opt) {
      case 'v': verbose = !verbose; break;
      case 'f': do_faqs = !do_faqs; break;
      case 'b': balance_factor = atof(optarg); break;
      case 'x': vtx_weight = true; break;
      case 'd': pst_weight = true; break;
      case 'u': pre_weight = true; break;
      case 'g': graph_filename = optarg; break;
      case 'o': output_filename = optarg; break;
      case '?':
        if (optopt == 'k')
          printf("Option -%c requires a long long.\n", optopt);
        else if (optopt == 'b')
          printf("Option -%c requires a double.\n", optopt);
        else if (optopt == 'g' || optopt == 'o')
          printf("Option -%c requires a string.\n", optopt);
        else
          printf("Unknown option character '\\x%x'.\n", optopt);
        return 1;
      default: abort();
    }
  }
  if (!(vtx_weight || pst_weight || pre_weight)) pst_weight = true;
  if (optind + 2 >= argc) {
    printf("USAGE: partition_tree [options] input_sequence input_tree parts [parts...]\n");
    return 1;
  }
  if (pre_weight) {
    printf("Option -u (pre weight) is not supported by this build.\n");
    return 1;
  }

  try {
    auto start_point = std::chrono::steady_clock::now();
    JNodeTable jnodes(argv[optind + 1]);
    jnodes.kids();   // the reference makes kids on load (jnode.cpp:101)
    if (verbose) printf("Loaded tree in: %f seconds\n", seconds_since(start_point));
    if (do_faqs) jnodes.getFacts().print();

    if (strcmp(graph_filename, "") == 0) {
      /* SIMPLE PARTITIONING — the reference parses argv[optind + 2] for every k
         (partition_tree.cpp:118); kept. */
      DeviceSequence seq = uploadSequence(readSequence(argv[optind]));
      for (int i = optind + 2; i != argc; ++i) {
        const short num_parts = atoi(argv[optind + 2]);
        Partition part(seq, jnodes, num_parts, balance_factor, vtx_weight, pst_weight, pre_weight);
        part.print();
      }
    } else if (strcmp(output_filename, "") == 0) {
      /* PARTITIONING AND EVALUATION */
      GraphWrapper graph(graph_filename);
      DeviceSequence seq = strcmp(argv[optind], "-") == 0 ? degreeSequence(graph)
                                                           : uploadSequence(readSequence(argv[optind]));
      for (int i = optind + 2; i != argc; ++i) {
        const short num_parts = atoi(argv[i]);
        auto partition_start = std::chrono::steady_clock::now();
        Partition part(seq, jnodes, num_parts, balance_factor, vtx_weight, pst_weight, pre_weight);
        if (verbose) printf("Partitioning took: %f seconds\n", seconds_since(partition_start));
        part.print();
        part.evaluate(graph, seq);
      }
    } else {
      /* PARTITIONING AND I/O (partition_tree.cpp:146-163): one k, files in input order */
      GraphWrapper graph(graph_filename);
      DeviceSequence seq = uploadSequence(strcmp(argv[optind], "-") == 0 ? fileSequence(graph_filename)
                                                                         : readSequence(argv[optind]));
      const short num_parts = atoi(argv[optind + 2]);
      auto partition_start = std::chrono::steady_clock::now();
      Partition part(seq, jnodes, num_parts, balance_factor, vtx_weight, pst_weight, pre_weight);
      if (verbose) printf("Partitioning took: %f seconds\n", seconds_since(partition_start));
      part.print();
      part.writePartitionedGraph(graph, seq, output_filename, true);
    }
    if (verbose) printf("Finished in: %f seconds\n", seconds_since(start_point));
  } catch (const std::out_of_range &e) {
    fprintf(stderr, "terminate called after throwing an instance of 'std::out_of_range'\n  what():  %s\n", e.what());
    return 134;
  } catch (const std::bad_alloc &) {
    fprintf(stderr, "terminate called after throwing an instance of 'std::bad_alloc'\n");
    return 134;
  } catch (const std::exception &e) {
    fprintf(stderr, "partition_tree: %s\n", e.what());
    return 1;
  }
  return 0;
}
