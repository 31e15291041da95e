// merge_trees — drop-in for chan150/sheep merge_trees.cpp (getopt "o:vkf") over
// libsheep_hip.so: merge two partial trees of the same sequence (the reduce step).
//
//   merge_trees [-o OUT -v -k -f] first.tre second.tre
//
// The output file is [end_id][lhs.size() JNodes] like the reference's mmapped table
// (jnode.cpp:52-74, header written on destruction :153-161).
#include <unistd.h>

#include <chrono>

#include "sheep/sheep.hpp"

using namespace sheep;

int main(int argc, char *argv[]) {
  const char *output_filename = "";
  bool verbose = false, do_faqs = false;

  opterr = 0;
  int opt;
  while ((opt = getopt(argc, argv, "o:vkf")) != -1) {
    switch (opt) {
      case 'o': output_filename = optarg; break;
      case 'v': verbose = !verbose; break;
      case 'k': break;   // make_kids: built on demand
      case 'f': do_faqs = !do_faqs; break;
      case '?':
        if (optopt == 'o')
          printf("Option -%c requires a string.\n", optopt);
        else
          printf("Unknown option character '\\x%x'.\n", optopt);
        return 1;
      default: abort();
    }
  }
  if (optind + 1 >= argc) {
    printf("USAGE: merge_trees [options ...] first.tree second.tree\n");
    return 1;
  }

  try {
    auto start_point = std::chrono::steady_clock::now();
    JNodeTable lhs(argv[optind]);
    JNodeTable rhs(argv[optind + 1]);
    auto load = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - start_point);
    if (verbose) printf("Loaded in: %lums\n", (unsigned long)load.count());

    JNodeTable jnodes(lhs.size());
    jnodes.merge(lhs, rhs);
    if (strcmp(output_filename, "") != 0) jnodes.save(output_filename);

    auto build = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - start_point) -
                 load;
    if (verbose) printf("Built in: %lums\n", (unsigned long)build.count());
    if (do_faqs) jnodes.getFacts().print();
  } catch (const std::bad_alloc &) {
    fprintf(stderr, "terminate called after throwing an instance of 'std::bad_alloc'\n");
    return 134;
  } catch (const std::exception &e) {
    fprintf(stderr, "merge_trees: %s\n", e.what());
    return 1;
  }
  return 0;
}
