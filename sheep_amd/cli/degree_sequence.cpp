// degree_sequence — drop-in for chan150/sheep degree_sequence.cpp over libsheep_hip.so:
// the file-based degree sequence (sequence.h:95-128, degrees counted on the GPU) written
// as a text sequence.
//
//   degree_sequence graph_file output_file
#include <chrono>

#include "sheep/sheep.hpp"

using namespace sheep;

int main(int argc, char *argv[]) {
  if (argc != 3) {
    printf("USAGE: degree_sequence graph_file output_file");
    return 1;
  }
  try {
    auto start_point = std::chrono::steady_clock::now();
    std::vector<vid_t> seq = fileSequence(argv[1]);
    writeSequence(seq, argv[2]);
    auto run = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - start_point);
    printf("Sorted in: %lums\n", (unsigned long)run.count());
  } catch (const std::bad_alloc &) {
    fprintf(stderr, "terminate called after throwing an instance of 'std::bad_alloc'\n");
    return 134;
  } catch (const std::exception &e) {
    fprintf(stderr, "degree_sequence: %s\n", e.what());
    return 1;
  }
  return 0;
}
