// world.hpp — graph2tree's MPI world (-i / -r, graph2tree.cpp:134-216) as ONE process
// over several GPUs of a node: rank r is device devices[r] (SHEEP_DEVICES, e.g. "0,1,2,3";
// default: every visible device).  Exchanges go over RCCL between distinct devices
// (sheep_group_* in include/sheep_hip.h); listing a device more than once rehearses
// several edge shards on one GPU.
#pragma once

#include <string>
#include <vector>

#include "sheep/sheep.hpp"

namespace sheep {

inline std::vector<int> world_devices() {
  std::vector<int> d;
  if (const char *e = getenv("SHEEP_DEVICES")) {
    std::string s = e;
    size_t a = 0;
    while (a < s.size()) {
      size_t b = s.find(',', a);
      if (b == std::string::npos) b = s.size();
      if (b > a) d.push_back(atoi(s.substr(a, b - a).c_str()));
      a = b + 1;
    }
  }
  if (d.empty()) {
    int n = 0;
    check(sheep_device_count(&n));
    for (int i = 0; i < n; ++i) d.push_back(i);
  }
  return d;
}

class World {
 public:
  explicit World(const std::vector<int> &devices) { check(sheep_group_create(devices.data(), (int)devices.size(), &g_)); }
  ~World() { sheep_group_destroy(g_); }
  World(const World &) = delete;
  World &operator=(const World &) = delete;
  int size() const { return sheep_group_size(g_); }
  sheep_ctx *ctx(int r) const { return sheep_group_ctx(g_, r); }
  sheep_group *handle() const { return g_; }

 private:
  sheep_group *g_ = nullptr;
};

// One rank's share of the world: its edge shard (records part r+1 of size, graph2tree -l
// semantics) and its copy of the sequence, on its device.
struct RankState {
  std::vector<sheep_xs1> host;   // the shard's records (the partition-file writer reads them)
  DeviceArray<sheep_xs1> rec;
  DeviceArray<uint32_t> seq, pos, deg;
  DeviceArray<sheep_jnode> tree;
  DeviceArray<int16_t> parts;
  uint64_t max_vid = 0;          // 1 + max vid of the shard
};

}  // namespace sheep
