// world.hpp — graph2tree's MPI world (-i / -r, graph2tree.cpp:134-216) over the GPUs of a
// node, in either of the two forms of include/sheep_hip.h's sheep_group:
//
//   * one process per rank, started by a launcher: `mpiexec -n W graph2tree ... -ir`
//     (MPICH PMI_RANK / PMI_SIZE, Open MPI OMPI_COMM_WORLD_*) or torchrun (RANK /
//     WORLD_SIZE).  Rank r runs on device SHEEP_DEVICES[local rank] (default: local rank
//     modulo the visible devices); the ranks meet over TCP at SHEEP_MASTER_ADDR /
//     SHEEP_MASTER_PORT (defaults: MASTER_ADDR or 127.0.0.1, MASTER_PORT + 1 or 29650);
//   * one process driving several ranks: SHEEP_DEVICES="0,1,2,3" without a launcher (a
//     device listed twice rehearses two shards on it).  Without SHEEP_DEVICES a plain
//     `graph2tree -i` is a world of one rank, as an MPI program started without mpiexec.
#pragma once

#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "sheep/sheep.hpp"

namespace sheep {

inline std::vector<int> env_devices() {
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
  return d;
}

// The rank of this process as a launcher (mpiexec / torchrun) set it; size 1 without one.
struct Launch {
  int rank = 0, size = 1, local = 0;
};
inline Launch launcher_env() {
  auto num = [](const char *a, const char *b, const char *c, int dflt) {
    for (const char *k : {a, b, c})
      if (k && getenv(k)) return atoi(getenv(k));
    return dflt;
  };
  Launch l;
  l.size = num("OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "WORLD_SIZE", 1);
  l.rank = num("OMPI_COMM_WORLD_RANK", "PMI_RANK", "RANK", 0);
  l.local = num("OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "LOCAL_RANK", l.rank);
  return l;
}

class World {
 public:
  // The world this graph2tree run belongs to (see the file comment).
  static std::unique_ptr<World> from_env() {
    const Launch l = launcher_env();
    std::vector<int> devs = env_devices();
    if (l.size > 1) {
      int dev;
      if (!devs.empty()) {
        dev = devs[(size_t)l.local % devs.size()];
      } else {
        int nd = 0;
        check(sheep_device_count(&nd));
        dev = nd > 0 ? l.local % nd : 0;
      }
      std::string host = getenv("SHEEP_MASTER_ADDR") ? getenv("SHEEP_MASTER_ADDR")
                         : getenv("MASTER_ADDR")     ? getenv("MASTER_ADDR")
                                                     : "127.0.0.1";
      int port = getenv("SHEEP_MASTER_PORT") ? atoi(getenv("SHEEP_MASTER_PORT"))
                 : getenv("MASTER_PORT")     ? atoi(getenv("MASTER_PORT")) + 1
                                             : 29650;
      return std::unique_ptr<World>(new World(dev, l.rank, l.size, host, port));
    }
    if (devs.empty()) devs.push_back(0);
    return std::unique_ptr<World>(new World(devs));
  }
  explicit World(const std::vector<int> &devices) { check(sheep_group_create(devices.data(), (int)devices.size(), &g_)); }
  World(int device, int rank, int size, const std::string &host, int port) {
    check(sheep_group_join(device, rank, size, host.c_str(), port, SHEEP_LINK_AUTO, &g_));
  }
  ~World() { sheep_group_destroy(g_); }
  World(const World &) = delete;
  World &operator=(const World &) = delete;
  int size() const { return sheep_group_size(g_); }            // ranks in the world
  int local() const { return sheep_group_local_count(g_); }    // ranks held by this process
  int rank(int i) const { return sheep_group_rank(g_, i); }    // global rank of local rank i
  sheep_ctx *ctx(int i) const { return sheep_group_ctx(g_, i); }
  sheep_group *handle() const { return g_; }
  void barrier() const { check(sheep_group_barrier(g_)); }

 private:
  sheep_group *g_ = nullptr;
};

// One rank's share of the world: its edge shard (records part r+1 of size, graph2tree -l
// semantics) and its copy of the sequence, on its device.
struct RankState {
  int rank = 0;
  DeviceArray<sheep_xs1> rec;    // the shard's records, read straight into HBM (loadRecords)
  uint64_t nrec = 0;
  DeviceArray<uint32_t> seq, pos, deg;
  DeviceArray<sheep_jnode> tree;
  DeviceArray<int16_t> parts;
  uint64_t max_vid = 0;          // 1 + max vid of the shard
};

}  // namespace sheep
