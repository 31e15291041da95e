// mesh.hpp — TCP links between the processes of one Sheep world (one process per rank):
// the bootstrap of the RCCL communicator (rank 0's ncclUniqueId goes to every rank), the
// barrier and the small host-value exchanges of a world, and the bulk transport of a
// world whose ranks cannot use RCCL (several ranks on one GPU: the one-GPU rehearsal).
//
// Rendezvous: rank 0 listens on host:port; every rank listens on an ephemeral port of its
// own and reports (rank, port, device bus id) to rank 0, which sends the table back; then
// rank j connects to every rank i < j.  Every pair of ranks has its own socket.
//
// Deadlines: every operation waits at most timeout_s seconds for its peer (poll on the
// socket, not a blocking send/recv), so a rank that stops taking part surfaces as an
// error on the others (naming the peer) instead of a hang.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace sheep {

class Mesh {
 public:
  // Blocks until all `world` ranks have joined (timeout_s: give up with an error).
  Mesh(int rank, int world, const std::string &host, int port, const std::string &bus_id, int timeout_s = 300);
  ~Mesh();
  Mesh(const Mesh &) = delete;
  Mesh &operator=(const Mesh &) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  // every rank's device bus id, by rank (known after the rendezvous)
  const std::vector<std::string> &bus_ids() const { return bus_; }

  int timeout_s() const { return timeout_s_; }
  void send(int peer, const void *buf, size_t bytes);
  void recv(int peer, void *buf, size_t bytes);
  // rank 0's bytes to every rank (star)
  void bcast(void *buf, size_t bytes);
  uint64_t allreduce_max(uint64_t v);
  uint64_t allreduce_sum(uint64_t v);
  void barrier();

 private:
  uint64_t allreduce(uint64_t v, bool is_max);
  int rank_, world_, timeout_s_;
  std::vector<int> fd_;           // socket per peer rank (-1 for self)
  std::vector<std::string> bus_;
};

}  // namespace sheep
