// mesh.hip — TCP links between the processes of one Sheep world (see mesh.hpp).
#include "mesh.hpp"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

#include "common.hpp"

namespace sheep {
namespace {

[[noreturn]] void fail(const std::string &what) {
  throw Error(SHEEP_ERR_HIP, "mesh: " + what + (errno ? std::string(": ") + strerror(errno) : std::string()));
}

void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
}

using Clock = std::chrono::steady_clock;
constexpr Clock::time_point NO_DEADLINE = Clock::time_point::max();

// waits until fd is ready for `events` or the deadline passes (then fails naming `who`)
void wait_ready(int fd, short events, Clock::time_point until, const std::string &who) {
  for (;;) {
    int ms = 1000;
    if (until != NO_DEADLINE) {
      const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(until - Clock::now()).count();
      if (left <= 0) { errno = 0; fail("timed out waiting for " + who); }
      ms = (int)std::min<long long>(left, 1000);
    }
    pollfd p{fd, events, 0};
    const int r = poll(&p, 1, ms);
    if (r < 0 && errno != EINTR) fail("poll");
    if (r > 0) return;   // ready, or an error / hang-up the next send / recv reports
  }
}

void put(int fd, const void *p, size_t n, Clock::time_point until = NO_DEADLINE, const std::string &who = "a peer") {
  const char *c = (const char *)p;
  while (n) {
    wait_ready(fd, POLLOUT, until, who);
    const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL | MSG_DONTWAIT);
    if (w < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) continue;
    if (w <= 0) fail("send to " + who);
    c += w;
    n -= (size_t)w;
  }
}

void get(int fd, void *p, size_t n, Clock::time_point until = NO_DEADLINE, const std::string &who = "a peer") {
  char *c = (char *)p;
  while (n) {
    wait_ready(fd, POLLIN, until, who);
    const ssize_t r = ::recv(fd, c, n, MSG_DONTWAIT);
    if (r < 0 && (errno == EINTR || errno == EAGAIN || errno == EWOULDBLOCK)) continue;
    if (r == 0) { errno = 0; fail(who + " closed the connection"); }
    if (r < 0) fail("recv from " + who);
    c += r;
    n -= (size_t)r;
  }
}

void put_u32(int fd, uint32_t v) { put(fd, &v, 4); }
uint32_t get_u32(int fd) { uint32_t v; get(fd, &v, 4); return v; }
void put_str(int fd, const std::string &s) { put_u32(fd, (uint32_t)s.size()); put(fd, s.data(), s.size()); }
std::string get_str(int fd) {
  const uint32_t n = get_u32(fd);
  if (n > 4096) { errno = 0; fail("bad handshake"); }
  std::string s(n, '\0');
  get(fd, &s[0], n);
  return s;
}

sockaddr_in resolve(const std::string &host, int port) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) { errno = 0; fail("cannot resolve " + host); }
    a.sin_addr = ((sockaddr_in *)res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  return a;
}

int listen_on(const sockaddr_in &a, int backlog) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) fail("socket");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (bind(fd, (const sockaddr *)&a, sizeof a) != 0) { close(fd); fail("bind port " + std::to_string(ntohs(a.sin_port))); }
  if (listen(fd, backlog) != 0) { close(fd); fail("listen"); }
  return fd;
}

int accept_within(int lfd, std::chrono::steady_clock::time_point until, in_addr *peer = nullptr) {
  for (;;) {
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(until - std::chrono::steady_clock::now());
    if (left.count() <= 0) { errno = 0; fail("timed out waiting for the other ranks"); }
    pollfd p{lfd, POLLIN, 0};
    const int r = poll(&p, 1, (int)std::min<long long>(left.count(), 1000));
    if (r < 0 && errno != EINTR) fail("poll");
    if (r <= 0) continue;
    sockaddr_in from{};
    socklen_t len = sizeof from;
    const int fd = accept(lfd, (sockaddr *)&from, &len);
    if (fd < 0) { if (errno == EINTR) continue; fail("accept"); }
    if (peer) *peer = from.sin_addr;
    tune(fd);
    return fd;
  }
}

int connect_within(const sockaddr_in &a, std::chrono::steady_clock::time_point until) {
  for (;;) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) fail("socket");
    if (connect(fd, (const sockaddr *)&a, sizeof a) == 0) {
      tune(fd);
      return fd;
    }
    close(fd);
    if (std::chrono::steady_clock::now() > until) fail("connect to rank at port " + std::to_string(ntohs(a.sin_port)));
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

}  // namespace

Mesh::Mesh(int rank, int world, const std::string &host, int port, const std::string &bus_id, int timeout_s)
    : rank_(rank), world_(world), timeout_s_(timeout_s), fd_(world, -1), bus_(world) {
  if (world < 1 || rank < 0 || rank >= world) { errno = 0; fail("bad rank / world"); }
  bus_[rank] = bus_id;
  if (world == 1) return;
  const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  const sockaddr_in root = resolve(host, port);
  // every rank's listening port and address: rank 0 learns a rank's address from its
  // accepted connection (the address the other ranks can reach it at, whichever host it
  // runs on) and relays the table
  std::vector<uint32_t> ports(world, 0), addrs(world, root.sin_addr.s_addr);
  int own = -1;
  try {
    if (rank == 0) {                                   // star: everyone reports to rank 0
      own = listen_on(root, world);
      for (int i = 1; i < world; ++i) {
        in_addr from{};
        const int fd = accept_within(own, until, &from);
        const uint32_t r = get_u32(fd);
        if (r == 0 || r >= (uint32_t)world || fd_[r] >= 0) { close(fd); errno = 0; fail("bad or repeated rank"); }
        fd_[r] = fd;
        ports[r] = get_u32(fd);
        addrs[r] = from.s_addr;
        bus_[r] = get_str(fd);
      }
      for (int r = 1; r < world; ++r) {
        for (int q = 0; q < world; ++q) { put_u32(fd_[r], ports[q]); put_u32(fd_[r], addrs[q]); put_str(fd_[r], bus_[q]); }
      }
    } else {
      sockaddr_in any{};
      any.sin_family = AF_INET;
      any.sin_addr.s_addr = htonl(INADDR_ANY);
      any.sin_port = 0;
      own = listen_on(any, world);
      sockaddr_in me{};
      socklen_t len = sizeof me;
      getsockname(own, (sockaddr *)&me, &len);
      fd_[0] = connect_within(root, until);
      put_u32(fd_[0], (uint32_t)rank);
      put_u32(fd_[0], ntohs(me.sin_port));
      put_str(fd_[0], bus_id);
      for (int q = 0; q < world; ++q) { ports[q] = get_u32(fd_[0]); addrs[q] = get_u32(fd_[0]); bus_[q] = get_str(fd_[0]); }
      for (int i = 1; i < rank; ++i) {                 // j connects to every 0 < i < j ...
        sockaddr_in a = root;
        a.sin_addr.s_addr = addrs[i];
        a.sin_port = htons((uint16_t)ports[i]);
        fd_[i] = connect_within(a, until);
        put_u32(fd_[i], (uint32_t)rank);
      }
      for (int k = rank + 1; k < world; ++k) {         // ... and accepts every j > i
        const int fd = accept_within(own, until);
        const uint32_t r = get_u32(fd);
        if (r <= (uint32_t)rank || r >= (uint32_t)world || fd_[r] >= 0) { close(fd); errno = 0; fail("bad peer rank"); }
        fd_[r] = fd;
      }
    }
  } catch (...) {
    if (own >= 0) close(own);
    for (int &f : fd_) if (f >= 0) { close(f); f = -1; }
    throw;
  }
  close(own);
}

Mesh::~Mesh() {
  for (int f : fd_) if (f >= 0) close(f);
}

namespace {
Clock::time_point deadline(int timeout_s) {
  return timeout_s > 0 ? Clock::now() + std::chrono::seconds(timeout_s) : NO_DEADLINE;
}
std::string peer_name(int r) { return "rank " + std::to_string(r); }
}  // namespace

void Mesh::send(int peer, const void *buf, size_t bytes) {
  put(fd_.at(peer), buf, bytes, deadline(timeout_s_), peer_name(peer));
}
void Mesh::recv(int peer, void *buf, size_t bytes) {
  get(fd_.at(peer), buf, bytes, deadline(timeout_s_), peer_name(peer));
}

void Mesh::bcast(void *buf, size_t bytes) {
  const auto until = deadline(timeout_s_);
  if (rank_ == 0) for (int r = 1; r < world_; ++r) put(fd_[r], buf, bytes, until, peer_name(r));
  else get(fd_[0], buf, bytes, until, peer_name(0));
}

uint64_t Mesh::allreduce(uint64_t v, bool is_max) {
  if (world_ == 1) return v;
  const auto until = deadline(timeout_s_);
  if (rank_ == 0) {
    for (int r = 1; r < world_; ++r) {
      uint64_t x;
      get(fd_[r], &x, 8, until, peer_name(r));
      v = is_max ? (x > v ? x : v) : v + x;
    }
  } else {
    put(fd_[0], &v, 8, until, peer_name(0));
  }
  bcast(&v, 8);
  return v;
}

uint64_t Mesh::allreduce_max(uint64_t v) { return allreduce(v, true); }
uint64_t Mesh::allreduce_sum(uint64_t v) { return allreduce(v, false); }
void Mesh::barrier() { (void)allreduce(0, true); }

}  // namespace sheep

// ---- C ABI: a host-only self-test of the links of a joined world ----------------------
// Forms the mesh, then: rank 0's buffer to every rank, every rank's buffer to its ring
// successor (sends on a helper thread), every rank's buffer to rank 0, the all-reduce max
// and sum of the ranks' checksums, a barrier.  *checksum_out = the sum over ranks of the
// checksums of all the buffers that rank received.  No device is touched (tests run it on
// CPUs: tests/test_dist.py).
namespace {
uint64_t fnv(const std::vector<uint8_t> &b) {
  uint64_t h = 1469598103934665603ull;
  for (uint8_t x : b) h = (h ^ x) * 1099511628211ull;
  return h;
}
std::vector<uint8_t> pattern(int rank, uint64_t bytes) {
  std::vector<uint8_t> b(bytes);
  uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(rank + 1);
  for (uint64_t i = 0; i < bytes; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b[i] = (uint8_t)x; }
  return b;
}
}  // namespace

extern "C" int sheep_mesh_selftest(int rank, int world, const char *host, int port, uint64_t bytes,
                                   uint64_t *checksum_out, uint64_t *max_out) {
  try {
    sheep::Mesh m(rank, world, host ? host : "127.0.0.1", port, "host" + std::to_string(rank), 60);
    uint64_t sum = 0;
    std::vector<uint8_t> root = pattern(0, bytes), mine = pattern(rank, bytes), got(bytes);
    if (rank != 0) root.assign(bytes, 0);
    m.bcast(root.data(), bytes);
    sum += fnv(root);
    if (world > 1) {
      std::thread t([&]() { m.send((rank + 1) % world, mine.data(), bytes); });
      m.recv((rank + world - 1) % world, got.data(), bytes);
      t.join();
      sum += fnv(got);
      if (rank == 0) {
        for (int r = 1; r < world; ++r) { m.recv(r, got.data(), bytes); sum += fnv(got); }
      } else {
        m.send(0, mine.data(), bytes);
      }
    }
    *max_out = m.allreduce_max(fnv(mine));
    *checksum_out = m.allreduce_sum(sum);
    m.barrier();
    return SHEEP_OK;
  } catch (const std::exception &e) {
    fprintf(stderr, "sheep_mesh_selftest: %s\n", e.what());
    return SHEEP_ERR_HIP;
  }
}

// The deadline of a joined world's links: rank `stall_rank` joins and then takes no part
// (it sleeps past the deadline); every other rank enters a barrier, which must fail within
// timeout_s instead of hanging.  *waited_s_out = how long the barrier waited (the stalled
// rank reports 0).  Returns SHEEP_OK on the stalled rank and the barrier's status (an
// error, with sheep_last_error naming the peer) on the others.  Host-only.
extern "C" int sheep_mesh_selftest_stall(int rank, int world, const char *host, int port, int stall_rank, int timeout_s,
                                         double *waited_s_out) {
  try {
    sheep::Mesh m(rank, world, host ? host : "127.0.0.1", port, "host" + std::to_string(rank), timeout_s);
    *waited_s_out = 0;
    if (rank == stall_rank) {
      std::this_thread::sleep_for(std::chrono::seconds(timeout_s + 3));
      return SHEEP_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    try {
      m.barrier();
    } catch (const sheep::Error &e) {
      *waited_s_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      sheep::set_error(e.what());
      return e.code;
    }
    *waited_s_out = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return SHEEP_OK;
  } catch (const std::exception &e) {
    sheep::set_error(e.what());
    return SHEEP_ERR_HIP;
  }
}
