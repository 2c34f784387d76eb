// Same-node exchange for the cross-process column split (SURVEY 8(e),
// include/mi_lp.h mi_lp_set_exchange): an all-gather of host byte strings
// through one POSIX shared-memory segment, in C++, so that no Python and no
// socket sits in a split solve's per-iteration path.
//
// The joined messages (the update row's list, a block's reduced costs, the
// filtered ratio-test breakpoints, the entering column's coefficient) are
// consumed by every rank's host control flow, so they are gathered where the
// host reads them. Layout: a header (one sequence word per rank on its own
// cache line) and two banks of `world` slots of `slot_bytes`. A round: each
// rank copies its chunk into its slot of bank (seq & 1), publishes seq
// (release), waits until every rank published seq (acquire) and copies the
// chunks out. Two banks suffice: a rank can start round seq + 1 only after
// every rank started round seq, i.e. finished reading round seq - 1's bank.
// Messages longer than a slot go in several rounds.
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>

#include "../../../include/mi_lp.h"

namespace {

constexpr uint32_t kMagic = 0x4d584348;  // "MXCH"
constexpr int kMaxWorld = 64;

struct alignas(64) SeqWord {
  std::atomic<uint64_t> v;
  char pad[64 - sizeof(std::atomic<uint64_t>)];
};

struct Header {
  std::atomic<uint32_t> magic;
  int32_t world;
  int64_t slot_bytes;
  std::atomic<int32_t> attached;
  int32_t pad;
  SeqWord seq[kMaxWorld];
  std::atomic<int32_t> pid[kMaxWorld];  // each rank's process, for liveness checks
};

// MILP_EXCHANGE_TIMEOUT_S: how long a rank waits for its peers in one
// all-gather round (default 0 = as long as every peer process is alive: a
// long refactorization or a slow first segment on one rank is not an error).
// Attaching waits at most MILP_EXCHANGE_ATTACH_S (default 120) seconds.
double EnvSeconds(const char* name, double fallback) {
  const char* e = std::getenv(name);
  return e != nullptr ? std::atof(e) : fallback;
}

bool PeerAlive(int32_t pid) { return pid <= 0 || kill(pid, 0) == 0 || errno != ESRCH; }

size_t SegmentBytes(int world, int64_t slot_bytes) {
  return sizeof(Header) + 2 * static_cast<size_t>(world) * static_cast<size_t>(slot_bytes);
}

// Waits until pred() or the timeout (seconds; <= 0: none) or alive()
// returns false (checked about once a second); spins, then yields.
template <typename Pred, typename Alive>
bool WaitFor(Pred pred, double timeout_s, Alive alive) {
  for (int i = 0; i < 4096; ++i) {
    if (pred()) return true;
  }
  const auto t0 = std::chrono::steady_clock::now();
  double next_check = 1.0;
  while (!pred()) {
    std::this_thread::yield();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s > 0 && s > timeout_s) return false;
    if (s > next_check) {
      if (!alive()) return false;
      next_check = s + 1.0;
    }
  }
  return true;
}

template <typename Pred>
bool WaitFor(Pred pred, double timeout_s) {
  return WaitFor(pred, timeout_s, [] { return true; });
}

}  // namespace

struct mi_exchange {
  int rank = 0;
  int world = 1;
  int64_t slot_bytes = 0;
  uint64_t seq = 0;
  double timeout_s = 0.0;
  Header* header = nullptr;
  char* slots = nullptr;
  size_t bytes = 0;
  char* Slot(uint64_t s, int r) const {
    return slots + (static_cast<size_t>(s & 1) * world + r) * static_cast<size_t>(slot_bytes);
  }
};

extern "C" {

int mi_exchange_open(const char* name, int32_t rank, int32_t world, int64_t slot_bytes,
                     mi_exchange** out) {
  if (name == nullptr || out == nullptr) return MI_LP_ERROR_NULL;
  *out = nullptr;
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world || slot_bytes < 64) {
    return MI_LP_ERROR_INVALID_PROBLEM;
  }
  slot_bytes = (slot_bytes + 63) & ~int64_t{63};
  const size_t bytes = SegmentBytes(world, slot_bytes);
  int fd = -1;
  if (rank == 0) {
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return MI_LP_ERROR_STATE;
    if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
      close(fd);
      shm_unlink(name);
      return MI_LP_ERROR_STATE;
    }
  } else {
    // Rank 0 creates the segment; wait for it (and for its full size).
    const bool ok = WaitFor([&]() {
      if (fd < 0) fd = shm_open(name, O_RDWR, 0600);
      if (fd < 0) return false;
      struct stat st;
      return fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) >= bytes;
    }, EnvSeconds("MILP_EXCHANGE_ATTACH_S", 120.0));
    if (!ok) {
      if (fd >= 0) close(fd);
      return MI_LP_ERROR_STATE;
    }
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (rank == 0) shm_unlink(name);
    return MI_LP_ERROR_STATE;
  }
  Header* h = static_cast<Header*>(p);
  if (rank == 0) {
    h->world = world;
    h->slot_bytes = slot_bytes;
    h->attached.store(0, std::memory_order_relaxed);
    for (int r = 0; r < kMaxWorld; ++r) {
      h->seq[r].v.store(0, std::memory_order_relaxed);
      h->pid[r].store(0, std::memory_order_relaxed);
    }
    h->magic.store(kMagic, std::memory_order_release);
  } else if (!WaitFor([&]() { return h->magic.load(std::memory_order_acquire) == kMagic; },
                      EnvSeconds("MILP_EXCHANGE_ATTACH_S", 120.0)) ||
             h->world != world || h->slot_bytes != slot_bytes) {
    munmap(p, bytes);
    return MI_LP_ERROR_INVALID_PROBLEM;
  }
  h->pid[rank].store(static_cast<int32_t>(getpid()), std::memory_order_release);
  h->attached.fetch_add(1, std::memory_order_acq_rel);
  // Everyone attached: the name can go (nothing is left in /dev/shm if a
  // rank dies later).
  if (!WaitFor([&]() { return h->attached.load(std::memory_order_acquire) == world; },
               EnvSeconds("MILP_EXCHANGE_ATTACH_S", 120.0))) {
    munmap(p, bytes);
    if (rank == 0) shm_unlink(name);
    return MI_LP_ERROR_STATE;
  }
  if (rank == 0) shm_unlink(name);
  mi_exchange* x = new (std::nothrow) mi_exchange();
  if (x == nullptr) {
    munmap(p, bytes);
    return MI_LP_ERROR_STATE;
  }
  x->rank = rank;
  x->world = world;
  x->slot_bytes = slot_bytes;
  x->header = h;
  x->slots = static_cast<char*>(p) + sizeof(Header);
  x->bytes = bytes;
  x->timeout_s = EnvSeconds("MILP_EXCHANGE_TIMEOUT_S", 0.0);
  *out = x;
  return MI_LP_OK;
}

// mi_lp_allgather_fn: every rank's bytes in rank order.
int mi_exchange_allgather(void* ctx, const void* send, int64_t send_bytes, void* recv,
                          const int64_t* recv_bytes) {
  mi_exchange* x = static_cast<mi_exchange*>(ctx);
  if (x == nullptr || recv_bytes == nullptr || (send_bytes > 0 && send == nullptr)) {
    return MI_LP_ERROR_NULL;
  }
  if (recv_bytes[x->rank] != send_bytes) return MI_LP_ERROR_INVALID_PROBLEM;
  int64_t longest = 0;
  int64_t offset[kMaxWorld];
  int64_t total = 0;
  for (int r = 0; r < x->world; ++r) {
    offset[r] = total;
    total += recv_bytes[r];
    if (recv_bytes[r] > longest) longest = recv_bytes[r];
  }
  const int64_t cap = x->slot_bytes;
  const int64_t rounds = longest == 0 ? 1 : (longest + cap - 1) / cap;
  const char* src = static_cast<const char*>(send);
  char* dst = static_cast<char*>(recv);
  for (int64_t round = 0; round < rounds; ++round) {
    const uint64_t s = ++x->seq;
    const int64_t at = round * cap;
    const int64_t mine = send_bytes - at < cap ? send_bytes - at : cap;
    if (mine > 0) std::memcpy(x->Slot(s, x->rank), src + at, static_cast<size_t>(mine));
    x->header->seq[x->rank].v.store(s, std::memory_order_release);
    for (int r = 0; r < x->world; ++r) {
      if (!WaitFor([&]() { return x->header->seq[r].v.load(std::memory_order_acquire) >= s; },
                   x->timeout_s,
                   [&]() { return PeerAlive(x->header->pid[r].load(std::memory_order_acquire)); })) {
        return MI_LP_ERROR_STATE;
      }
    }
    for (int r = 0; r < x->world; ++r) {
      const int64_t n = recv_bytes[r] - at < cap ? recv_bytes[r] - at : cap;
      if (n > 0) std::memcpy(dst + offset[r] + at, x->Slot(s, r), static_cast<size_t>(n));
    }
  }
  return MI_LP_OK;
}

void mi_exchange_close(mi_exchange* x) {
  if (x == nullptr) return;
  munmap(x->header, x->bytes);
  delete x;
}

}  // extern "C"
