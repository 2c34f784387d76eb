// Device simplex segment on gfx950: one workgroup runs the phase-II dual loop
// (sdual_core.h) or the primal loop (sprimal_core.h) of one LP over its arena
// in HBM until the loop needs the host (SdExit). DeviceLp owns the arena, a
// pinned staging image and the transfers; RevisedSimplex (engine/simplex.cc)
// packs and unpacks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../engine/device_lp.h"
#include "../engine/fibers.h"
#include "sdual_core.h"

namespace milp {
namespace {
inline hipStream_t Stream(void* p) { return reinterpret_cast<hipStream_t>(p); }
}  // namespace

// Dynamic LDS of a segment workgroup: the staged dense vector of the
// triangular sweeps and rank-one products (32 KB), then the reduction and
// metadata scratch (SdScratch, 4.5 KB): four workgroups per CU keep the
// 1 024-group pool resident.
constexpr int kLdsDoubles = 4096;
extern __shared__ double sd_lds[];
// TriangularMatrix::stored_ (m flags, zero between uses) in LDS for m up to
// this many rows.
constexpr int kLdsStoredBytes = 2560;
constexpr int kLdsTotalDoubles = kLdsDoubles + sdual::kSdScratchDoubles + kLdsStoredBytes / 8;
// The segment's LDS: the staging / working vector area (zeroed), the stored
// flags when they fit (zeroed; the arena pointer is put back before the
// header leaves), the scratch.
__device__ inline char* sd_lds_enter(sdual::Lp* lp) {
  lp->lds = sd_lds;
  lp->lds_doubles = kLdsDoubles;
  lp->lds_scratch = sd_lds + kLdsDoubles;
  lp->lds_busy = 0;
  for (int i = threadIdx.x; i < kLdsDoubles; i += blockDim.x) sd_lds[i] = 0.0;  // SdLdsVec
  char* saved = lp->stored;
  if (lp->m <= kLdsStoredBytes) {
    char* st = reinterpret_cast<char*>(sd_lds + kLdsDoubles + sdual::kSdScratchDoubles);
    for (int i = threadIdx.x; i < kLdsStoredBytes; i += blockDim.x) st[i] = 0;
    lp->stored = st;
  }
  __syncthreads();
  return saved;
}

// One thread walks Glop's loop; the header lives in the arena.
__global__ __launch_bounds__(64) void sdual_segment_kernel(sdual::Lp* lp) {
  char* stored = sd_lds_enter(lp);
  // every lane (sdual_core.h: the wave); primal segments: sprimal_core.h
  if (lp->primal) {
    sdual::sp_run(*lp);
  } else {
    sdual::sd_run(*lp);
  }
  __syncthreads();
  lp->stored = stored;
}

// ---------------------------------------------------------------------------
// Persistent segment pool (the batch APIs): one launch per device keeps
// kPoolGroups workgroups resident. Workgroup 0 is the dispatcher: it alone
// polls the host queue (coherent mapped memory, ~4 us between polls, so the
// PCIe link stays free) and republishes new entries in device memory. The
// others claim the next index, wait on the device-side tail, move the LP's
// staging image in, run its segment, move it out and raise the LP's mailbox
// flag to 3. The dispatcher stops on the stop word or after kIdleSpins polls
// without work; the workers follow, so the grid always drains.
//
// Both queues are rings of `cap` slots (kCap, or less for the wrap-around
// test: MILP_SDUAL_QUEUE_CAP) indexed by a running count:
//  * the host publishes entry t into q->entry[t % cap] only while
//    t - q->seen < cap, i.e. the dispatcher has copied the slot's previous
//    occupant;
//  * the dispatcher republishes entry k into ring->entry[k % cap] only when
//    the slot's previous occupant (k - cap) was read: ring->ack[slot] holds
//    the last index read from the slot + 1 (slots last used by an earlier
//    grid are free: that grid read everything it republished before it quit);
//  * a worker that claimed index idx reads it once ring->tail > idx.
// A grid that drained leaves q->seen behind: the next launch starts there, so
// an entry published while the old grid was quitting is served, once.
struct SdQueue {
  static constexpr int kCap = 1 << 14;
  int64_t tail;  // entries [0, tail) published (host)
  int64_t seen;  // entries [0, seen) copied into the device ring (dispatcher)
  int32_t stop;
  int32_t pad;
  int64_t dbg[8];  // MILP_SDUAL_DEBUG progress words
  uint64_t entry[kCap];  // device view of an LP's staging image
};
__device__ inline void pool_dbg(SdQueue* q, int k, int64_t v) {
  __hip_atomic_store(&q->dbg[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
struct SdRing {
  unsigned long long head;  // next index a worker claims
  long long tail;           // entries [0, tail) republished
  int quit;
  int pad;
  uint64_t entry[SdQueue::kCap];
  long long ack[SdQueue::kCap];  // per slot: last index read from it + 1
};
constexpr int kPoolGroups = 1024;
constexpr int kMinPoolGroups = 33;
constexpr int64_t kIdleSpins = 1 << 20;  // ~4 s of dispatcher polls

// Cooperative copy by the workgroup (16-byte words; regions are 256-byte
// aligned and padded).
__device__ inline void team_copy(char* dst, const char* src, int64_t bytes) {
  const int64_t words = (bytes + 15) / 16;
  uint4* d = reinterpret_cast<uint4*>(dst);
  const uint4* s = reinterpret_cast<const uint4*>(src);
  for (int64_t w = threadIdx.x; w < words; w += blockDim.x) d[w] = s[w];
}
__device__ inline void team_copy_store_prefix(const sdual::Store& st, const char* from_base,
                                              char* to_base, uint64_t arena) {
  // st's pointers are arena addresses; its starts are readable at from_base.
  const int64_t* starts = reinterpret_cast<const int64_t*>(
      from_base + (reinterpret_cast<uint64_t>(st.starts) - arena));
  const int64_t used = starts[st.num_cols];
  const uint64_t r = reinterpret_cast<uint64_t>(st.rows) - arena;
  const uint64_t c = reinterpret_cast<uint64_t>(st.coefs) - arena;
  team_copy(to_base + r, from_base + r, used * 4);
  team_copy(to_base + c, from_base + c, used * 8);
}

__global__ __launch_bounds__(64) void sdual_pool_kernel(SdQueue* q, SdRing* ring,
                                                        long long head_base, long long cap) {
  if (blockIdx.x == 0) {
    if (threadIdx.x != 0) return;
    long long seen = head_base;
    __hip_atomic_store(&q->seen, static_cast<int64_t>(seen), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    int64_t idle = 0;
    while (true) {
      // Relaxed polls bypass the caches for the polled word only; the acquire
      // fence (one cache invalidation) follows a change.
      const long long t = static_cast<long long>(
          __hip_atomic_load(&q->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      if (t > seen) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        long long k = seen;
        for (; k < t; ++k) {
          const long long slot = k % cap;
          // The slot's previous occupant must have been read (see above).
          if (k - cap >= head_base &&
              __hip_atomic_load(&ring->ack[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                  k - cap + 1) {
            break;
          }
          ring->entry[slot] = __hip_atomic_load(&q->entry[slot], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (k > seen) {
          __hip_atomic_store(&ring->tail, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          seen = k;
          __hip_atomic_store(&q->seen, static_cast<int64_t>(seen), __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_SYSTEM);
          pool_dbg(q, 0, seen);
        }
        idle = 0;  // entries wait (a full ring waits for the workers)
      } else if (__hip_atomic_load(&q->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
                 ++idle > kIdleSpins) {
        __hip_atomic_store(&ring->quit, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      __builtin_amdgcn_s_sleep(127);
    }
  }
  __shared__ uint64_t entry_shared;
  __shared__ int quit;
  while (true) {
    if (threadIdx.x == 0) {
      quit = 0;
      const unsigned long long idx = atomicAdd(&ring->head, 1ull);
      while (true) {
        if (static_cast<long long>(idx) <
            __hip_atomic_load(&ring->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          const long long slot = static_cast<long long>(idx) % cap;
          entry_shared = __hip_atomic_load(&ring->entry[slot], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ring->ack[slot], static_cast<long long>(idx) + 1, __ATOMIC_RELEASE,
                             __HIP_MEMORY_SCOPE_AGENT);
          pool_dbg(q, 1, static_cast<int64_t>(idx) + 1);
          pool_dbg(q, 2, 1);
          break;
        }
        if (__hip_atomic_load(&ring->quit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
          quit = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(64);
      }
    }
    __syncthreads();
    if (quit) return;
    // The entry is the staging image (device view of pinned host memory):
    // move it into the arena, run, move the mutable part back.
    const sdual::Lp* sh = reinterpret_cast<const sdual::Lp*>(entry_shared);
    const char* stage = reinterpret_cast<const char*>(sh);
    const uint64_t t_claim = wall_clock64();
    char* arena = reinterpret_cast<char*>(sh->arena_dev);
    const uint64_t arena_addr = sh->arena_dev;
    team_copy(arena, stage, sizeof(sdual::Lp));
    team_copy(arena + sh->mutable_begin, stage + sh->mutable_begin,
              sh->fixed_end - sh->mutable_begin);
    {
      uint4* z = reinterpret_cast<uint4*>(arena + sh->scratch_begin);
      const int64_t words = (sh->scratch_end - sh->scratch_begin + 15) / 16;
      for (int64_t w = threadIdx.x; w < words; w += blockDim.x) z[w] = make_uint4(0, 0, 0, 0);
    }
    team_copy_store_prefix(sh->storage, stage, arena, arena_addr);
    team_copy_store_prefix(sh->right_storage, stage, arena, arena_addr);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) pool_dbg(q, 2, 2);
    sdual::Lp* lp = reinterpret_cast<sdual::Lp*>(arena);
    lp->phase_ticks[13] += wall_clock64() - t_claim;  // staging image in
    char* stored = sd_lds_enter(lp);
    if (lp->primal) {
      sdual::sp_run(*lp);
    } else {
      sdual::sd_run(*lp);
    }
    __syncthreads();
    lp->stored = stored;  // every lane (sdual_core.h: the wave)
    const uint64_t t_out = wall_clock64();
    if (threadIdx.x == 0) {
      pool_dbg(q, 2, 3);
      pool_dbg(q, 3, lp->num_iterations);
    }
    __threadfence();
    __syncthreads();
    char* stage_out = const_cast<char*>(stage);
    if (threadIdx.x == 0) {
      pool_dbg(q, 4, lp->mutable_end - lp->mutable_begin);
      pool_dbg(q, 5, reinterpret_cast<int64_t>(stage_out));
    }
    team_copy(stage_out, arena, sizeof(sdual::Lp));
    if (threadIdx.x == 0) pool_dbg(q, 2, 31);
    team_copy(stage_out + lp->mutable_begin, arena + lp->mutable_begin,
              lp->mutable_end - lp->mutable_begin);
    if (threadIdx.x == 0) pool_dbg(q, 2, 32);
    team_copy_store_prefix(lp->storage, arena, stage_out, arena_addr);
    team_copy_store_prefix(lp->right_storage, arena, stage_out, arena_addr);
    if (threadIdx.x == 0) pool_dbg(q, 2, 33);
    if (lp->coeff_out != nullptr) {
      for (int c = threadIdx.x; c < lp->N; c += blockDim.x) lp->coeff_out[c] = lp->coeff[c];
    }
    if (threadIdx.x == 0) pool_dbg(q, 2, 34);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
      reinterpret_cast<sdual::Lp*>(stage_out)->phase_ticks[14] =
          lp->phase_ticks[14] + (wall_clock64() - t_out);  // staging image out
    }
    if (threadIdx.x == 0) pool_dbg(q, 2, 35);
    __syncthreads();
    if (threadIdx.x == 0) pool_dbg(q, 2, 36);
    __threadfence_system();
    if (threadIdx.x == 0) {
      pool_dbg(q, 2, 4);
      __hip_atomic_store(&lp->mb->flag, 3, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

namespace {
// A stream with a CU mask gets a hardware queue of its own: the resident grid
// never sits in front of another stream's work (streams otherwise share the
// GPU_MAX_HW_QUEUES queues round-robin, in order).
bool CreateOwnQueueStream(int device, hipStream_t* s) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
      cus <= 0) {
    return false;
  }
  std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
  if (cus % 32 != 0) mask.back() = (1u << (cus % 32)) - 1;
  return hipExtStreamCreateWithCUMask(s, static_cast<uint32_t>(mask.size()), mask.data()) ==
         hipSuccess;
}

// One pool per device. Never destroyed (like SmallBatcher): the runtime may
// be gone at process exit; the kernel drains on its idle limit.
class SdualPool {
 public:
  static SdualPool& Get(int device) {
    std::lock_guard<std::mutex> lock(RegistryMutex());
    std::vector<SdualPool*>& all = Registry();
    if (static_cast<int>(all.size()) <= device) all.resize(device + 1, nullptr);
    if (all[device] == nullptr) {
      all[device] = new SdualPool(device);
      RegisterDeviceShutdown();
    }
    return *all[device];
  }
  // Process teardown (mi_lp_shutdown, or the atexit handler registered with
  // the first pool): the resident grid drains on the stop word before the HIP
  // runtime, and any profiler hooked into it, goes away. Waits at most ~10 s.
  static void ShutdownAll() {
    std::lock_guard<std::mutex> lock(RegistryMutex());
    for (SdualPool* p : Registry()) {
      if (p != nullptr) p->Shutdown();
    }
  }
  void Shutdown() {
    std::lock_guard<std::mutex> lock(mu_);
    if (!running_) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device_);
    __atomic_store_n(&q_->stop, 1, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    while (hipStreamQuery(stream_) == hipErrorNotReady &&
           std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10)) {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    running_ = false;
    // The CU-masked queue goes too: left to the runtime's exit-time teardown,
    // a profiler's own teardown (rocprofiler-sdk's static destructors) later
    // calls into HSA on it and faults (symbolized with MILP_CRASH_REPORT,
    // profiles/r05_pmc). Launch creates a new one when needed.
    (void)hipStreamDestroy(stream_);
    stream_ = nullptr;
    (void)hipSetDevice(prev);
  }
  // Publishes one arena; (re)launches the kernel when it is not running. A
  // full host ring (kCap entries the dispatcher has not copied yet) waits.
  void Enqueue(void* lp) {
    while (true) {
      {
        std::lock_guard<std::mutex> lock(mu_);
        if (running_ && inflight_ == 0 && launched_groups_ < GroupsFor(lps_) &&
            hipStreamQuery(stream_) == hipErrorNotReady) {
          // A grid launched for fewer LPs (a single solve's few dozen
          // workers) would serve a batch on too few workgroups: stop it (no
          // entry can be published while mu_ is held, so its dispatcher goes
          // idle and quits) and relaunch at the batch's size; Launch waits
          // for the old grid and starts at the first uncopied entry. Only
          // with no segment in flight: one could wait for a factorization
          // this thread's fibers would serve.
          __atomic_store_n(&q_->stop, 1, __ATOMIC_RELEASE);
          Launch();
        }
        if (!running_ || hipStreamQuery(stream_) == hipSuccess) Launch();
        const int64_t t = q_->tail;
        if (t - __atomic_load_n(&q_->seen, __ATOMIC_ACQUIRE) < cap_) {
          ++inflight_;
          __atomic_store_n(&q_->entry[t % cap_], reinterpret_cast<uint64_t>(lp),
                           __ATOMIC_RELEASE);
          __atomic_store_n(&q_->tail, t + 1, __ATOMIC_RELEASE);
          return;
        }
      }
      if (InFiber()) {
        FiberYield(false);
      } else {
        std::this_thread::yield();
      }
    }
  }
  // A segment published by Enqueue has completed (its mailbox flag read 3).
  void Done() {
    std::lock_guard<std::mutex> lock(mu_);
    --inflight_;
  }
  int64_t Tail() const { return q_->tail; }
  const int64_t* Dbg() const { return q_->dbg; }
  // False when the kernel is gone (idle limit) before serving a request.
  bool Alive() {
    std::lock_guard<std::mutex> lock(mu_);
    return running_ && hipStreamQuery(stream_) == hipErrorNotReady;
  }
  // A published entry waits for a grid: relaunch one if the last drained
  // (idle limit or stop word) before copying it. The new grid starts at the
  // old one's seen, so the entry is served once.
  void EnsureRunning() {
    std::lock_guard<std::mutex> lock(mu_);
    if (!running_ || hipStreamQuery(stream_) == hipSuccess) Launch();
  }
  // The batch calls in progress on this device (BatchScope): the last one to
  // end raises the stop word, so the resident grid leaves the CUs to single
  // solves instead of spinning out its idle limit.
  // `lps`: the LPs the batch call may have in flight on this device; a grid
  // launched meanwhile has one workgroup per LP (plus the dispatcher), up to
  // kPoolGroups. A pool wave holds a whole SIMD's registers, so a grid larger
  // than the work would lock the engine's other kernels out of the CUs.
  void Acquire(int lps) {
    std::lock_guard<std::mutex> lock(mu_);
    lps_ += lps;
    if (users_++ == 0) __atomic_store_n(&q_->stop, 0, __ATOMIC_RELEASE);
  }
  void Release(int lps) {
    std::lock_guard<std::mutex> lock(mu_);
    lps_ -= lps;
    if (--users_ == 0 && running_) __atomic_store_n(&q_->stop, 1, __ATOMIC_RELEASE);
  }

 private:
  explicit SdualPool(int device) : device_(device) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    if (hipHostMalloc(reinterpret_cast<void**>(&q_), sizeof(SdQueue),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&d_q_), q_, 0) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_ring_), sizeof(SdRing)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&h_ring_), sizeof(SdRing),
                      hipHostMallocDefault) != hipSuccess ||
        !CreateOwnQueueStream(device, &stream_)) {
      (void)hipSetDevice(prev);
      throw DeviceError("sdual pool: allocation failed");
    }
    std::memset(q_, 0, sizeof(SdQueue));
    if (hipMemset(d_ring_, 0, sizeof(SdRing)) != hipSuccess) {
      (void)hipSetDevice(prev);
      throw DeviceError("sdual pool: ring clear failed");
    }
    if (const char* e = std::getenv("MILP_SDUAL_QUEUE_CAP")) {  // wrap-around tests
      cap_ = std::max<int64_t>(2, std::min<int64_t>(SdQueue::kCap, std::atoll(e)));
    }
    (void)hipSetDevice(prev);
  }
  // Called with mu_ held: waits for the previous grid (if any) to drain; the
  // new one starts at the first entry the old dispatcher did not copy.
  void Launch() {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device_);
    if (running_) (void)hipStreamSynchronize(stream_);
    if (stream_ == nullptr && !CreateOwnQueueStream(device_, &stream_)) {
      (void)hipSetDevice(prev);
      throw DeviceError("sdual pool: stream");
    }
    head_base_ = __atomic_load_n(&q_->seen, __ATOMIC_ACQUIRE);
    // The grid claims queue indices from head_base_ on (a synchronous copy:
    // the launch below must see it).
    std::memset(h_ring_, 0, offsetof(SdRing, entry));
    h_ring_->head = static_cast<unsigned long long>(head_base_);
    h_ring_->tail = head_base_;
    if (hipMemcpy(d_ring_, h_ring_, offsetof(SdRing, entry), hipMemcpyHostToDevice) !=
        hipSuccess) {
      (void)hipSetDevice(prev);
      throw DeviceError("sdual pool: ring reset failed");
    }
    __atomic_store_n(&q_->stop, 0, __ATOMIC_RELEASE);
    // Outside batch calls (single solves): a few dozen workers.
    const int groups = GroupsFor(lps_);
    launched_groups_ = groups;
    hipLaunchKernelGGL(sdual_pool_kernel, dim3(groups), dim3(64), kLdsTotalDoubles * sizeof(double), stream_, d_q_, d_ring_,
                       static_cast<long long>(head_base_), static_cast<long long>(cap_));
    const hipError_t e = hipGetLastError();
    (void)hipSetDevice(prev);
    if (e != hipSuccess) throw DeviceError("sdual pool: launch failed");
    running_ = true;
  }

  static int GroupsFor(int lps) { return std::max(kMinPoolGroups, std::min(kPoolGroups, lps + 1)); }
  static std::mutex& RegistryMutex() {
    static std::mutex* mu = new std::mutex();
    return *mu;
  }
  static std::vector<SdualPool*>& Registry() {
    static std::vector<SdualPool*>* all = new std::vector<SdualPool*>();
    return *all;
  }

  int device_;
  std::mutex mu_;
  SdQueue* q_ = nullptr;
  SdQueue* d_q_ = nullptr;
  SdRing* d_ring_ = nullptr;
  SdRing* h_ring_ = nullptr;
  hipStream_t stream_ = nullptr;
  bool running_ = false;
  int64_t head_base_ = 0;
  int64_t cap_ = SdQueue::kCap;
  int users_ = 0;
  int lps_ = 0;
  int launched_groups_ = 0;
  int inflight_ = 0;
};
}  // namespace

void SdualPoolScope(int device, bool begin, int lps) {
  SdualPool& pool = SdualPool::Get(device);
  if (begin) {
    pool.Acquire(lps);
  } else {
    pool.Release(lps);
  }
}

// MILP_SDUAL_PROFILE: reallocations of the arena / mailbox and their time.
namespace {
// How long pooled-segment fibers were away between their polls.
struct GapSum {
  std::atomic<int64_t> total_ns{0}, last_ns{0}, max_ns{0}, polls{0}, segments{0};
  ~GapSum() {
    if (std::getenv("MILP_SDUAL_PROFILE") == nullptr) return;
    std::fprintf(stderr,
                 "  host fiber polls %lld, away %.1f us total, max %.1f us; last gap %.1f us "
                 "over %lld segments\n",
                 static_cast<long long>(polls.load()), total_ns.load() / 1e3, max_ns.load() / 1e3,
                 last_ns.load() / 1e3, static_cast<long long>(segments.load()));
    std::fprintf(stderr, "  host fiber slices > 1 ms: %lld, %.1f us; longest %.1f us\n",
                 static_cast<long long>(fiber_detail::g_slices.long_count.load()),
                 fiber_detail::g_slices.long_ns.load() / 1e3,
                 fiber_detail::g_slices.max_ns.load() / 1e3);
  }
};
GapSum gaps;
// When the pooled segments were enqueued and seen done (ns since the last
// profile reset): the batch's ramp and tail.
struct Timeline {
  std::mutex mu;
  std::chrono::steady_clock::time_point epoch = std::chrono::steady_clock::now();
  std::vector<int64_t> enq, done;
  int64_t Now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                epoch).count();
  }
  static void Print(const char* what, std::vector<int64_t> v) {
    if (v.empty()) return;
    std::sort(v.begin(), v.end());
    auto q = [&](double f) { return v[std::min(v.size() - 1, static_cast<size_t>(f * v.size()))] / 1e6; };
    std::fprintf(stderr, "  host %s ms: p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f\n", what,
                 q(0.0), q(0.1), q(0.5), q(0.9), q(1.0));
  }
  ~Timeline() {
    if (std::getenv("MILP_SDUAL_PROFILE") == nullptr) return;
    Print("segment enqueued at", enq);
    Print("segment done at", done);
  }
};
Timeline timeline;

struct ReserveStats {
  std::atomic<int64_t> reallocs{0}, ns{0};
  ~ReserveStats() {
    if (std::getenv("MILP_SDUAL_PROFILE") == nullptr) return;
    std::fprintf(stderr, "  host reserve reallocs %lld, %.1f us\n",
                 static_cast<long long>(reallocs.load()), ns.load() / 1e3);
  }
};
ReserveStats g_reserve_stats;
}  // namespace

void SdualProfileReset() {
  {
    std::lock_guard<std::mutex> lock(timeline.mu);
    timeline.epoch = std::chrono::steady_clock::now();
    timeline.enq.clear();
    timeline.done.clear();
  }
  for (auto* a : {&gaps.total_ns, &gaps.last_ns, &gaps.max_ns, &gaps.polls, &gaps.segments,
                  &g_reserve_stats.reallocs, &g_reserve_stats.ns, &fiber_detail::g_slices.long_ns,
                  &fiber_detail::g_slices.long_count, &fiber_detail::g_slices.max_ns}) {
    a->store(0);
  }
}

// The arena and staging image grow to twice the first request (a later
// segment's LU or rank-one storage may need more); a reallocation frees the
// old buffers, which waits on the device.
void DeviceLp::SdualReserve(size_t bytes, int rows, int64_t lu_cap) {
  const auto t0 = std::chrono::steady_clock::now();
  bool realloc = false;
  if (bytes > sdual_cap_) {
    realloc = true;
    const size_t cap = std::max(2 * bytes, static_cast<size_t>(1) << 20);
    if (sdual_arena_ != nullptr) {
      Check(hipStreamSynchronize(Stream(stream_)), "sdual sync");
      Check(hipFree(sdual_arena_), "hipFree");
      Check(hipHostFree(sdual_staging_), "hipHostFree");
      sdual_arena_ = nullptr;
      sdual_staging_ = nullptr;
    }
    Check(hipMalloc(&sdual_arena_, cap), "hipMalloc sdual arena");
    Check(hipHostMalloc(&sdual_staging_, cap, hipHostMallocMapped | hipHostMallocCoherent),
          "hipHostMalloc sdual");
    Check(hipHostGetDevicePointer(&sdual_staging_dev_, sdual_staging_, 0), "staging pointer");
    sdual_cap_ = cap;
  }
  const size_t basis_off = 256;
  const size_t image_off = basis_off + ((sizeof(int32_t) * static_cast<size_t>(rows) + 255) & ~size_t{255});
  const size_t mb_bytes = image_off + static_cast<size_t>(lu_cap);
  if (mb_bytes > sdual_mb_cap_) {
    realloc = true;
    if (sdual_mb_block_ != nullptr) Check(hipHostFree(sdual_mb_block_), "hipHostFree mailbox");
    const size_t cap = 2 * mb_bytes;
    Check(hipHostMalloc(&sdual_mb_block_, cap, hipHostMallocMapped | hipHostMallocCoherent),
          "hipHostMalloc mailbox");
    Check(hipHostGetDevicePointer(&sdual_mb_device_, sdual_mb_block_, 0), "mailbox pointer");
    sdual_mb_cap_ = cap;
  }
  char* base = static_cast<char*>(sdual_mb_block_);
  sdual_mb_ = reinterpret_cast<sdual::Mailbox*>(base);
  sdual_mb_basis_ = reinterpret_cast<int32_t*>(base + basis_off);
  sdual_mb_image_ = base + image_off;
  std::memset(base, 0, sizeof(sdual::Mailbox));
  sdual_mb_->image_cap = lu_cap;
  if (realloc) {
    ++g_reserve_stats.reallocs;
    g_reserve_stats.ns += std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0).count();
  }
}

void DeviceLp::SdualMailboxDevice(sdual::Mailbox** mb, int32_t** basis, char** image) const {
  char* d = static_cast<char*>(sdual_mb_device_);
  const char* h = static_cast<const char*>(sdual_mb_block_);
  *mb = reinterpret_cast<sdual::Mailbox*>(d);
  *basis = reinterpret_cast<int32_t*>(d + (reinterpret_cast<const char*>(sdual_mb_basis_) - h));
  *image = d + (sdual_mb_image_ - h);
}

void DeviceLp::SdualFree() {
  if (sdual_arena_ != nullptr) {
    (void)hipStreamSynchronize(Stream(stream_));
    (void)hipFree(sdual_arena_);
    (void)hipHostFree(sdual_staging_);
  }
  if (sdual_mb_block_ != nullptr) (void)hipHostFree(sdual_mb_block_);
  sdual_arena_ = nullptr;
  sdual_staging_ = nullptr;
  sdual_cap_ = 0;
  sdual_mb_block_ = nullptr;
  sdual_mb_cap_ = 0;
}

void DeviceLp::SdualMatrix(const int64_t** starts, const int32_t** rows, const double** vals,
                           const int64_t** t_starts, const int32_t** t_cols,
                           const double** t_vals) const {
  *starts = d_starts_;
  *rows = d_rows_;
  *vals = d_vals_;
  *t_starts = d_t_starts_;
  *t_cols = d_t_cols_;
  *t_vals = d_t_vals_;
}

void DeviceLp::SdualRun(size_t bytes, const double* arena_coeff, int n, void (*serve)(void*),
                        void* ctx) {
  static const bool pool = [] {
    const char* e = std::getenv("MILP_SDUAL_POOL");
    return e == nullptr || std::atoi(e) != 0;
  }();
  if (pool) {
    SdualRunPooled(bytes, arena_coeff, n, serve, ctx);
    return;
  }
  DeviceOp("sdual segment");
  if (batch_pending_) WaitSmallBatch();
  BeginKernel(MI_K_SDUAL);
  Check(hipMemcpyAsync(sdual_arena_, sdual_staging_, bytes, hipMemcpyHostToDevice,
                       Stream(stream_)),
        "sdual H2D");
  hipLaunchKernelGGL(sdual_segment_kernel, dim3(1), dim3(64), kLdsTotalDoubles * sizeof(double), Stream(stream_),
                     reinterpret_cast<sdual::Lp*>(sdual_arena_));
  Check(hipGetLastError(), "sdual launch");
  // The segment's last update row becomes the device copy that later device
  // update-row reads see (update_row.cc coefficient_, non-listed positions
  // included).
  if (d_coeff_ != nullptr && n > 0) {
    Check(hipMemcpyAsync(d_coeff_, arena_coeff, sizeof(double) * static_cast<size_t>(n),
                         hipMemcpyDeviceToDevice, Stream(stream_)),
          "sdual coefficients");
  }
  Check(hipMemcpyAsync(sdual_staging_, sdual_arena_, bytes, hipMemcpyDeviceToHost,
                       Stream(stream_)),
        "sdual D2H");
  EndKernel(MI_K_SDUAL, 2.0 * static_cast<double>(bytes));
  // Answer factorization requests until the stream (kernel, copies) is done.
  int32_t* flag = &sdual_mb_->flag;
  bool idle = false;  // the slice since the last resume found nothing to do
  while (true) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == 1) {
      DeviceOp("sdual factorization request");
      serve(ctx);
      __atomic_store_n(flag, 2, __ATOMIC_RELEASE);
      idle = false;
      continue;
    }
    const hipError_t q = hipStreamQuery(Stream(stream_));
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) Check(q, "sdual segment");
    if (InFiber()) {
      FiberYield(idle);
      idle = true;
      RestoreDevice();
    } else {
      std::this_thread::yield();
    }
  }
  DeviceOp("sdual segment done");
}

// ---------------------------------------------------------------------------
// LU servers: with hundreds of LPs on a few host threads' fibers, a fiber sees
// its segment's factorization request only when the round robin comes back to
// it (a whole cycle of other LPs' host work). Server threads
// (MILP_SDUAL_SERVERS, default 4; 0 = the fibers alone) scan the mailboxes of
// the running pooled segments and answer at once. The mailbox flag arbitrates:
// whoever moves it 1 -> 4 serves, then stores 2. The requesting LP's host
// objects are idle meanwhile (its fiber waits in SdualRunPooled), and the
// answer is published by the release store of 2.
class LuServers {
 public:
  static constexpr int kSlots = 8192;
  static LuServers* Get() {
    static LuServers* s = [] {
      LuServers* created = new LuServers();  // never destroyed; threads joined by Shutdown
      g_instance.store(created, std::memory_order_release);
      RegisterDeviceShutdown();
      return created;
    }();
    return s;
  }
  // Process teardown: the server threads stop polling the mailboxes (mapped
  // host memory the HIP runtime frees at exit) and are joined; later
  // segments are served by their own fibers.
  static void ShutdownAll() {
    LuServers* s = g_instance.load(std::memory_order_acquire);
    if (s == nullptr) return;
    s->stop_.store(true, std::memory_order_release);
    for (std::thread& t : s->workers_) {
      if (t.joinable()) t.join();
    }
    s->threads_ = 0;
  }
  bool enabled() const { return threads_ > 0 && !stop_.load(std::memory_order_acquire); }
  int Register(int32_t* flag, void (*serve)(void*), void* ctx) {
    std::lock_guard<std::mutex> lock(mu_);
    int slot;
    if (!free_.empty()) {
      slot = free_.back();
      free_.pop_back();
    } else {
      if (used_ >= kSlots) return -1;
      slot = used_++;
    }
    Slot& sl = slots_[slot];
    sl.serve = serve;
    sl.ctx = ctx;
    sl.flag.store(flag, std::memory_order_release);
    if (slot + 1 > hi_.load(std::memory_order_relaxed)) hi_.store(slot + 1, std::memory_order_release);
    return slot;
  }
  // Returns once no server is inside this slot's service.
  void Unregister(int slot) {
    if (slot < 0) return;
    Slot& sl = slots_[slot];
    sl.flag.store(nullptr, std::memory_order_seq_cst);
    while (sl.busy.load(std::memory_order_seq_cst)) std::this_thread::yield();
    std::lock_guard<std::mutex> lock(mu_);
    free_.push_back(slot);
  }
  // Claims a pending request of `flag` (1 -> 4) for the caller to serve.
  static bool Claim(int32_t* flag) {
    int32_t expected = 1;
    return __atomic_compare_exchange_n(flag, &expected, 4, false, __ATOMIC_ACQ_REL,
                                       __ATOMIC_ACQUIRE);
  }

 private:
  struct Slot {
    std::atomic<int32_t*> flag{nullptr};
    std::atomic<bool> busy{false};
    void (*serve)(void*) = nullptr;
    void* ctx = nullptr;
  };
  LuServers() {
    int n = 4;
    if (const char* e = std::getenv("MILP_SDUAL_SERVERS")) n = std::max(0, std::atoi(e));
    threads_ = n;
    for (int t = 0; t < n; ++t) workers_.emplace_back([this, t, n] { Loop(t, n); });
  }
  void Loop(int t, int n) {
    int idle = 0;
    while (!stop_.load(std::memory_order_acquire)) {
      bool served = false;
      const int hi = hi_.load(std::memory_order_acquire);
      for (int i = t; i < hi; i += n) {
        Slot& sl = slots_[i];
        int32_t* flag = sl.flag.load(std::memory_order_acquire);
        if (flag == nullptr || __atomic_load_n(flag, __ATOMIC_ACQUIRE) != 1) continue;
        sl.busy.store(true, std::memory_order_seq_cst);
        // Re-read after raising busy: Unregister clears the flag pointer first.
        if (sl.flag.load(std::memory_order_seq_cst) == flag && Claim(flag)) {
          sl.serve(sl.ctx);
          __atomic_store_n(flag, 2, __ATOMIC_RELEASE);
          served = true;
        }
        sl.busy.store(false, std::memory_order_release);
      }
      if (served) {
        idle = 0;
      } else if (++idle > 64) {
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      } else {
        std::this_thread::yield();
      }
    }
  }
  static std::atomic<LuServers*> g_instance;
  int threads_ = 0;
  std::atomic<bool> stop_{false};
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::vector<int> free_;
  int used_ = 0;
  std::atomic<int> hi_{0};
  Slot slots_[kSlots];
};

std::atomic<LuServers*> LuServers::g_instance{nullptr};

void SdualShutdown() {
  LuServers::ShutdownAll();
  SdualPool::ShutdownAll();
}

// The same segment through the device's persistent pool kernel: a resident
// workgroup moves the staging image in and out itself (no stream work, so
// nothing queues behind the resident grid), and signals completion through
// the mailbox flag (3). Many LPs' segments run at once.
void DeviceLp::SdualRunPooled(size_t bytes, const double* arena_coeff, int n,
                              void (*serve)(void*), void* ctx) {
  (void)bytes;
  (void)arena_coeff;
  (void)n;
  DeviceOp("sdual pooled segment");
  WaitStream();  // nothing of this handle's may still write d_coeff_
  sdual::Lp* hs = reinterpret_cast<sdual::Lp*>(sdual_staging_);
  hs->staging_dev = reinterpret_cast<uint64_t>(sdual_staging_dev_);
  hs->coeff_out = d_coeff_;
  int32_t* flag = &sdual_mb_->flag;
  __atomic_store_n(flag, 0, __ATOMIC_RELEASE);
  SdualPool& pool = SdualPool::Get(device_);
  LuServers* servers = LuServers::Get();
  const int slot = servers->enabled() ? servers->Register(flag, serve, ctx) : -1;
  struct Unreg {
    LuServers* s;
    int slot;
    ~Unreg() { s->Unregister(slot); }
  } unreg{servers, slot};
  if (std::getenv("MILP_SDUAL_PROFILE") != nullptr) {
    std::lock_guard<std::mutex> lock(timeline.mu);
    timeline.enq.push_back(timeline.Now());
  }
  // Algorithmic work of the segment: Glop's own operation counts (the
  // deterministic-time counters, 2e-9 s per operation, lp_types.h:421-424),
  // 12 bytes per operation (an 8-byte value and a 4-byte index), plus the
  // arena bytes the workgroup moves in and out.
  const double dt_before = sdual::rs_deterministic_time(*hs);
  const double moved = 2.0 * sizeof(sdual::Lp) +
                       static_cast<double>(hs->fixed_end - hs->mutable_begin) +
                       static_cast<double>(hs->scratch_end - hs->scratch_begin);
  pool.Enqueue(sdual_staging_dev_);
  int64_t polls = 0;
  static const bool debug = std::getenv("MILP_SDUAL_DEBUG") != nullptr;
  // MILP_SDUAL_PROFILE: how long the fiber was away between its polls (the
  // last gap bounds the delay in seeing the segment done).
  static const bool prof = std::getenv("MILP_SDUAL_PROFILE") != nullptr;
  int64_t gap_ns = 0;
  bool idle = false;  // the slice since the last resume found nothing to do
  const auto t0 = std::chrono::steady_clock::now();
  int64_t next_report = 1;
  while (true) {
    const int32_t f = __atomic_load_n(flag, __ATOMIC_ACQUIRE);
    if (debug) {
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (s > next_report) {
        const volatile int64_t* d = pool.Dbg();
        std::fprintf(stderr,
                     "sdual pooled: %.0fs flag=%d alive=%d tail=%lld seen=%lld claimed=%lld "
                     "stage=%lld iterations=%lld out=%lld stage_ptr=%llx staging_dev=%p\n",
                     s, f, pool.Alive() ? 1 : 0, static_cast<long long>(pool.Tail()),
                     static_cast<long long>(d[0]), static_cast<long long>(d[1]),
                     static_cast<long long>(d[2]), static_cast<long long>(d[3]),
                     static_cast<long long>(d[4]), static_cast<unsigned long long>(d[5]),
                     sdual_staging_dev_);
        next_report += 1;
      }
    }
    if (f == 3) {
      pool.Done();
      if (prof) {
        gaps.last_ns += gap_ns;
        ++gaps.segments;
        std::lock_guard<std::mutex> lock(timeline.mu);
        timeline.done.push_back(timeline.Now());
      }
      break;
    }
    if (f == 1 && LuServers::Claim(flag)) {
      DeviceOp("sdual factorization request");
      serve(ctx);
      __atomic_store_n(flag, 2, __ATOMIC_RELEASE);
      idle = false;
      continue;
    }
    if ((++polls & 1023) == 0 && __atomic_load_n(flag, __ATOMIC_ACQUIRE) == 0) {
      // The grid may have drained (idle limit, stop word) before copying this
      // entry: a new grid starts from the first uncopied entry.
      pool.EnsureRunning();
    }
    const auto y0 = prof ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
    if (InFiber()) {
      FiberYield(idle);
      idle = true;
      RestoreDevice();
    } else {
      std::this_thread::yield();
    }
    if (prof) {
      gap_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now() - y0).count();
      gaps.total_ns += gap_ns;
      ++gaps.polls;
      int64_t m = gaps.max_ns.load();
      while (gap_ns > m && !gaps.max_ns.compare_exchange_weak(m, gap_ns)) {
      }
    }
  }
  ++stats_.launches[MI_K_SDUAL];
  {
    const double ops = (sdual::rs_deterministic_time(*hs) - dt_before) / 2e-9;
    stats_.algorithmic_bytes[MI_K_SDUAL] +=
        12.0 * ops + moved + static_cast<double>(hs->mutable_end - hs->mutable_begin);
    // The workgroup's own time (wall_clock64, 100 MHz): the loop phases and
    // the arena transfers.
    uint64_t ticks = 0;
    for (int k : {0, 1, 2, 3, 4, 5, 6, 7, 8, 13, 14}) ticks += hs->phase_ticks[k];
    stats_.device_ms[MI_K_SDUAL] += static_cast<double>(ticks) / 1e5;
  }
  DeviceOp("sdual pooled segment done");
}

}  // namespace milp
