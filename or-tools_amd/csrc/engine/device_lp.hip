// DeviceLp: device buffers + kernel launch plumbing (see device_lp.h).
#include "device_lp.h"
#include "fibers.h"
#include "host_pool.h"

#include <algorithm>
#include <hip/hip_runtime.h>

#include <atomic>
#include <limits>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <rocprim/device/device_radix_sort.hpp>

#include <chrono>
#include <cstdlib>
#include <cstring>

#include "lp_data.h"

#include "../kernels/kernel_args.h"

namespace milp {

namespace {
inline hipStream_t S(void* p) { return reinterpret_cast<hipStream_t>(p); }

// Host wall time of one public DeviceLp call, accumulated into call_ms[id].
struct CallTimer {
  mi_lp_kernel_stats* stats;
  int id;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  CallTimer(mi_lp_kernel_stats* s, int i) : stats(s), id(i) {}
  ~CallTimer() {
    stats->call_ms[id] += std::chrono::duration<double, std::milli>(
                              std::chrono::steady_clock::now() - t0)
                              .count();
  }
};
}  // namespace

void DeviceLp::Check(int err, const char* what) {
  if (err != hipSuccess) {
    throw DeviceError(std::string(what) + ": " +
                      hipGetErrorString(static_cast<hipError_t>(err)));
  }
}

namespace {
void StartWatchdog();
}  // namespace

void ReleaseSmallBatchSlot(int device, int slot);  // below, with SmallBatcher

DeviceLp::~DeviceLp() {
  if (device_ >= 0) (void)hipSetDevice(device_);
  bool slot_idle = true;
  try {
    WaitSmallBatch();  // a batched request may still write this handle's buffers
  } catch (const std::exception&) {
    // The request never completed: its slot is not returned to the pool (a
    // later owner would take the stale sequence number for its own).
    slot_idle = false;
  }
  if (batch_slot_ >= 0 && slot_idle) ReleaseSmallBatchSlot(device_, batch_slot_);
  if (stream_ != nullptr) (void)hipStreamSynchronize(S(stream_));
  SdualFree();
  FreeTriBuffers();
  for (void* p : allocations_) (void)hipFree(p);
  if (h_pin_i_) (void)hipHostFree(h_pin_i_);
  if (h_pin_d_) (void)hipHostFree(h_pin_d_);
  if (h_pin_d2_) (void)hipHostFree(h_pin_d2_);
  if (h_pin_w_) (void)hipHostFree(h_pin_w_);
  if (h_upd_in_) (void)hipHostFree(h_upd_in_);
  if (h_pin_count_) (void)hipHostFree(h_pin_count_);
  if (h_map_) (void)hipHostFree(h_map_);
  if (h_small_in_) (void)hipHostFree(h_small_in_);
  if (h_scan_fail_) (void)hipHostFree(h_scan_fail_);
  for (void* p : {static_cast<void*>(h_cand_col_), static_cast<void*>(h_cand_coeff_),
                  static_cast<void*>(h_cand_rc_), static_cast<void*>(h_dual_counts_),
                  static_cast<void*>(h_cb_cols_), static_cast<void*>(h_cb_bits_),
                  static_cast<void*>(h_flip_cols_), static_cast<void*>(h_flip_flags_)}) {
    if (p) (void)hipHostFree(p);
  }
  if (ev_flips_ != nullptr) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev_flips_));
  for (void* e : ev_cb_) {
    if (e) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e));
  }
  if (h_mask_diff_) (void)hipHostFree(h_mask_diff_);
  for (int k = 0; k < kNumMasks; ++k) {
    if (h_pin_mask_[k]) (void)hipHostFree(h_pin_mask_[k]);
    if (ev_mask_[k]) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev_mask_[k]));
  }
  if (ev_start_) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev_start_));
  if (ev_stop_) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev_stop_));
  for (const PendingTiming& t : ev_pending_) {
    ev_pool_.push_back(t.start);
    ev_pool_.push_back(t.stop);
  }
  if (ev_open_ != nullptr) ev_pool_.push_back(ev_open_);
  for (void* e : ev_pool_) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e));
  if (stream_) (void)hipStreamDestroy(S(stream_));
}

void DeviceLp::Init(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
    throw DeviceError("no HIP device visible (the MI355X engine has no CPU fallback)");
  }
  if (device < 0 || device >= count) throw DeviceError("bad device ordinal");
  device_ = device;
  Check(hipSetDevice(device), "hipSetDevice");
  // The stream starts at the default priority; UploadMatrix sets it
  // (SetStreamPriority).
  if (const char* v = std::getenv("MILP_STREAM_PRIORITY")) stream_priority_ = std::atoi(v) != 0;
  stream_priority_env_ = stream_priority_;
  hipStream_t s;
  Check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
  stream_prioritized_ = false;
  hipEvent_t a, b;
  Check(hipEventCreate(&a), "hipEventCreate");
  Check(hipEventCreate(&b), "hipEventCreate");
  ev_start_ = a;
  ev_stop_ = b;
  for (int k = 0; k < kNumMasks; ++k) {
    hipEvent_t e;
    Check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    ev_mask_[k] = e;
  }
  if (const char* u = std::getenv("MILP_DENSE_UNROLL")) {
    const int v = std::atoi(u);
    if (v == 8 || v == 16 || v == 32) dense_unroll_ = v;
  }
  if (const char* t = std::getenv("MILP_DUAL_TIGHTEN_MIN")) {
    tighten_min_candidates_ = std::atoi(t);
  }
  if (const char* t = std::getenv("MILP_DUAL_TIGHTEN_SORT")) tighten_sort_ = std::atoi(t) != 0;
  tighten_target_ = milp_kernels::kTightenTarget;
  if (const char* t = std::getenv("MILP_TIGHTEN_TARGET")) tighten_target_ = std::atoi(t);
  if (const char* r = std::getenv("MILP_ROWWISE_CHUNK_MAX_ROWS")) {
    rowwise_chunk_max_rows_ = std::atoi(r);
  }
  if (const char* f = std::getenv("MILP_FULL_ROWS")) {
    full_rows_enabled_ = std::strcmp(f, "off") != 0;
  }
  if (const char* f = std::getenv("MILP_SMALL_FUSED")) {
    small_fused_enabled_ = std::strcmp(f, "off") != 0;
  }
  if (const char* r = std::getenv("MILP_SMALL_SERIAL_ROWS")) small_serial_rows_ = std::atoi(r);
  if (const char* r = std::getenv("MILP_SMALL_THREADS")) small_threads_ = std::atoi(r);
  if (const char* f = std::getenv("MILP_MEDIUM")) medium_enabled_ = std::strcmp(f, "off") != 0;
  if (const char* v = std::getenv("MILP_DEVICE_SOLVE")) {
    if (std::strcmp(v, "force") == 0) tri_mode_ = 1;
    if (std::strcmp(v, "off") == 0) tri_mode_ = 2;
  }
  if (const char* v = std::getenv("MILP_DEVICE_SOLVE_MIN_ROWS")) tri_min_rows_ = std::atoi(v);
  if (const char* v = std::getenv("MILP_TRI_WIDE")) tri_wide_level_ = std::atoi(v);
  // MILP_TRI_GRAPH=0: launch the plan kernel by kernel instead of replaying
  // a captured graph; MILP_TRI_TAU=0: the tau worker keeps the host loop.
  if (const char* v = std::getenv("MILP_TRI_GRAPH")) tri_graph_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_TAU")) tri_tau_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_MAPPED")) tri_mapped_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_SYNCFREE")) tri_syncfree_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_LOWER")) tri_lower_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_BTRAN")) tri_btran_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_PAIR")) tri_pair_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_SPEC_FLIP")) spec_flip_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_EARLY_FLIPS")) early_flips_on_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_PAD")) tri_pad_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_DENSE_TAIL")) dense_tail_mode_ = std::atoi(v);
  if (const char* v = std::getenv("MILP_DENSE_TAIL_MIN_ENTRIES")) {
    dense_tail_min_entries_ = std::atoll(v);
  }
  if (const char* v = std::getenv("MILP_DENSE_TAIL_MIN_COLS")) {
    dense_tail_min_cols_ = std::max(1, std::atoi(v));
  }
  if (const char* v = std::getenv("MILP_TRI_MIN_WIDTH")) tri_min_width_ = std::atoi(v);
  if (const char* v = std::getenv("MILP_TRI_CHAIN")) tri_chain_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_CHAIN_WIDTH")) tri_chain_width_ = std::atoi(v);
  if (const char* v = std::getenv("MILP_TRI_CHAIN_MIN_LEVELS")) {
    tri_chain_min_levels_ = std::max(1, std::atoi(v));
  }
  if (const char* v = std::getenv("MILP_TRI_SYNCFREE_MIN_LEVELS")) {
    tri_syncfree_min_levels_ = std::atoi(v);
  }
  if (const char* v = std::getenv("MILP_TRI_FUSE0")) tri_fuse0_ = std::atoi(v) != 0;
  if (const char* v = std::getenv("MILP_TRI_POLL_MAX")) tri_poll_max_ = std::max(1, std::atoi(v));
  if (const char* v = std::getenv("MILP_TRI_PERSIST")) {
    tri_persist_groups_ = std::max(0, std::min(256, std::atoi(v)));
  }
  if (const char* v = std::getenv("MILP_TRI_XCD")) tri_xcd_stride_ = std::atoi(v) != 0 ? 8 : 1;
  if (const char* v = std::getenv("MILP_SMALL_BATCH")) small_batch_ = std::atoi(v) != 0;
  CreateShards();
  StartWatchdog();
}

template <typename T>
T* DeviceLp::Alloc(size_t n) {
  void* p = nullptr;
  Check(hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)), "hipMalloc");
  allocations_.push_back(p);
  return static_cast<T*>(p);
}

void DeviceLp::Upload(void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return;
  if (batch_pending_) WaitSmallBatch();  // stream work after a batched request
  Check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, S(stream_)), "H2D");
}

// MILP_WATCHDOG_S=k: a thread that reports the last device operation when
// none has started or finished for k seconds (hang diagnosis on the GPU box).
std::atomic<const char*> g_dev_op{"none"};
std::atomic<uint64_t> g_dev_ops{0};

void DeviceOp(const char* what) {
  g_dev_op.store(what, std::memory_order_relaxed);
  g_dev_ops.fetch_add(1, std::memory_order_relaxed);
}

namespace {
void StartWatchdog() {
  static std::once_flag once;
  std::call_once(once, []() {
    const char* e = std::getenv("MILP_WATCHDOG_S");
    if (e == nullptr || std::atoi(e) <= 0) return;
    const int secs = std::atoi(e);
    std::thread([secs]() {
      uint64_t last = ~0ull;
      int still = 0;
      while (true) {
        std::this_thread::sleep_for(std::chrono::seconds(1));
        const uint64_t n = g_dev_ops.load(std::memory_order_relaxed);
        still = n == last ? still + 1 : 0;
        last = n;
        if (still == secs) {
          std::fprintf(stderr, "[watchdog] no device operation for %d s; last: %s (#%llu)\n",
                       secs, g_dev_op.load(std::memory_order_relaxed),
                       static_cast<unsigned long long>(n));
          std::fflush(stderr);
        }
      }
    }).detach();
  });
}
}  // namespace

// ---------------------------------------------------------------------------
// SmallBatcher: one per device. Handles of small LPs post their one-launch
// update rows (and list dots) as requests; whichever thread finds no launch
// under way becomes the launcher and sends every pending request of a kind
// in one launch of small_batch_kernel (one workgroup per request) on the
// batcher's stream, until nothing is pending. A request's completion is a
// sequence number the kernel writes into mapped memory: waiting costs no HIP
// call. Many small LPs then cost one HIP launch per batch instead of one per
// LP iteration (the HIP launch path serializes launches from many threads).
namespace {
class SmallBatcher {
 public:
  static constexpr int kMaxSlots = 2048;
  static SmallBatcher& Get(int device) {
    // Never destroyed: the launcher thread is stopped and joined by
    // ShutdownAll (mi_lp_shutdown / the atexit handler) before the HIP
    // runtime goes away.
    std::lock_guard<std::mutex> lock(RegistryMutex());
    std::vector<SmallBatcher*>& all = Registry();
    if (static_cast<int>(all.size()) <= device) all.resize(device + 1, nullptr);
    if (all[device] == nullptr) {
      all[device] = new SmallBatcher(device);
      RegisterDeviceShutdown();
    }
    return *all[device];
  }
  static void ShutdownAll() {
    std::lock_guard<std::mutex> lock(RegistryMutex());
    for (SmallBatcher* b : Registry()) {
      if (b != nullptr) b->Stop();
    }
  }
  int AddSlot() {
    std::lock_guard<std::mutex> lock(mu_);
    if (!free_slots_.empty()) {
      const int id = free_slots_.back();
      free_slots_.pop_back();
      return id;
    }
    if (next_slot_ >= kMaxSlots) throw DeviceError("small batch: too many handles");
    return next_slot_++;
  }
  // A slot whose last request has completed goes back to the pool; its done
  // word keeps the last sequence number, the next owner starts above it.
  void FreeSlot(int id) {
    std::lock_guard<std::mutex> lock(mu_);
    free_slots_.push_back(id);
  }
  milp_kernels::SmallSlot* slot(int id) { return h_slots_ + id; }
  unsigned long long done(int id) const {
    return __atomic_load_n(h_done_ + id, __ATOMIC_ACQUIRE);
  }
  void Submit(int kind, int id) {
    {
      std::unique_lock<std::mutex> lock(mu_);
      // A Stop() in progress owns the launcher and the streams until it has
      // joined the one and destroyed the others; a restart waits for it.
      stopped_cv_.wait(lock, [&] { return !stopping_; });
      pending_[kind].push_back(id);
      ++num_pending_;
      if (!launcher_.joinable()) {  // stopped by ShutdownAll: start again
        stop_ = false;
        CreateStreams();
        launcher_ = std::thread([this] { LauncherLoop(); });
      }
    }
    cv_.notify_one();
  }

  ~SmallBatcher() { Stop(); }
  // The launcher finishes the requests already pending, then exits. The
  // thread object moves out under the lock and `stopping_` holds off
  // restarts (Submit) and other Stop() calls until the streams are gone.
  void Stop() {
    std::thread launcher;
    {
      std::unique_lock<std::mutex> lock(mu_);
      stopped_cv_.wait(lock, [&] { return !stopping_; });
      if (!launcher_.joinable()) return;  // never started, or already stopped
      stop_ = true;
      stopping_ = true;
      launcher = std::move(launcher_);
    }
    cv_.notify_one();
    launcher.join();
    {
      std::lock_guard<std::mutex> lock(mu_);
      for (hipStream_t& st : streams_) {
        if (st != nullptr) (void)hipStreamDestroy(st);
        st = nullptr;
      }
      stopping_ = false;
    }
    stopped_cv_.notify_all();
  }

 private:
  void CreateStreams() {
    (void)hipSetDevice(device_);
    if (const char* e = std::getenv("MILP_SMALL_BATCH_STREAMS")) {
      streams_used_ = std::max(1, std::min(kStreams, std::atoi(e)));
    }
    for (int i = 0; i < kStreams; ++i) {
      hipStream_t st;
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        throw DeviceError("small batch: stream");
      }
      streams_[i] = st;
      if (events_[i] == nullptr &&
          hipEventCreateWithFlags(&events_[i], hipEventDisableTiming) != hipSuccess) {
        throw DeviceError("small batch: event");
      }
      in_flight_[i] = false;
    }
  }
  static std::mutex& RegistryMutex() {
    static std::mutex* mu = new std::mutex();
    return *mu;
  }
  static std::vector<SmallBatcher*>& Registry() {
    static std::vector<SmallBatcher*>* all = new std::vector<SmallBatcher*>();
    return *all;
  }
  // The launcher: takes every pending request, launches one kernel per kind
  // (a workgroup per request) on one of its streams, repeats. Up to
  // `streams_used_` batches are in flight (MILP_SMALL_BATCH_STREAMS, default
  // 4): a request that arrives while batches run is launched at once on a
  // free stream instead of waiting for the running batch (whose time is its
  // slowest request: the mid-size LPs' update rows made every small LP wait
  // for them). With every stream busy the launcher waits for the oldest
  // batch; meanwhile the other LPs' requests gather into the next one.
  void LauncherLoop() {
    (void)hipSetDevice(device_);
    std::vector<int> batch[milp_kernels::kSmallKinds];
    int next = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lock(mu_);
        cv_.wait(lock, [&] { return stop_ || num_pending_ > 0; });
        if (stop_ && num_pending_ == 0) break;
      }
      // A free stream: the next in turn, once its last batch has completed.
      const int s = next;
      next = (next + 1) % streams_used_;
      if (in_flight_[s]) {
        (void)hipEventSynchronize(events_[s]);
        in_flight_[s] = false;
      }
      {
        std::lock_guard<std::mutex> lock(mu_);
        for (int k = 0; k < milp_kernels::kSmallKinds; ++k) {
          batch[k].swap(pending_[k]);
          pending_[k].clear();
        }
        num_pending_ = 0;
      }
      bool failed = false;
      for (int k = 0; k < milp_kernels::kSmallKinds && !failed; ++k) {
        for (size_t at = 0; at < batch[k].size(); at += milp_kernels::kSmallBatchMax) {
          milp_kernels::SmallBatchArgs a{};
          a.slots = m_slots_;
          a.done = m_done_;
          a.count = static_cast<int>(
              std::min<size_t>(milp_kernels::kSmallBatchMax, batch[k].size() - at));
          for (int i = 0; i < a.count; ++i) a.ids[i] = batch[k][at + i];
          if (milp_launch::small_batch(k, a, streams_[s]) != hipSuccess) failed = true;
        }
        batch[k].clear();
      }
      // A failed launch leaves its requests without a done word: their
      // owners time out and report a DeviceError.
      if (hipEventRecord(events_[s], streams_[s]) == hipSuccess) {
        in_flight_[s] = true;
      } else {
        (void)hipStreamSynchronize(streams_[s]);
      }
    }
    for (int s = 0; s < streams_used_; ++s) {
      if (in_flight_[s]) (void)hipEventSynchronize(events_[s]);
      in_flight_[s] = false;
    }
  }

 private:
  explicit SmallBatcher(int device) : device_(device) {
    CreateStreams();
    void* p = nullptr;
    void* d = nullptr;
    if (hipHostMalloc(&p, sizeof(milp_kernels::SmallSlot) * kMaxSlots, hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
      throw DeviceError("small batch: slots");
    }
    std::memset(p, 0, sizeof(milp_kernels::SmallSlot) * kMaxSlots);
    h_slots_ = static_cast<milp_kernels::SmallSlot*>(p);
    m_slots_ = static_cast<const milp_kernels::SmallSlot*>(d);
    if (hipHostMalloc(&p, sizeof(unsigned long long) * kMaxSlots, hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
      throw DeviceError("small batch: done words");
    }
    std::memset(p, 0, sizeof(unsigned long long) * kMaxSlots);
    h_done_ = static_cast<unsigned long long*>(p);
    m_done_ = static_cast<unsigned long long*>(d);
    launcher_ = std::thread([this] { LauncherLoop(); });
  }
  int device_;
  static constexpr int kStreams = 8;
  int streams_used_ = 4;
  hipStream_t streams_[kStreams] = {};
  hipEvent_t events_[kStreams] = {};  // each stream's last batch
  bool in_flight_[kStreams] = {};
  std::mutex mu_;
  std::condition_variable cv_;
  std::condition_variable stopped_cv_;  // a Stop() in progress has finished
  bool stopping_ = false;
  std::thread launcher_;
  bool stop_ = false;
  int num_pending_ = 0;
  std::vector<int> pending_[milp_kernels::kSmallKinds];
  int next_slot_ = 0;
  std::vector<int> free_slots_;
  milp_kernels::SmallSlot* h_slots_ = nullptr;
  const milp_kernels::SmallSlot* m_slots_ = nullptr;
  unsigned long long* h_done_ = nullptr;
  unsigned long long* m_done_ = nullptr;
};

void SetSlotArgs(milp_kernels::SmallSlot* s, const milp_kernels::RowWiseSmallArgs& a) { s->rw = a; }
void SetSlotArgs(milp_kernels::SmallSlot* s, const milp_kernels::ColWiseSmallArgs& a) { s->cw = a; }
void SetSlotArgs(milp_kernels::SmallSlot* s, const milp_kernels::ListDotsSmallArgs& a) { s->ld = a; }
void SetSlotArgs(milp_kernels::SmallSlot* s, const milp_kernels::RowWiseSmallColArgs& a) {
  s->rc = a;
}
}  // namespace

void ReleaseSmallBatchSlot(int device, int slot) { SmallBatcher::Get(device).FreeSlot(slot); }

void ShutdownDevices() {
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  SdualShutdown();
  SmallBatcher::ShutdownAll();
}

// std::atexit from the first long-lived device object: registered after the
// HIP runtime initialized, so it runs before the runtime's own exit-time
// teardown (atexit handlers and static destructors run in reverse order of
// registration).
void RegisterDeviceShutdown() {
  static std::once_flag once;
  std::call_once(once, [] { std::atexit([] { ShutdownDevices(); }); });
}

template <typename Args>
void DeviceLp::LaunchSmall(int kind, const Args& args) {
  // The dual device mode reads the update row on this handle's own stream
  // without a host wait in between: its small LPs keep the single launch.
  if (!small_batch_ || dual_ready_) {
    hipError_t e = hipSuccess;
    switch (kind) {
      case milp_kernels::kSmallRowWise:
        e = milp_launch::row_wise_update_small(
            reinterpret_cast<const milp_kernels::RowWiseSmallArgs&>(args), small_threads_,
            S(stream_));
        break;
      case milp_kernels::kMediumRowWise:
        e = milp_launch::row_wise_update_medium(
            reinterpret_cast<const milp_kernels::RowWiseSmallArgs&>(args), S(stream_));
        break;
      case milp_kernels::kSmallColWise:
        e = milp_launch::column_wise_update_small(
            reinterpret_cast<const milp_kernels::ColWiseSmallArgs&>(args), S(stream_));
        break;
      case milp_kernels::kSmallListDots:
        e = milp_launch::list_dots_small(
            reinterpret_cast<const milp_kernels::ListDotsSmallArgs&>(args), S(stream_));
        break;
      case milp_kernels::kMediumListDots:
        e = milp_launch::list_dots_medium(
            reinterpret_cast<const milp_kernels::ListDotsSmallArgs&>(args), S(stream_));
        break;
      default:
        e = milp_launch::row_wise_update_small_by_column(
            reinterpret_cast<const milp_kernels::RowWiseSmallColArgs&>(args), S(stream_));
        break;
    }
    Check(e, "small launch");
    return;
  }
  // The batch kernel runs on the batcher's stream: this handle's own stream
  // must have nothing in flight that the request reads.
  if (hipStreamQuery(S(stream_)) != hipSuccess) Check(hipStreamSynchronize(S(stream_)), "sync");
  if (batch_pending_) WaitSmallBatch();
  SmallBatcher& b = SmallBatcher::Get(device_);
  if (batch_slot_ < 0) {
    batch_slot_ = b.AddSlot();
    batch_seq_ = b.done(batch_slot_);  // continue above the previous owner's numbers
  }
  milp_kernels::SmallSlot* slot = b.slot(batch_slot_);
  SetSlotArgs(slot, args);
  slot->kind = kind;
  slot->seq = ++batch_seq_;
  batch_pending_ = true;
  b.Submit(kind, batch_slot_);
}

void DeviceLp::SetSmallBatch(bool on) {
  if (!on) WaitSmallBatch();  // the last request completes before single launches resume
  if (const char* v = std::getenv("MILP_SMALL_BATCH")) on = std::atoi(v) != 0;
  small_batch_ = on;
}

void DeviceLp::SetBatchPriority(bool high) {
  stream_priority_ = high || stream_priority_env_;
  if (m_ > 0) SetStreamPriority(stream_priority_);
  // A prioritized LP launches its own kernels on its stream instead of
  // joining the batched launches (whose cycle is set by the light LPs'
  // requests); MILP_BATCH_PRIORITY_DIRECT=0 keeps it in the batches.
  static const bool direct = [] {
    const char* e = std::getenv("MILP_BATCH_PRIORITY_DIRECT");
    return e == nullptr || std::atoi(e) != 0;
  }();
  if (high && direct) SetSmallBatch(false);
}

void DeviceLp::WaitSmallBatch() {
  if (!batch_pending_) return;
  SmallBatcher& b = SmallBatcher::Get(device_);
  const auto t0 = std::chrono::steady_clock::now();
  int spins = 0;
  while (b.done(batch_slot_) != batch_seq_) {
    if (InFiber()) {
      FiberYield(spins > 0);
      RestoreDevice();
    } else {
      __builtin_ia32_pause();
    }
    if (++spins == 1 << 16) {
      spins = 0;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20)) {
        throw DeviceError("small batch: request not completed within 20 s");
      }
    }
  }
  batch_pending_ = false;
}

// Fibers of one host thread may belong to handles on different GPUs: the
// thread's current device is whatever the last fiber set, so a fiber that
// resumes makes its own handle's device current again before any HIP call
// (allocations and launches use the current device).
void DeviceLp::RestoreDevice() {
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != device_) Check(hipSetDevice(device_), "hipSetDevice");
}

// The stream wait of this handle. On a fiber of a batched solve (fibers.h)
// the fiber yields while the stream is busy, so the thread runs another LP's
// host work instead of spinning.
void DeviceLp::WaitStream() {
  WaitSmallBatch();
  if (InFiber()) {
    bool polled = false;  // later rounds of this wait only poll
    while (hipStreamQuery(S(stream_)) == hipErrorNotReady) {
      FiberYield(polled);
      polled = true;
      RestoreDevice();
    }
  }
  Check(hipStreamSynchronize(S(stream_)), "sync");
}

void DeviceLp::Download(void* dst, const void* src, size_t bytes) {
  if (bytes == 0) return;
  Check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, S(stream_)), "D2H");
  WaitStream();
}

void DeviceLp::Synchronize() {
  DeviceOp("Synchronize");
  WaitStream();
  DeviceOp("Synchronize done");
  small_inflight_ = false;
  for (auto& d : shards_) {
    if (d) d->Synchronize();
  }
}

void DeviceLp::ResetStats() {
  DrainTimings();
  std::memset(&stats_, 0, sizeof(stats_));
  for (auto& d : shards_) {
    if (d) d->ResetStats();
  }
}

const mi_lp_kernel_stats& DeviceLp::stats() {
  DrainTimings();
  if (shards_.empty()) return stats_;
  ShardedStats();
  return agg_stats_;
}

// Kernel timing: every logical launch is bracketed by two events recorded on
// the stream; their elapsed times are collected later (when the stats are
// read, or every 512 launches), so timing adds no synchronization to the
// iteration it measures.
void* DeviceLp::TakeEvent() {
  if (!ev_pool_.empty()) {
    void* e = ev_pool_.back();
    ev_pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  Check(hipEventCreate(&e), "hipEventCreate");
  return e;
}

void DeviceLp::DrainTimings() {
  for (const PendingTiming& t : ev_pending_) {
    Check(hipEventSynchronize(reinterpret_cast<hipEvent_t>(t.stop)), "ev sync");
    float ms = 0.0f;
    Check(hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(t.start),
                              reinterpret_cast<hipEvent_t>(t.stop)),
          "ev time");
    stats_.device_ms[t.id] += ms;
    ev_pool_.push_back(t.start);
    ev_pool_.push_back(t.stop);
  }
  ev_pending_.clear();
}

void DeviceLp::BeginKernel(int id) {
  static const char* const kNames[] = {"pricing", "update_row", "primal_norms", "rc_update",
                                       "tri_solve", "col_norms", "spmv_rows", "single_row",
                                       "dual_ratio", "readback", "tri_solve_tau", "tri_solve_l",
                                       "?", "?", "?", "?"};
  DeviceOp(kNames[id & 15]);
  if (batch_pending_) WaitSmallBatch();  // kernels after a batched request see its results
  if (!Timed(id)) return;
  if (ev_open_ == nullptr) ev_open_ = TakeEvent();
  Check(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_open_), S(stream_)), "ev");
}

void DeviceLp::EndKernel(int id, double bytes, bool count_launch) {
  Check(hipGetLastError(), "kernel launch");
  if (count_launch) stats_.launches[id] += 1;
  stats_.algorithmic_bytes[id] += bytes;
  if (Timed(id) && ev_open_ != nullptr) {
    void* stop = TakeEvent();
    Check(hipEventRecord(reinterpret_cast<hipEvent_t>(stop), S(stream_)), "ev");
    ev_pending_.push_back(PendingTiming{ev_open_, stop, id});
    ev_open_ = nullptr;
    if (ev_pending_.size() >= 512) DrainTimings();
  }
}

// MILP_STREAM_PRIORITY=1: the solver thread's stream at the highest priority
// and the tau worker's solve stream at the lowest. Off by default: an A/B on
// C5 alone read +3-4 %, but the full bench with priorities came out lower on
// every section (C5 575-600 vs 657 it/s, C3 45-61 vs 64, C4 1 740-1 860 vs
// 2 800 LPs/s) and config-4 probes lost 5-35 % (scripts/gpu_c4_ab.sh).
void DeviceLp::SetStreamPriority(bool high) {
  if (high == stream_prioritized_) return;
  Check(hipStreamSynchronize(S(stream_)), "sync");
  FreeTriBuffers();  // its contexts hold the old stream (rebuilt on demand)
  Check(hipStreamDestroy(S(stream_)), "hipStreamDestroy");
  hipStream_t s;
  if (high) {
    int least = 0, greatest = 0;
    Check(hipDeviceGetStreamPriorityRange(&least, &greatest), "priority range");
    Check(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest), "hipStreamCreate");
  } else {
    Check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  }
  stream_ = s;
  stream_prioritized_ = high;
}

void DeviceLp::UploadMatrix(const CompactSparseMatrix& csc, const CompactSparseMatrix& csr) {
  Check(hipSetDevice(device_), "hipSetDevice");
  SetStreamPriority(stream_priority_);
  for (void* p : allocations_) (void)hipFree(p);
  allocations_.clear();
  m_ = csc.num_rows();
  n_total_ = csc.num_cols();
  nnz_ = csc.num_entries();
  avg_col_len_ = n_total_ > 0 ? static_cast<double>(nnz_) / n_total_ : 0.0;
  max_col_len_ = 0;
  for (int c = 0; c < n_total_; ++c) {
    max_col_len_ = std::max<int64_t>(max_col_len_, csc.starts_[c + 1] - csc.starts_[c]);
  }
  h_starts_ = csc.starts_;
  h_t_starts_ = csr.starts_;
  // Full rows: every structural column present (then entry j is column j).
  num_structural_ = n_total_ - m_;
  h_row_full_.assign(m_, 0);
  for (int r = 0; r < m_; ++r) {
    h_row_full_[r] = (csr.starts_[r + 1] - csr.starts_[r] == int64_t(num_structural_) + 1) ? 1 : 0;
  }
  d_starts_ = Alloc<int64_t>(n_total_ + 1);
  d_rows_ = Alloc<int32_t>(nnz_);
  d_vals_ = Alloc<double>(nnz_);
  d_t_starts_ = Alloc<int64_t>(m_ + 1);
  d_t_cols_ = Alloc<int32_t>(nnz_);
  d_t_vals_ = Alloc<double>(nnz_);
  Upload(d_starts_, csc.starts_.data(), (n_total_ + 1) * sizeof(int64_t));
  Upload(d_rows_, csc.rows_.data(), nnz_ * sizeof(int32_t));
  Upload(d_vals_, csc.coefficients_.data(), nnz_ * sizeof(double));
  Upload(d_t_starts_, csr.starts_.data(), (m_ + 1) * sizeof(int64_t));
  Upload(d_t_cols_, csr.rows_.data(), nnz_ * sizeof(int32_t));
  Upload(d_t_vals_, csr.coefficients_.data(), nnz_ * sizeof(double));
  mask_words_ = (n_total_ + 63) / 64;
  for (int k = 0; k < kNumMasks; ++k) {
    d_masks_[k] = Alloc<uint64_t>(mask_words_);
    h_masks_[k].assign(mask_words_, ~0ull);  // force first upload
    mask_on_device_[k] = false;               // and no changed-word update before it
    Check(hipEventSynchronize(reinterpret_cast<hipEvent_t>(ev_mask_[k])), "mask event");
    if (h_pin_mask_[k]) (void)hipHostFree(h_pin_mask_[k]);
    Check(hipHostMalloc(reinterpret_cast<void**>(&h_pin_mask_[k]),
                        std::max(1, mask_words_) * sizeof(uint64_t)),
          "pin");
  }
  if (h_mask_diff_ == nullptr) {
    Check(hipHostMalloc(reinterpret_cast<void**>(&h_mask_diff_),
                        size_t(kNumMasks) * kMaskDiffMax * 12, hipHostMallocMapped),
          "hipHostMalloc (mapped)");
    void* dev = nullptr;
    Check(hipHostGetDevicePointer(&dev, h_mask_diff_, 0), "mapped pointer");
    m_mask_diff_ = static_cast<char*>(dev);
  }
  d_vec_m_ = Alloc<double>(m_);
  d_vec_m2_ = Alloc<double>(m_);
  d_vec_w_ = Alloc<double>(m_);
  fused_ready_ = false;
  d_vec_n_ = Alloc<double>(n_total_);
  d_coeff_ = Alloc<double>(n_total_);
  d_flags_ = Alloc<uint8_t>(n_total_);
  d_list_ = Alloc<int32_t>(n_total_);
  d_count_ = Alloc<int>(1);
  d_out_n_ = Alloc<double>(n_total_);
  d_out_n2_ = Alloc<double>(n_total_);
  d_out_list_ = Alloc<double>(std::max(n_total_, m_));
  d_cols_ = Alloc<int32_t>(std::max(n_total_, m_));
  // Row-wise update-row inputs: rows, multipliers, CSR offsets (one upload).
  const size_t upd_bytes = size_t(m_ + 2) * (sizeof(int32_t) + 2 * sizeof(double));
  d_upd_in_ = Alloc<uint8_t>(upd_bytes);
  d_row_tag_ = Alloc<uint32_t>(m_);
  d_row_pos_ = Alloc<int32_t>(m_);
  Check(hipMemsetAsync(d_row_tag_, 0, std::max(1, m_) * sizeof(uint32_t), S(stream_)), "memset");
  row_tag_ = 0;
  Check(hipMemsetAsync(d_coeff_, 0, n_total_ * sizeof(double), S(stream_)), "memset");
  // Tile status words and tickets of the ordered compactions.
  const int tiles = milp_launch::scan_tiles(n_total_);
  d_scan_status_ = Alloc<unsigned long long>(tiles);
  d_scan_ticket_ = Alloc<unsigned int>(2);
  Check(hipMemsetAsync(d_scan_status_, 0, tiles * sizeof(unsigned long long), S(stream_)),
        "memset");
  Check(hipMemsetAsync(d_scan_ticket_, 0, 2 * sizeof(unsigned int), S(stream_)), "memset");
  scan_epoch_ = 0;
  if (h_scan_fail_ == nullptr) {
    Check(hipHostMalloc(reinterpret_cast<void**>(&h_scan_fail_), 64, hipHostMallocMapped),
          "hipHostMalloc (mapped)");
    void* d = nullptr;
    Check(hipHostGetDevicePointer(&d, h_scan_fail_, 0), "mapped pointer");
    m_scan_fail_ = static_cast<int*>(d);
  }
  *h_scan_fail_ = 0;
  if (h_pin_i_) (void)hipHostFree(h_pin_i_);
  if (h_pin_d_) (void)hipHostFree(h_pin_d_);
  if (h_pin_d2_) (void)hipHostFree(h_pin_d2_);
  if (h_pin_w_) (void)hipHostFree(h_pin_w_);
  if (h_upd_in_) (void)hipHostFree(h_upd_in_);
  Check(hipHostMalloc(&h_upd_in_, upd_bytes), "pin");
  const size_t big = std::max(n_total_, m_) + 1;
  Check(hipHostMalloc(reinterpret_cast<void**>(&h_pin_i_), big * sizeof(int32_t)), "pin");
  Check(hipHostMalloc(reinterpret_cast<void**>(&h_pin_d_), big * sizeof(double)), "pin");
  Check(hipHostMalloc(reinterpret_cast<void**>(&h_pin_d2_), big * sizeof(double)), "pin");
  Check(hipHostMalloc(reinterpret_cast<void**>(&h_pin_w_), (m_ + 1) * sizeof(double)), "pin");
  if (h_pin_count_ == nullptr) {
    Check(hipHostMalloc(reinterpret_cast<void**>(&h_pin_count_), sizeof(int)), "pin");
  }
  // Mapped host buffer for the small-N compaction result: count, list, values.
  if (h_map_ != nullptr) (void)hipHostFree(h_map_);
  h_map_ = nullptr;
  d_map_count_ = nullptr;
  d_map_list_ = nullptr;
  d_map_vals_ = nullptr;
  {
    const size_t list_off = 64;
    const size_t vals_off = (list_off + size_t(n_total_) * sizeof(int32_t) + 63) / 64 * 64;
    const size_t bytes = vals_off + size_t(n_total_) * sizeof(double);
    Check(hipHostMalloc(&h_map_, bytes, hipHostMallocMapped), "mapped");
    char* base = static_cast<char*>(h_map_);
    h_map_count_ = reinterpret_cast<int*>(base);
    h_map_list_ = reinterpret_cast<int32_t*>(base + list_off);
    h_map_vals_ = reinterpret_cast<double*>(base + vals_off);
    void* dev = nullptr;
    Check(hipHostGetDevicePointer(&dev, h_map_, 0), "mapped pointer");
    char* dbase = static_cast<char*>(dev);
    d_map_count_ = reinterpret_cast<int*>(dbase);
    d_map_list_ = reinterpret_cast<int32_t*>(dbase + list_off);
    d_map_vals_ = reinterpret_cast<double*>(dbase + vals_off);
  }
  if (h_small_in_ != nullptr) (void)hipHostFree(h_small_in_);
  h_small_in_ = nullptr;
  small_inflight_ = false;
  mask_dirty_ = false;
  medium_ = small_fused_enabled_ && medium_enabled_ && n_total_ > milp_kernels::kSmallLdsCols &&
            n_total_ <= milp_kernels::kMediumCols;
  if (n_total_ <= milp_kernels::kSmallLdsCols || medium_) {
    const int cap = std::max(1, m_);  // filtered rows
    const size_t rho_off = (size_t(cap) * sizeof(int32_t) + 63) / 64 * 64;
    const size_t mask_off = rho_off + size_t(cap) * sizeof(double);
    const size_t y_off = mask_off + size_t(mask_words_) * sizeof(uint64_t);
    const size_t w_off = y_off + size_t(m_) * sizeof(double);
    const size_t out_off = w_off + size_t(m_) * sizeof(double);
    const size_t dots_off = out_off + size_t(n_total_) * sizeof(double);
    Check(hipHostMalloc(&h_small_in_, dots_off + size_t(n_total_) * sizeof(double),
                        hipHostMallocMapped),
          "mapped");
    char* base = static_cast<char*>(h_small_in_);
    h_small_rows_ = reinterpret_cast<int32_t*>(base);
    h_small_rho_ = reinterpret_cast<double*>(base + rho_off);
    h_small_mask_ = reinterpret_cast<uint64_t*>(base + mask_off);
    void* dev = nullptr;
    Check(hipHostGetDevicePointer(&dev, h_small_in_, 0), "mapped pointer");
    const char* dbase = static_cast<const char*>(dev);
    d_small_rows_ = reinterpret_cast<const int32_t*>(dbase);
    d_small_rho_ = reinterpret_cast<const double*>(dbase + rho_off);
    d_small_mask_ = reinterpret_cast<const uint64_t*>(dbase + mask_off);
    h_small_y_ = reinterpret_cast<double*>(base + y_off);
    h_small_out_ = reinterpret_cast<double*>(base + out_off);
    d_small_y_ = reinterpret_cast<const double*>(dbase + y_off);
    d_small_out_ = reinterpret_cast<double*>(const_cast<char*>(dbase) + out_off);
    h_small_w_ = reinterpret_cast<double*>(base + w_off);
    h_small_dots_ = reinterpret_cast<double*>(base + dots_off);
    d_small_w_ = reinterpret_cast<const double*>(dbase + w_off);
    d_small_dots_ = reinterpret_cast<double*>(const_cast<char*>(dbase) + dots_off);
  }
  mapped_result_ = false;
  list_count_ = 0;
  dual_ready_ = false;
  last_list_len_ = 0;
  ++list_epoch_;
  BuildDenseBlock();
  Synchronize();
  if (!shards_.empty()) ShardedUpload(csc);
}

// Full structural columns go to the value-only dense block (8 B per entry
// instead of 12, unit-stride chains). MILP_DENSE_BLOCK=off|force|auto
// (auto: at least 256 full columns and 32 rows).
void DeviceLp::BuildDenseBlock() {
  nd_ = 0;
  ns_ = n_total_;
  h_is_dense_.assign(n_total_, 0);
  h_dense_words_.assign(mask_words_, 0);
  sparse_entries_ = nnz_;
  const char* env = std::getenv("MILP_DENSE_BLOCK");
  const std::string mode = env ? env : "auto";
  if (mode == "off" || m_ <= 0) return;
  std::vector<int32_t> dense, sparse;
  for (int c = 0; c < n_total_; ++c) {
    if (h_starts_[c + 1] - h_starts_[c] == m_) dense.push_back(c); else sparse.push_back(c);
  }
  const bool use = mode == "force" ? !dense.empty()
                                   : (dense.size() >= 256 && m_ >= 32);
  if (!use) return;
  nd_ = static_cast<int>(dense.size());
  ns_ = static_cast<int>(sparse.size());
  for (const int c : dense) {
    h_is_dense_[c] = 1;
    h_dense_words_[c >> 6] |= 1ull << (c & 63);
  }
  sparse_entries_ = nnz_ - static_cast<int64_t>(nd_) * m_;
  const int steps = m_ >> 2;
  d_dense_body_ = Alloc<double>(static_cast<size_t>(steps) * nd_ * 4);
  d_dense_tail_ = Alloc<double>(static_cast<size_t>(m_ - 4 * steps) * nd_);
  d_dense_cols_ = Alloc<int32_t>(nd_);
  d_sparse_cols_ = Alloc<int32_t>(ns_);
  d_is_dense_ = Alloc<uint8_t>(n_total_);
  Upload(d_dense_cols_, dense.data(), nd_ * sizeof(int32_t));
  Upload(d_sparse_cols_, sparse.data(), ns_ * sizeof(int32_t));
  Upload(d_is_dense_, h_is_dense_.data(), n_total_);
  Synchronize();  // the host vectors above are pageable and go out of scope
  Check(milp_launch::dense_pack(d_starts_, d_vals_, d_dense_cols_, nd_, m_, d_dense_body_,
                                d_dense_tail_, S(stream_)),
        "dense pack");
}

void DeviceLp::LaunchColumnDots(int mode, const double* d_y, const double* d_c,
                                double* d_out, const double* d_y2, double* d_out2) {
  FlushRelevantMask();
  milp_kernels::DotArgs a{};
  a.starts = d_starts_;
  a.rows = d_rows_;
  a.vals = d_vals_;
  a.y = d_y;
  a.c = d_c;
  a.out = d_out;
  a.y2 = d_y2;
  a.out2 = d_out2;
  a.mask = d_masks_[kRelevant];
  a.flags = d_flags_;
  a.drop_tolerance = 0.0;
  if (mode == 2) {  // dots over the update-row list
    a.ncols = list_count_;
    a.col_list = d_list_;
    a.flags = nullptr;  // every listed column is active
  } else {
    a.ncols = nd_ > 0 ? ns_ : n_total_;
    a.col_list = nd_ > 0 ? d_sparse_cols_ : nullptr;
  }
  a.skip = nd_ > 0 ? d_is_dense_ : nullptr;
  const double sparse_avg =
      (nd_ > 0 ? (ns_ > 0 ? double(sparse_entries_) / ns_ : 0.0) : avg_col_len_);
  a.drop_tolerance = drop_;
  Check(milp_launch::column_dot(mode, sparse_avg >= 32.0, a, S(stream_)), "column dots");
  if (nd_ > 0) {
    milp_kernels::DenseArgs d{};
    d.body = d_dense_body_;
    d.tail = d_dense_tail_;
    d.dense_cols = d_dense_cols_;
    d.nd = nd_;
    d.m = m_;
    d.y = d_y;
    d.mask = d_masks_[kRelevant];
    d.c = d_c;
    d.out = d_out;
    d.y2 = d_y2;
    d.out2 = d_out2;
    d.flags = d_flags_;
    d.drop_tolerance = drop_;
    Check(milp_launch::dense_dot(mode, dense_unroll_, d, S(stream_)), "dense dots");
  }
}

void DeviceLp::SetMask(Mask which, const uint64_t* words, int num_words) {
  if (!shards_.empty()) return ShardedSetMask(which, words, num_words);
  std::vector<uint64_t>& h = h_masks_[which];
  if (num_words != mask_words_) throw DeviceError("mask size mismatch");
  // Unchanged words are skipped only once the device holds a copy: a mask
  // equal to the all-ones placeholder (e.g. a column shard with every column
  // relevant) must still reach the device the first time.
  if (mask_on_device_[which] && std::memcmp(h.data(), words, num_words * sizeof(uint64_t)) == 0) {
    return;
  }
  if (which == kRelevant && small_fused_enabled_ && h_small_in_ != nullptr &&
      (!medium_ || small_batch_)) {
    // Small LPs: the relevant set changes every pivot and the small update
    // row reads it from mapped host memory; other kernels flush it first.
    std::memcpy(h.data(), words, num_words * sizeof(uint64_t));
    mask_dirty_ = true;
    return;
  }
  if (h_mask_diff_ != nullptr && mask_on_device_[which] && !(which == kRelevant && mask_dirty_)) {
    // A pivot moves a few bits: send only the changed words (mapped pairs +
    // one small kernel) instead of the whole mask through the copy engine.
    hipEvent_t done = reinterpret_cast<hipEvent_t>(ev_mask_[which]);
    Check(hipEventSynchronize(done), "mask event");
    char* slot = h_mask_diff_ + size_t(which) * kMaskDiffMax * 12;
    int32_t* idx = reinterpret_cast<int32_t*>(slot);
    uint64_t* val = reinterpret_cast<uint64_t*>(slot + kMaskDiffMax * 4);
    int count = 0;
    for (int w = 0; w < num_words && count <= kMaskDiffMax; ++w) {
      if (h[w] != words[w]) {
        if (count < kMaskDiffMax) {
          idx[count] = w;
          val[count] = words[w];
        }
        ++count;
      }
    }
    if (count <= kMaskDiffMax) {
      std::memcpy(h.data(), words, num_words * sizeof(uint64_t));
      char* dslot = m_mask_diff_ + size_t(which) * kMaskDiffMax * 12;
      Check(milp_launch::set_mask_words(reinterpret_cast<const int32_t*>(dslot),
                                        reinterpret_cast<const uint64_t*>(dslot + kMaskDiffMax * 4),
                                        count, d_masks_[which], S(stream_)),
            "mask words");
      Check(hipEventRecord(done, S(stream_)), "mask event");
      return;
    }
  }
  std::memcpy(h.data(), words, num_words * sizeof(uint64_t));
  UploadMask(which);
}

void DeviceLp::UploadMask(Mask which) {
  // Asynchronous copy from a pinned slot; the slot is reused only once its
  // previous copy has completed.
  hipEvent_t done = reinterpret_cast<hipEvent_t>(ev_mask_[which]);
  Check(hipEventSynchronize(done), "mask event");
  std::memcpy(h_pin_mask_[which], h_masks_[which].data(), mask_words_ * sizeof(uint64_t));
  Upload(d_masks_[which], h_pin_mask_[which], mask_words_ * sizeof(uint64_t));
  Check(hipEventRecord(done, S(stream_)), "mask event");
  mask_on_device_[which] = true;
  if (which == kRelevant) mask_dirty_ = false;
}

void DeviceLp::FlushRelevantMask() {
  if (mask_dirty_) UploadMask(kRelevant);
}

// Compaction of the update-row flags into the ascending list of listed
// positions plus their coefficients. No host synchronization here: the count
// comes back with the list in FetchUpdateRow (one round trip per update row).
void DeviceLp::Compact(int n) {
  if (n <= milp_launch::kSmallCompactMax) {
    // One workgroup: flags -> list + coefficients + count in a single launch.
    // The result also lands in mapped host memory: the readback is the sync.
    Check(milp_launch::compact_small(d_flags_, n, d_coeff_, d_list_, d_out_list_, d_count_,
                                     d_map_list_, d_map_vals_, d_map_count_, S(stream_)),
          "compact small");
    mapped_result_ = true;
  } else {
    // Ordered single-pass compaction over the chip, the list also into
    // mapped host memory.
    Check(milp_launch::compact_flags(d_flags_, n, d_coeff_, d_list_, d_out_list_, d_count_,
                                     list_mirror_ ? d_map_list_ : nullptr,
                                     list_mirror_ ? d_map_vals_ : nullptr,
                                     list_mirror_ ? d_map_count_ : nullptr, NextScan(),
                                     S(stream_)),
          "compact");
    mapped_result_ = list_mirror_;
  }
  list_count_ = -1;  // known after FetchUpdateRow
  ++list_epoch_;
}

void DeviceLp::UpdateRowColumnWise(const std::vector<double>& rho, double drop,
                                   int64_t relevant_entries, const std::vector<double>* w) {
  if (!shards_.empty()) return ShardedUpdateRowColumnWise(rho, drop, relevant_entries, w);
  CallTimer timer(&stats_, MI_K_UPDATE_ROW);
  small_dots_mapped_ = false;
  if (small_fused_enabled_ && h_small_in_ != nullptr && !medium_ && nd_ == 0 &&
      m_ <= milp_kernels::kSmallColWiseRows) {
    UpdateRowColumnWiseSmall(rho, drop, relevant_entries, w);
    return;
  }
  std::memcpy(h_pin_d_, rho.data(), m_ * sizeof(double));
  Upload(d_vec_m_, h_pin_d_, m_ * sizeof(double));
  if (w != nullptr) {
    std::memcpy(h_pin_d2_, w->data(), m_ * sizeof(double));
    Upload(d_vec_w_, h_pin_d2_, m_ * sizeof(double));
    fused_w_ = *w;
  }
  fused_ready_ = false;
  drop_ = drop;
  // Algorithmic bytes: every relevant column is read (12 B per CSC entry,
  // 8 B per dense-block entry), rho once, coefficients + flags written.
  int64_t dense_rel = 0;
  if (nd_ > 0) {
    const uint64_t* rel = h_masks_[kRelevant].data();
    for (int w = 0; w < mask_words_; ++w) {
      dense_rel += __builtin_popcountll(rel[w] & h_dense_words_[w]);
    }
  }
  const double dense_entries = double(dense_rel) * m_;
  BeginKernel(MI_K_UPDATE_ROW);
  if (w != nullptr) {
    LaunchColumnDots(4, d_vec_m_, nullptr, d_coeff_, d_vec_w_, d_out_n_);
  } else {
    LaunchColumnDots(0, d_vec_m_, nullptr, d_coeff_);
  }
  // The fused variant also reads w and writes one more double per listed
  // column (counted as up to N).
  EndKernel(MI_K_UPDATE_ROW, 12.0 * (double(relevant_entries) - dense_entries) +
                                 8.0 * dense_entries + 8.0 * m_ + 9.0 * n_total_ +
                                 (w != nullptr ? 8.0 * m_ : 0.0));
  Compact(n_total_);
  fused_ready_ = (w != nullptr);
}

// Small LPs: rho (and w), the relevant mask, and the results through mapped
// host memory, one launch; the w dots come back in list order with the list.
void DeviceLp::UpdateRowColumnWiseSmall(const std::vector<double>& rho, double drop,
                                        int64_t relevant_entries,
                                        const std::vector<double>* w) {
  if (small_inflight_) Synchronize();
  std::memcpy(h_small_y_, rho.data(), m_ * sizeof(double));
  if (w != nullptr) {
    std::memcpy(h_small_w_, w->data(), m_ * sizeof(double));
    fused_w_ = *w;
  }
  std::memcpy(h_small_mask_, h_masks_[kRelevant].data(), mask_words_ * sizeof(uint64_t));
  fused_ready_ = false;
  drop_ = drop;
  milp_kernels::ColWiseSmallArgs a{};
  a.starts = d_starts_;
  a.rows = d_rows_;
  a.vals = d_vals_;
  a.rho = d_small_y_;
  a.w = w != nullptr ? d_small_w_ : nullptr;
  a.m = m_;
  a.num_cols = n_total_;
  a.relevant = d_small_mask_;
  a.coefficient = d_coeff_;
  a.flags = d_flags_;
  a.out2 = d_out_n_;
  a.drop_tolerance = drop;
  a.list = d_list_;
  a.vals_out = d_out_list_;
  a.count = d_count_;
  a.host_list = d_map_list_;
  a.host_vals = d_map_vals_;
  a.host_count = d_map_count_;
  a.host_dots = d_small_dots_;
  BeginKernel(MI_K_UPDATE_ROW);
  LaunchSmall(milp_kernels::kSmallColWise, a);
  EndKernel(MI_K_UPDATE_ROW, 12.0 * double(relevant_entries) + 8.0 * m_ + 9.0 * n_total_ +
                                 (w != nullptr ? 8.0 * m_ : 0.0));
  small_inflight_ = true;
  mapped_result_ = true;
  list_count_ = -1;  // known after FetchUpdateRow
  ++list_epoch_;
  fused_ready_ = (w != nullptr);
  small_dots_mapped_ = (w != nullptr);
}

void DeviceLp::UpdateRowRowWise(const std::vector<int>& filtered_rows,
                                const std::vector<double>& rho, int algorithm,
                                double drop) {
  if (!shards_.empty()) return ShardedUpdateRowRowWise(filtered_rows, rho, algorithm, drop);
  CallTimer timer(&stats_, algorithm == 0 ? MI_K_SINGLE_ROW : MI_K_UPDATE_ROW);
  const int k = static_cast<int>(filtered_rows.size());
  fused_ready_ = false;
  if (small_fused_enabled_ && h_small_in_ != nullptr) {
    double entries = 0.0;
    for (int r : filtered_rows) entries += double(h_t_starts_[r + 1] - h_t_starts_[r]);
    // Few short rows: applied row by row; otherwise column by column.
    const bool serial = k <= small_serial_rows_ && k <= milp_kernels::kSmallRowsMax &&
                        entries <= milp_kernels::kSmallEntries;
    if (!medium_ || (serial && small_batch_)) {
      UpdateRowRowWiseSmall(filtered_rows, rho, algorithm, drop, entries, serial);
      return;
    }
  }
  FlushRelevantMask();
  bool all_full = full_rows_enabled_ && k > 0;
  for (int i = 0; i < k && all_full; ++i) all_full = h_row_full_[filtered_rows[i]] != 0;
  // One upload: the rows, their multipliers and (full rows) their CSR offsets.
  const size_t rho_off = (size_t(k) * sizeof(int32_t) + 7) / 8 * 8;
  const size_t offs_off = rho_off + size_t(k) * sizeof(double);
  char* hin = static_cast<char*>(h_upd_in_);
  int32_t* h_rows = reinterpret_cast<int32_t*>(hin);
  double* h_rho = reinterpret_cast<double*>(hin + rho_off);
  int64_t* h_offs = reinterpret_cast<int64_t*>(hin + offs_off);
  std::memcpy(h_rows, filtered_rows.data(), k * sizeof(int32_t));
  for (int i = 0; i < k; ++i) h_rho[i] = rho[filtered_rows[i]];
  if (all_full) {
    for (int i = 0; i < k; ++i) h_offs[i] = h_t_starts_[filtered_rows[i]];
  }
  Upload(d_upd_in_, h_upd_in_, all_full ? offs_off + size_t(k) * sizeof(int64_t) : offs_off);
  char* din = static_cast<char*>(d_upd_in_);
  const int32_t* d_rows = reinterpret_cast<const int32_t*>(din);
  const double* d_rho = reinterpret_cast<const double*>(din + rho_off);
  const int64_t* d_offs = reinterpret_cast<const int64_t*>(din + offs_off);
  milp_kernels::RowWiseArgs a{};
  a.t_starts = d_t_starts_;
  a.t_cols = d_t_cols_;
  a.t_vals = d_t_vals_;
  a.filtered_rows = d_rows;
  a.rho = d_rho;
  a.num_filtered = k;
  a.num_cols = n_total_;
  a.relevant = d_masks_[kRelevant];
  a.coefficient = d_coeff_;
  a.flags = d_flags_;
  a.drop_tolerance = drop;
  a.algorithm = algorithm;
  const int id = algorithm == 0 ? MI_K_SINGLE_ROW : MI_K_UPDATE_ROW;
  BeginKernel(id);
  if (all_full) {
    // Full rows: a thread per column reads each row's entry directly.
    NextRowTag();
    Check(milp_launch::tag_rows(d_rows, k, row_tag_, d_row_tag_, d_row_pos_, S(stream_)),
          "tag rows");
    milp_kernels::RowWiseFullArgs f{};
    f.t_starts = d_t_starts_;
    f.t_vals = d_t_vals_;
    f.row_offsets = d_offs;
    f.rho = d_rho;
    f.num_filtered = k;
    f.num_structural = num_structural_;
    f.num_cols = n_total_;
    f.row_tag = d_row_tag_;
    f.row_pos = d_row_pos_;
    f.tag = row_tag_;
    f.relevant = d_masks_[kRelevant];
    f.coefficient = d_coeff_;
    f.flags = d_flags_;
    f.drop_tolerance = drop;
    f.algorithm = algorithm;
    Check(milp_launch::row_wise_update_full_rows(f, S(stream_)), "rowwise full rows");
    // Values only (the column index of entry j is j), the list, the outputs.
    EndKernel(id, 8.0 * double(k) * (num_structural_ + 1) + 12.0 * k + 9.0 * n_total_);
    Compact(n_total_);
    return;
  }
  if (k <= rowwise_chunk_max_rows_ || max_col_len_ > kColumnKernelMaxColumnLength) {
    // Few rows: workgroups own column chunks and merge the rows in order.
    Check(milp_launch::row_wise_update(a, S(stream_)), "rowwise");
  } else {
    // Many rows: one thread per column gathers its filtered entries from the
    // CSC copy (same arithmetic, same order).
    NextRowTag();
    Check(milp_launch::tag_rows(d_rows, k, row_tag_, d_row_tag_, d_row_pos_, S(stream_)),
          "tag rows");
    milp_kernels::RowWiseColArgs c{};
    c.starts = d_starts_;
    c.rows = d_rows_;
    c.vals = d_vals_;
    c.row_tag = d_row_tag_;
    c.row_pos = d_row_pos_;
    c.tag = row_tag_;
    c.rho = d_rho;
    c.num_cols = n_total_;
    c.relevant = d_masks_[kRelevant];
    c.coefficient = d_coeff_;
    c.flags = d_flags_;
    c.drop_tolerance = drop;
    c.algorithm = algorithm;
    Check(milp_launch::row_wise_update_by_column(c, S(stream_)), "rowwise by column");
  }
  double entries = 0.0;
  for (int r : filtered_rows) entries += double(h_t_starts_[r + 1] - h_t_starts_[r]);
  EndKernel(id, 12.0 * entries + 12.0 * k + 9.0 * n_total_);
  Compact(n_total_);
}

// Small LPs: inputs in mapped host memory, one launch, the list comes back in
// mapped host memory (FetchUpdateRow's stream sync is the only round trip).
void DeviceLp::UpdateRowRowWiseSmall(const std::vector<int>& filtered_rows,
                                     const std::vector<double>& rho, int algorithm,
                                     double drop, double entries, bool serial) {
  const int k = static_cast<int>(filtered_rows.size());
  // The previous launch may still be reading the inputs when no sync came
  // in between (not the case in the simplex loop, which fetches every row).
  if (small_inflight_) Synchronize();
  for (int i = 0; i < k; ++i) {
    h_small_rows_[i] = filtered_rows[i];
    h_small_rho_[i] = rho[filtered_rows[i]];
  }
  std::memcpy(h_small_mask_, h_masks_[kRelevant].data(), mask_words_ * sizeof(uint64_t));
  const int id = algorithm == 0 ? MI_K_SINGLE_ROW : MI_K_UPDATE_ROW;
  if (!serial) {
    milp_kernels::RowWiseSmallColArgs c{};
    c.starts = d_starts_;
    c.rows = d_rows_;
    c.vals = d_vals_;
    c.filtered_rows = d_small_rows_;
    c.rho = d_small_rho_;
    c.num_filtered = k;
    c.m = m_;
    c.num_cols = n_total_;
    c.relevant = d_small_mask_;
    c.coefficient = d_coeff_;
    c.flags = d_flags_;
    c.drop_tolerance = drop;
    c.algorithm = algorithm;
    c.list = d_list_;
    c.list_vals = d_out_list_;
    c.count = d_count_;
    c.host_list = d_map_list_;
    c.host_vals = d_map_vals_;
    c.host_count = d_map_count_;
    BeginKernel(id);
    LaunchSmall(milp_kernels::kSmallRowWiseByColumn, c);
    // The whole CSC copy, the filtered rows and multipliers, flags/coefficients.
    EndKernel(id, 12.0 * double(nnz_) + 8.0 * (n_total_ + 1) + 12.0 * k + 9.0 * n_total_);
    small_inflight_ = true;
    mapped_result_ = true;
    list_count_ = -1;
    ++list_epoch_;
    return;
  }
  milp_kernels::RowWiseSmallArgs a{};
  a.t_starts = d_t_starts_;
  a.t_cols = d_t_cols_;
  a.t_vals = d_t_vals_;
  a.filtered_rows = d_small_rows_;
  a.rho = d_small_rho_;
  a.num_filtered = k;
  a.num_cols = n_total_;
  a.relevant = d_small_mask_;
  a.coefficient = d_coeff_;
  a.flags = d_flags_;
  a.drop_tolerance = drop;
  a.algorithm = algorithm;
  a.list = d_list_;
  a.vals = d_out_list_;
  a.count = d_count_;
  a.host_list = d_map_list_;
  a.host_vals = d_map_vals_;
  a.host_count = d_map_count_;
  BeginKernel(id);
  LaunchSmall(medium_ ? milp_kernels::kMediumRowWise : milp_kernels::kSmallRowWise, a);
  // Rows and multipliers, the CSR entries, N-sized flags/coefficients, the list.
  EndKernel(id, 12.0 * entries + 12.0 * k + 9.0 * n_total_);
  small_inflight_ = true;
  mapped_result_ = true;
  list_count_ = -1;  // known after FetchUpdateRow
  ++list_epoch_;
}

void DeviceLp::NextRowTag() {
  if (++row_tag_ == 0) {  // wrapped: clear the marks
    Check(hipMemsetAsync(d_row_tag_, 0, m_ * sizeof(uint32_t), S(stream_)), "memset");
    row_tag_ = 1;
  }
}

void DeviceLp::FetchUpdateRow(std::vector<int>* positions, std::vector<double>* values) {
  if (!shards_.empty()) return ShardedFetchUpdateRow(positions, values);
  CallTimer timer(&stats_, MI_K_READBACK);
  if (mapped_result_) {
    Synchronize();
    CheckScan();
    const int n = *h_map_count_;
    if (n < 0 || n > n_total_) throw DeviceError("bad update-row count");
    list_count_ = n;
    last_list_len_ = n;
    positions->assign(h_map_list_, h_map_list_ + n);
    values->assign(h_map_vals_, h_map_vals_ + n);
    AccountList(*positions);
    return;
  }
  // Count, and a prefix of the list sized from the previous update row, in
  // one round trip; the rest (if any) in a second one.
  const int cap = std::min<int64_t>(
      n_total_, std::max<int64_t>(4096, int64_t(last_list_len_) + last_list_len_ / 4));
  Check(hipMemcpyAsync(h_pin_count_, d_count_, sizeof(int), hipMemcpyDeviceToHost, S(stream_)),
        "D2H");
  Check(hipMemcpyAsync(h_pin_i_, d_list_, cap * sizeof(int32_t), hipMemcpyDeviceToHost,
                       S(stream_)),
        "D2H");
  Download(h_pin_d_, d_out_list_, cap * sizeof(double));
  const int n = *h_pin_count_;
  if (n < 0 || n > n_total_) throw DeviceError("bad update-row count");
  if (n > cap) {
    Check(hipMemcpyAsync(h_pin_i_ + cap, d_list_ + cap, (n - cap) * sizeof(int32_t),
                         hipMemcpyDeviceToHost, S(stream_)),
          "D2H");
    Download(h_pin_d_ + cap, d_out_list_ + cap, (n - cap) * sizeof(double));
  }
  list_count_ = n;
  last_list_len_ = n;
  positions->resize(n);
  values->resize(n);
  if (n > 0) {
    CopyHost(positions->data(), h_pin_i_, n * sizeof(int32_t));
    CopyHost(values->data(), h_pin_d_, n * sizeof(double));
  }
  AccountList(*positions);
}

// Byte accounting of the listed columns (ListDotsOverUpdateRow).
void DeviceLp::AccountList(const std::vector<int>& positions) {
  int64_t part_entries[16] = {0};
  int64_t part_dense[16] = {0};
  const bool has_dense = !h_is_dense_.empty();
  const int parts = ParallelRanges(static_cast<int64_t>(positions.size()), 16384, 1,
                                   [&](int p, int64_t b, int64_t e) {
    int64_t entries = 0;
    int64_t dense = 0;
    for (int64_t k = b; k < e; ++k) {
      const int c = positions[k];
      if (has_dense && h_is_dense_[c]) {
        ++dense;
      } else {
        entries += h_starts_[c + 1] - h_starts_[c];
      }
    }
    part_entries[p] = entries;
    part_dense[p] = dense;
  });
  list_entries_ = 0;
  list_dense_ = 0;
  for (int p = 0; p < parts; ++p) {
    list_entries_ += part_entries[p];
    list_dense_ += part_dense[p];
  }
}

// memcpy split over the host pool (large host <-> pinned staging copies).
void DeviceLp::CopyHost(void* dst, const void* src, size_t bytes) {
  ParallelRanges(static_cast<int64_t>(bytes), 1 << 18, 4096, [&](int, int64_t b, int64_t e) {
    std::memcpy(static_cast<char*>(dst) + b, static_cast<const char*>(src) + b, e - b);
  });
}

double DeviceLp::ReadCoefficient(int col) {
  if (!shards_.empty()) return ShardedReadCoefficient(col);
  CallTimer timer(&stats_, MI_K_READBACK);
  double v = 0.0;
  Download(h_pin_d2_, d_coeff_ + col, sizeof(double));
  v = h_pin_d2_[0];
  return v;
}

void DeviceLp::ListDotsOverUpdateRow(const std::vector<double>& v, std::vector<double>* out) {
  if (!shards_.empty()) return ShardedListDotsOverUpdateRow(v, out);
  CallTimer timer(&stats_, MI_K_PRIMAL_NORMS);
  if (list_count_ < 0) throw DeviceError("update-row list used before FetchUpdateRow");
  const int n = list_count_;
  out->resize(n);
  if (n == 0) return;
  if (fused_ready_ && v.size() == fused_w_.size() &&
      std::memcmp(v.data(), fused_w_.data(), v.size() * sizeof(double)) == 0) {
    // Computed by the fused update-row pass: only the gather remains.
    fused_ready_ = false;
    if (small_dots_mapped_) {  // already gathered, in list order
      small_dots_mapped_ = false;
      std::memcpy(out->data(), h_small_dots_, n * sizeof(double));
      return;
    }
    Check(milp_launch::gather(d_list_, n, d_out_n_, d_out_list_, S(stream_)), "gather");
    Download(h_pin_d_, d_out_list_, n * sizeof(double));
    std::memcpy(out->data(), h_pin_d_, n * sizeof(double));
    return;
  }
  fused_ready_ = false;
  if (small_fused_enabled_ && h_small_in_ != nullptr && nd_ == 0 &&
      (m_ <= milp_kernels::kSmallLdsCols || (medium_ && m_ <= milp_kernels::kMediumListRows))) {
    // Small or mid-size LP: one launch, v in and the dots out through mapped
    // host memory.
    if (small_inflight_) Synchronize();
    std::memcpy(h_small_y_, v.data(), m_ * sizeof(double));
    milp_kernels::ListDotsSmallArgs a{};
    a.starts = d_starts_;
    a.rows = d_rows_;
    a.vals = d_vals_;
    a.y = d_small_y_;
    a.m = m_;
    a.list = d_list_;
    a.n = n;
    a.out = d_small_out_;
    BeginKernel(MI_K_PRIMAL_NORMS);
    LaunchSmall(m_ <= milp_kernels::kSmallLdsCols ? milp_kernels::kSmallListDots
                                                  : milp_kernels::kMediumListDots,
                a);
    EndKernel(MI_K_PRIMAL_NORMS, 12.0 * double(list_entries_) + 8.0 * m_ + 4.0 * n + 8.0 * n);
    Synchronize();
    std::memcpy(out->data(), h_small_out_, n * sizeof(double));
    return;
  }
  std::memcpy(h_pin_d2_, v.data(), m_ * sizeof(double));
  Upload(d_vec_m_, h_pin_d2_, m_ * sizeof(double));
  BeginKernel(MI_K_PRIMAL_NORMS);
  LaunchColumnDots(2, d_vec_m_, nullptr, d_out_n_);
  Check(milp_launch::gather(d_list_, n, d_out_n_, d_out_list_, S(stream_)), "gather");
  EndKernel(MI_K_PRIMAL_NORMS, 12.0 * double(list_entries_) + 8.0 * double(list_dense_) * m_ +
                                   8.0 * m_ + 4.0 * n + 8.0 * n);
  Download(h_pin_d_, d_out_list_, n * sizeof(double));
  std::memcpy(out->data(), h_pin_d_, n * sizeof(double));
}

void DeviceLp::ListDots(const std::vector<int>& cols, const std::vector<double>& v,
                        std::vector<double>* out) {
  if (!shards_.empty()) return ShardedListDots(cols, v, out);
  CallTimer timer(&stats_, MI_K_PRIMAL_NORMS);
  fused_ready_ = false;  // d_out_n_ is reused below
  const int n = static_cast<int>(cols.size());
  out->resize(n);
  if (n == 0) return;
  std::memcpy(h_pin_i_, cols.data(), n * sizeof(int32_t));
  Upload(d_cols_, h_pin_i_, n * sizeof(int32_t));
  std::memcpy(h_pin_d2_, v.data(), m_ * sizeof(double));
  Upload(d_vec_m_, h_pin_d2_, m_ * sizeof(double));
  milp_kernels::DotArgs a{};
  a.starts = d_starts_;
  a.rows = d_rows_;
  a.vals = d_vals_;
  a.y = d_vec_m_;
  a.ncols = n;
  a.col_list = d_cols_;
  a.out = d_out_n_;
  double entries = 0.0;
  for (int c : cols) entries += double(h_starts_[c + 1] - h_starts_[c]);
  BeginKernel(MI_K_PRIMAL_NORMS);
  Check(milp_launch::column_dot(2, avg_col_len_ >= 32.0, a, S(stream_)), "listdots");
  Check(milp_launch::gather(d_cols_, n, d_out_n_, d_out_list_, S(stream_)), "gather");
  EndKernel(MI_K_PRIMAL_NORMS, 12.0 * entries + 8.0 * m_ + 12.0 * n);
  Download(h_pin_d_, d_out_list_, n * sizeof(double));
  std::memcpy(out->data(), h_pin_d_, n * sizeof(double));
}

void DeviceLp::Pricing(const std::vector<double>& c, const std::vector<double>& y,
                       std::vector<double>* rc, const std::vector<double>* w,
                       std::vector<double>* list_dots) {
  if (!shards_.empty()) return ShardedPricing(c, y, rc, w, list_dots);
  CallTimer timer(&stats_, MI_K_PRICING);
  fused_ready_ = false;  // d_out_n_ is reused below
  const bool fused = (w != nullptr);
  if (fused && list_dots == nullptr) throw DeviceError("fused pricing needs list_dots");
  CopyHost(h_pin_d_, c.data(), n_total_ * sizeof(double));
  Upload(d_vec_n_, h_pin_d_, n_total_ * sizeof(double));
  std::memcpy(h_pin_d2_, y.data(), m_ * sizeof(double));
  Upload(d_vec_m_, h_pin_d2_, m_ * sizeof(double));
  if (fused) {
    std::memcpy(h_pin_w_, w->data(), m_ * sizeof(double));
    Upload(d_vec_w_, h_pin_w_, m_ * sizeof(double));
  }
  if (fused && list_count_ < 0) throw DeviceError("update-row list used before FetchUpdateRow");
  const int n_list = fused ? list_count_ : 0;
  BeginKernel(MI_K_PRICING);
  if (fused) {
    LaunchColumnDots(5, d_vec_m_, d_vec_n_, d_out_n_, d_vec_w_, d_out_n2_);
    Check(milp_launch::gather(d_list_, n_list, d_out_n2_, d_out_list_, S(stream_)), "gather");
  } else {
    LaunchColumnDots(1, d_vec_m_, d_vec_n_, d_out_n_);
  }
  // 12 B per CSC entry of [A|I] (8 B per dense-block entry) + column starts
  // + y + c in + rc out; the fused pass also reads w, the flags,
  // and writes + gathers one dot per listed column.
  const double dense_entries = double(nd_) * m_;
  EndKernel(MI_K_PRICING, 12.0 * double(sparse_entries_) + 8.0 * dense_entries +
                              8.0 * (n_total_ + 1) + 8.0 * m_ + 16.0 * n_total_ +
                              (fused ? 8.0 * m_ + 1.0 * n_total_ + 28.0 * n_list : 0.0));
  rc->resize(n_total_);
  if (fused) {
    list_dots->resize(n_list);
    // Same stream: runs after the kernel, before the synchronizing download.
    if (n_list > 0) {
      Check(hipMemcpyAsync(h_pin_d2_, d_out_list_, n_list * sizeof(double),
                           hipMemcpyDeviceToHost, S(stream_)),
            "D2H");
    }
  }
  Download(h_pin_d_, d_out_n_, n_total_ * sizeof(double));
  CopyHost(rc->data(), h_pin_d_, n_total_ * sizeof(double));
  if (fused && n_list > 0) CopyHost(list_dots->data(), h_pin_d2_, n_list * sizeof(double));
}

void DeviceLp::ColumnSquaredNorms(std::vector<double>* out) {
  if (!shards_.empty()) FlushOwnMasks();
  CallTimer timer(&stats_, MI_K_COL_NORMS);
  fused_ready_ = false;  // d_out_n_ is reused below
  FlushRelevantMask();
  BeginKernel(MI_K_COL_NORMS);
  Check(milp_launch::column_squared_norms(d_starts_, d_vals_, d_masks_[kRelevant], n_total_,
                                          d_out_n_, S(stream_)),
        "colnorms");
  EndKernel(MI_K_COL_NORMS, 8.0 * nnz_ + 8.0 * (n_total_ + 1) + 8.0 * n_total_);
  out->resize(n_total_);
  Download(h_pin_d_, d_out_n_, n_total_ * sizeof(double));
  std::memcpy(out->data(), h_pin_d_, n_total_ * sizeof(double));
}

void DeviceLp::RowSums(const std::vector<double>& x, bool skip_basic, double sign,
                       std::vector<double>* out) {
  if (!shards_.empty()) FlushOwnMasks();
  CallTimer timer(&stats_, MI_K_SPMV_ROWS);
  std::memcpy(h_pin_d_, x.data(), n_total_ * sizeof(double));
  Upload(d_vec_n_, h_pin_d_, n_total_ * sizeof(double));
  milp_kernels::RowSumArgs a{};
  a.t_starts = d_t_starts_;
  a.t_cols = d_t_cols_;
  a.t_vals = d_t_vals_;
  a.x = d_vec_n_;
  a.skip = skip_basic ? d_masks_[kBasic] : nullptr;
  a.sign = sign;
  a.num_rows = m_;
  a.out = d_vec_m2_;
  BeginKernel(MI_K_SPMV_ROWS);
  Check(milp_launch::row_sums(a, S(stream_)), "rowsums");
  EndKernel(MI_K_SPMV_ROWS, 12.0 * nnz_ + 8.0 * (m_ + 1) + 8.0 * n_total_ + 8.0 * m_);
  out->resize(m_);
  Download(h_pin_d_, d_vec_m2_, m_ * sizeof(double));
  std::memcpy(out->data(), h_pin_d_, m_ * sizeof(double));
}


// ---------------------------------------------------------------------------
// Dual device mode.
namespace {
template <typename T>
void PinnedResize(T** p, size_t n) {
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(p), std::max<size_t>(1, n) * sizeof(T)) !=
      hipSuccess) {
    throw DeviceError("hipHostMalloc");
  }
}
// Pinned host memory the kernels write directly (device pointer in *dev).
template <typename T>
void MappedResize(T** p, T** dev, size_t n) {
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *dev = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(p), std::max<size_t>(1, n) * sizeof(T),
                    hipHostMallocMapped) != hipSuccess) {
    throw DeviceError("hipHostMalloc (mapped)");
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, *p, 0) != hipSuccess) throw DeviceError("mapped pointer");
  *dev = static_cast<T*>(d);
}
}  // namespace

void DeviceLp::DualBegin(const std::vector<double>& rc, const std::vector<uint8_t>& colbits,
                         const std::vector<double>& bound_diff) {
  if (!shards_.empty()) return ShardedDualBegin(rc, colbits, bound_diff);
  if (!dual_ready_) {
    d_rc_ = Alloc<double>(n_total_);
    d_colbits_ = Alloc<uint8_t>(n_total_);
    d_bound_diff_ = Alloc<double>(n_total_);
    d_best_ = Alloc<unsigned long long>(2);  // alternating pass-1 slots
    Check(hipMemsetAsync(d_best_, 0xff, 2 * sizeof(unsigned long long), S(stream_)), "memset");
    dual_calls_ = 0;
    d_slot_flags_ = Alloc<uint8_t>(n_total_);
    d_slots_ = Alloc<int32_t>(n_total_);
    d_num_slots_ = Alloc<int>(1);
    d_cand_col_ = Alloc<int32_t>(n_total_);
    d_cand_coeff_ = Alloc<double>(n_total_);
    d_cand_rc_ = Alloc<double>(n_total_);
    d_small_cols_ = Alloc<int32_t>(n_total_);
    d_small_bits_ = Alloc<uint8_t>(n_total_);
    d_best2_ = Alloc<unsigned long long>(2);
    d_tighten_ = Alloc<milp_kernels::TightenState>(1);
    d_keys_in_ = Alloc<unsigned long long>(n_total_);
    d_keys_out_ = Alloc<unsigned long long>(n_total_);
    d_sorted_slots_ = Alloc<int32_t>(n_total_);
    sort_temp_bytes_ = 0;
    Check(rocprim::radix_sort_pairs(nullptr, sort_temp_bytes_, d_keys_in_, d_keys_out_,
                                             d_slots_, d_sorted_slots_, n_total_, 0, 64,
                                             S(stream_)),
          "radix sizing");
    d_sort_temp_ = Alloc<uint8_t>(sort_temp_bytes_);
    Synchronize();  // the pinned buffers below may still feed earlier copies
    MappedResize(&h_cand_col_, &m_cand_col_, n_total_);
    MappedResize(&h_cand_coeff_, &m_cand_coeff_, n_total_);
    MappedResize(&h_cand_rc_, &m_cand_rc_, n_total_);
    MappedResize(&h_dual_counts_, &m_dual_counts_, 2);
    // Column-bit changes and the listed boxed flips go through mapped memory
    // (kernels read their inputs and write the flags there: no copies).
    MappedResize(&h_cb_cols_, &m_cb_cols_, 2 * size_t(n_total_));
    MappedResize(&h_cb_bits_, &m_cb_bits_, 2 * size_t(n_total_));
    MappedResize(&h_flip_cols_, &m_flip_cols_, n_total_);
    MappedResize(&h_flip_flags_, &m_flip_flags_, n_total_);
    if (ev_flips_ == nullptr) {
      hipEvent_t e;
      Check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
      ev_flips_ = e;
    }
    for (void*& ev : ev_cb_) {
      if (ev == nullptr) {
        hipEvent_t e;
        Check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        ev = e;
      }
    }
    last_candidates_ = 0;
    dual_ready_ = true;
  }
  if (static_cast<int>(rc.size()) != n_total_ || static_cast<int>(colbits.size()) != n_total_ ||
      static_cast<int>(bound_diff.size()) != n_total_) {
    throw DeviceError("dual device mode: size mismatch");
  }
  WaitEarlyFlips();
  ++rc_epoch_;
  Upload(d_rc_, rc.data(), n_total_ * sizeof(double));
  Upload(d_colbits_, colbits.data(), n_total_);
  Upload(d_bound_diff_, bound_diff.data(), n_total_ * sizeof(double));
  Synchronize();  // pageable sources
}

void DeviceLp::DualSetColBits(const std::vector<int32_t>& cols,
                              const std::vector<uint8_t>& bits) {
  if (!shards_.empty()) return ShardedDualSetColBits(cols, bits);
  const int n = static_cast<int>(cols.size());
  if (n == 0) return;
  if (n > n_total_) throw DeviceError("dual device mode: too many column changes");
  if (early_flips_.pending) {
    early_flips_.cols_changed.insert(early_flips_.cols_changed.end(), cols.begin(), cols.end());
  }
  // Two alternating slots of mapped memory: the host fills one while the
  // kernel of the previous call may still read the other.
  const int slot = cb_slot_;
  cb_slot_ ^= 1;
  hipEvent_t done = reinterpret_cast<hipEvent_t>(ev_cb_[slot]);
  Check(hipEventSynchronize(done), "colbits event");
  const size_t off = size_t(slot) * n_total_;
  std::memcpy(h_cb_cols_ + off, cols.data(), n * sizeof(int32_t));
  std::memcpy(h_cb_bits_ + off, bits.data(), n);
  Check(milp_launch::set_colbits(m_cb_cols_ + off, m_cb_bits_ + off, n, d_colbits_, S(stream_)),
        "colbits");
  Check(hipEventRecord(done, S(stream_)), "colbits event");
}

void DeviceLp::DualTakePricedReducedCosts() {
  if (!shards_.empty()) return ShardedDualTakePricedReducedCosts();
  ++rc_epoch_;
  Check(hipMemcpyAsync(d_rc_, d_out_n_, n_total_ * sizeof(double), hipMemcpyDeviceToDevice,
                       S(stream_)),
        "D2D");
}

void DeviceLp::DualDownloadReducedCosts(std::vector<double>* rc) {
  if (!shards_.empty()) return ShardedDualDownloadReducedCosts(rc);
  CallTimer timer(&stats_, MI_K_READBACK);
  rc->resize(n_total_);
  Download(h_pin_d_, d_rc_, n_total_ * sizeof(double));
  std::memcpy(rc->data(), h_pin_d_, n_total_ * sizeof(double));
}

void DeviceLp::DualSetReducedCost(int col, double value) {
  if (!shards_.empty()) return ShardedDualSetReducedCost(col, value);
  ++rc_epoch_;
  Check(milp_launch::set_double(d_rc_ + col, value, S(stream_)), "set rc");
}

milp_kernels::ScanState DeviceLp::NextScan() {
  if (++scan_epoch_ == 0) scan_epoch_ = 1;  // 0 is the zeroed status words' epoch
  return milp_kernels::ScanState{d_scan_status_, d_scan_ticket_, scan_epoch_, m_scan_fail_};
}

void DeviceLp::CheckScan() {
  if (*static_cast<volatile int*>(h_scan_fail_) != 0) {
    throw DeviceError("ordered compaction: look-back wait timed out at tile " +
                      std::to_string(*h_scan_fail_ - 1));
  }
}

// Two launches: pass 1 (the bound B), then pass 2 fused with its ordered
// compaction and the candidate gather into mapped host memory; one stream
// synchronization, no copies. Only a large pass-2 set (rare) adds the
// tightening round (keys, radix sort, walk, pass 2 again).
// MILP_TIGHTEN_STATS=1: at exit, how many breakpoints the tightening passes
// sorted (k1) and how far the walk went, by powers of two.
struct TightenStats {
  static inline const bool on = std::getenv("MILP_TIGHTEN_STATS") != nullptr;
  std::mutex mu;
  int64_t calls = 0, no_accept = 0, k1_hist[32] = {}, walk_hist[32] = {};
  void Add(int k1, int walk, bool none) {
    std::lock_guard<std::mutex> l(mu);
    ++calls;
    no_accept += none ? 1 : 0;
    ++k1_hist[std::min(31, 32 - __builtin_clz(static_cast<unsigned>(std::max(k1, 1))))];
    ++walk_hist[std::min(31, 32 - __builtin_clz(static_cast<unsigned>(std::max(walk, 1))))];
  }
  ~TightenStats() {
    if (!on || calls == 0) return;
    std::fprintf(stderr, "[tighten] calls %lld, walks without acceptance %lld\n",
                 static_cast<long long>(calls), static_cast<long long>(no_accept));
    for (int b = 0; b < 32; ++b) {
      if (k1_hist[b] == 0 && walk_hist[b] == 0) continue;
      std::fprintf(stderr, "[tighten] < 2^%2d: k1 %lld walk %lld\n", b,
                   static_cast<long long>(k1_hist[b]), static_cast<long long>(walk_hist[b]));
    }
  }
};
TightenStats g_tighten_stats;

void DeviceLp::DualRatioCandidates(double sign, double threshold, double harris_tolerance,
                                   double minimum_delta, double variation_magnitude,
                                   DualCandidates* out) {
  if (!shards_.empty()) {
    return ShardedDualRatioCandidates(sign, threshold, harris_tolerance, minimum_delta,
                                      variation_magnitude, out);
  }
  CallTimer timer(&stats_, MI_K_DUAL_RATIO);
  milp_kernels::DualRatioArgs a{};
  a.list = d_list_;
  a.list_coeff = d_out_list_;
  a.count = d_count_;
  a.max_count = n_total_;
  a.rc = d_rc_;
  a.colbits = d_colbits_;
  a.bound_diff = d_bound_diff_;
  a.sign = sign;
  a.threshold = threshold;
  a.harris_tolerance = harris_tolerance;
  a.minimum_delta = minimum_delta;
  a.variation_magnitude = variation_magnitude;
  const int slot = static_cast<int>(dual_calls_++ & 1);
  a.best = d_best_ + slot;
  a.best_next = d_best_ + (slot ^ 1);
  a.bound = a.best;
  milp_kernels::DualSelectOut sel{};
  sel.slots = d_slots_;
  sel.num_slots = d_num_slots_;
  sel.cand_col = m_cand_col_;
  sel.cand_coeff = m_cand_coeff_;
  sel.cand_rc = m_cand_rc_;
  sel.counts = m_dual_counts_;
  // Past tighten_min_candidates_ a second pass follows and writes the host
  // copy: this one keeps its candidates on the device.
  sel.host_cap = std::max(0, tighten_min_candidates_);
  BeginKernel(MI_K_DUAL_RATIO);
  Check(milp_launch::dual_ratio_bound(a, S(stream_)), "dual ratio bound");
  Check(milp_launch::dual_ratio_select(a, sel, NextScan(), S(stream_)), "dual ratio select");
  EndKernel(MI_K_DUAL_RATIO, 0.0);  // bytes added once the list length is known
  Synchronize();
  CheckScan();
  const int k1 = h_dual_counts_[0];
  // Many breakpoints under B: tighten the bound by walking them in pop order.
  if (k1 > tighten_min_candidates_) {
    if (k1 > n_total_) throw DeviceError("dual ratio test: bad counts");
    BeginKernel(MI_K_DUAL_RATIO);
    if (tighten_sort_) {
      Check(milp_launch::dual_ratio_keys(a, d_slots_, k1, d_keys_in_, S(stream_)), "keys");
      size_t bytes = sort_temp_bytes_;
      Check(rocprim::radix_sort_pairs(d_sort_temp_, bytes, d_keys_in_, d_keys_out_, d_slots_,
                                      d_sorted_slots_, k1, 0, 64, S(stream_)),
            "radix sort");
      Check(milp_launch::dual_flip_walk(a, d_sorted_slots_, k1, d_best2_, S(stream_)), "walk");
    } else {
      Check(milp_launch::dual_tighten(a, d_slots_, k1, d_keys_in_, d_tighten_, d_best2_,
                                      tighten_target_, S(stream_)),
            "tighten");
    }
    a.bound = d_best2_;
    sel.host_cap = std::numeric_limits<int>::max();
    Check(milp_launch::dual_ratio_select(a, sel, NextScan(), S(stream_)), "dual ratio select");
    EndKernel(MI_K_DUAL_RATIO, 0.0, /*count_launch=*/false);  // same logical launch
    Synchronize();
    CheckScan();
    if (TightenStats::on) {
      unsigned long long w = 0;
      Check(hipMemcpy(&w, d_best2_ + 1, sizeof(w), hipMemcpyDeviceToHost), "walk length");
      g_tighten_stats.Add(k1, static_cast<int>(w & 0xffffffffull), (w >> 40) != 0);
    }
  }
  const int k = h_dual_counts_[0];
  const int count = h_dual_counts_[1];
  if (k < 0 || k > n_total_ || count < 0 || count > n_total_) {
    throw DeviceError("dual ratio test: bad counts");
  }
  last_candidates_ = k;
  dual_list_count_ = count;
  // Algorithmic bytes: per list slot its position and coefficient, and the
  // reduced cost, column byte and bound difference of its column (29 B), once
  // per pass; the candidates written (20 B) and their tightening keys.
  const bool tightened = k1 > tighten_min_candidates_;
  stats_.algorithmic_bytes[MI_K_DUAL_RATIO] +=
      (tightened ? 3.0 : 2.0) * 29.0 * count + 20.0 * k + (tightened ? 20.0 * k1 + 36.0 * k1 : 0.0);
  out->col.assign(h_cand_col_, h_cand_col_ + k);
  out->coeff.assign(h_cand_coeff_, h_cand_coeff_ + k);
  out->rc.assign(h_cand_rc_, h_cand_rc_ + k);
  out->list_count = count;
}

void DeviceLp::DualUpdateReducedCosts(double mult, int leaving_col, double leaving_value,
                                      int entering_col) {
  if (!shards_.empty()) {
    return ShardedDualUpdateReducedCosts(mult, leaving_col, leaving_value, entering_col);
  }
  CallTimer timer(&stats_, MI_K_RC_UPDATE);
  ++rc_epoch_;
  BeginKernel(MI_K_RC_UPDATE);
  Check(milp_launch::update_reduced_costs(d_list_, d_out_list_, d_count_, n_total_, mult,
                                          leaving_col, leaving_value, entering_col, d_rc_,
                                          S(stream_)),
        "rc update");
  // The list (position + coefficient) and a read-modify-write of rc.
  EndKernel(MI_K_RC_UPDATE, 28.0 * dual_list_count_);
}

void DeviceLp::DualBoxedFlips(const std::vector<int>* cols, double threshold,
                              std::vector<uint8_t>* flags) {
  if (!shards_.empty()) return ShardedDualBoxedFlips(cols, threshold, flags);
  CallTimer timer(&stats_, MI_K_DUAL_RATIO);
  const int n = cols != nullptr ? static_cast<int>(cols->size()) : n_total_;
  flags->assign(n, 0);
  if (early_flips_.pending) {
    const EarlyFlips& e = early_flips_;
    bool same = cols != nullptr && n == e.n && threshold == e.threshold &&
                rc_epoch_ == e.rc_epoch &&
                std::memcmp(cols->data(), h_flip_cols_, size_t(n) * sizeof(int32_t)) == 0;
    for (size_t i = 0; same && i < e.cols_changed.size(); ++i) {
      same = std::find(cols->begin(), cols->end(), e.cols_changed[i]) == cols->end();
    }
    WaitEarlyFlips();  // its buffers are reused below either way
    if (same) {
      std::memcpy(flags->data(), h_flip_flags_, n);
      return;
    }
  }
  if (n == 0) return;
  if (cols != nullptr) {
    // A list (the candidates of one ratio test): columns in and flags out
    // through mapped memory; the stream sync is the only round trip.
    // (The previous listed call ended with a sync: the buffers are free.)
    std::memcpy(h_flip_cols_, cols->data(), n * sizeof(int32_t));
    Check(milp_launch::boxed_flips(m_flip_cols_, n, d_rc_, d_colbits_, threshold, m_flip_flags_,
                                   S(stream_)),
          "boxed flips");
    Synchronize();
    std::memcpy(flags->data(), h_flip_flags_, n);
    return;
  }
  Check(milp_launch::boxed_flips(nullptr, n, d_rc_, d_colbits_, threshold, d_slot_flags_,
                                 S(stream_)),
        "boxed flips");
  Download(h_flip_flags_, d_slot_flags_, n);
  std::memcpy(flags->data(), h_flip_flags_, n);
}

void DeviceLp::DualBoxedFlipsEarly(const std::vector<int>& cols, double threshold) {
  if (!early_flips_on_ || !shards_.empty() || !dual_ready_) return;
  const int n = static_cast<int>(cols.size());
  if (n == 0 || n > n_total_) return;
  WaitEarlyFlips();
  std::memcpy(h_flip_cols_, cols.data(), size_t(n) * sizeof(int32_t));
  Check(milp_launch::boxed_flips(m_flip_cols_, n, d_rc_, d_colbits_, threshold, m_flip_flags_,
                                 S(stream_)),
        "boxed flips (early)");
  Check(hipEventRecord(reinterpret_cast<hipEvent_t>(ev_flips_), S(stream_)), "flips event");
  early_flips_.pending = true;
  early_flips_.n = n;
  early_flips_.threshold = threshold;
  early_flips_.rc_epoch = rc_epoch_;
  early_flips_.cols_changed.clear();
}

void DeviceLp::WaitEarlyFlips() {
  if (!early_flips_.pending) return;
  early_flips_.pending = false;
  Check(hipEventSynchronize(reinterpret_cast<hipEvent_t>(ev_flips_)), "flips event");
}

}  // namespace milp
