// Fork-join pool for the engine's O(N) host loops.
//
// Only element-independent work is split: every element is computed by the
// same expression as in the serial loop and written to its own slot, and
// anything order-dependent (the DynamicMaximum top-k heap, RNG draws) is
// replayed serially afterwards, in the serial loop's order. Results therefore
// do not depend on the number of threads or on the partition.
//
// One process-wide pool. A caller that finds it busy (another handle's loop)
// runs all parts itself. MILP_HOST_THREADS sets the thread count (caller
// included, default 16 and at most the hardware's threads; 1 disables the
// pool).
#ifndef MILP_HOST_POOL_H_
#define MILP_HOST_POOL_H_

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace milp {

// A thread that runs one LP of a batch (mi_lp_batch_solve's workers): the
// batch already keeps every core busy, so its loops run serially instead of
// waking the pool (whose spinning workers would take cores from the other
// LPs). The results are the same either way.
inline thread_local bool t_host_serial = false;
struct HostSerialScope {
  bool saved;
  explicit HostSerialScope(bool on) : saved(t_host_serial) { t_host_serial = on; }
  ~HostSerialScope() { t_host_serial = saved; }
};

class HostPool {
 public:
  static HostPool& Get() {
    static HostPool pool;
    return pool;
  }
  int threads() const { return t_host_serial ? 1 : num_threads_; }

  // fn(part) for part in [0, parts); part 0 runs on the caller.
  void Run(int parts, const std::function<void(int)>& fn) {
    if (parts <= 1 || threads() <= 1) {
      for (int p = 0; p < parts; ++p) fn(p);
      return;
    }
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) {
      for (int p = 0; p < parts; ++p) fn(p);
      return;
    }
    // Publish the job (its pointer last), then wake the workers; sleeping
    // ones need the condition variable, spinning ones see the generation.
    next_part_.store(1, std::memory_order_relaxed);
    pending_.store(parts - 1, std::memory_order_relaxed);
    job_parts_.store(parts, std::memory_order_relaxed);
    job_.store(&fn, std::memory_order_release);
    generation_.fetch_add(1, std::memory_order_acq_rel);
    if (sleepers_.load(std::memory_order_acquire) > 0) {
      { std::lock_guard<std::mutex> l(mu_); }
      cv_.notify_all();
    }
    fn(0);
    // The caller helps with the parts no worker has picked up yet.
    for (int p = next_part_.fetch_add(1, std::memory_order_acq_rel); p < parts;
         p = next_part_.fetch_add(1, std::memory_order_acq_rel)) {
      fn(p);
      pending_.fetch_sub(1, std::memory_order_acq_rel);
    }
    while (pending_.load(std::memory_order_acquire) != 0) Pause();
    // Retire the job; return only when no worker can still be reading it.
    // The retire store and the active_ load are seq_cst, as are the worker's
    // active_ increment and job_ load: release/acquire would let this load be
    // ordered before the store (store-load reordering), and a worker that
    // registers in that window would still read the retired job.
    job_.store(nullptr, std::memory_order_seq_cst);
    while (active_.load(std::memory_order_seq_cst) != 0) Pause();
  }

  ~HostPool() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_.store(true, std::memory_order_release);
      generation_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (std::thread& t : workers_) t.join();
  }

 private:
  HostPool() {
    int n = 16;  // the GPU box's CPU share per GPU
    if (const char* e = std::getenv("MILP_HOST_THREADS")) n = std::atoi(e);
    const int hw = static_cast<int>(std::thread::hardware_concurrency());
    if (hw > 0) n = std::min(n, hw);
    num_threads_ = std::max(1, std::min(n, 16));
    for (int i = 1; i < num_threads_; ++i) workers_.emplace_back([this]() { Work(); });
  }
  static void Pause() { __builtin_ia32_pause(); }

  void Work() {
    uint64_t seen = 0;
    while (true) {
      // Spin (the engine's loops come every few hundred microseconds while
      // a solve runs), then sleep until the next job.
      uint64_t g = generation_.load(std::memory_order_acquire);
      if (g == seen) {
        const auto start = std::chrono::steady_clock::now();
        for (int spin = 1; g == seen; ++spin) {
          Pause();
          g = generation_.load(std::memory_order_acquire);
          if ((spin & 1023) == 0 &&
              std::chrono::steady_clock::now() - start > std::chrono::milliseconds(5)) {
            break;
          }
        }
      }
      if (g == seen) {
        std::unique_lock<std::mutex> l(mu_);
        sleepers_.fetch_add(1, std::memory_order_acq_rel);
        cv_.wait(l, [&]() { return generation_.load(std::memory_order_acquire) != seen; });
        sleepers_.fetch_sub(1, std::memory_order_acq_rel);
        g = generation_.load(std::memory_order_acquire);
      }
      seen = g;
      if (stop_.load(std::memory_order_acquire)) return;
      active_.fetch_add(1, std::memory_order_seq_cst);
      const std::function<void(int)>* job = job_.load(std::memory_order_seq_cst);
      if (job != nullptr) {
        const int parts = job_parts_.load(std::memory_order_relaxed);
        for (int p = next_part_.fetch_add(1, std::memory_order_acq_rel); p < parts;
             p = next_part_.fetch_add(1, std::memory_order_acq_rel)) {
          (*job)(p);
          pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
      }
      active_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }

  int num_threads_ = 1;
  std::vector<std::thread> workers_;
  std::mutex run_mu_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> generation_{0};
  std::atomic<int> next_part_{0};
  std::atomic<int> pending_{0};
  std::atomic<int> active_{0};
  std::atomic<const std::function<void(int)>*> job_{nullptr};
  std::atomic<int> job_parts_{0};
  std::atomic<int> sleepers_{0};
  std::atomic<bool> stop_{false};
};

// Splits [0, n) into at most HostPool threads parts whose boundaries are
// multiples of `align` (64 keeps bitset words whole), and runs
// fn(part, begin, end) on each. Runs serially when n < min_parallel.
// MILP_HOST_PARALLEL_MIN overrides every size threshold (tests set it low to
// run the split loops on small LPs).
inline int64_t ParallelMinOverride() {
  const char* e = std::getenv("MILP_HOST_PARALLEL_MIN");
  return e != nullptr ? std::atoll(e) : -1;
}

// The split of [0, n) ParallelRanges uses: `parts` parts of `per` elements
// (the last one shorter). Two-pass callers plan once and run both passes on
// the same plan, whatever MILP_HOST_THREADS reads between them.
struct RangePlan {
  int parts = 1;
  int64_t per = 0;
};

inline RangePlan PlanRanges(int64_t n, int64_t min_parallel, int64_t align) {
  HostPool& pool = HostPool::Get();
  const int64_t override_min = ParallelMinOverride();
  if (override_min >= 0) min_parallel = override_min;
  int parts = (n >= min_parallel && n > 0) ? pool.threads() : 1;
  if (const char* cap = std::getenv("MILP_HOST_THREADS")) {  // read per call: probes vary it
    parts = std::max(1, std::min(parts, std::atoi(cap)));
  }
  RangePlan plan;
  if (parts <= 1) {
    plan.per = n;
    return plan;
  }
  plan.per = ((n + parts - 1) / parts + align - 1) / align * align;
  plan.parts = static_cast<int>((n + plan.per - 1) / plan.per);
  return plan;
}

template <typename F>
int RunRanges(const RangePlan& plan, int64_t n, F&& fn) {
  if (plan.parts <= 1) {
    fn(0, int64_t{0}, n);
    return 1;
  }
  const int64_t per = plan.per;
  const std::function<void(int)> job = [&](int p) {
    const int64_t b = p * per;
    const int64_t e = std::min(n, b + per);
    fn(p, b, e);
  };
  HostPool::Get().Run(plan.parts, job);
  return plan.parts;
}

template <typename F>
int ParallelRanges(int64_t n, int64_t min_parallel, int64_t align, F&& fn) {
  return RunRanges(PlanRanges(n, min_parallel, align), n, std::forward<F>(fn));
}

// Appends to *rows the indices r in [begin, n) with v[r] != 0 in increasing
// order (and their values to *vals if not null), scanning the range in
// parallel parts that are concatenated in order: the same output as the
// serial loop. Returns the largest |v[r]| over the appended entries when
// max_abs is requested (std::max over |v| in index order, as the serial
// scan: a NaN is never selected).
template <typename Real>
void ParallelAppendNonZeros(const Real* v, int64_t begin, int64_t n, std::vector<int>* rows,
                            std::vector<Real>* vals, Real* max_abs = nullptr) {
  constexpr int kMaxParts = 16;
  int64_t part_count[kMaxParts] = {};
  Real part_max[kMaxParts] = {};
  const int64_t len = n > begin ? n - begin : 0;
  // Pass 1: count (and the largest magnitude) per part; pass 2: each part
  // writes its entries at its offset. Both passes run on one plan.
  const RangePlan plan = PlanRanges(len, 65536, 64);
  const int parts = RunRanges(plan, len, [&](int p, int64_t b, int64_t e) {
    int64_t c = 0;
    Real m = 0;
    for (int64_t i = begin + b; i < begin + e; ++i) {
      if (v[i] != 0.0) {
        ++c;
        m = std::max(m, std::fabs(v[i]));
      }
    }
    part_count[p] = c;
    part_max[p] = m;
  });
  const size_t base = rows->size();
  const size_t vbase = vals != nullptr ? vals->size() : 0;
  int64_t offset[kMaxParts + 1];
  offset[0] = 0;
  for (int p = 0; p < parts; ++p) offset[p + 1] = offset[p] + part_count[p];
  rows->resize(base + static_cast<size_t>(offset[parts]));
  if (vals != nullptr) vals->resize(vbase + static_cast<size_t>(offset[parts]));
  int* out_rows = rows->data() + base;
  Real* out_vals = vals != nullptr ? vals->data() + vbase : nullptr;
  RunRanges(plan, len, [&](int p, int64_t b, int64_t e) {
    int64_t at = offset[p];
    for (int64_t i = begin + b; i < begin + e; ++i) {
      if (v[i] != 0.0) {
        out_rows[at] = static_cast<int>(i);
        if (out_vals != nullptr) out_vals[at] = v[i];
        ++at;
      }
    }
  });
  Real m = max_abs != nullptr ? *max_abs : Real(0);
  for (int p = 0; p < parts; ++p) m = std::max(m, part_max[p]);
  if (max_abs != nullptr) *max_abs = m;
}

}  // namespace milp

#endif  // MILP_HOST_POOL_H_
