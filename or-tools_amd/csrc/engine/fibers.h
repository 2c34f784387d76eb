// Cooperative fibers for the batched small-LP solves (configs 3 and 4).
//
// A small LP's iteration is ~15 us of host work around one device round trip
// of ~24 us. With one LP per host thread, the thread idles in
// the stream wait. Here one host thread drives several LPs, each on a fiber of
// its own: where the engine waits for its stream (DeviceLp::WaitStream), a
// fiber whose stream is not done yields, and the thread runs another LP's host
// work meanwhile. The LPs are independent solver instances (one handle and
// one stream each); nothing is shared between fibers except the thread, so
// every LP's arithmetic and results are unchanged. Outside a fiber pool the
// yield is a no-op and the wait is the plain stream synchronization.
#ifndef MILP_FIBERS_H_
#define MILP_FIBERS_H_

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

// Context switch (engine/simplex.cc, x86-64 SysV): saves the callee-saved
// registers, MXCSR and the x87 control word on the current stack, stores the
// stack pointer to *save_sp, and resumes the context saved at load_sp. No
// system call (swapcontext's signal-mask save costs two per switch, which
// dominated a batch whose fibers mostly poll).
extern "C" void milp_fiber_switch(void** save_sp, void* load_sp);
extern "C" void milp_fiber_trampoline();

namespace milp {

namespace fiber_detail {
struct Fiber {
  void* sp = nullptr;
  std::function<void()> fn;
  std::unique_ptr<char[]> stack;
  bool done = false;
  double weight = 0.0;  // SetFiberWeight: the scheduler favours the heaviest
};
inline thread_local void** t_sched_sp = nullptr;  // where the scheduler's sp is saved
inline thread_local Fiber* t_current = nullptr;
inline thread_local bool t_slice_idle = false;
// MILP_SDUAL_PROFILE: slices over 1 ms (a fiber holding its thread).
struct SliceStats {
  std::atomic<int64_t> long_ns{0}, long_count{0}, max_ns{0};
};
inline SliceStats g_slices;
inline bool SliceProfile() {
  static const bool on = std::getenv("MILP_SDUAL_PROFILE") != nullptr;
  return on;
}

// First code a fiber runs (through milp_fiber_trampoline): never returns.
extern "C" inline void milp_fiber_entry(Fiber* f) {
  f->fn();
  f->done = true;
  milp_fiber_switch(&f->sp, *t_sched_sp);
  __builtin_unreachable();
}
}  // namespace fiber_detail

// True inside a fiber of a running pool.
inline bool InFiber() { return fiber_detail::t_current != nullptr; }

// The current fiber's work estimate (0 = none). A pool gives its heaviest
// fiber every other slice: a large LP is host-bound and would otherwise get
// a 1/k share of its thread while the light LPs it shares the thread with
// mostly wait for the device; the light ones now run in its device waits.
inline void SetFiberWeight(double w) {
  if (fiber_detail::t_current != nullptr) fiber_detail::t_current->weight = w;
}
inline bool FiberPriorityEnabled() {
  static const bool on = [] {
    const char* e = std::getenv("MILP_BATCH_PRIORITY");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

// Gives the thread to the next fiber of the pool; returns when this fiber is
// scheduled again. A no-op outside a pool. idle: the slice since the last
// resume only found its wait unfinished (the scheduler backs off when a whole
// round was idle).
inline void FiberYield(bool idle = false) {
  using namespace fiber_detail;
  Fiber* f = t_current;
  if (f == nullptr) return;
  t_slice_idle = idle;
  milp_fiber_switch(&f->sp, *t_sched_sp);
}

// Runs every task as a fiber on the calling thread, round robin at the
// yields, until all have returned. Tasks must not throw (RunSolve catches).
// After two rounds in which every fiber only polled the thread yields its CPU
// between rounds; after 4 096 such rounds (a long device wait) it sleeps ~20 us
// per round, so the CPU quota stays with the threads that work.
inline void RunFibers(std::vector<std::function<void()>> tasks, size_t stack_bytes = 4u << 20) {
  using namespace fiber_detail;
  if (tasks.size() == 1) {  // nothing to interleave
    tasks[0]();
    return;
  }
  std::vector<std::unique_ptr<Fiber>> fibers;
  for (auto& t : tasks) {
    auto f = std::make_unique<Fiber>();
    f->fn = std::move(t);
    f->stack.reset(new char[stack_bytes]);
    // Initial frame popped by milp_fiber_switch: control words, r15, r14,
    // r13 = entry, r12 = fiber, rbx, rbp, return address = trampoline.
    uintptr_t top = reinterpret_cast<uintptr_t>(f->stack.get()) + stack_bytes;
    top &= ~uintptr_t{15};
    uint64_t* sp = reinterpret_cast<uint64_t*>(top - 80);
    sp[0] = 0x037Full << 32 | 0x1F80u;  // MXCSR default, x87 control word default
    sp[1] = 0;
    sp[2] = 0;
    sp[3] = reinterpret_cast<uint64_t>(&milp_fiber_entry);
    sp[4] = reinterpret_cast<uint64_t>(f.get());
    sp[5] = 0;
    sp[6] = 0;
    sp[7] = reinterpret_cast<uint64_t>(&milp_fiber_trampoline);
    f->sp = sp;
    fibers.push_back(std::move(f));
  }
  void* sched_sp = nullptr;
  void** saved_sched = t_sched_sp;
  Fiber* saved_current = t_current;
  t_sched_sp = &sched_sp;
  size_t remaining = fibers.size();
  int idle_rounds = 0;
  const bool priority = FiberPriorityEnabled();
  while (remaining > 0) {
    bool all_idle = true;
    auto run_slice = [&](Fiber* f) {
      t_current = f;
      t_slice_idle = false;
      const bool prof = SliceProfile();
      const auto s0 = prof ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
      milp_fiber_switch(&sched_sp, f->sp);
      if (prof) {
        const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - s0).count();
        if (ns > 1000000) {
          g_slices.long_ns += ns;
          ++g_slices.long_count;
        }
        int64_t m = g_slices.max_ns.load();
        while (ns > m && !g_slices.max_ns.compare_exchange_weak(m, ns)) {
        }
      }
      t_current = nullptr;
      if (!t_slice_idle) all_idle = false;
      if (f->done) --remaining;
    };
    // The heaviest running fiber (weights are set by the tasks) runs before
    // every other fiber's slice.
    Fiber* heavy = nullptr;
    if (priority) {
      for (auto& f : fibers) {
        if (!f->done && f->weight > 0.0 && (heavy == nullptr || f->weight > heavy->weight)) {
          heavy = f.get();
        }
      }
    }
    for (auto& f : fibers) {
      if (f->done || f.get() == heavy) continue;
      if (heavy != nullptr && !heavy->done) run_slice(heavy);
      run_slice(f.get());
    }
    if (heavy != nullptr && !heavy->done) run_slice(heavy);
    idle_rounds = all_idle ? idle_rounds + 1 : 0;
    static const int idle_us = [] {  // MILP_FIBER_IDLE_US=k: sleep k us per idle round
      const char* e = std::getenv("MILP_FIBER_IDLE_US");
      return e != nullptr ? std::atoi(e) : 0;
    }();
    if (idle_rounds >= 4096) {
      std::this_thread::sleep_for(std::chrono::microseconds(20));  // long device waits
    } else if (idle_rounds >= 2) {
      if (idle_us > 0) {
        std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
      } else {
        std::this_thread::yield();
      }
    }
  }
  t_sched_sp = saved_sched;
  t_current = saved_current;
}

}  // namespace milp

#endif  // MILP_FIBERS_H_
