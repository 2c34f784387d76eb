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

#include <ucontext.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

namespace milp {

namespace fiber_detail {
struct Fiber {
  ucontext_t ctx;
  std::function<void()> fn;
  std::unique_ptr<char[]> stack;
  bool done = false;
};
inline thread_local ucontext_t* t_scheduler = nullptr;
inline thread_local Fiber* t_current = nullptr;

inline void Entry(unsigned lo, unsigned hi) {
  Fiber* f = reinterpret_cast<Fiber*>((static_cast<uintptr_t>(hi) << 32) | lo);
  f->fn();
  f->done = true;  // returning resumes the scheduler (uc_link)
}
}  // namespace fiber_detail

// True inside a fiber of a running pool.
inline bool InFiber() { return fiber_detail::t_current != nullptr; }

// Gives the thread to the next fiber of the pool; returns when this fiber is
// scheduled again. A no-op outside a pool.
inline void FiberYield() {
  using namespace fiber_detail;
  Fiber* f = t_current;
  if (f == nullptr) return;
  swapcontext(&f->ctx, t_scheduler);
}

// Runs every task as a fiber on the calling thread, round robin at the
// yields, until all have returned. Tasks must not throw (RunSolve catches).
inline void RunFibers(std::vector<std::function<void()>> tasks, size_t stack_bytes = 4u << 20) {
  using namespace fiber_detail;
  if (tasks.size() == 1) {  // nothing to interleave
    tasks[0]();
    return;
  }
  ucontext_t scheduler;
  std::vector<std::unique_ptr<Fiber>> fibers;
  for (auto& t : tasks) {
    auto f = std::make_unique<Fiber>();
    f->fn = std::move(t);
    f->stack.reset(new char[stack_bytes]);
    getcontext(&f->ctx);
    f->ctx.uc_stack.ss_sp = f->stack.get();
    f->ctx.uc_stack.ss_size = stack_bytes;
    f->ctx.uc_link = &scheduler;
    const uintptr_t p = reinterpret_cast<uintptr_t>(f.get());
    makecontext(&f->ctx, reinterpret_cast<void (*)()>(&Entry), 2,
                static_cast<unsigned>(p & 0xffffffffu), static_cast<unsigned>(p >> 32));
    fibers.push_back(std::move(f));
  }
  ucontext_t* saved_scheduler = t_scheduler;
  Fiber* saved_current = t_current;
  t_scheduler = &scheduler;
  size_t remaining = fibers.size();
  while (remaining > 0) {
    for (auto& f : fibers) {
      if (f->done) continue;
      t_current = f.get();
      swapcontext(&scheduler, &f->ctx);
      t_current = nullptr;
      if (f->done) --remaining;
    }
  }
  t_scheduler = saved_scheduler;
  t_current = saved_current;
}

}  // namespace milp

#endif  // MILP_FIBERS_H_
