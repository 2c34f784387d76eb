// Host sampling profiler for the engine's own threads (development aid).
// MILP_SAMPLE_PROFILE=<us>: SIGPROF every <us> of process CPU time records
// the interrupted thread's call stack with its CLOCK_MONOTONIC time. At exit
// the samples inside MILP_SAMPLE_WINDOW=t0,t1 (ns; scripts/probe.py sets it
// to its timed window) are summed per function, self and inclusive, and
// printed to stderr. Nothing runs unless the variable is set. With
// MILP_SAMPLE_WALL the samples are wall-clock ticks of the first thread that
// enters RevisedSimplex::Solve instead of process CPU time.
#include <cxxabi.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/time.h>
#include <time.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace milp {
namespace {

constexpr int kDepth = 24;
constexpr int kMaxSamples = 1 << 18;

struct Sample {
  int64_t t_ns;
  int depth;
  void* pc[kDepth];
};

Sample* g_samples = nullptr;
std::atomic<int> g_count{0};

// The interrupted PC, then the callers found by unwinding (MILP_SAMPLE_STACK=1;
// the unwinder is not async-signal-safe everywhere, so off by default).
bool g_stack = false;
void OnProf(int, siginfo_t*, void* ctx) {
  if (g_samples == nullptr) return;
  const int k = g_count.fetch_add(1, std::memory_order_relaxed);
  if (k >= kMaxSamples) return;
  Sample& s = g_samples[k];
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  s.t_ns = static_cast<int64_t>(ts.tv_sec) * 1000000000 + ts.tv_nsec;
  const ucontext_t* uc = static_cast<const ucontext_t*>(ctx);
  s.pc[0] = nullptr;
  s.pc[1] = nullptr;
  s.pc[2] = reinterpret_cast<void*>(uc->uc_mcontext.gregs[REG_RIP]);
  s.depth = 3;
  if (g_stack) {
    void* frames[kDepth];
    const int n = backtrace(frames, kDepth);
    // frames[0..1]: this handler and the signal trampoline; frames[2] is the
    // interrupted function again.
    for (int f = 3; f < n && s.depth < kDepth; ++f) s.pc[s.depth++] = frames[f];
  }
}

std::string Name(void* pc) {
  Dl_info info;
  if (dladdr(pc, &info) == 0) return "?";
  if (info.dli_sname == nullptr) {
    const char* f = info.dli_fname != nullptr ? info.dli_fname : "?";
    const char* slash = std::strrchr(f, '/');
    return std::string(slash != nullptr ? slash + 1 : f) + "+?";
  }
  int status = 0;
  char* d = abi::__cxa_demangle(info.dli_sname, nullptr, nullptr, &status);
  std::string n = status == 0 && d != nullptr ? d : info.dli_sname;
  std::free(d);
  // Drop the argument lists: the function is what is summed.
  const size_t p = n.find('(');
  if (p != std::string::npos && p > 0) n = n.substr(0, p);
  return n.size() > 90 ? n.substr(0, 90) : n;
}

int g_interval_us = 0;
std::atomic<bool> g_attached{false};
timer_t g_timer;
bool g_timer_set = false;

struct Sampler {
  Sampler() {
    const char* e = std::getenv("MILP_SAMPLE_PROFILE");
    if (e == nullptr) return;
    const int us = std::max(50, std::atoi(e));
    g_interval_us = us;
    g_samples = static_cast<Sample*>(std::calloc(kMaxSamples, sizeof(Sample)));
    if (g_samples == nullptr) return;
    g_stack = std::getenv("MILP_SAMPLE_STACK") != nullptr;
    void* warm[2];
    backtrace(warm, 2);  // loads the unwinder outside the handler
    struct sigaction sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = OnProf;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, nullptr);
    // MILP_SAMPLE_WALL: wall-clock samples of the first solver thread only
    // (SamplerAttachThread), blocked time included.
    if (std::getenv("MILP_SAMPLE_WALL") != nullptr) return;
    itimerval tv;
    tv.it_interval.tv_sec = 0;
    tv.it_interval.tv_usec = us;
    tv.it_value = tv.it_interval;
    setitimer(ITIMER_PROF, &tv, nullptr);
  }
  ~Sampler() {
    if (g_samples == nullptr) return;
    itimerval off;
    std::memset(&off, 0, sizeof(off));
    setitimer(ITIMER_PROF, &off, nullptr);
    int64_t t0 = 0, t1 = INT64_MAX;
    if (const char* w = std::getenv("MILP_SAMPLE_WINDOW")) {
      long long a = 0, b = 0;
      if (std::sscanf(w, "%lld,%lld", &a, &b) == 2) {
        t0 = a;
        t1 = b;
      }
    }
    const int n = std::min(g_count.load(), kMaxSamples);
    std::map<void*, std::string> names;
    std::map<std::string, int> self, incl;
    int used = 0;
    for (int k = 0; k < n; ++k) {
      const Sample& s = g_samples[k];
      if (s.t_ns < t0 || s.t_ns > t1 || s.depth <= 2) continue;
      ++used;
      std::set<std::string> seen;
      // Frames 0-1 are the handler and the signal trampoline.
      for (int f = 2; f < s.depth; ++f) {
        auto it = names.find(s.pc[f]);
        if (it == names.end()) it = names.emplace(s.pc[f], Name(s.pc[f])).first;
        if (f == 2) ++self[it->second];
        if (seen.insert(it->second).second) ++incl[it->second];
      }
    }
    std::fprintf(stderr, "[sampler] %d samples (%d in window)\n", n, used);
    auto top = [&](const std::map<std::string, int>& m, const char* what) {
      std::vector<std::pair<int, std::string>> v;
      for (const auto& kv : m) v.emplace_back(kv.second, kv.first);
      std::sort(v.rbegin(), v.rend());
      std::fprintf(stderr, "[sampler] %s:\n", what);
      for (size_t i = 0; i < v.size() && i < 45; ++i) {
        std::fprintf(stderr, "  %6.2f%%  %s\n", 100.0 * v[i].first / std::max(1, used),
                     v[i].second.c_str());
      }
    };
    top(self, "self");
    top(incl, "inclusive");
  }
};
Sampler g_sampler;

}  // namespace

namespace {
bool WallMode(bool batch) {
  const char* w = std::getenv("MILP_SAMPLE_WALL");
  if (g_samples == nullptr || w == nullptr) return false;
  return (std::strcmp(w, "batch") == 0) == batch;
}
void AttachCaller();
}  // namespace

// MILP_SAMPLE_WALL=1: the first thread entering RevisedSimplex::Solve;
// MILP_SAMPLE_WALL=batch: the first batch worker thread (its fibers).
void SamplerAttachThread() {
  if (WallMode(false)) AttachCaller();
}
void SamplerAttachBatchThread() {
  if (WallMode(true)) AttachCaller();
}
// A batch call starts: its first worker thread is the one sampled (the
// previous call's workers have exited).
void SamplerBatchCallBegin() {
  if (!WallMode(true)) return;
  if (g_timer_set) {
    timer_delete(g_timer);
    g_timer_set = false;
  }
  g_attached.store(false);
}

namespace {
void AttachCaller() {
  if (g_attached.exchange(true)) return;
  sigevent ev;
  std::memset(&ev, 0, sizeof(ev));
  ev.sigev_notify = SIGEV_THREAD_ID;
  ev.sigev_signo = SIGPROF;
  ev._sigev_un._tid = static_cast<pid_t>(syscall(SYS_gettid));
  timer_t& timer = g_timer;
  if (timer_create(CLOCK_MONOTONIC, &ev, &timer) != 0) return;
  g_timer_set = true;
  itimerspec its;
  its.it_interval.tv_sec = 0;
  its.it_interval.tv_nsec = static_cast<long>(g_interval_us) * 1000;
  its.it_value = its.it_interval;
  timer_settime(timer, 0, &its, nullptr);
}
}  // namespace
}  // namespace milp
