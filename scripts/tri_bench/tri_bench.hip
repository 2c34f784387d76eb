// Development harness: the config-5 U solve (TransposeLowerSolve of U^T,
// sparse.cc:899-955) as standalone kernels, timed with HIP events and checked
// bit for bit against the host loop. Input: scripts/tri_bench/make_input.py.
//   tri_bench <data.bin> [reps]
// Variants differ only in how outputs are scheduled and how waits are done;
// every output is evaluated in Glop's order (groups of four from the column's
// end, then the 1-3 remaining one by one, then the division).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,               \
                   hipGetErrorString(e_));                                         \
      std::exit(2);                                                                \
    }                                                                              \
  } while (0)

constexpr unsigned long long kPending = 0x7ff0deadbeef0001ull;
constexpr uint64_t kMaxWait = 20000000;  // 0.2 s at 100 MHz

struct Sched {
  int num_pos, l0_end;
  const int* row;       // position -> row
  const int* cnt;       // entries
  const int* est;       // entry start (evaluation order)
  const int* epos;      // entry input position
  const double* eval;   // entry value
  const double* diag;   // per position
  const double* rhs;    // by row
  double* y;            // by position (sentinel until final)
  int* fail;
  int poll_max;
};

__device__ __forceinline__ double ld(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool pend(double v) {
  return static_cast<unsigned long long>(__double_as_longlong(v)) == kPending;
}

__global__ void init_kernel(Sched s) {
  const double p = __longlong_as_double(static_cast<long long>(kPending));
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < s.num_pos; k += gridDim.x * blockDim.x) {
    st(s.y + k, k < s.l0_end ? s.rhs[s.row[k]] / s.diag[k] : p);
  }
}

// Output k: waits for its inputs window by window (8 loads in flight), folds
// the groups as they become final, stores.
__device__ __forceinline__ void output(const Sched& s, int k) {
  const int n = s.cnt[k];
  const int e0 = s.est[k];
  const int end = e0 + n;
  double sum = s.rhs[s.row[k]];
  const double d = s.diag[k];
  int e = e0;
  int backoff = 1;
  uint64_t t_prog = wall_clock64();
  // The loop's exit is wave-uniform (every lane stays until all are done):
  // the store of a finished lane then sits inside the loop body and cannot be
  // sunk below the loop, where a waiting lane of the same wave would never
  // let the wave reach it.
  bool done = false;
  while (__ballot(!done) != 0) {
    if (done) continue;
    const int before = e;
    while (e < end) {
      double v[8];
      int ps[8];
      double cs[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ps[i] = e + i < end ? s.epos[e + i] : 0;
        cs[i] = e + i < end ? s.eval[e + i] : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = e + i < end ? ld(s.y + ps[i]) : 0.0;
      int took = 0;
      // Entry j of the output is group j / 4 while 4 remain, then singles.
#pragma unroll
      for (int g = 0; g < 8; g += 4) {
        if (took != g || e + g + 3 >= end) continue;
        if (pend(v[g]) || pend(v[g + 1]) || pend(v[g + 2]) || pend(v[g + 3])) continue;
        sum -= cs[g] * v[g] + cs[g + 1] * v[g + 1] + cs[g + 2] * v[g + 2] + cs[g + 3] * v[g + 3];
        took = g + 4;
      }
      const int left = end - e - took;
      if (took < 8 && left > 0 && left < 4 && took + left <= 8) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (i < left) ok = ok && !pend(v[took + i]);
        }
        if (ok) {
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            if (i < left) sum -= cs[took + i] * v[took + i];
          }
          took += left;
        }
      }
      e += took;
      if (took < 8) break;
    }
    if (e == end) {
      st(s.y + k, sum / d);
      done = true;
      continue;
    }
    if (e != before) {
      t_prog = wall_clock64();
      backoff = 1;
    } else if (wall_clock64() - t_prog > kMaxWait) {
      atomicExch(s.fail, 1);
      done = true;
    } else {
      for (int i = 0; i < backoff; ++i) __builtin_amdgcn_s_sleep(1);
      backoff = min(backoff * 2, s.poll_max);
    }
  }
}

// A: one thread per output, every output resident (the engine's sync-free).
__global__ __launch_bounds__(256) void all_resident_kernel(Sched s) {
  const int k = s.l0_end + blockIdx.x * blockDim.x + threadIdx.x;
  if (k < s.num_pos) output(s, k);
}

// B: persistent stride walk over T = gridDim.x * blockDim.x threads (only the
// frontier polls). Blocks with blockIdx % xcd != 0 leave at once (placement
// on one XCD per the round-robin dealing when xcd = 8).
__global__ __launch_bounds__(256) void stride_kernel(Sched s, int xcd) {
  if (blockIdx.x % xcd != 0) return;
  const int g = blockIdx.x / xcd;
  const int T = (gridDim.x / xcd) * blockDim.x;
  // Every lane of a wave holds positions of the same round: the for loop's
  // trip count is wave-uniform up to the last round, where output() keeps
  // the exit uniform itself.
  for (int k0 = s.l0_end + g * blockDim.x; k0 < s.num_pos; k0 += T) {
    const int k = k0 + threadIdx.x;
    if (__ballot(k < s.num_pos) == 0) break;
    if (k < s.num_pos) output(s, k);
  }
}

// A: over a position range [lo, hi) only (the wide levels).
__global__ __launch_bounds__(256) void range_resident_kernel(Sched s, int lo, int hi) {
  const int k = lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (k < hi) output(s, k);
}

// E: one 1024-thread workgroup computes positions [lo, hi) (hi - lo <= kSeg)
// with its own outputs in LDS: a value slot holds the pending mark until the
// output is final, so the slot is its own flag (LDS stores are seen by the
// other waves of the CU in order). Inputs below lo are final in y (earlier
// launches). Thread t takes lo + t, lo + t + 1024, ... and loads the record,
// the first 8 entries and their values below lo for its NEXT output while it
// waits on the current one (one output of look-ahead), so a hop costs an LDS
// round trip, not a global load.
constexpr int kSeg = 16384;
constexpr int kE = 1024;
struct Pre {
  int row, n, est;
  double d, in;
  int ps[8];
  double cs[8];
  double vs[8];  // value when the input is below lo, else 0 (read from LDS)
};

__device__ __forceinline__ void prefetch(const Sched& s, int k, int lo, Pre* p) {
  p->row = s.row[k];
  p->n = s.cnt[k];
  p->est = s.est[k];
  p->d = s.diag[k];
  p->in = s.rhs[p->row];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool in = i < p->n;
    p->ps[i] = in ? s.epos[p->est + i] : lo;
    p->cs[i] = in ? s.eval[p->est + i] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) p->vs[i] = (i < p->n && p->ps[i] < lo) ? s.y[p->ps[i]] : 0.0;
}

__device__ __forceinline__ double lds_ld(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The window of up to 8 entries starting at entry e of an output: positions,
// coefficients, values (the pending mark for this segment's not-yet-final
// outputs; inputs below lo are final in y).
__device__ __forceinline__ void load_window(const Sched& s, int est, int n, int e, int lo,
                                            int* ps, double* cs, double* v) {
  const double pm = __longlong_as_double(static_cast<long long>(kPending));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool in = e + i < n;
    ps[i] = in ? s.epos[est + e + i] : lo;
    cs[i] = in ? s.eval[est + e + i] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (e + i < n && ps[i] < lo) ? s.y[ps[i]] : (e + i < n ? pm : 0.0);
}

__global__ __launch_bounds__(kE) void chain_lds_kernel(Sched s, int lo, int hi) {
  __shared__ double vals[kSeg];
  const double pm = __longlong_as_double(static_cast<long long>(kPending));
  for (int i = threadIdx.x; i < hi - lo; i += kE) vals[i] = pm;
  __syncthreads();
  int k = lo + threadIdx.x;
  // Current output: record, window at entry e; next output: prefetched.
  bool active = k < hi;
  Pre cur{}, nxt{};
  if (active) prefetch(s, k, lo, &cur);
  if (active && k + kE < hi) prefetch(s, k + kE, lo, &nxt);
  int e = 0;
  double sum = cur.in;
  double v[8];
  int ps[8];
  double cs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ps[i] = cur.ps[i];
    cs[i] = cur.cs[i];
    v[i] = (i < cur.n && cur.ps[i] >= lo) ? pm : cur.vs[i];
  }
  uint64_t t_prog = wall_clock64();
  // One loop body polls, folds and stores, so a lane whose output another
  // lane of its wave waits for stores before the wave polls again; the loop
  // exit is wave-uniform so that no store can be sunk below it.
  while (__ballot(active) != 0) {
    if (!active) continue;
    const int n = cur.n;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (pend(v[i])) v[i] = lds_ld(vals + (ps[i] - lo));
    }
    // Window-relative fold: groups of 4 while 4 remain, then singles.
    int took = 0;
#pragma unroll
    for (int g = 0; g < 8; g += 4) {
      if (took != g || e + g + 3 >= n) continue;
      if (pend(v[g]) || pend(v[g + 1]) || pend(v[g + 2]) || pend(v[g + 3])) continue;
      sum -= cs[g] * v[g] + cs[g + 1] * v[g + 1] + cs[g + 2] * v[g + 2] + cs[g + 3] * v[g + 3];
      took = g + 4;
    }
    const int left = n - e - took;
    if (took < 8 && left > 0 && left < 4 && took + left <= 8) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (i < left) ok = ok && !pend(v[took + i]);
      }
      if (ok) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (i < left) sum -= cs[took + i] * v[took + i];
        }
        took += left;
      }
    }
    e += took;
    if (e == n) {
      const double out = sum / cur.d;
      __hip_atomic_store(vals + (k - lo), out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      s.y[k] = out;
      t_prog = wall_clock64();
      k += kE;
      if (k >= hi) {
        active = false;
      } else {
        cur = nxt;
        if (k + kE < hi) prefetch(s, k + kE, lo, &nxt);
        e = 0;
        sum = cur.in;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          ps[i] = cur.ps[i];
          cs[i] = cur.cs[i];
          v[i] = (i < cur.n && cur.ps[i] >= lo) ? pm : cur.vs[i];
        }
      }
    } else if (took == 8) {
      load_window(s, cur.est, n, e, lo, ps, cs, v);  // long output: the next 8
      t_prog = wall_clock64();
    } else if (took > 0) {
      // A partial window: shift the rest down (keeps the loaded values).
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int j = i + took;
        ps[i] = j < 8 ? ps[j] : lo;
        cs[i] = j < 8 ? cs[j] : 0.0;
        v[i] = j < 8 ? v[j] : 0.0;
      }
      if (e + (8 - took) < n) {
        // Refill the tail of the window from global memory.
        double rv[8];
        int rp[8];
        double rc[8];
        load_window(s, cur.est, n, e, lo, rp, rc, rv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (i >= 8 - took) {
            ps[i] = rp[i];
            cs[i] = rc[i];
            v[i] = rv[i];
          }
        }
      }
      t_prog = wall_clock64();
    } else {
      if (wall_clock64() - t_prog > kMaxWait) {
        atomicExch(s.fail, 1);
        active = false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

struct Host {
  int n = 0;
  int64_t nnz = 0;
  std::vector<int64_t> starts;
  std::vector<int> rows;
  std::vector<double> vals, diag, rhs;
};

Host Read(const char* path) {
  Host h;
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    std::perror(path);
    std::exit(2);
  }
  auto rd = [&](void* p, size_t b) {
    if (std::fread(p, 1, b, f) != b) {
      std::fprintf(stderr, "short read\n");
      std::exit(2);
    }
  };
  rd(&h.n, 4);
  rd(&h.nnz, 8);
  h.starts.resize(h.n + 1);
  h.rows.resize(h.nnz);
  h.vals.resize(h.nnz);
  h.diag.resize(h.n);
  h.rhs.resize(h.n);
  rd(h.starts.data(), 8 * (h.n + 1));
  rd(h.rows.data(), 4 * h.nnz);
  rd(h.vals.data(), 8 * h.nnz);
  rd(h.diag.data(), 8 * h.n);
  rd(h.rhs.data(), 8 * h.n);
  std::fclose(f);
  return h;
}

// Glop's loop (sparse.cc:899-955), all columns computed.
std::vector<double> Reference(const Host& h) {
  std::vector<double> x = h.rhs;
  for (int col = h.n - 1; col >= 0; --col) {
    double sum = x[col];
    int64_t i = h.starts[col + 1] - 1;
    const int64_t i_end = h.starts[col];
    for (; i >= i_end + 3; i -= 4) {
      sum -= h.vals[i] * x[h.rows[i]] + h.vals[i - 1] * x[h.rows[i - 1]] +
             h.vals[i - 2] * x[h.rows[i - 2]] + h.vals[i - 3] * x[h.rows[i - 3]];
    }
    if (i >= i_end) {
      sum -= h.vals[i] * x[h.rows[i]];
      if (i >= i_end + 1) {
        sum -= h.vals[i - 1] * x[h.rows[i - 1]];
        if (i >= i_end + 2) sum -= h.vals[i - 2] * x[h.rows[i - 2]];
      }
    }
    x[col] = sum / h.diag[col];
  }
  return x;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: tri_bench data.bin [reps]\n");
    return 2;
  }
  const int reps = argc > 2 ? std::atoi(argv[2]) : 200;
  Host h = Read(argv[1]);
  const int n = h.n;
  // Levels: output c reads rows r > c of its column.
  std::vector<int> level(n, 0);
  int levels = 1;
  for (int c = n - 1; c >= 0; --c) {
    int lv = -1;
    for (int64_t i = h.starts[c]; i < h.starts[c + 1]; ++i) lv = std::max(lv, level[h.rows[i]]);
    level[c] = lv + 1;
    levels = std::max(levels, lv + 2);
  }
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return level[a] < level[b]; });
  std::vector<int> pos_of(n);
  for (int p = 0; p < n; ++p) pos_of[order[p]] = p;
  int l0_end = 0;
  while (l0_end < n && level[order[l0_end]] == 0) ++l0_end;
  std::vector<int> cnt(n), est(n), epos, rowv(n);
  std::vector<double> eval, dg(n);
  for (int p = 0; p < n; ++p) {
    const int c = order[p];
    rowv[p] = c;
    dg[p] = h.diag[c];
    est[p] = static_cast<int>(epos.size());
    for (int64_t i = h.starts[c + 1] - 1; i >= h.starts[c]; --i) {
      epos.push_back(pos_of[h.rows[i]]);
      eval.push_back(h.vals[i]);
    }
    cnt[p] = static_cast<int>(epos.size()) - est[p];
  }
  std::printf("n %d nnz %lld levels %d level0 %d\n", n, static_cast<long long>(h.nnz), levels,
              l0_end);
  std::vector<double> ref = Reference(h);

  auto up = [](const void* src, size_t bytes) {
    void* d = nullptr;
    CHECK(hipMalloc(&d, std::max<size_t>(bytes, 8)));
    if (bytes) CHECK(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice));
    return d;
  };
  Sched s{};
  s.num_pos = n;
  s.l0_end = l0_end;
  s.row = static_cast<const int*>(up(rowv.data(), 4 * n));
  s.cnt = static_cast<const int*>(up(cnt.data(), 4 * n));
  s.est = static_cast<const int*>(up(est.data(), 4 * n));
  s.epos = static_cast<const int*>(up(epos.data(), 4 * epos.size()));
  s.eval = static_cast<const double*>(up(eval.data(), 8 * eval.size()));
  s.diag = static_cast<const double*>(up(dg.data(), 8 * n));
  s.rhs = static_cast<const double*>(up(h.rhs.data(), 8 * n));
  CHECK(hipMalloc(&s.y, 8 * n));
  CHECK(hipMalloc(&s.fail, 4));
  CHECK(hipMemset(s.fail, 0, 4));
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int init_blocks = std::min(1024, (n + 255) / 256);

  auto check = [&](const char* name) {
    std::vector<double> y(n);
    CHECK(hipMemcpy(y.data(), s.y, 8 * n, hipMemcpyDeviceToHost));
    int fail = 0;
    CHECK(hipMemcpy(&fail, s.fail, 4, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int p = 0; p < n; ++p) {
      if (std::memcmp(&y[p], &ref[rowv[p]], 8) != 0) ++bad;
    }
    if (bad || fail) std::printf("  %s: %lld MISMATCHES, fail=%d\n", name, (long long)bad, fail);
    return bad == 0 && fail == 0;
  };
  auto time_it = [&](const char* name, auto launch) {
    // warm-up + check
    init_kernel<<<init_blocks, 256, 0, st>>>(s);
    launch();
    CHECK(hipStreamSynchronize(st));
    const bool ok = check(name);
    if (!ok && std::strcmp(name, "init only") != 0) {
      std::printf("%-40s WRONG (not timed)\n", name);
      CHECK(hipMemset(s.fail, 0, 4));
      return;
    }
    CHECK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) {
      init_kernel<<<init_blocks, 256, 0, st>>>(s);
      launch();
    }
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("%-40s %8.1f us per solve (init included) %s\n", name, 1000.0 * ms / reps,
                ok ? "exact" : "WRONG");
    std::fflush(stdout);
  };
  time_it("init only", [&] {});
  for (int pm : {1, 4, 16, 64}) {
    s.poll_max = pm;
    char name[64];
    std::snprintf(name, sizeof name, "A all-resident poll_max %d", pm);
    time_it(name, [&] {
      all_resident_kernel<<<(n - l0_end + 255) / 256, 256, 0, st>>>(s);
    });
  }
  s.poll_max = 4;
  for (int xcd : {1, 8}) {
    for (int groups : {32, 64, 128, 256, 512}) {
      if (xcd == 8 && groups > 128) continue;
      char name[64];
      std::snprintf(name, sizeof name, "B stride groups %d xcd %d", groups, xcd);
      time_it(name, [&] { stride_kernel<<<groups * xcd, 256, 0, st>>>(s, xcd); });
    }
  }
  // Hybrid: the wide levels [1, K] on the whole chip (A over their range),
  // then the narrow ones in LDS chain segments of at most kSeg positions.
  std::vector<int> lstart(levels + 1, 0);
  for (int p = 0; p < n; ++p) lstart[level[order[p]] + 1] = p + 1;
  for (int l = 1; l <= levels; ++l) lstart[l] = std::max(lstart[l], lstart[l - 1]);
  for (int K : {0, 3, 5, 7, 9}) {
    const int wide_hi = lstart[K + 1];
    std::vector<int> segs;  // chain segment boundaries from wide_hi, cut at level ends
    int a = std::max(wide_hi, l0_end);
    while (a < n) {
      int b = a;
      for (int l = 1; l <= levels; ++l) {
        if (lstart[l] > a && lstart[l] - a <= kSeg) b = lstart[l];
      }
      if (b == a) b = std::min(n, a + kSeg);  // a level wider than a segment
      segs.push_back(a);
      segs.push_back(b);
      a = b;
    }
    char name[96];
    std::snprintf(name, sizeof name, "H wide levels 1..%d + %zu LDS chain segs", K, segs.size() / 2);
    time_it(name, [&] {
      if (wide_hi > l0_end) {
        range_resident_kernel<<<(wide_hi - l0_end + 255) / 256, 256, 0, st>>>(s, l0_end, wide_hi);
      }
      for (size_t i = 0; i < segs.size(); i += 2) {
        chain_lds_kernel<<<1, kE, 0, st>>>(s, segs[i], segs[i + 1]);
      }
    });
  }
  return 0;
}
