// Dense tail of the forward U^T solve (BTRAN's TriangularMatrix::
// TransposeUpperSolve, sparse.cc:848-897) on the device.
//
// The host loop computes, column by column from the first non-identity one,
//
//   sum = x[c]; for each group of four entries (i, i+1, i+2, i+3) of column c
//   from its start while four remain: sum -= v_i x[r_i] + v_{i+1} x[r_{i+1}]
//   + v_{i+2} x[r_{i+2}] + v_{i+3} x[r_{i+3}]; then the 1-3 remaining entries
//   one subtraction each; x[c] = sum / diag[c] (or sum with a unit diagonal).
//
// Every column reads rows < c only. When the last T columns (the tail, from
// t) hold most of the entries -- config 2's dense kernel: ~1 500 columns that
// each read ~8 500 slack rows before the kernel's own rows -- the rows < t
// are final before the tail starts (the host computes columns [fni, t)
// first). So each tail column's leading groups that read rows < t only can
// be folded for all tail columns at once (dense_tail_prefix_kernel: one
// workgroup per column computes the group sums in parallel and folds them in
// order: the same operations in the same order as the loop); what is left of
// each chain reads the tail's own outputs, and dense_tail_walk_kernel runs
// it on one workgroup with the tail's values in LDS: lane j owns columns
// t + j, t + j + 1024, ..., folds a group as soon as its four inputs are
// final, and publishes its output through LDS -- a hand-off is an LDS round
// trip, not a launch or a trip through L2.
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace milp_kernels {

namespace {
constexpr unsigned long long kTailPending = 0x7ff0deadbeef0002ull;  // a NaN no arithmetic makes
constexpr uint64_t kTailMaxWaitTicks = 20000000;                    // 0.2 s at 100 MHz

__device__ __forceinline__ bool tail_pending(double v) {
  return static_cast<unsigned long long>(__double_as_longlong(v)) == kTailPending;
}
}  // namespace

__global__ __launch_bounds__(256) void dense_tail_copy_in_kernel(DenseTailArgs a) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
    a.x[i] = a.host_x[i];
  }
}

__global__ __launch_bounds__(256) void dense_tail_copy_out_kernel(DenseTailArgs a) {
  const int T = a.n - a.t;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < T; i += gridDim.x * blockDim.x) {
    a.host_out[i] = a.x[a.t + i];
  }
}

// One workgroup per tail column: the group sums of its leading groups (each
// the loop's own expression, products summed left to right), staged in LDS
// by chunks, then folded into the running sum in order by one lane.
constexpr int kPrefixThreads = 256;
constexpr int kPrefixChunk = 4096;  // group sums per LDS chunk (32 KB)
__global__ __launch_bounds__(kPrefixThreads) void dense_tail_prefix_kernel(DenseTailArgs a) {
  __shared__ double gs[kPrefixChunk];
  const int j = blockIdx.x;
  const int64_t s0 = a.starts[j];
  const int64_t groups = (a.split[j] - s0) / 4;
  double sum = a.x[a.t + j];
  for (int64_t g0 = 0; g0 < groups; g0 += kPrefixChunk) {
    const int cnt = static_cast<int>(min<int64_t>(kPrefixChunk, groups - g0));
    for (int k = threadIdx.x; k < cnt; k += kPrefixThreads) {
      const int64_t i = s0 + 4 * (g0 + k);
      gs[k] = a.vals[i] * a.x[a.rows[i]] + a.vals[i + 1] * a.x[a.rows[i + 1]] +
              a.vals[i + 2] * a.x[a.rows[i + 2]] + a.vals[i + 3] * a.x[a.rows[i + 3]];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int k = 0; k < cnt; ++k) sum -= gs[k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) a.pre[j] = sum;
}

// The tail's dependency walk on one workgroup. A lane keeps a window of its
// column's next 16 entries in registers (rows, values, and the inputs below
// t, all loaded together), folds the groups whose four inputs are final
// (tail rows: LDS, pending until published), then the 1-3 remaining entries
// one by one, divides and publishes. The loop exit is wave-uniform, so a
// lane's stores stay inside the loop body (a reader in the same wave sees
// them on its next pass).
constexpr int kWin = 16;
__global__ __launch_bounds__(kTailThreads) void dense_tail_walk_kernel(DenseTailArgs a) {
  __shared__ double xt[kTailMaxCols];
  const int T = a.n - a.t;
  const double pend = __longlong_as_double(static_cast<long long>(kTailPending));
  for (int k = threadIdx.x; k < T; k += kTailThreads) xt[k] = pend;
  __syncthreads();
  int j = threadIdx.x;
  bool active = j < T;
  int64_t i = 0, end = 0;
  double sum = 0.0;
  int64_t wb = 0;  // entry index of window slot 0
  int wr[kWin];
  double wc[kWin], wv[kWin];
  auto load_window = [&]() {
    wb = i;
#pragma unroll
    for (int q = 0; q < kWin; ++q) {
      const bool in = wb + q < end;
      wr[q] = in ? a.rows[wb + q] : a.t;
      wc[q] = in ? a.vals[wb + q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kWin; ++q) wv[q] = (wb + q < end && wr[q] < a.t) ? a.x[wr[q]] : pend;
  };
  auto start_column = [&]() {
    i = a.split[j];
    end = a.starts[j + 1];
    sum = a.pre[j];
    load_window();
  };
  if (active) start_column();
  uint64_t t_progress = wall_clock64();
  while (__ballot(active) != 0) {
    if (!active) continue;
    // Refresh the pending tail inputs of the window from LDS.
#pragma unroll
    for (int q = 0; q < kWin; ++q) {
      if (wb + q < end && tail_pending(wv[q]) && wr[q] >= a.t) {
        wv[q] = __hip_atomic_load(xt + (wr[q] - a.t), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    bool moved = false;
    // Groups of four in order while four entries remain and all are final.
#pragma unroll
    for (int g = 0; g < kWin; g += 4) {
      const int o = static_cast<int>(i - wb);
      if (o != g || end - i < 4) continue;
      if (tail_pending(wv[g]) || tail_pending(wv[g + 1]) || tail_pending(wv[g + 2]) ||
          tail_pending(wv[g + 3])) {
        continue;
      }
      sum -= wc[g] * wv[g] + wc[g + 1] * wv[g + 1] + wc[g + 2] * wv[g + 2] + wc[g + 3] * wv[g + 3];
      i += 4;
      moved = true;
    }
    // The 1-3 remaining entries (inside the window: the window starts on a
    // group boundary and holds whole groups), one subtraction each.
    const int64_t left = end - i;
    if (left > 0 && left < 4 && i - wb + left <= kWin) {
      // (Static window indices: a register array indexed at run time would
      // live in scratch.)
      const int o = static_cast<int>(i - wb);
      const int e = o + static_cast<int>(left);
      bool ready = true;
#pragma unroll
      for (int q = 0; q < kWin; ++q) {
        if (q >= o && q < e) ready = ready && !tail_pending(wv[q]);
      }
      if (ready) {
#pragma unroll
        for (int q = 0; q < kWin; ++q) {
          if (q >= o && q < e) sum -= wc[q] * wv[q];
        }
        i = end;
        moved = true;
      }
    }
    if (i == end) {
      const double out = a.diag != nullptr ? sum / a.diag[j] : sum;
      a.x[a.t + j] = out;
      __hip_atomic_store(xt + j, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      j += kTailThreads;
      if (j >= T) {
        active = false;
      } else {
        start_column();
      }
      t_progress = wall_clock64();
    } else if (moved) {
      if (i - wb >= kWin) load_window();  // the window is used up: the next 16
      t_progress = wall_clock64();
    } else if (wall_clock64() - t_progress > kTailMaxWaitTicks) {
      if (a.fail != nullptr) {
        __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      active = false;
    } else {
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

}  // namespace milp_kernels

namespace milp_launch {

hipError_t dense_tail_upper_solve(const milp_kernels::DenseTailArgs& a, hipStream_t s) {
  const int T = a.n - a.t;
  if (T <= 0 || T > milp_kernels::kTailMaxCols) return hipErrorInvalidValue;
  const int blocks = std::max(1, std::min(1024, (a.n + 255) / 256));
  milp_kernels::dense_tail_copy_in_kernel<<<blocks, 256, 0, s>>>(a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  milp_kernels::dense_tail_prefix_kernel<<<T, milp_kernels::kPrefixThreads, 0, s>>>(a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  milp_kernels::dense_tail_walk_kernel<<<1, milp_kernels::kTailThreads, 0, s>>>(a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  milp_kernels::dense_tail_copy_out_kernel<<<std::max(1, std::min(256, (T + 255) / 256)), 256, 0,
                                             s>>>(a);
  return hipGetLastError();
}

}  // namespace milp_launch
