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

__global__ __launch_bounds__(256) void dense_tail_copy_pre_kernel(DenseTailArgs a) {
  const int T = a.n - a.t;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < T; i += gridDim.x * blockDim.x) {
    a.host_out[i] = a.pre[i];
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

// The tail's own triangle on one workgroup, by blocks of 64 columns. Each
// tail column keeps a cursor (the next entry of its chain) and its running
// sum in LDS. Block k: (A) every later column folds its whole groups whose
// rows are all final -- below the block's first column (rows ascend within a
// column, so a group's last row decides) -- one lane per column, in the
// column's own order; (B) the block's 64 columns finish their chains with one
// wave, lane j = column j of the block: the entries left are staged in LDS,
// a group is folded when its inputs (earlier columns of the block, in LDS)
// are final, then the 1-3 remaining entries one by one, the division, and the
// value is published in LDS for the next lanes and the next blocks. The
// lane loop's exit is wave-uniform, so a lane publishes inside the loop body.
constexpr int kTailBlock = 64;
constexpr int kStageEntries = 72;  // per block column: < 64 rows of the block + a group

__global__ __launch_bounds__(kTailThreads) void dense_tail_walk_kernel(DenseTailArgs a) {
  __shared__ double xt[kTailMaxCols];
  __shared__ double run[kTailMaxCols];    // running sums
  __shared__ int cur[kTailMaxCols];       // chain cursors (relative entry index)
  __shared__ int st_row[kTailBlock * kStageEntries];
  __shared__ double st_val[kTailBlock * kStageEntries];
  __shared__ double st_diag[kTailBlock];
  const int T = a.n - a.t;
  const int tid = threadIdx.x;
  const double pend = __longlong_as_double(static_cast<long long>(kTailPending));
  for (int c = tid; c < T; c += kTailThreads) {
    xt[c] = pend;
    run[c] = a.pre[c];
    cur[c] = static_cast<int>(a.split[c]);
  }
  __syncthreads();
  // The value of row r (r < t: final in x; a tail row below the current
  // block: final in LDS).
  auto value = [&](int r) -> double { return r < a.t ? a.x[r] : xt[r - a.t]; };
  for (int b0 = 0; b0 < T; b0 += kTailBlock) {
    const int b1 = min(T, b0 + kTailBlock);
    const int limit = a.t + b0;  // rows below are final
    // (A) every column of this block and later: whole groups below `limit`.
    for (int c = b0 + tid; c < T; c += kTailThreads) {
      int i = cur[c];
      const int end = static_cast<int>(a.starts[c + 1]);
      double sum = run[c];
      while (i + 3 < end) {
        const int r0 = a.rows[i], r1 = a.rows[i + 1], r2 = a.rows[i + 2], r3 = a.rows[i + 3];
        if (max(max(r0, r1), max(r2, r3)) >= limit) break;
        sum -= a.vals[i] * value(r0) + a.vals[i + 1] * value(r1) + a.vals[i + 2] * value(r2) +
               a.vals[i + 3] * value(r3);
        i += 4;
      }
      cur[c] = i;
      run[c] = sum;
    }
    __syncthreads();
    // Stage the entries the block's columns have left (all below their own
    // column: at most the block's rows plus one straddling group).
    for (int k = tid; k < (b1 - b0) * kStageEntries; k += kTailThreads) {
      const int c = b0 + k / kStageEntries;
      const int q = k % kStageEntries;
      const int i = cur[c] + q;
      const bool in = i < static_cast<int>(a.starts[c + 1]);
      st_row[k] = in ? a.rows[i] : -1;
      st_val[k] = in ? a.vals[i] : 0.0;
    }
    for (int c = b0 + tid; c < b1; c += kTailThreads) {
      st_diag[c - b0] = a.diag != nullptr ? a.diag[c] : 1.0;
    }
    __syncthreads();
    // (B) the block's own triangle on wave 0.
    if (tid < 64) {
      const int c = b0 + tid;
      bool active = c < b1;
      const int left0 = active ? static_cast<int>(a.starts[c + 1]) - cur[c] : 0;
      int e = 0;  // staged entries consumed
      double sum = active ? run[c] : 0.0;
      // Entry e of the chain left: staged (the first kStageEntries), else
      // in global memory (a column whose rows are not ascending can hold
      // more entries behind a block row).
      const int base = active ? cur[c] : 0;
      auto row_at = [&](int e) {
        return e < kStageEntries ? st_row[tid * kStageEntries + e] : a.rows[base + e];
      };
      auto val_at = [&](int e) {
        return e < kStageEntries ? st_val[tid * kStageEntries + e] : a.vals[base + e];
      };
      uint64_t t_progress = wall_clock64();
      while (__ballot(active) != 0) {
        if (!active) continue;
        bool moved = false;
        // Whole groups while four entries remain and their inputs are final.
        while (left0 - e >= 4) {
          const double v0 = value(row_at(e)), v1 = value(row_at(e + 1));
          const double v2 = value(row_at(e + 2)), v3 = value(row_at(e + 3));
          if (tail_pending(v0) || tail_pending(v1) || tail_pending(v2) || tail_pending(v3)) {
            break;
          }
          sum -= val_at(e) * v0 + val_at(e + 1) * v1 + val_at(e + 2) * v2 + val_at(e + 3) * v3;
          e += 4;
          moved = true;
        }
        if (left0 - e < 4 && e < left0) {
          const int left = left0 - e;
          bool ready = true;
          for (int q = 0; q < left; ++q) ready = ready && !tail_pending(value(row_at(e + q)));
          if (ready) {
            for (int q = 0; q < left; ++q) sum -= val_at(e + q) * value(row_at(e + q));
            e = left0;
            moved = true;
          }
        }
        if (e == left0) {
          const double out = a.diag != nullptr ? sum / st_diag[tid] : sum;
          a.x[a.t + c] = out;
          __hip_atomic_store(xt + c, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          active = false;
        } else if (moved) {
          t_progress = wall_clock64();
        } else if (wall_clock64() - t_progress > kTailMaxWaitTicks) {
          if (a.fail != nullptr) {
            __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          active = false;
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace milp_kernels

namespace milp_launch {

hipError_t dense_tail_prefix(const milp_kernels::DenseTailArgs& a, hipStream_t s) {
  const int T = a.n - a.t;
  if (T <= 0) return hipErrorInvalidValue;
  const int blocks = std::max(1, std::min(1024, (a.n + 255) / 256));
  milp_kernels::dense_tail_copy_in_kernel<<<blocks, 256, 0, s>>>(a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  milp_kernels::dense_tail_prefix_kernel<<<T, milp_kernels::kPrefixThreads, 0, s>>>(a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // The prefixes out (to host_out, T values).
  milp_kernels::dense_tail_copy_pre_kernel<<<std::max(1, std::min(256, (T + 255) / 256)), 256, 0,
                                             s>>>(a);
  return hipGetLastError();
}

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
