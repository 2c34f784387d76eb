// Dense triangular solve of the basis factorization on one CU.
//
// Replaces TriangularMatrix::TransposeLowerSolve (lp_data/sparse.cc:899-955),
// which Glop runs for the U part of an FTRAN whenever the result is too
// dense for the hypersparse path (lu_factorization.cc:314-331). In that
// row-oriented ("gather") form every output
//
//   x[c] = (x[c] - sum over the entries (r, v) of column c of v * x[r]) / diag[c]
//
// reads only rows r > c, and the subtraction order of one output is fixed by
// its own entries: groups of four products, summed left to right, subtracted
// one group at a time, then the 1-3 remaining products one by one, entries
// taken from the end of the column. A thread that computes x[c] from its
// entries in that order gets Glop's bits, whatever the order in which the
// outputs are computed, as long as every x[r] it reads is final.
//
// Schedule: the host lists the outputs by dependency level (level 0: no
// entries), entries in evaluation order (engine/device_solve.hip). One
// 1024-thread workgroup (one CU, so every hand-off stays inside one L1/L2)
// computes the levels in turn with a barrier between them. x values are read
// at agent scope (L2), never from a possibly stale L1 line.

#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace milp_kernels {

__device__ __forceinline__ double load_final(const double* x, int r) {
  return __hip_atomic_load(x + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Glop's evaluation of one output from its entries e0, e1, ... (evaluation
// order): groups of four products summed left to right, each group
// subtracted, then the 1-3 remaining products one by one.
__device__ __forceinline__ double group_sum(const TriSolveArgs& a, const double* x, int e) {
  return a.entry_coef[e] * load_final(x, a.entry_row[e]) +
         a.entry_coef[e + 1] * load_final(x, a.entry_row[e + 1]) +
         a.entry_coef[e + 2] * load_final(x, a.entry_row[e + 2]) +
         a.entry_coef[e + 3] * load_final(x, a.entry_row[e + 3]);
}

__device__ __forceinline__ double tail_subtract(const TriSolveArgs& a, const double* x,
                                                double sum, int e, int end) {
  if (e < end) {
    sum -= a.entry_coef[e] * load_final(x, a.entry_row[e]);
    if (e + 1 < end) {
      sum -= a.entry_coef[e + 1] * load_final(x, a.entry_row[e + 1]);
      if (e + 2 < end) sum -= a.entry_coef[e + 2] * load_final(x, a.entry_row[e + 2]);
    }
  }
  return sum;
}

// Entries of one output, in evaluation order, by batches of 8 (2 groups):
// the 8 x loads of a batch are independent and go out together.
__device__ __forceinline__ double subtract_entries(const TriSolveArgs& a, const double* x,
                                                   double sum, int e, int end) {
  for (; e + 7 < end; e += 8) {
    double p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = a.entry_coef[e + i] * load_final(x, a.entry_row[e + i]);
    sum -= p[0] + p[1] + p[2] + p[3];
    sum -= p[4] + p[5] + p[6] + p[7];
  }
  for (; e + 3 < end; e += 4) sum -= group_sum(a, x, e);
  return tail_subtract(a, x, sum, e, end);
}

// One output c from its entries (evaluation order) and the final x.
__device__ __forceinline__ double solve_output(const TriSolveArgs& a, const double* x, int k,
                                               int c, int beg, int end) {
  double sum = x[c];
  const int n = end - beg;
  if (n <= 4) {
    // Short rows (almost all of them): the 4 loads go out together.
    int r[4];
    double v[4], xr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      r[i] = i < n ? a.entry_row[beg + i] : c;
      v[i] = i < n ? a.entry_coef[beg + i] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) xr[i] = i < n ? load_final(x, r[i]) : 0.0;
    if (n == 4) {
      sum -= v[0] * xr[0] + v[1] * xr[1] + v[2] * xr[2] + v[3] * xr[3];
    } else {
      if (n > 0) sum -= v[0] * xr[0];
      if (n > 1) sum -= v[1] * xr[1];
      if (n > 2) sum -= v[2] * xr[2];
    }
  } else {
    sum = subtract_entries(a, x, sum, beg, end);
  }
  return a.diag != nullptr ? sum / a.diag[k] : sum;
}

// Level-synchronous: the outputs of one level depend only on earlier
// levels, so the workgroup computes a level, then meets at a barrier
// (every store has completed: explicit s_waitcnt vmcnt(0), s_barrier), then the
// next. Inside a level each thread takes up to kTriUnroll outputs at once so
// that their loads overlap.
__global__ __launch_bounds__(kTriThreads) void tri_transpose_lower_kernel(TriSolveArgs a) {
  double* x = a.x;
  const int tid = threadIdx.x;
  if (a.clock != nullptr && tid == 0) a.clock[0] = wall_clock64();
  for (int l = 0; l < a.num_levels; ++l) {
    const int lb = a.level_start[l];
    const int le = a.level_start[l + 1];
    for (int base = lb; base < le; base += kTriUnroll * kTriThreads) {
      int kk[kTriUnroll], cc[kTriUnroll], bb[kTriUnroll], ee[kTriUnroll];
#pragma unroll
      for (int j = 0; j < kTriUnroll; ++j) {
        kk[j] = base + j * kTriThreads + tid;
        cc[j] = kk[j] < le ? a.work_row[kk[j]] : a.top + 1;
        bb[j] = kk[j] < le ? a.work_begin[kk[j]] : 0;
        ee[j] = kk[j] < le ? a.work_begin[kk[j] + 1] : 0;
      }
      double out[kTriUnroll];
#pragma unroll
      for (int j = 0; j < kTriUnroll; ++j) {
        if (cc[j] <= a.top) out[j] = solve_output(a, x, kk[j], cc[j], bb[j], ee[j]);
      }
#pragma unroll
      for (int j = 0; j < kTriUnroll; ++j) {
        if (cc[j] <= a.top) x[cc[j]] = out[j];
      }
    }
    // The level's stores must have reached L2 before any wave reads them:
    // __syncthreads alone does not wait for them here (workgroup scope).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (a.clock != nullptr && tid == 0) a.clock[l + 1] = wall_clock64();
  }
}

}  // namespace milp_kernels

namespace milp_launch {

hipError_t tri_transpose_lower(const milp_kernels::TriSolveArgs& args, hipStream_t s) {
  if (args.num_work <= 0) return hipSuccess;
  milp_kernels::tri_transpose_lower_kernel<<<1, milp_kernels::kTriThreads, 0, s>>>(args);
  return hipGetLastError();
}

}  // namespace milp_launch
