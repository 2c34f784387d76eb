// Dense triangular solve of the basis factorization.
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
// taken from the end of the column. Computing x[c] from its entries in that
// order gives Glop's bits, whatever the order in which the outputs are
// computed, as long as every x[r] read is final.
//
// Layout (engine/device_solve.hip builds it once per factorization): the
// outputs are listed by dependency level (level 0: no entries) and the
// values live in that order, y[k] = x[row(k)], so that an output's own read
// and write are coalesced and its entries are positions into y. Per
// position, structure-of-arrays records: row, entry count, up to 4 entries
// (positions and values) inline, the diagonal; longer outputs point into
// overflow arrays. A solve permutes x into y, computes the levels, permutes
// back.
//
// Schedule: the level sequence is cut into segments. A wide level (thousands
// of independent outputs, e.g. the diagonal-only level 0) is one launch over
// the whole chip. A run of narrow levels is one launch of one 1024-thread
// workgroup (one CU: every hand-off stays inside one L1/L2) that computes the
// levels in turn with a barrier between them; the next level's records are
// loaded while the current one computes. Values written in the same launch
// are read at agent scope (L2), never from a possibly stale L1 line.
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace milp_kernels {

__device__ __forceinline__ double load_final(const double* y, int k) {
  return __hip_atomic_load(y + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The structure of one listed output.
struct TriRec {
  int row;  // top + 1 when the position is empty
  int n;
  int4 e;   // entry positions (n <= 4); e.x = overflow start when n > 4
  double v[4];
  double d;
};

__device__ __forceinline__ void tri_load(const TriSolveArgs& a, int k, int le, int top,
                                         TriRec* r) {
  const bool in = k < le;
  const int kk = in ? k : 0;  // a valid address for an empty slot
  r->row = in ? a.rec_row[kk] : top + 1;
  r->n = a.rec_n[kk];
  r->e = a.rec_entry[kk];
  const double2 v01 = a.rec_value[2 * kk];
  const double2 v23 = a.rec_value[2 * kk + 1];
  r->v[0] = v01.x;
  r->v[1] = v01.y;
  r->v[2] = v23.x;
  r->v[3] = v23.y;
  r->d = a.diag != nullptr ? a.diag[kk] : 1.0;
}

// Entries of a long output (overflow arrays), in evaluation order, by batches
// of 8 whose loads go out together.
__device__ __forceinline__ double subtract_overflow(const TriSolveArgs& a, const double* y,
                                                   double sum, int e, int end) {
  for (; e + 7 < end; e += 8) {
    double p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = a.ovf_value[e + i] * load_final(y, a.ovf_pos[e + i]);
    sum -= p[0] + p[1] + p[2] + p[3];
    sum -= p[4] + p[5] + p[6] + p[7];
  }
  for (; e + 3 < end; e += 4) {
    sum -= a.ovf_value[e] * load_final(y, a.ovf_pos[e]) +
           a.ovf_value[e + 1] * load_final(y, a.ovf_pos[e + 1]) +
           a.ovf_value[e + 2] * load_final(y, a.ovf_pos[e + 2]) +
           a.ovf_value[e + 3] * load_final(y, a.ovf_pos[e + 3]);
  }
  if (e < end) {
    sum -= a.ovf_value[e] * load_final(y, a.ovf_pos[e]);
    if (e + 1 < end) {
      sum -= a.ovf_value[e + 1] * load_final(y, a.ovf_pos[e + 1]);
      if (e + 2 < end) sum -= a.ovf_value[e + 2] * load_final(y, a.ovf_pos[e + 2]);
    }
  }
  return sum;
}

// LowerSolve's order (sparse.cc:793-812 seen from one output): one
// subtraction per entry in ascending column order, an entry whose value is
// zero contributes nothing (the host skips that column). Loads by batches of 8.
__device__ __forceinline__ double subtract_sequential(const TriSolveArgs& a, const double* y,
                                                     double sum, int e, int end) {
  for (; e < end; e += 8) {
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = e + i < end ? load_final(y, a.ovf_pos[e + i]) : 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (e + i < end && v[i] != 0.0) sum -= v[i] * a.ovf_value[e + i];
    }
  }
  return sum;
}

// A scatter loop's own column (sparse.cc:792-846): a zero is skipped, so it
// keeps its bits and is not divided; anything else is divided by the
// diagonal (nothing to do for a unit one). Consumers skip the columns whose
// final value is zero, as the loop does (bit-identical except where value /
// diagonal underflows to zero, which the loop would still scatter).
__device__ __forceinline__ double tri_sequential_divide(const TriSolveArgs& a, double sum,
                                                        double d) {
  return (a.diag != nullptr && sum != 0.0) ? sum / d : sum;
}

// The output's value from its input `sum` and its entries (final values).
__device__ __forceinline__ double tri_apply(const TriSolveArgs& a, const double* y, double sum,
                                            const TriRec& r) {
  if (a.sequential) {
    if (r.n <= 4) {
      const int n = r.n;
      const double y0 = n > 0 ? load_final(y, r.e.x) : 0.0;
      const double y1 = n > 1 ? load_final(y, r.e.y) : 0.0;
      const double y2 = n > 2 ? load_final(y, r.e.z) : 0.0;
      const double y3 = n > 3 ? load_final(y, r.e.w) : 0.0;
      if (y0 != 0.0) sum -= y0 * r.v[0];
      if (y1 != 0.0) sum -= y1 * r.v[1];
      if (y2 != 0.0) sum -= y2 * r.v[2];
      if (y3 != 0.0) sum -= y3 * r.v[3];
    } else {
      sum = subtract_sequential(a, y, sum, r.e.x, r.e.x + r.n);
    }
    return tri_sequential_divide(a, sum, r.d);
  }
  if (r.n <= 4) {
    const int n = r.n;
    const double y0 = n > 0 ? load_final(y, r.e.x) : 0.0;
    const double y1 = n > 1 ? load_final(y, r.e.y) : 0.0;
    const double y2 = n > 2 ? load_final(y, r.e.z) : 0.0;
    const double y3 = n > 3 ? load_final(y, r.e.w) : 0.0;
    if (n == 4) {
      sum -= r.v[0] * y0 + r.v[1] * y1 + r.v[2] * y2 + r.v[3] * y3;
    } else {
      if (n > 0) sum -= r.v[0] * y0;
      if (n > 1) sum -= r.v[1] * y1;
      if (n > 2) sum -= r.v[2] * y2;
    }
  } else {
    sum = subtract_overflow(a, y, sum, r.e.x, r.e.x + r.n);
  }
  return a.diag != nullptr ? sum / r.d : sum;
}

__device__ __forceinline__ void tri_compute(const TriSolveArgs& a, double* y, int k, int top,
                                            const TriRec& r) {
  if (r.row > top) return;
  y[k] = tri_apply(a, y, y[k], r);
}

// Zero-copy staging in and out of device-visible host memory (coalesced
// PCIe reads and writes, inside the captured plan: no copy engine calls).
__global__ __launch_bounds__(256) void tri_copy_in_kernel(TriSolveArgs a0) {
  const TriSolveArgs a = TriRhs(a0, blockIdx.y);
  const int n = a.num_rows - a.first_col;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    a.x[a.first_col + i] = a.host_x[a.first_col + i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *a.top = *reinterpret_cast<const int*>(a.host_x + a.num_rows);
  }
}

__global__ __launch_bounds__(256) void tri_copy_out_kernel(TriSolveArgs a0) {
  const TriSolveArgs a = TriRhs(a0, blockIdx.y);
  const int end = *a.top + 1;
  for (int i = a.first_col + blockIdx.x * blockDim.x + threadIdx.x; i < end;
       i += gridDim.x * blockDim.x) {
    a.host_x[i] = a.x[i];
  }
}

// y[k] = x[row(k)] for every position (listed or not).
__global__ __launch_bounds__(256) void tri_gather_kernel(TriSolveArgs a) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < a.num_pos;
       k += gridDim.x * blockDim.x) {
    a.y[k] = a.x[a.pos_row[k]];
  }
}

// The gather with level 0 fused: y[k] = x[row(k)], divided by the diagonal
// for the listed outputs of level 0 (no entries: tri_apply's sum is the input
// itself, then the division).
__global__ __launch_bounds__(256) void tri_gather_level0_kernel(TriSolveArgs a) {
  const int top = *a.top;
  const int l0_end = a.level_start[1];
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < a.num_pos;
       k += gridDim.x * blockDim.x) {
    double v = a.x[a.pos_row[k]];
    if (k < l0_end && a.rec_row[k] <= top) {  // padding rows: INT32_MAX
      v = a.sequential ? tri_sequential_divide(a, v, a.diag[k]) : v / a.diag[k];
    }
    a.y[k] = v;
  }
}

// x[row(k)] = y[k] for the computed outputs.
__global__ __launch_bounds__(256) void tri_scatter_kernel(TriSolveArgs a) {
  const int top = *a.top;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < a.num_work;
       k += gridDim.x * blockDim.x) {
    const int row = a.rec_row[k];
    if (row <= top) a.x[row] = a.y[k];
  }
}

// One wide level over the whole chip; kernel boundaries order it with the
// other levels.
__global__ __launch_bounds__(256) void tri_level_grid_kernel(TriSolveArgs a, int level) {
  const int top = *a.top;
  const int lb = a.level_start[level];
  const int le = a.level_start[level + 1];
  for (int k = lb + blockIdx.x * blockDim.x + threadIdx.x; k < le;
       k += gridDim.x * blockDim.x) {
    TriRec r;
    tri_load(a, k, le, top, &r);
    tri_compute(a, a.y, k, top, r);
  }
}

// The value of position p inside a single-CU run: outputs of this run
// ([seg_lo, seg_hi)) from LDS; every other position -- outputs of earlier
// launches, and the read-only rows listed after all levels -- from global
// memory, where an earlier launch left it final (plain loads are safe across
// a kernel boundary).
struct TriRunValues {
  const double* y;
  const double* lds;
  int seg_lo, seg_hi;
  __device__ __forceinline__ double operator()(int p) const {
    return (p >= seg_lo && p < seg_hi) ? lds[p - seg_lo] : y[p];
  }
};

// tri_apply with the values read through `val` (same terms, same order).
template <typename Val>
__device__ __forceinline__ double tri_apply_vals(const TriSolveArgs& a, const Val& val, double sum,
                                                 const TriRec& r) {
  if (a.sequential) {
    if (r.n <= 4) {
      const int n = r.n;
      const double y0 = n > 0 ? val(r.e.x) : 0.0;
      const double y1 = n > 1 ? val(r.e.y) : 0.0;
      const double y2 = n > 2 ? val(r.e.z) : 0.0;
      const double y3 = n > 3 ? val(r.e.w) : 0.0;
      if (y0 != 0.0) sum -= y0 * r.v[0];
      if (y1 != 0.0) sum -= y1 * r.v[1];
      if (y2 != 0.0) sum -= y2 * r.v[2];
      if (y3 != 0.0) sum -= y3 * r.v[3];
    } else {
      for (int e = r.e.x, end = r.e.x + r.n; e < end; ++e) {
        const double v = val(a.ovf_pos[e]);
        if (v != 0.0) sum -= v * a.ovf_value[e];
      }
    }
    return tri_sequential_divide(a, sum, r.d);
  }
  if (r.n <= 4) {
    const int n = r.n;
    const double y0 = n > 0 ? val(r.e.x) : 0.0;
    const double y1 = n > 1 ? val(r.e.y) : 0.0;
    const double y2 = n > 2 ? val(r.e.z) : 0.0;
    const double y3 = n > 3 ? val(r.e.w) : 0.0;
    if (n == 4) {
      sum -= r.v[0] * y0 + r.v[1] * y1 + r.v[2] * y2 + r.v[3] * y3;
    } else {
      if (n > 0) sum -= r.v[0] * y0;
      if (n > 1) sum -= r.v[1] * y1;
      if (n > 2) sum -= r.v[2] * y2;
    }
  } else {
    // subtract_overflow's grouping: batches of 8 as two groups of 4, then 4s,
    // then the 1-3 remaining one by one.
    int e = r.e.x;
    const int end = r.e.x + r.n;
    for (; e + 7 < end; e += 8) {
      double p[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) p[i] = a.ovf_value[e + i] * val(a.ovf_pos[e + i]);
      sum -= p[0] + p[1] + p[2] + p[3];
      sum -= p[4] + p[5] + p[6] + p[7];
    }
    for (; e + 3 < end; e += 4) {
      sum -= a.ovf_value[e] * val(a.ovf_pos[e]) + a.ovf_value[e + 1] * val(a.ovf_pos[e + 1]) +
             a.ovf_value[e + 2] * val(a.ovf_pos[e + 2]) +
             a.ovf_value[e + 3] * val(a.ovf_pos[e + 3]);
    }
    if (e < end) {
      sum -= a.ovf_value[e] * val(a.ovf_pos[e]);
      if (e + 1 < end) {
        sum -= a.ovf_value[e + 1] * val(a.ovf_pos[e + 1]);
        if (e + 2 < end) sum -= a.ovf_value[e + 2] * val(a.ovf_pos[e + 2]);
      }
    }
  }
  return a.diag != nullptr ? sum / r.d : sum;
}

// Narrow levels [level_begin, level_end) on one CU, one level after the
// other. The run's own outputs live in LDS (written there and to global
// memory for the later launches), so a level hands its values to the next
// through LDS with one barrier, not through L2 with a store drain.
__global__ __launch_bounds__(kTriThreads) void tri_levels_cu_kernel(TriSolveArgs a,
                                                                    int level_begin,
                                                                    int level_end) {
  __shared__ double lds_y[kTriLdsVals];
  double* y = a.y;
  const int tid = threadIdx.x;
  const int top = *a.top;
  const int seg_lo = a.level_start[level_begin];
  const TriRunValues val{y, lds_y, seg_lo, a.level_start[level_end]};
  if (a.clock != nullptr && tid == 0) a.clock[level_begin] = wall_clock64();
  TriRec pre[kTriPrefetch];
  {
    const int lb = a.level_start[level_begin];
    const int le = a.level_start[level_begin + 1];
#pragma unroll
    for (int j = 0; j < kTriPrefetch; ++j) {
      tri_load(a, lb + j * kTriThreads + tid, le, top, &pre[j]);
    }
  }
  for (int l = level_begin; l < level_end; ++l) {
    const int lb = a.level_start[l];
    const int le = a.level_start[l + 1];
    TriRec cur[kTriPrefetch];
#pragma unroll
    for (int j = 0; j < kTriPrefetch; ++j) cur[j] = pre[j];
    if (l + 1 < level_end) {
      const int nb = a.level_start[l + 1];
      const int ne = a.level_start[l + 2];
#pragma unroll
      for (int j = 0; j < kTriPrefetch; ++j) {
        tri_load(a, nb + j * kTriThreads + tid, ne, top, &pre[j]);
      }
    }
    auto compute = [&](int k, const TriRec& r) {
      if (k >= le) return;
      // Not computed (row above top, or padding): the input, as tri_compute
      // leaves it in y.
      const double out = r.row > top ? y[k] : tri_apply_vals(a, val, y[k], r);
      lds_y[k - seg_lo] = out;
      if (r.row <= top) y[k] = out;
    };
#pragma unroll
    for (int j = 0; j < kTriPrefetch; ++j) compute(lb + j * kTriThreads + tid, cur[j]);
    // Positions beyond the prefetched ones (levels wider than the prefetch).
    for (int k = lb + kTriPrefetch * kTriThreads + tid; k < le; k += kTriThreads) {
      TriRec r;
      tri_load(a, k, le, top, &r);
      compute(k, r);
    }
    __syncthreads();
    if (a.clock != nullptr && tid == 0) a.clock[l + 1] = wall_clock64();
  }
}

// ---------------------------------------------------------------------------
// Dependency-driven ("sync-free") variant: one thread per listed output, all
// resident at once, no level barriers and no per-level launches. An output's
// slot in y holds kTriPending until its final value is stored there, so the
// value is its own ready flag; a thread waits for the entries it reads, then
// computes with the same arithmetic as tri_compute and stores. Waits only go
// to lower positions (earlier levels), which belong to the same or earlier
// workgroups, dispatched first: every wait ends. The wait, the computation
// and the store sit in one loop body, so a lane whose reader shares its wave
// stores before the wave spins again.
constexpr unsigned long long kTriPending = 0x7ff0deadbeef0001ull;  // a NaN no arithmetic makes
constexpr uint64_t kTriMaxWaitTicks = 20000000;  // 0.2 s of the 100 MHz wall clock

__device__ __forceinline__ bool tri_pending(double v) {
  return static_cast<unsigned long long>(__double_as_longlong(v)) == kTriPending;
}

// y[k] = x[row(k)], or "pending" for the outputs this solve computes; the
// outputs of a fused level 0 (k < level0_end: no entries) are computed here,
// their input divided as tri_apply divides it, and scattered to x.
__global__ __launch_bounds__(256) void tri_init_kernel(TriSolveArgs a0) {
  const TriSolveArgs a = TriRhs(a0, blockIdx.y);
  const int top = *a.top;
  const double pending = __longlong_as_double(static_cast<long long>(kTriPending));
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < a.num_pos;
       k += gridDim.x * blockDim.x) {
    const int row = a.pos_row[k];
    double v;
    if (k < a.level0_end) {
      const int rrow = a.rec_row[k];  // INT32_MAX for padding
      v = a.x[row];
      if (rrow <= top) {
        if (a.diag != nullptr) {
          v = a.sequential ? tri_sequential_divide(a, v, a.diag[k]) : v / a.diag[k];
        }
        a.x[row] = v;  // the scatter, fused
      }
    } else {
      v = (k < a.num_work && row <= top) ? pending : a.x[row];
    }
    // Write-through (sc1) stores: a plain store would leave the line valid in
    // this XCD's L2, and a reader on this XCD would then poll that stale copy
    // (pending) until the line is evicted, long after its producer on
    // another XCD stored the final value.
    __hip_atomic_store(a.y + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Backoff between polls: `units` s_sleep(1) (64 clocks each), doubling up to
// a.poll_max; fewer polls in flight leave the memory queues to the hand-offs.
__device__ __forceinline__ void tri_backoff(const TriSolveArgs& a, int* units) {
  for (int i = 0; i < *units; ++i) __builtin_amdgcn_s_sleep(1);
  *units = min(*units * 2, a.poll_max);
}

__device__ __forceinline__ int tri_entry_pos(const TriSolveArgs& a, const int4& e, int n, int j) {
  if (n > 4) return a.ovf_pos[e.x + j];
  return j == 0 ? e.x : j == 1 ? e.y : j == 2 ? e.z : e.w;
}

// tri_apply for n <= 4 with the entry values already in registers.
__device__ __forceinline__ double tri_apply4(const TriSolveArgs& a, double sum, const TriRec& r,
                                             double y0, double y1, double y2, double y3) {
  const int n = r.n;
  if (a.sequential) {
    if (y0 != 0.0) sum -= y0 * r.v[0];
    if (y1 != 0.0) sum -= y1 * r.v[1];
    if (y2 != 0.0) sum -= y2 * r.v[2];
    if (y3 != 0.0) sum -= y3 * r.v[3];
    return tri_sequential_divide(a, sum, r.d);
  }
  if (n == 4) {
    sum -= r.v[0] * y0 + r.v[1] * y1 + r.v[2] * y2 + r.v[3] * y3;
  } else {
    if (n > 0) sum -= r.v[0] * y0;
    if (n > 1) sum -= r.v[1] * y1;
    if (n > 2) sum -= r.v[2] * y2;
  }
  return a.diag != nullptr ? sum / r.d : sum;
}

// Output k of the sync-free solve: wait for its entries, compute, store.
//
// The wait loop's exit is wave-uniform (`__ballot` over the lanes still
// waiting): a lane that finishes stores inside the loop body, the same pass.
// With a per-lane exit the compiler sinks the division and the stores below
// the loop, so a wave published its 64 outputs only when its slowest lane was
// done: every level paid the wave's slowest input, not each output's own.
__device__ __forceinline__ void tri_syncfree_output(const TriSolveArgs& a, int k, int top) {
  TriRec r;
  tri_load(a, k, a.num_work, top, &r);
  bool done = r.row > top;  // not computed: y[k] already holds x[row]
  double* y = a.y;
  const double in = done ? 0.0 : a.x[r.row];
  int backoff = 1;
  const uint64_t t0 = wall_clock64();  // 100 MHz
  const double pend = __longlong_as_double(static_cast<long long>(kTriPending));
  // n <= 4: one poll round loads the entries still pending at once and keeps
  // them: the values that end the wait are the ones the output is computed
  // from (a hop is one round trip, not a readiness walk plus a reload), and a
  // final value is never loaded twice.
  const int n = r.n;
  double y0 = n > 0 ? pend : 0.0, y1 = n > 1 ? pend : 0.0;
  double y2 = n > 2 ? pend : 0.0, y3 = n > 3 ? pend : 0.0;
  // n > 4: the output folds its entries in evaluation order as they become
  // final (the same operations as subtract_overflow / subtract_sequential,
  // so the same bits): by the time its last input arrives only the groups
  // after the last stall are left, and a deep chain of long outputs advances
  // by one group fold per hop instead of one whole sum. The wait bound
  // restarts on progress (a stall detector, not a budget for the chain).
  double sum = in;
  int e = r.e.x;
  const int end = r.e.x + r.n;
  uint64_t t_progress = t0;
  while (__ballot(!done) != 0) {
    if (done) continue;
    if (n <= 4) {
      if (tri_pending(y0)) y0 = load_final(y, r.e.x);
      if (tri_pending(y1)) y1 = load_final(y, r.e.y);
      if (tri_pending(y2)) y2 = load_final(y, r.e.z);
      if (tri_pending(y3)) y3 = load_final(y, r.e.w);
      const bool pending = tri_pending(y0) || tri_pending(y1) || tri_pending(y2) ||
                           tri_pending(y3);
      if (!pending) {
        const double out = tri_apply4(a, in, r, y0, y1, y2, y3);
        a.x[r.row] = out;  // the scatter, fused
        __hip_atomic_store(y + k, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done = true;
      } else if (wall_clock64() - t0 > kTriMaxWaitTicks) {
        // Bounded wait (never expected): report and leave, the host fails loudly.
        if (a.fail != nullptr) __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        done = true;
      } else {
        tri_backoff(a, &backoff);
      }
      continue;
    }
    const int e0 = e;
    while (e < end) {
      // Up to 8 values per round, their loads in flight together.
      double v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = e + i < end ? load_final(y, a.ovf_pos[e + i]) : 0.0;
      int took = 0;
      if (a.sequential) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (took != i || e + i >= end || tri_pending(v[i])) continue;
          if (v[i] != 0.0) sum -= v[i] * a.ovf_value[e + i];
          took = i + 1;
        }
      } else {
#pragma unroll
        for (int g = 0; g < 8; g += 4) {
          if (took != g || e + g + 3 >= end) continue;
          if (tri_pending(v[g]) || tri_pending(v[g + 1]) || tri_pending(v[g + 2]) ||
              tri_pending(v[g + 3])) {
            continue;
          }
          sum -= a.ovf_value[e + g] * v[g] + a.ovf_value[e + g + 1] * v[g + 1] +
                 a.ovf_value[e + g + 2] * v[g + 2] + a.ovf_value[e + g + 3] * v[g + 3];
          took = g + 4;
        }
        // The tail (fewer than 4 left), one subtraction per entry, all final.
        const int left = end - e - took;
        if (took < 8 && left > 0 && left < 4) {
          const int t = took;
          bool ready = true;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            if (i < left && t + i < 8) ready = ready && !tri_pending(v[t + i]);
          }
          if (ready && t + left <= 8) {
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              if (i < left) sum -= a.ovf_value[e + t + i] * v[t + i];
            }
            took = t + left;
          }
        }
      }
      e += took;
      if (took < 8) break;  // a pending value, or the end
    }
    if (e == end) {
      const double out = a.sequential ? tri_sequential_divide(a, sum, r.d)
                                      : (a.diag != nullptr ? sum / r.d : sum);
      a.x[r.row] = out;  // the scatter, fused
      __hip_atomic_store(y + k, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      done = true;
    } else if (e != e0) {
      t_progress = wall_clock64();
      backoff = 1;
    } else if (wall_clock64() - t_progress > kTriMaxWaitTicks) {
      if (a.fail != nullptr) __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      done = true;
    } else {
      tri_backoff(a, &backoff);
    }
  }
}

__global__ __launch_bounds__(256) void tri_syncfree_kernel(TriSolveArgs a0) {
  const TriSolveArgs a = TriRhs(a0, blockIdx.y);
  const int k = a.seg_begin + blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.seg_end) return;
  tri_syncfree_output(a, k, *a.top);
}

// Persistent form: the working workgroups' threads walk the outputs in level
// order, thread t taking t, t + T, t + 2T, ... (T threads in all). Every wait
// goes to a lower position; the thread owning it is at a position no higher
// than the waiter's (same stride walk), so the lowest waiting output always
// has its entries computed or computable: all waits end with every working
// workgroup resident (a handful per XCD). With xcd_stride 8 only the blocks
// b with b % 8 == 0 work: they share one XCD under the observed round-robin
// dealing, so hand-offs stay in one L2 (speed only; the stores and loads are
// agent scope, correct under any placement).
__global__ __launch_bounds__(kTriThreads) void tri_syncfree_persistent_kernel(TriSolveArgs a,
                                                                              int xcd_stride) {
  if (blockIdx.x % xcd_stride != 0) return;
  const int group = blockIdx.x / xcd_stride;
  const int total = (gridDim.x / xcd_stride) * kTriThreads;
  const int top = *a.top;
  for (int k = group * kTriThreads + threadIdx.x; k < a.num_work; k += total) {
    if (k >= a.level0_end) tri_syncfree_output(a, k, top);  // level 0: the init's
  }
}

// A narrow segment of the schedule (positions [seg_begin, seg_end), levels
// unpadded) on one workgroup per right-hand side: a hand-off between two of
// its outputs is an LDS store and load inside one CU (a fraction of a
// microsecond) instead of a trip through the L2s of two XCDs. Thread t walks
// the segment's positions t, t + T, ... in order; every output reads lower
// positions only, so the lowest unfinished output is always computable and
// all waits end (one workgroup, all its waves resident). Each output is
// evaluated exactly as tri_syncfree_output evaluates it (same operations in
// the same order, long outputs folding as their inputs arrive); earlier
// segments are final in y, and the outputs go to y for later ones.
//
// The segment's inputs x[row] are loaded into LDS by the whole workgroup
// first, with a ready word per position (1: final -- an output of this
// segment once computed, or a position it does not compute), so an output's
// input comes from LDS and only its record from global memory. A value is
// stored before its ready word (workgroup release / acquire).
__device__ __forceinline__ double tri_chain_load(const TriSolveArgs& a, const double* vals,
                                                 const int* ready, int p) {
  if (p >= a.seg_begin && p < a.seg_end) {
    if (__hip_atomic_load(ready + (p - a.seg_begin), __ATOMIC_ACQUIRE,
                          __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
      return __longlong_as_double(static_cast<long long>(kTriPending));
    }
    return vals[p - a.seg_begin];
  }
  return load_final(a.y, p);
}

// An entry's value when an output starts: earlier segments' values are final
// in y (loaded once, kept in registers), this segment's come from LDS when
// ready, else the pending mark; polls then re-read only pending entries,
// from LDS.
__device__ __forceinline__ double tri_chain_first(const TriSolveArgs& a, const double* vals,
                                                  const int* ready, int p) {
  if (p >= a.seg_begin && p < a.seg_end) return tri_chain_load(a, vals, ready, p);
  return load_final(a.y, p);
}
__device__ __forceinline__ double tri_chain_refresh(const TriSolveArgs& a, const double* vals,
                                                    const int* ready, int p, double cur) {
  return tri_pending(cur) ? tri_chain_load(a, vals, ready, p) : cur;
}

__global__ __launch_bounds__(kTriThreads) void tri_chain_kernel(TriSolveArgs a0) {
  const TriSolveArgs a = TriRhs(a0, blockIdx.y);
  __shared__ double vals[kTriChainVals];
  __shared__ int ready[kTriChainVals];
  const int cs = a.seg_begin;
  const int ce = a.seg_end;
  const int top = *a.top;
  {
    // Eight positions per thread in flight: the rows, then their inputs.
    for (int k0 = cs + threadIdx.x; k0 < ce; k0 += 8 * kTriThreads) {
      int row[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * kTriThreads;
        row[u] = k < ce ? a.rec_row[k] : INT32_MAX;
      }
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = row[u] < a.num_rows ? a.x[row[u]] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u * kTriThreads;
        if (k < ce) {
          vals[k - cs] = v[u];
          ready[k - cs] = row[u] <= top ? 0 : 1;
        }
      }
    }
  }
  __syncthreads();
  // Thread t's outputs are positions t, t + T, ... of the segment, taken in
  // that order by a uniform outer loop: every lane of a wave loads its
  // output's record and entries (global loads) together, then the wave polls
  // LDS only until all its lanes are done. A lane waiting on LDS is never held
  // behind another lane's global load (a hand-off costs an LDS round trip).
  // Long outputs fold their entries by windows of 8 as they become final.
  uint64_t t_progress = wall_clock64();
  bool failed = false;
  for (int k = cs + threadIdx.x; k < ce && !failed; k += kTriThreads) {
    if (ready[k - cs] != 0) continue;  // not computed: keeps its input
    TriRec r;
    tri_load(a, k, ce, top, &r);
    double sum = vals[k - cs];
    int e = 0, end = 0;
    int wpos[8];
    double wval[8];
    double v[8];  // entry values, the pending mark until final
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = 0.0;
    if (r.n > 4) {
      e = r.e.x;
      end = r.e.x + r.n;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        wpos[u] = e + u < end ? a.ovf_pos[e + u] : 0;
        wval[u] = e + u < end ? a.ovf_value[e + u] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = e + u < end ? tri_chain_first(a, vals, ready, wpos[u]) : 0.0;
    } else {
      const int n = r.n;
      v[0] = n > 0 ? tri_chain_first(a, vals, ready, r.e.x) : 0.0;
      v[1] = n > 1 ? tri_chain_first(a, vals, ready, r.e.y) : 0.0;
      v[2] = n > 2 ? tri_chain_first(a, vals, ready, r.e.z) : 0.0;
      v[3] = n > 3 ? tri_chain_first(a, vals, ready, r.e.w) : 0.0;
    }
    int polls = 0;
    while (true) {
      bool finished = false;
      bool progress = false;
      double out = 0.0;
      if (r.n <= 4) {
        if (!(tri_pending(v[0]) || tri_pending(v[1]) || tri_pending(v[2]) || tri_pending(v[3]))) {
          out = tri_apply4(a, sum, r, v[0], v[1], v[2], v[3]);
          finished = true;
        }
      } else {
        int took = 0;
        if (a.sequential) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            if (took != u || e + u >= end || tri_pending(v[u])) continue;
            if (v[u] != 0.0) sum -= v[u] * wval[u];
            took = u + 1;
          }
        } else {
#pragma unroll
          for (int g = 0; g < 8; g += 4) {
            if (took != g || e + g + 3 >= end) continue;
            if (tri_pending(v[g]) || tri_pending(v[g + 1]) || tri_pending(v[g + 2]) ||
                tri_pending(v[g + 3])) {
              continue;
            }
            sum -= wval[g] * v[g] + wval[g + 1] * v[g + 1] + wval[g + 2] * v[g + 2] +
                   wval[g + 3] * v[g + 3];
            took = g + 4;
          }
          const int left = end - e - took;
          if (took < 8 && left > 0 && left < 4) {
            const int t = took;
            bool all_final = true;
#pragma unroll
            for (int u = 0; u < 3; ++u) {
              if (u < left && t + u < 8) all_final = all_final && !tri_pending(v[t + u]);
            }
            if (all_final && t + left <= 8) {
#pragma unroll
              for (int u = 0; u < 3; ++u) {
                if (u < left) sum -= wval[t + u] * v[t + u];
              }
              took = t + left;
            }
          }
        }
        if (took > 0) {
          e += took;
          progress = true;
          if (e == end) {
            out = a.sequential ? tri_sequential_divide(a, sum, r.d)
                               : (a.diag != nullptr ? sum / r.d : sum);
            finished = true;
          } else {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              wpos[u] = e + u < end ? a.ovf_pos[e + u] : 0;
              wval[u] = e + u < end ? a.ovf_value[e + u] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              v[u] = e + u < end ? tri_chain_first(a, vals, ready, wpos[u]) : 0.0;
            }
          }
        }
      }
      if (finished) {
        vals[k - cs] = out;
        __hip_atomic_store(ready + (k - cs), 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(a.y + k, out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        a.x[r.row] = out;  // the scatter, fused
        break;
      }
      // A wave none of whose lanes moved yields its issue slots for a moment
      // (the LDS polls of 16 waves would otherwise crowd the producers).
      if (__ballot(progress) == 0) __builtin_amdgcn_s_sleep(1);
      if (progress) {
        polls = 0;
      } else if (++polls % 64 == 0) {
        const uint64_t now = wall_clock64();
        if (polls == 64) t_progress = now;  // first stalled check of this wait
        if (now - t_progress > kTriMaxWaitTicks) {
          if (a.fail != nullptr) __hip_atomic_store(a.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          failed = true;
          break;
        }
      }
      if (r.n <= 4) {
        v[0] = tri_chain_refresh(a, vals, ready, r.e.x, v[0]);
        v[1] = tri_chain_refresh(a, vals, ready, r.e.y, v[1]);
        v[2] = tri_chain_refresh(a, vals, ready, r.e.z, v[2]);
        v[3] = tri_chain_refresh(a, vals, ready, r.e.w, v[3]);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = tri_chain_refresh(a, vals, ready, wpos[u], v[u]);
      }
    }
  }
}

}  // namespace milp_kernels

namespace milp_launch {

hipError_t tri_transpose_lower_syncfree(const milp_kernels::TriSolveArgs& args,
                                        const int* segs, int num_segs, hipStream_t s,
                                        int num_rhs) {
  if (args.num_work <= 0) return hipSuccess;
  const int row_blocks =
      std::max(1, std::min(1024, (args.num_rows - args.first_col + 255) / 256));
  hipError_t e;
  if (args.host_x != nullptr) {
    milp_kernels::tri_copy_in_kernel<<<dim3(row_blocks, num_rhs), 256, 0, s>>>(args);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int pos_blocks = std::max(1, std::min(1024, (args.num_pos + 255) / 256));
  milp_kernels::tri_init_kernel<<<dim3(pos_blocks, num_rhs), 256, 0, s>>>(args);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  milp_kernels::TriSolveArgs a = args;
  for (int i = 0; i < num_segs; ++i) {
    // Positions of a fused level 0 were computed by the init kernel.
    a.seg_begin = std::max(segs[3 * i], args.level0_end);
    a.seg_end = segs[3 * i + 1];
    if (a.seg_end <= a.seg_begin) continue;
    if (segs[3 * i + 2] != 0) {
      milp_kernels::tri_chain_kernel<<<dim3(1, num_rhs), milp_kernels::kTriThreads, 0, s>>>(a);
    } else {
      // One thread per listed output and right-hand side: every workgroup
      // resident (100k outputs = 391 workgroups of 256 per vector on 256 CUs).
      milp_kernels::tri_syncfree_kernel<<<dim3((a.seg_end - a.seg_begin + 255) / 256, num_rhs),
                                          256, 0, s>>>(a);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (args.host_x == nullptr) return hipSuccess;
  milp_kernels::tri_copy_out_kernel<<<dim3(row_blocks, num_rhs), 256, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t tri_transpose_lower_persistent(const milp_kernels::TriSolveArgs& args, int groups,
                                          int xcd_stride, hipStream_t s) {
  if (args.num_work <= 0) return hipSuccess;
  const int row_blocks =
      std::max(1, std::min(1024, (args.num_rows - args.first_col + 255) / 256));
  hipError_t e;
  if (args.host_x != nullptr) {
    milp_kernels::tri_copy_in_kernel<<<row_blocks, 256, 0, s>>>(args);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int pos_blocks = std::max(1, std::min(1024, (args.num_pos + 255) / 256));
  milp_kernels::tri_init_kernel<<<pos_blocks, 256, 0, s>>>(args);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  milp_kernels::tri_syncfree_persistent_kernel<<<groups * xcd_stride, milp_kernels::kTriThreads,
                                                 0, s>>>(args, xcd_stride);
  e = hipGetLastError();
  if (e != hipSuccess || args.host_x == nullptr) return e;
  milp_kernels::tri_copy_out_kernel<<<row_blocks, 256, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t tri_transpose_lower(const milp_kernels::TriSolveArgs& args, const int* segments,
                               int num_segments, hipStream_t s) {
  if (args.num_work <= 0) return hipSuccess;
  const int row_blocks =
      std::max(1, std::min(1024, (args.num_rows - args.first_col + 255) / 256));
  hipError_t e;
  if (args.host_x != nullptr) {
    milp_kernels::tri_copy_in_kernel<<<row_blocks, 256, 0, s>>>(args);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int pos_blocks = std::min(1024, (args.num_pos + 255) / 256);
  // Level 0 alone over the chip (the first segment is (-1, blocks)) and a
  // diagonal to divide by: fused into the gather.
  const bool fuse0 = args.fuse_level0 && args.diag != nullptr && num_segments > 0 &&
                     segments[0] == -1;
  if (fuse0) {
    milp_kernels::tri_gather_level0_kernel<<<pos_blocks, 256, 0, s>>>(args);
  } else {
    milp_kernels::tri_gather_kernel<<<pos_blocks, 256, 0, s>>>(args);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  for (int i = fuse0 ? 1 : 0; i < num_segments; ++i) {
    const int lb = segments[2 * i];
    const int le = segments[2 * i + 1];
    if (le <= lb) continue;
    if (lb < 0) {  // a wide level on the whole chip: (-level - 1, blocks)
      milp_kernels::tri_level_grid_kernel<<<le, 256, 0, s>>>(args, -lb - 1);
    } else {
      milp_kernels::tri_levels_cu_kernel<<<1, milp_kernels::kTriThreads, 0, s>>>(args, lb, le);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const int work_blocks = std::min(1024, (args.num_work + 255) / 256);
  // (A scatter straight into mapped host memory, tri_scatter_host_kernel,
  // measured 80 us against 5 + 15 us for this scatter plus the coalesced
  // copy-out: scattered 8-byte PCIe writes.)
  milp_kernels::tri_scatter_kernel<<<work_blocks, 256, 0, s>>>(args);
  if (args.host_x == nullptr) return hipGetLastError();
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  milp_kernels::tri_copy_out_kernel<<<row_blocks, 256, 0, s>>>(args);
  return hipGetLastError();
}

}  // namespace milp_launch
