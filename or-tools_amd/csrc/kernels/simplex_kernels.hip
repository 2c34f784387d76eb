// CDNA4 (gfx950) kernels for the O(nnz(A)) inner loops of Glop's revised
// simplex. Every kernel reproduces the floating-point evaluation order of the
// Glop loop it replaces, so results are bit-identical to the host code:
//   * CompactSparseMatrix::ColumnScalarProduct (lp_data/sparse.h:514-542):
//     four strided accumulators r1..r4 over the column, ((r1+r2)+r3)+r4, then
//     the <=3 tail terms in order.
//   * ColumnAddMultipleToDenseColumn scatter (sparse.h:389-399) summed per row
//     in increasing column order, zero multipliers skipped.
//   * UpdateRow row-wise algorithms (update_row.cc:196-280): per output column
//     the filtered rho rows are accumulated in increasing row order.
// Compiled with -ffp-contract=off: no FMA contraction anywhere.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_args.h"

namespace milp_kernels {

constexpr int kWave = 64;

__device__ __forceinline__ bool bit_set(const uint64_t* words, int i) {
  return (words[i >> 6] >> (i & 63)) & 1ull;
}

// ---------------------------------------------------------------------------
// Column dot product with Glop's 4-accumulator order, one wave per column.
// The 64 lanes load 64 consecutive entries of the column (coalesced), each
// computes its product, and lanes 0..3 (accumulator k = lane & 3) fold the 16
// products of their chain in order by reading them with __shfl. The chain
// index of entry e (relative to the column start) is e & 3 and entries of one
// chain are visited in increasing e, exactly as in sparse.h:527-532.
__device__ __forceinline__ double wave_column_dot(const int64_t s, const int64_t e,
                                                  const int32_t* __restrict__ rows,
                                                  const double* __restrict__ vals,
                                                  const double* __restrict__ y,
                                                  int lane) {
  const int64_t len = e - s;
  const int64_t full = (len >= 4) ? (len / 4) * 4 : 0;  // entries in 4-blocks
  double acc = 0.0;  // lanes 0..3: r1..r4
  for (int64_t base = 0; base < full; base += kWave) {
    const int64_t idx = base + lane;
    double p = 0.0;
    if (idx < full) p = vals[s + idx] * y[rows[s + idx]];
    const int64_t nvalid = (full - base) < kWave ? (full - base) : kWave;
    // nvalid is a multiple of 4: each chain has nvalid/4 terms in this chunk.
    const int nt = static_cast<int>(nvalid >> 2);
#pragma unroll 4
    for (int t = 0; t < 16; ++t) {
      const double q = __shfl(p, (t << 2) + (lane & 3), kWave);
      if (t < nt) acc += q;
    }
  }
  const double r2 = __shfl(acc, 1, kWave);
  const double r3 = __shfl(acc, 2, kWave);
  const double r4 = __shfl(acc, 3, kWave);
  double result = acc + r2 + r3 + r4;
  // Tail (sparse.h:534-541), same on every lane.
  for (int64_t i = s + full; i < e; ++i) result += vals[i] * y[rows[i]];
  return result;
}

// Quarter-wave variant for short columns: 4 lanes per column, lane k owns
// chain k and walks it sequentially (16 columns per wave).
__device__ __forceinline__ double quad_column_dot(const int64_t s, const int64_t e,
                                                  const int32_t* __restrict__ rows,
                                                  const double* __restrict__ vals,
                                                  const double* __restrict__ y,
                                                  int sub, int lane) {
  const int64_t len = e - s;
  const int64_t full = (len >= 4) ? (len / 4) * 4 : 0;
  double acc = 0.0;
  for (int64_t i = s + sub; i < s + full; i += 4) acc += vals[i] * y[rows[i]];
  const int g = lane & ~3;
  const double r1 = __shfl(acc, g + 0, kWave);
  const double r2 = __shfl(acc, g + 1, kWave);
  const double r3 = __shfl(acc, g + 2, kWave);
  const double r4 = __shfl(acc, g + 3, kWave);
  double result = r1 + r2 + r3 + r4;
  for (int64_t i = s + full; i < e; ++i) result += vals[i] * y[rows[i]];
  return result;
}

// One thread per column, the four chains in registers: the same terms in the
// same order as quad_column_dot (chain k = entries s+k, s+k+4, ...), for the
// one-workgroup kernels of small LPs whose columns are a few entries long.
__device__ __forceinline__ double thread_column_dot(const int64_t s, const int64_t e,
                                                    const int32_t* __restrict__ rows,
                                                    const double* __restrict__ vals,
                                                    const double* __restrict__ y) {
  const int64_t len = e - s;
  const int64_t full = (len >= 4) ? (len / 4) * 4 : 0;
  double r1 = 0.0, r2 = 0.0, r3 = 0.0, r4 = 0.0;
  for (int64_t i = s; i < s + full; i += 4) {
    r1 += vals[i] * y[rows[i]];
    r2 += vals[i + 1] * y[rows[i + 1]];
    r3 += vals[i + 2] * y[rows[i + 2]];
    r4 += vals[i + 3] * y[rows[i + 3]];
  }
  double result = r1 + r2 + r3 + r4;
  for (int64_t i = s + full; i < e; ++i) result += vals[i] * y[rows[i]];
  return result;
}

// Modes of the column-dot kernel.
enum DotMode : int {
  kUpdateRowColumnWise = 0,  // update_row.cc:282-306 over relevant columns
  kPricing = 1,              // reduced_costs.cc:372-381: rc = c - a_j.y
  kListDots = 2,             // primal_edge_norms.cc:229-233 over a column list
  kFullUpdateRow = 3,        // update_row.cc:311-332 over non-basic columns
  // Column-wise update row fused with the primal edge-norm dots
  // (primal_edge_norms.cc:229-233): one pass over A yields rho.a_j and w.a_j.
  kUpdateRowWithDots = 4,
  // Pricing fused with the edge-norm dots deferred from the previous pivot:
  // rc_j = c_j - a_j.y for every column and w.a_j for the columns flagged as
  // listed in that pivot's update row. One pass over A instead of two.
  kPricingWithDots = 5
};


template <int MODE, bool WAVE_PER_COL>
__global__ __launch_bounds__(256) void column_dot_kernel(DotArgs a) {
  const int lane = threadIdx.x & 63;
  int col_slot;
  int sub = 0;
  if (WAVE_PER_COL) {
    col_slot = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  } else {
    col_slot = blockIdx.x * (blockDim.x >> 2) + (threadIdx.x >> 2);
    sub = threadIdx.x & 3;
  }
  // All lanes that share a column must stay converged through the shuffles,
  // so out-of-range slots compute on column 0 and just skip the epilogue.
  const bool in_range = col_slot < a.ncols;
  const int slot = in_range ? col_slot : 0;
  const int col = a.col_list != nullptr ? a.col_list[slot] : slot;
  bool active = in_range;
  if (a.skip != nullptr) active = active && !a.skip[col];
  if (MODE == kUpdateRowColumnWise || MODE == kFullUpdateRow || MODE == kUpdateRowWithDots) {
    active = active && bit_set(a.mask, col);
  } else if (MODE == kListDots && a.flags != nullptr) {
    active = active && a.flags[col];
  }
  const int64_t s = a.starts[col];
  const int64_t e = active ? a.starts[col + 1] : s;
  const double dot = WAVE_PER_COL ? wave_column_dot(s, e, a.rows, a.vals, a.y, lane)
                                  : quad_column_dot(s, e, a.rows, a.vals, a.y, sub, lane);
  double dot2 = 0.0;
  bool listed = false;
  if (MODE == kUpdateRowWithDots) {  // second sweep of the same column (cache hot)
    dot2 = WAVE_PER_COL ? wave_column_dot(s, e, a.rows, a.vals, a.y2, lane)
                        : quad_column_dot(s, e, a.rows, a.vals, a.y2, sub, lane);
  } else if (MODE == kPricingWithDots) {
    // Only listed columns sweep again; the others walk an empty range so the
    // lanes of a column stay converged through the shuffles.
    listed = active && a.flags[col] != 0;
    const int64_t e2 = listed ? e : s;
    dot2 = WAVE_PER_COL ? wave_column_dot(s, e2, a.rows, a.vals, a.y2, lane)
                        : quad_column_dot(s, e2, a.rows, a.vals, a.y2, sub, lane);
  }
  const bool writer = WAVE_PER_COL ? (lane == 0) : (sub == 0);
  if (!writer || !in_range) return;
  if (a.skip != nullptr && a.skip[col]) return;  // owned by the dense block
  if (MODE == kUpdateRowWithDots) {
    const bool keep = active && fabs(dot) > a.drop_tolerance;
    a.flags[col] = keep ? 1 : 0;
    if (keep) {
      a.out[col] = dot;
      a.out2[col] = dot2;
    }
  } else if (MODE == kUpdateRowColumnWise) {
    const bool keep = active && fabs(dot) > a.drop_tolerance;
    a.flags[col] = keep ? 1 : 0;
    if (keep) a.out[col] = dot;
  } else if (MODE == kPricing) {
    a.out[col] = a.c[col] - dot;
  } else if (MODE == kPricingWithDots) {
    a.out[col] = a.c[col] - dot;
    if (listed) a.out2[col] = dot2;
  } else if (MODE == kListDots) {
    if (active) a.out[col] = dot;
  } else {  // kFullUpdateRow
    if (active && fabs(dot) > a.drop_tolerance) a.out[col] = dot;
  }
}

// ---------------------------------------------------------------------------
// Dense block dots (layout in kernel_args.h). A workgroup owns 64 dense
// columns; its wave k streams chain k (Glop's accumulator r_{k+1} in
// ColumnScalarProduct, sparse.h:514-542) of those columns, lane j walking
// column j sequentially, two chain elements per 16-byte load: one wave step
// is one contiguous 1-KiB load. The chain index is wave-uniform, so the y
// (and w) elements a step needs are the same for every lane and come from
// scalar loads: the vector memory path carries only A. UNROLL loads are
// issued ahead of the dependent adds. The four partial sums meet in LDS and
// lane j of wave 0 folds ((r1 + r2) + r3) + r4, then adds the <= 3 tail
// terms in order, exactly as ColumnScalarProduct.
typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int kDenseColsPerBlock = 64;

template <int MODE, int UNROLL>
__global__ __launch_bounds__(256) void dense_dot_kernel(DenseArgs a) {
  constexpr bool kTwo = MODE == kUpdateRowWithDots || MODE == kPricingWithDots;
  __shared__ double part[4][kDenseColsPerBlock];
  __shared__ double part2[kTwo ? 4 : 1][kDenseColsPerBlock];
  const int lane = threadIdx.x & 63;
  const int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // chain of this wave
  const int j = blockIdx.x * kDenseColsPerBlock + lane;
  const int nd = a.nd;
  const bool in_range = j < nd;
  const int col = in_range ? a.dense_cols[j] : 0;
  bool active = in_range;
  if (MODE == kUpdateRowColumnWise || MODE == kUpdateRowWithDots)
    active = active && bit_set(a.mask, col);
  if (MODE == kListDots) active = active && a.flags[col];
  const int steps = a.m >> 2;
  const int pairs = steps >> 1;
  double acc = 0.0;
  double acc2 = 0.0;
  if (active) {
    const dbl2* __restrict__ p =
        reinterpret_cast<const dbl2*>(a.body) + static_cast<int64_t>(k) * nd + j;
    const double* __restrict__ y = a.y + k;
    const double* __restrict__ y2 = kTwo ? a.y2 + k : nullptr;
    const int64_t stride = static_cast<int64_t>(nd) * 4;  // double2 per pair step
    int t = 0;
    for (; t + UNROLL <= pairs; t += UNROLL) {
      dbl2 v[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(p + (t + u) * stride);
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const int r = (t + u) * 8;
        acc += v[u].x * y[r];
        acc += v[u].y * y[r + 4];
        if (kTwo) {
          acc2 += v[u].x * y2[r];
          acc2 += v[u].y * y2[r + 4];
        }
      }
    }
    for (; t < pairs; ++t) {
      const dbl2 v = p[t * stride];
      acc += v.x * y[t * 8];
      acc += v.y * y[t * 8 + 4];
      if (kTwo) {
        acc2 += v.x * y2[t * 8];
        acc2 += v.y * y2[t * 8 + 4];
      }
    }
    if (steps & 1) {
      const double v = a.body[static_cast<int64_t>(pairs) * nd * 8 +
                              static_cast<int64_t>(k) * nd + j];
      acc += v * y[(steps - 1) * 4];
      if (kTwo) acc2 += v * y2[(steps - 1) * 4];
    }
  }
  part[k][lane] = acc;
  if (kTwo) part2[k][lane] = acc2;
  __syncthreads();
  if (k != 0 || !in_range) return;
  double result = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
  double result2 = 0.0;
  if (kTwo) result2 = part2[0][lane] + part2[1][lane] + part2[2][lane] + part2[3][lane];
  const int base = steps * 4;
  for (int r = 0; base + r < a.m; ++r) {
    const double v = a.tail[static_cast<int64_t>(r) * nd + j];
    result += v * a.y[base + r];
    if (kTwo) result2 += v * a.y2[base + r];
  }
  if (MODE == kUpdateRowColumnWise || MODE == kUpdateRowWithDots) {
    const bool keep = active && fabs(result) > a.drop_tolerance;
    a.flags[col] = keep ? 1 : 0;
    if (keep) {
      a.out[col] = result;
      if (kTwo) a.out2[col] = result2;
    }
  } else if (MODE == kPricing) {
    a.out[col] = a.c[col] - result;
  } else if (MODE == kPricingWithDots) {
    a.out[col] = a.c[col] - result;
    if (a.flags[col]) a.out2[col] = result2;  // listed in the deferred update row
  } else if (MODE == kListDots) {
    if (active) a.out[col] = result;
  }
}

// Builds the dense block from the CSC arrays; one thread per destination
// element so the stores are contiguous.
__global__ __launch_bounds__(256) void dense_pack_kernel(const int64_t* starts,
                                                         const double* vals,
                                                         const int32_t* dense_cols, int nd,
                                                         int m, double* body, double* tail) {
  const int steps = m >> 2;
  const int pairs = steps >> 1;
  const int64_t pair_total = static_cast<int64_t>(pairs) * nd * 8;
  const int64_t odd_total = (steps & 1) ? static_cast<int64_t>(nd) * 4 : 0;
  const int64_t tail_total = static_cast<int64_t>(m - 4 * steps) * nd;
  const int64_t total = pair_total + odd_total + tail_total;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    if (e < pair_total) {  // e = ((t2 * 4 + k) * nd + j) * 2 + h
      const int h = static_cast<int>(e & 1);
      const int64_t q = e >> 1;
      const int j = static_cast<int>(q % nd);
      const int64_t q2 = q / nd;
      const int k = static_cast<int>(q2 & 3);
      const int t2 = static_cast<int>(q2 >> 2);
      body[e] = vals[starts[dense_cols[j]] + 4 * (2 * t2 + h) + k];
    } else if (e < pair_total + odd_total) {  // f = k * nd + j
      const int64_t f = e - pair_total;
      const int k = static_cast<int>(f / nd);
      const int j = static_cast<int>(f % nd);
      body[e] = vals[starts[dense_cols[j]] + 4 * (steps - 1) + k];
    } else {
      const int64_t f = e - pair_total - odd_total;
      const int j = static_cast<int>(f % nd);
      const int r = static_cast<int>(f / nd);
      tail[f] = vals[starts[dense_cols[j]] + 4 * steps + r];
    }
  }
}

__global__ void gather_kernel(const int32_t* list, int n, const double* src, double* dst) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    dst[i] = src[list[i]];
}

// Update-row compaction for small N in one workgroup: thread t owns a
// contiguous slice of the flags, a block-wide exclusive scan of the slice
// counts gives each thread its output offset, so the list comes out in
// ascending position order, as rocprim::select would produce it.
constexpr int kCompactThreads = 1024;
__global__ __launch_bounds__(kCompactThreads) void compact_small_kernel(
    const uint8_t* flags, int n, const double* coeff, int32_t* list, double* vals, int* count,
    int32_t* host_list, double* host_vals, int* host_count) {
  __shared__ int sums[kCompactThreads];
  const int t = threadIdx.x;
  const int per = (n + kCompactThreads - 1) / kCompactThreads;
  const int b = min(n, t * per);
  const int e = min(n, b + per);
  int c = 0;
  for (int i = b; i < e; ++i) c += flags[i] != 0;
  sums[t] = c;
  __syncthreads();
  for (int off = 1; off < kCompactThreads; off <<= 1) {
    const int v = t >= off ? sums[t - off] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  int pos = sums[t] - c;
  for (int i = b; i < e; ++i) {
    if (flags[i] != 0) {
      const double v = coeff[i];
      list[pos] = i;
      vals[pos] = v;
      if (host_list != nullptr) {  // zero-copy readback into mapped host memory
        host_list[pos] = i;
        host_vals[pos] = v;
      }
      ++pos;
    }
  }
  if (t == kCompactThreads - 1) {
    *count = sums[t];
    if (host_count != nullptr) *host_count = sums[t];
  }
}

// ---------------------------------------------------------------------------
// Ordered single-pass compaction over many workgroups. A workgroup takes the
// next tile ticket (tiles are taken in order by running workgroups, so a
// predecessor never waits on an unscheduled one), counts its kept slots,
// publishes the count, walks back over its predecessors' published values to
// its exclusive prefix and publishes the inclusive one. Status words carry
// the launch epoch: words of earlier launches read as "not yet published".
constexpr unsigned long long kScanAggregate = 1ull << 30;
constexpr unsigned long long kScanInclusive = 2ull << 30;
constexpr unsigned long long kScanCountMask = (1ull << 30) - 1;

__device__ __forceinline__ void scan_publish(const ScanState& st, int tile,
                                             unsigned long long flag, int value) {
  const unsigned long long w =
      (static_cast<unsigned long long>(st.epoch) << 32) | flag | static_cast<unsigned>(value);
  __hip_atomic_store(st.status + tile, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Thread 0 only: the exclusive prefix of `tile`, whose own count is `count`.
__device__ int scan_look_back(const ScanState& st, int tile, int count) {
  if (tile == 0) {
    scan_publish(st, 0, kScanInclusive, count);
    return 0;
  }
  scan_publish(st, tile, kScanAggregate, count);
  int prefix = 0;
  const uint64_t t0 = wall_clock64();  // 100 MHz
  for (int j = tile - 1; j >= 0;) {
    const unsigned long long w =
        __hip_atomic_load(st.status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long flag = w & (3ull << 30);
    if ((w >> 32) != st.epoch || flag == 0) {
      if (wall_clock64() - t0 > 20000000) {  // 0.2 s: never expected; the host fails loudly
        if (st.fail != nullptr) {
          __hip_atomic_store(st.fail, tile + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    prefix += static_cast<int>(w & kScanCountMask);
    if (flag == kScanInclusive) break;
    --j;
  }
  scan_publish(st, tile, kScanInclusive, prefix + count);
  return prefix;
}

// Block-wide exclusive scan of one int per thread (kScanThreads threads).
__device__ __forceinline__ int scan_block_exclusive(int c, int* total, int* lds_waves) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  int x = c;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int y = __shfl_up(x, off, kWave);
    if (lane >= off) x += y;
  }
  if (lane == kWave - 1) lds_waves[wave] = x;
  __syncthreads();
  int before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kScanThreads / kWave; ++w) {
    const int v = lds_waves[w];
    before += w < wave ? v : 0;
    all += v;
  }
  *total = all;
  return before + x - c;
}

__device__ __forceinline__ int scan_take_tile(const ScanState& st, int* lds_tile) {
  if (threadIdx.x == 0) *lds_tile = static_cast<int>(atomicAdd(st.ticket, 1u));
  __syncthreads();
  return *lds_tile;
}

// The last workgroup to finish rewinds the tickets for the next launch.
__device__ __forceinline__ void scan_finish(const ScanState& st) {
  if (threadIdx.x == 0) {
    const unsigned int done = atomicAdd(st.ticket + 1, 1u);
    if (done == gridDim.x - 1) {
      __hip_atomic_store(st.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(st.ticket + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ __launch_bounds__(kScanThreads) void compact_flags_kernel(
    const uint8_t* flags, int n, const double* coeff, int32_t* list, double* vals, int* count,
    int32_t* host_list, double* host_vals, int* host_count, ScanState st) {
  __shared__ int lds_tile, lds_prefix;
  __shared__ int lds_waves[kScanThreads / kWave];
  const int tile = scan_take_tile(st, &lds_tile);
  const int base = tile * kScanTile + threadIdx.x * kScanItems;
  // Eight flag bytes per thread in one load when the slice is whole.
  unsigned keep = 0;
  if (base + kScanItems <= n) {
    const uint2 f = *reinterpret_cast<const uint2*>(flags + base);
#pragma unroll
    for (int i = 0; i < 4; ++i) keep |= ((f.x >> (8 * i)) & 0xff) ? (1u << i) : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) keep |= ((f.y >> (8 * i)) & 0xff) ? (1u << (4 + i)) : 0u;
  } else {
    for (int i = 0; i < kScanItems; ++i) {
      if (base + i < n && flags[base + i] != 0) keep |= 1u << i;
    }
  }
  int total;
  const int excl = scan_block_exclusive(__popc(keep), &total, lds_waves);
  if (threadIdx.x == 0) lds_prefix = scan_look_back(st, tile, total);
  __syncthreads();
  int pos = lds_prefix + excl;
  while (keep != 0) {
    const int i = __ffs(keep) - 1;
    keep &= keep - 1;
    const int slot = base + i;
    const double v = coeff[slot];
    list[pos] = slot;
    vals[pos] = v;
    if (host_list != nullptr) {  // zero-copy readback into mapped host memory
      host_list[pos] = slot;
      host_vals[pos] = v;
    }
    ++pos;
  }
  if (tile == static_cast<int>(gridDim.x) - 1 && threadIdx.x == 0) {
    const int all = lds_prefix + total;
    *count = all;
    if (host_count != nullptr) *host_count = all;
  }
  scan_finish(st);
}

// ---------------------------------------------------------------------------
// Row-wise update row (update_row.cc:196-280). The filtered non-zeros of rho
// (ascending rows) are merged column-chunk by column-chunk: a workgroup owns
// kChunk consecutive columns of the update row, and walks the CSR rows of the
// transposed matrix in increasing order, binary-searching the first entry in
// its chunk. Each column therefore receives its contributions in increasing
// row order, as in the host scatter loops. Accumulators live in LDS.
constexpr int kChunk = 256;


__global__ __launch_bounds__(256) void row_wise_update_kernel(RowWiseArgs a) {
  __shared__ double acc[kChunk];
  __shared__ uint8_t touched[kChunk];
  const int c0 = blockIdx.x * kChunk;
  const int c1 = min(c0 + kChunk, a.num_cols);
  for (int i = threadIdx.x; i < kChunk; i += blockDim.x) {
    acc[i] = 0.0;
    touched[i] = 0;
  }
  __syncthreads();
  for (int k = 0; k < a.num_filtered; ++k) {
    const int r = a.filtered_rows[k];
    const double multiplier = a.rho[k];  // compacted: rho values of filtered rows
    int64_t lo = a.t_starts[r];
    int64_t hi = a.t_starts[r + 1];
    // lower_bound of c0 within the row (all threads compute the same value).
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (a.t_cols[mid] < c0) lo = mid + 1; else hi = mid;
    }
    const int64_t row_end = a.t_starts[r + 1];
    for (int64_t i = lo + threadIdx.x; i < row_end; i += blockDim.x) {
      const int pos = a.t_cols[i];
      if (pos >= c1) break;
      const double v = multiplier * a.t_vals[i];
      const int l = pos - c0;
      if (a.algorithm == 0) {
        acc[l] = v;  // single row: one contribution per position
      } else if (a.algorithm == 1) {
        acc[l] = touched[l] ? acc[l] + v : v;  // hypersparse: first is assigned
      } else {
        acc[l] = touched[l] ? acc[l] + v : 0.0 + v;  // row-wise: 0.0 += v
      }
      touched[l] = 1;
    }
    __syncthreads();  // rows are applied in order
  }
  for (int l = threadIdx.x; l < c1 - c0; l += blockDim.x) {
    const int pos = c0 + l;
    const double v = acc[l];
    const bool rel = bit_set(a.relevant, pos);
    bool listed;
    if (a.algorithm == 0) {
      listed = touched[l] && rel && fabs(v) > a.drop_tolerance;
      if (listed) a.coefficient[pos] = v;
    } else if (a.algorithm == 1) {
      listed = touched[l] && rel && fabs(v) > a.drop_tolerance;
      if (touched[l]) a.coefficient[pos] = v;
    } else {
      listed = rel && fabs(v) > a.drop_tolerance;
      a.coefficient[pos] = touched[l] ? v : 0.0;
    }
    a.flags[pos] = listed ? 1 : 0;
  }
}

// ---------------------------------------------------------------------------
// Small LPs: the row-wise update row, its epilogue and the compaction in one
// workgroup and one launch (RowWiseSmallArgs), with no copies: for LPs with a
// few thousand columns the queue latency per operation, not the bytes, bounds
// an iteration, and a serial walk over global memory would pay a memory
// round trip per row. So every global load is issued in one of two parallel
// waves (row extents, then all entries, products formed on the way), the
// accumulation runs out of LDS, and the list goes straight to mapped host
// memory. Arithmetic as row_wise_update_kernel: the rows are applied in list
// order with a barrier between rows (a position appears once per row, so one
// thread owns it within a row), with the same first-write rule per algorithm.
template <int THREADS>
__device__ __forceinline__ void row_wise_small_body(const RowWiseSmallArgs& a) {
  __shared__ double acc[kSmallLdsCols];
  __shared__ uint8_t touched[kSmallLdsCols];
  __shared__ uint64_t rel[kSmallLdsCols / 64];
  __shared__ int32_t ent_pos[kSmallEntries];
  __shared__ double ent_val[kSmallEntries];
  __shared__ double s_rho[kSmallRowsMax];
  __shared__ int64_t s_off[kSmallRowsMax];
  __shared__ int s_beg[kSmallRowsMax + 1];
  __shared__ int sums[THREADS];
  const int t = threadIdx.x;
  const int n = a.num_cols;
  const int k_rows = a.num_filtered;
  for (int i = t; i < n; i += THREADS) touched[i] = 0;
  for (int w = t; w < (n + 63) / 64; w += THREADS) rel[w] = a.relevant[w];
  // Wave 1: row extents (one row per thread; k_rows <= THREADS).
  int len = 0;
  if (t < k_rows) {
    const int r = a.filtered_rows[t];
    s_rho[t] = a.rho[t];
    const int64_t b = a.t_starts[r];
    s_off[t] = b;
    len = static_cast<int>(a.t_starts[r + 1] - b);
  }
  sums[t] = len;
  __syncthreads();
  for (int off = 1; off < THREADS; off <<= 1) {
    const int v = t >= off ? sums[t - off] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  if (t < k_rows) s_beg[t] = sums[t] - len;
  if (t == 0) s_beg[k_rows] = sums[THREADS - 1];
  __syncthreads();
  // Wave 2: every entry of every filtered row, product rho_k * A[r_k, pos].
  const int num_entries = s_beg[k_rows];  // <= kSmallEntries (host-checked)
  for (int e = t; e < num_entries; e += THREADS) {
    int lo = 0;
    int hi = k_rows - 1;
    while (lo < hi) {  // last row k with s_beg[k] <= e
      const int mid = (lo + hi + 1) >> 1;
      if (s_beg[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const int64_t i = s_off[lo] + (e - s_beg[lo]);
    ent_pos[e] = a.t_cols[i];
    ent_val[e] = s_rho[lo] * a.t_vals[i];
  }
  __syncthreads();
  for (int k = 0; k < k_rows; ++k) {
    for (int e = s_beg[k] + t; e < s_beg[k + 1]; e += THREADS) {
      const int pos = ent_pos[e];
      const double v = ent_val[e];
      double out;
      if (a.algorithm == 0) {
        out = v;
      } else if (!touched[pos]) {
        out = a.algorithm == 2 ? 0.0 + v : v;
      } else {
        out = acc[pos] + v;
      }
      acc[pos] = out;
      touched[pos] = 1;
    }
    __syncthreads();  // rows are applied in order
  }
  // Epilogue over this thread's slice of positions (<= 32 with N <= 8192).
  const int per = (n + THREADS - 1) / THREADS;
  const int b = min(n, t * per);
  const int e = min(n, b + per);
  uint32_t listed_bits = 0;
  int c = 0;
  for (int pos = b; pos < e; ++pos) {
    const bool was_touched = touched[pos] != 0;
    const double v = was_touched ? acc[pos] : 0.0;
    const bool is_rel = (rel[pos >> 6] >> (pos & 63)) & 1ull;
    bool listed;
    if (a.algorithm == 0) {
      listed = was_touched && is_rel && fabs(v) > a.drop_tolerance;
      if (listed) a.coefficient[pos] = v;
    } else if (a.algorithm == 1) {
      listed = was_touched && is_rel && fabs(v) > a.drop_tolerance;
      if (was_touched) a.coefficient[pos] = v;
    } else {
      listed = is_rel && fabs(v) > a.drop_tolerance;
      a.coefficient[pos] = was_touched ? v : 0.0;
    }
    a.flags[pos] = listed ? 1 : 0;
    listed_bits |= uint32_t(listed) << (pos - b);
    c += listed;
  }
  __syncthreads();
  sums[t] = c;
  __syncthreads();
  for (int off = 1; off < THREADS; off <<= 1) {
    const int v = t >= off ? sums[t - off] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  int out_pos = sums[t] - c;
  for (int pos = b; pos < e; ++pos) {
    if ((listed_bits >> (pos - b)) & 1u) {
      const double v = acc[pos];  // a listed position was touched: its value
      a.list[out_pos] = pos;
      a.vals[out_pos] = v;
      a.host_list[out_pos] = pos;
      a.host_vals[out_pos] = v;
      ++out_pos;
    }
  }
  if (t == THREADS - 1) {
    *a.count = sums[t];
    *a.host_count = sums[t];
  }
}

template <int THREADS>
__global__ __launch_bounds__(THREADS) void row_wise_small_kernel(RowWiseSmallArgs a) {
  row_wise_small_body<THREADS>(a);
}

// Medium LPs (N <= kMediumCols): row_wise_small_body's algorithm with the
// accumulators in an LDS hash table instead of an N-sized LDS array. A request
// has at most kSmallEntries entries, so at most that many positions are
// touched; kMediumSlots > kSmallEntries slots with linear probing always find
// a free slot or the key. The slots are assigned before the row loop, so the
// rows are applied in turn out of LDS with a barrier between rows, exactly as
// the small kernel does (same arithmetic, order and first-write rule). The
// epilogue looks positions up in the table: flags and coefficients
// position-interleaved (coalesced), the listed bits into LDS, then thread t
// compacts word t, so the list is in increasing position order.
constexpr int kMediumSlots = 5120;
static_assert(kMediumSlots > kSmallEntries, "the table must never fill");

// Multiplicative hash, mapped to [0, kMediumSlots) by its high bits (a
// modulo of the low bits would send positions equal mod 1024 to the same 5
// home slots: long probe runs).
__device__ __forceinline__ int medium_hash(int pos) {
  const uint32_t h = static_cast<uint32_t>(pos) * 2654435761u;
  return static_cast<int>((static_cast<uint64_t>(h) * kMediumSlots) >> 32);
}

// Slot holding `pos`, or -1. Probes end at an empty slot or after every slot.
__device__ __forceinline__ int medium_find(const int32_t* keys, int pos) {
  int sl = medium_hash(pos);
  for (int i = 0; i < kMediumSlots; ++i) {
    const int k = keys[sl];
    if (k == pos) return sl;
    if (k < 0) return -1;
    sl = sl + 1 == kMediumSlots ? 0 : sl + 1;
  }
  return -1;
}

__device__ __forceinline__ void row_wise_medium_body(const RowWiseSmallArgs& a) {
  constexpr int THREADS = kCompactThreads;
  __shared__ int32_t keys[kMediumSlots];
  __shared__ double acc[kMediumSlots];
  __shared__ uint8_t written[kMediumSlots];
  __shared__ uint64_t rel[kMediumCols / 64];
  __shared__ unsigned long long listed_w[kMediumCols / 64];
  __shared__ unsigned long long touched_w[kMediumCols / 64];  // positions in the table
  __shared__ int16_t ent_slot[kSmallEntries];
  __shared__ double ent_val[kSmallEntries];
  __shared__ double s_rho[kSmallRowsMax];
  __shared__ int64_t s_off[kSmallRowsMax];
  __shared__ int s_beg[kSmallRowsMax + 1];
  __shared__ int sums[THREADS];
  const int t = threadIdx.x;
  const int n = a.num_cols;
  const int k_rows = a.num_filtered;
  for (int i = t; i < kMediumSlots; i += THREADS) {
    keys[i] = -1;
    written[i] = 0;
  }
  for (int w = t; w < (n + 63) / 64; w += THREADS) {
    rel[w] = a.relevant[w];
    listed_w[w] = 0;
    touched_w[w] = 0;
  }
  int len = 0;
  if (t < k_rows) {
    const int r = a.filtered_rows[t];
    s_rho[t] = a.rho[t];
    const int64_t b = a.t_starts[r];
    s_off[t] = b;
    len = static_cast<int>(a.t_starts[r + 1] - b);
  }
  sums[t] = len;
  __syncthreads();
  for (int off = 1; off < THREADS; off <<= 1) {
    const int v = t >= off ? sums[t - off] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  if (t < k_rows) s_beg[t] = sums[t] - len;
  if (t == 0) s_beg[k_rows] = sums[THREADS - 1];
  __syncthreads();
  const int num_entries = s_beg[k_rows];  // <= kSmallEntries (host-checked)
  for (int e = t; e < num_entries; e += THREADS) {
    int lo = 0;
    int hi = k_rows - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_beg[mid] <= e) lo = mid; else hi = mid - 1;
    }
    const int64_t i = s_off[lo] + (e - s_beg[lo]);
    const int pos = a.t_cols[i];
    ent_val[e] = s_rho[lo] * a.t_vals[i];
    int sl = medium_hash(pos);
    for (int probe = 0; probe < kMediumSlots; ++probe) {
      const int old = atomicCAS(&keys[sl], -1, pos);
      if (old == -1 || old == pos) break;
      sl = sl + 1 == kMediumSlots ? 0 : sl + 1;
    }
    ent_slot[e] = static_cast<int16_t>(sl);
    atomicOr(&touched_w[pos >> 6], 1ull << (pos & 63));
  }
  __syncthreads();
  for (int k = 0; k < k_rows; ++k) {
    for (int e = s_beg[k] + t; e < s_beg[k + 1]; e += THREADS) {
      const int sl = ent_slot[e];
      const double v = ent_val[e];
      double out;
      if (a.algorithm == 0) {
        out = v;
      } else if (!written[sl]) {
        out = a.algorithm == 2 ? 0.0 + v : v;
      } else {
        out = acc[sl] + v;
      }
      acc[sl] = out;
      written[sl] = 1;
    }
    __syncthreads();  // rows are applied in order
  }
  for (int pos = t; pos < n; pos += THREADS) {
    // Only positions an entry touched are in the table: the others skip the
    // probe (it would walk to an empty slot).
    const bool in_table = (touched_w[pos >> 6] >> (pos & 63)) & 1ull;
    const int sl = in_table ? medium_find(keys, pos) : -1;
    const bool was_touched = sl >= 0 && written[sl] != 0;
    const double v = was_touched ? acc[sl] : 0.0;
    const bool is_rel = (rel[pos >> 6] >> (pos & 63)) & 1ull;
    bool listed;
    if (a.algorithm == 0) {
      listed = was_touched && is_rel && fabs(v) > a.drop_tolerance;
      if (listed) a.coefficient[pos] = v;
    } else if (a.algorithm == 1) {
      listed = was_touched && is_rel && fabs(v) > a.drop_tolerance;
      if (was_touched) a.coefficient[pos] = v;
    } else {
      listed = is_rel && fabs(v) > a.drop_tolerance;
      a.coefficient[pos] = was_touched ? v : 0.0;
    }
    a.flags[pos] = listed ? 1 : 0;
    if (listed) atomicOr(&listed_w[pos >> 6], 1ull << (pos & 63));
  }
  __syncthreads();
  const uint64_t mine = t < (n + 63) / 64 ? listed_w[t] : 0ull;
  const int c = __popcll(mine);
  sums[t] = c;
  __syncthreads();
  for (int off = 1; off < THREADS; off <<= 1) {
    const int v = t >= off ? sums[t - off] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  int out_pos = sums[t] - c;
  for (uint64_t bits = mine; bits != 0; bits &= bits - 1) {
    const int pos = t * 64 + __builtin_ctzll(bits);
    const double v = acc[medium_find(keys, pos)];  // a listed position was touched
    a.list[out_pos] = pos;
    a.vals[out_pos] = v;
    a.host_list[out_pos] = pos;
    a.host_vals[out_pos] = v;
    ++out_pos;
  }
  if (t == THREADS - 1) {
    *a.count = sums[t];
    *a.host_count = sums[t];
  }
}

static_assert(kMediumCols == 64 * kCompactThreads, "one listed word per thread");

__global__ __launch_bounds__(kCompactThreads) void row_wise_medium_kernel(RowWiseSmallArgs a) {
  row_wise_medium_body(a);
}

// Small LPs: the column-wise update row (with the primal edge-norm dots when
// w is given) and its compaction in one launch (ColWiseSmallArgs). Per column
// the arithmetic and the write rule are column_dot_kernel's: kept columns
// (relevant, |rho.a_j| > drop) get coefficient and w.a_j, the others keep their
// stale coefficient. One thread per column (thread_column_dot).
__device__ __forceinline__ void column_wise_small_body(const ColWiseSmallArgs& a) {
  __shared__ double s_y[kSmallColWiseRows];
  __shared__ double s_w[kSmallColWiseRows];
  __shared__ uint8_t keep_flag[kSmallLdsCols];
  __shared__ int sums[kCompactThreads];
  const int t = threadIdx.x;
  const int n = a.num_cols;
  const bool with_dots = a.w != nullptr;
  for (int i = t; i < a.m; i += kCompactThreads) {
    s_y[i] = a.rho[i];
    if (with_dots) s_w[i] = a.w[i];
  }
  __syncthreads();
  for (int col = t; col < n; col += kCompactThreads) {
    const bool active = bit_set(a.relevant, col);
    const int64_t s = a.starts[col];
    const int64_t e = active ? a.starts[col + 1] : s;
    const double dot = thread_column_dot(s, e, a.rows, a.vals, s_y);
    const bool keep = active && fabs(dot) > a.drop_tolerance;
    a.flags[col] = keep ? 1 : 0;
    keep_flag[col] = keep ? 1 : 0;
    if (keep) {
      a.coefficient[col] = dot;
      if (with_dots) a.out2[col] = thread_column_dot(s, e, a.rows, a.vals, s_w);
    }
  }
  __syncthreads();
  const int per = (n + kCompactThreads - 1) / kCompactThreads;
  const int b = min(n, t * per);
  const int e = min(n, b + per);
  int c = 0;
  for (int pos = b; pos < e; ++pos) c += keep_flag[pos];
  sums[t] = c;
  __syncthreads();
  for (int off = 1; off < kCompactThreads; off <<= 1) {
    const int v = t >= off ? sums[t - off] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  int out_pos = sums[t] - c;
  for (int pos = b; pos < e; ++pos) {
    if (keep_flag[pos]) {
      const double v = a.coefficient[pos];  // written above by this workgroup
      a.list[out_pos] = pos;
      a.vals_out[out_pos] = v;
      a.host_list[out_pos] = pos;
      a.host_vals[out_pos] = v;
      if (with_dots) a.host_dots[out_pos] = a.out2[pos];
      ++out_pos;
    }
  }
  if (t == kCompactThreads - 1) {
    *a.count = sums[t];
    *a.host_count = sums[t];
  }
}

__global__ __launch_bounds__(kCompactThreads) void column_wise_small_kernel(ColWiseSmallArgs a) {
  column_wise_small_body(a);
}

// Small LPs: the primal edge-norm dots over the update-row list in one launch
// (ListDotsSmallArgs), one thread per listed column; y (m <= kRows) in LDS.
template <int kRows>
__device__ __forceinline__ void list_dots_body(const ListDotsSmallArgs& a) {
  __shared__ double s_y[kRows];
  const int t = threadIdx.x;
  for (int i = t; i < a.m; i += kCompactThreads) s_y[i] = a.y[i];
  __syncthreads();
  for (int slot = t; slot < a.n; slot += kCompactThreads) {
    const int col = a.list[slot];
    a.out[slot] = thread_column_dot(a.starts[col], a.starts[col + 1], a.rows, a.vals, s_y);
  }
}

__global__ __launch_bounds__(kCompactThreads) void list_dots_small_kernel(ListDotsSmallArgs a) {
  list_dots_body<kSmallLdsCols>(a);
}

// Mid-size LPs (kSmallLdsCols < m <= kMediumListRows): the same with 128 KB of y.
__global__ __launch_bounds__(kCompactThreads) void list_dots_medium_kernel(ListDotsSmallArgs a) {
  list_dots_body<kMediumListRows>(a);
}

// ---------------------------------------------------------------------------
// The row-wise update row for many filtered rows, one thread per column.
// Per column the result must be the host scatter's: contributions
// rho_k * A[r_k, j] accumulated in the order k of the filtered list (which
// need not be ascending in r). The thread collects its column's filtered
// entries (a CSC column holds ~nnz/N of them), orders them by k with an
// in-register insertion sort, and accumulates in that order with the same
// first-write rule as row_wise_update_kernel. Columns with more than
// kMaxColumnHits filtered entries fall back to repeated minimum selection.
constexpr int kMaxColumnHits = 32;  // = DeviceLp::kColumnKernelMaxColumnLength

__device__ __forceinline__ double row_wise_accumulate(double acc, bool first, double v,
                                                      int algorithm) {
  if (!first) return acc + v;
  return algorithm == 2 ? 0.0 + v : v;  // AssignToZero then +=, or first assign
}

// Per-column accumulation of the row-wise update row from the CSC copy:
// k_of(r) = list position of row r, or -1 if r is not filtered. The hits are
// ordered by k (insertion in registers, or repeated minimum selection past
// kMaxColumnHits) and accumulated with the first-write rule of the algorithm.
template <typename KOf>
__device__ __forceinline__ double column_hits_accumulate(int64_t s, int64_t e,
                                                         const int32_t* rows,
                                                         const double* vals,
                                                         const double* rho, KOf k_of,
                                                         int algorithm, bool* touched) {
  int hits = 0;
  for (int64_t i = s; i < e; ++i) hits += k_of(rows[i]) >= 0 ? 1 : 0;
  double acc = 0.0;
  if (hits > 0 && hits <= kMaxColumnHits) {
    int ks[kMaxColumnHits];
    double vs[kMaxColumnHits];
    int c = 0;
    for (int64_t i = s; i < e; ++i) {
      const int k = k_of(rows[i]);
      if (k < 0) continue;
      const double v = rho[k] * vals[i];
      int p = c;
#pragma unroll
      for (int q = kMaxColumnHits - 1; q > 0; --q) {
        if (q <= c && ks[q - 1] > k) {
          ks[q] = ks[q - 1];
          vs[q] = vs[q - 1];
          p = q - 1;
        }
      }
#pragma unroll
      for (int q = 0; q < kMaxColumnHits; ++q) {
        if (q == p) {
          ks[q] = k;
          vs[q] = v;
        }
      }
      ++c;
    }
#pragma unroll
    for (int q = 0; q < kMaxColumnHits; ++q) {
      if (q < c) acc = row_wise_accumulate(acc, q == 0, vs[q], algorithm);
    }
  } else if (hits > kMaxColumnHits) {
    int last = -1;
    for (int h = 0; h < hits; ++h) {
      int best_k = 0x7fffffff;
      double best_v = 0.0;
      for (int64_t i = s; i < e; ++i) {
        const int k = k_of(rows[i]);
        if (k > last && k < best_k) {
          best_k = k;
          best_v = rho[k] * vals[i];
        }
      }
      acc = row_wise_accumulate(acc, h == 0, best_v, algorithm);
      last = best_k;
    }
  }
  *touched = hits > 0;
  return acc;
}

// The update-row write rule per algorithm (update_row.cc:196-280); returns
// whether the position is listed.
__device__ __forceinline__ bool row_wise_store(int algorithm, bool touched, bool rel, double acc,
                                               double drop_tolerance, double* coefficient,
                                               int col) {
  bool listed;
  if (algorithm == 0) {
    listed = touched && rel && fabs(acc) > drop_tolerance;
    if (listed) coefficient[col] = acc;
  } else if (algorithm == 1) {
    listed = touched && rel && fabs(acc) > drop_tolerance;
    if (touched) coefficient[col] = acc;
  } else {
    listed = rel && fabs(acc) > drop_tolerance;
    coefficient[col] = touched ? acc : 0.0;
  }
  return listed;
}

__global__ __launch_bounds__(256) void row_wise_by_column_kernel(RowWiseColArgs a) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= a.num_cols) return;
  auto k_of = [&](int r) { return a.row_tag[r] == a.tag ? a.row_pos[r] : -1; };
  bool touched = false;
  const double acc = column_hits_accumulate(a.starts[col], a.starts[col + 1], a.rows, a.vals,
                                            a.rho, k_of, a.algorithm, &touched);
  const bool listed = row_wise_store(a.algorithm, touched, bit_set(a.relevant, col), acc,
                                     a.drop_tolerance, a.coefficient, col);
  a.flags[col] = listed ? 1 : 0;
}

// Small LPs with many filtered rows: the same per-column accumulation in one
// workgroup (row positions in LDS instead of the tag pass), then the
// compaction into mapped host memory, as row_wise_small_kernel.
__device__ __forceinline__ void row_wise_small_by_column_body(const RowWiseSmallColArgs& a) {
  __shared__ int32_t s_pos[kSmallLdsCols];
  __shared__ double s_rho[kSmallLdsCols];
  __shared__ uint64_t rel[kSmallLdsCols / 64];
  __shared__ int sums[kCompactThreads];
  const int t = threadIdx.x;
  const int n = a.num_cols;
  for (int r = t; r < a.m; r += kCompactThreads) s_pos[r] = -1;
  for (int w = t; w < (n + 63) / 64; w += kCompactThreads) rel[w] = a.relevant[w];
  __syncthreads();
  for (int k = t; k < a.num_filtered; k += kCompactThreads) {
    s_pos[a.filtered_rows[k]] = k;
    s_rho[k] = a.rho[k];
  }
  __syncthreads();
  auto k_of = [&](int r) { return s_pos[r]; };
  const int per = (n + kCompactThreads - 1) / kCompactThreads;
  const int b = min(n, t * per);
  const int e = min(n, b + per);
  uint32_t listed_bits = 0;
  int c = 0;
  for (int col = b; col < e; ++col) {
    bool touched = false;
    const double acc = column_hits_accumulate(a.starts[col], a.starts[col + 1], a.rows, a.vals,
                                              s_rho, k_of, a.algorithm, &touched);
    const bool is_rel = (rel[col >> 6] >> (col & 63)) & 1ull;
    const bool listed = row_wise_store(a.algorithm, touched, is_rel, acc, a.drop_tolerance,
                                       a.coefficient, col);
    a.flags[col] = listed ? 1 : 0;
    listed_bits |= uint32_t(listed) << (col - b);
    c += listed;
  }
  sums[t] = c;
  __syncthreads();
  for (int off = 1; off < kCompactThreads; off <<= 1) {
    const int v = t >= off ? sums[t - off] : 0;
    __syncthreads();
    sums[t] += v;
    __syncthreads();
  }
  int out_pos = sums[t] - c;
  for (int col = b; col < e; ++col) {
    if ((listed_bits >> (col - b)) & 1u) {
      const double v = a.coefficient[col];  // this thread's own store above
      a.list[out_pos] = col;
      a.list_vals[out_pos] = v;
      a.host_list[out_pos] = col;
      a.host_vals[out_pos] = v;
      ++out_pos;
    }
  }
  if (t == kCompactThreads - 1) {
    *a.count = sums[t];
    *a.host_count = sums[t];
  }
}

__global__ __launch_bounds__(kCompactThreads) void row_wise_small_by_column_kernel(
    RowWiseSmallColArgs a) {
  row_wise_small_by_column_body(a);
}

// ---------------------------------------------------------------------------
// Batched small-LP launches: one workgroup per request of many LPs (one launch
// instead of one per LP; the HIP launch path, not the GPU, bounds many
// concurrent small LPs). A request's arguments sit in a slot of mapped host
// memory; the workgroup stages them through LDS once, runs the same body as
// the single launch, then publishes its slot's sequence number (system
// scope, after a system fence: the results are visible to the host and to
// later launches on other streams when the host sees the number).
template <int KIND>
__global__ __launch_bounds__(kCompactThreads) void small_batch_kernel(SmallBatchArgs b) {
  __shared__ SmallSlot s_slot;
  const SmallSlot* src = b.slots + b.ids[blockIdx.x];
  {
    const uint32_t* from = reinterpret_cast<const uint32_t*>(src);
    uint32_t* to = reinterpret_cast<uint32_t*>(&s_slot);
    for (int i = threadIdx.x; i < int(sizeof(SmallSlot) / 4); i += blockDim.x) to[i] = from[i];
  }
  __syncthreads();
  if constexpr (KIND == kSmallRowWise) {
    const RowWiseSmallArgs a = s_slot.rw;
    row_wise_small_body<kCompactThreads>(a);
  } else if constexpr (KIND == kSmallColWise) {
    const ColWiseSmallArgs a = s_slot.cw;
    column_wise_small_body(a);
  } else if constexpr (KIND == kMediumRowWise) {
    const RowWiseSmallArgs a = s_slot.rw;
    row_wise_medium_body(a);
  } else if constexpr (KIND == kSmallListDots) {
    const ListDotsSmallArgs a = s_slot.ld;
    list_dots_body<kSmallLdsCols>(a);
  } else if constexpr (KIND == kMediumListDots) {
    const ListDotsSmallArgs a = s_slot.ld;
    list_dots_body<kMediumListRows>(a);
  } else {
    const RowWiseSmallColArgs a = s_slot.rc;
    row_wise_small_by_column_body(a);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(b.done + b.ids[blockIdx.x], s_slot.seq, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------------------
// Row-wise update row over full rows (config 2's dense A). A thread owns one
// column and reads that column's entry of each filtered row directly (no
// search): lanes of a wave read consecutive entries of one CSR row, and the
// row start (uploaded per filtered row) and rho value are wave-uniform
// (scalar loads). The loads of
// kFullRowsUnroll rows are in flight before their products are accumulated,
// in list order k, with the first-write rule of row_wise_update_kernel.
constexpr int kFullRowsUnroll = 16;

__global__ __launch_bounds__(256) void row_wise_full_rows_kernel(RowWiseFullArgs a) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= a.num_cols) return;
  double acc = 0.0;
  bool touched = false;
  if (col < a.num_structural) {
    const int num = a.num_filtered;
    int k = 0;
    for (; k + kFullRowsUnroll <= num; k += kFullRowsUnroll) {
      double v[kFullRowsUnroll];
#pragma unroll
      for (int u = 0; u < kFullRowsUnroll; ++u) {
        v[u] = a.t_vals[a.row_offsets[k + u] + col];
      }
#pragma unroll
      for (int u = 0; u < kFullRowsUnroll; ++u) {
        acc = row_wise_accumulate(acc, !touched, a.rho[k + u] * v[u], a.algorithm);
        touched = true;
      }
    }
    for (; k < num; ++k) {
      acc = row_wise_accumulate(acc, !touched, a.rho[k] * a.t_vals[a.row_offsets[k] + col],
                                a.algorithm);
      touched = true;
    }
  } else {
    const int r = col - a.num_structural;
    if (a.row_tag[r] == a.tag) {
      const int k = a.row_pos[r];
      acc = row_wise_accumulate(0.0, true, a.rho[k] * a.t_vals[a.t_starts[r + 1] - 1],
                                a.algorithm);
      touched = true;
    }
  }
  const bool rel = bit_set(a.relevant, col);
  bool listed;
  if (a.algorithm == 0) {
    listed = touched && rel && fabs(acc) > a.drop_tolerance;
    if (listed) a.coefficient[col] = acc;
  } else if (a.algorithm == 1) {
    listed = touched && rel && fabs(acc) > a.drop_tolerance;
    if (touched) a.coefficient[col] = acc;
  } else {
    listed = rel && fabs(acc) > a.drop_tolerance;
    a.coefficient[col] = touched ? acc : 0.0;
  }
  a.flags[col] = listed ? 1 : 0;
}

__global__ void tag_rows_kernel(const int32_t* filtered_rows, int n, uint32_t tag,
                                uint32_t* row_tag, int32_t* row_pos) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const int r = filtered_rows[k];
    row_tag[r] = tag;
    row_pos[r] = k;
  }
}

// ---------------------------------------------------------------------------
// Dual device mode: the bound-flipping ratio test filter, the reduced-cost
// update and the boxed dual-feasibility decisions where the update row and
// the reduced costs already are.

// One update-row slot as a breakpoint candidate (entering_variable.cc:68-96,
// same expressions): returns false if the slot is not eligible.
__device__ __forceinline__ bool dual_breakpoint(const DualRatioArgs& a, int slot, double* ratio,
                                                double* harris, bool* sets_bound,
                                                double* flip_delta = nullptr) {
  const int col = a.list[slot];
  const double c = a.list_coeff[slot];
  const double coeff = a.sign > 0.0 ? c : -c;
  const uint8_t bits = a.colbits[col];
  double reduced_cost, magnitude;
  if ((bits & kColCanDecrease) && coeff > a.threshold) {
    reduced_cost = -a.rc[col];
    magnitude = coeff;
  } else if ((bits & kColCanIncrease) && coeff < -a.threshold) {
    reduced_cost = a.rc[col];
    magnitude = -coeff;
  } else {
    return false;
  }
  *ratio = reduced_cost / magnitude;
  *harris = fmax(a.minimum_delta / magnitude, *ratio + a.harris_tolerance / magnitude);
  *sets_bound = !(bits & kColBoxed) || (a.bound_diff[col] * magnitude >= a.variation_magnitude);
  // Variation a bound flip of this breakpoint absorbs (0: not boxed).
  if (flip_delta != nullptr) *flip_delta = (bits & kColBoxed) ? a.bound_diff[col] * magnitude : 0.0;
  return true;
}

// Pass 1: B = min Harris ratio over the breakpoints that can never be bound
// flipped. In the host loop such a breakpoint, once popped, bounds the
// search by a value <= B, so no breakpoint with ratio > B is ever popped.
__global__ __launch_bounds__(256) void dual_ratio_bound_kernel(DualRatioArgs a) {
  __shared__ unsigned long long block_min[4];
  const int n = *a.count;
  // The other slot of the pair was last used by the previous call (ordered
  // before this launch): it starts the next call at "none", no memset.
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.best_next != nullptr) *a.best_next = ~0ull;
  unsigned long long best = ~0ull;
  for (int slot = blockIdx.x * blockDim.x + threadIdx.x; slot < n;
       slot += gridDim.x * blockDim.x) {
    double ratio, harris;
    bool sets_bound;
    if (dual_breakpoint(a, slot, &ratio, &harris, &sets_bound) && sets_bound) {
      const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(harris));
      best = b < best ? b : best;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_down(best, off, kWave);
    best = o < best ? o : best;
  }
  if ((threadIdx.x & 63) == 0) block_min[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = block_min[0];
    for (int w = 1; w < (blockDim.x >> 6); ++w) m = block_min[w] < m ? block_min[w] : m;
    if (m != ~0ull) atomicMin(a.best, m);
  }
}

// Pass 2 with its compaction: the kept slots come out in list order, their
// candidates go straight to host memory; the workgroup of the last list tile
// writes the counts. Grid: scan_tiles(max_count) tiles, those past the list
// length only take their ticket.
__global__ __launch_bounds__(kScanThreads) void dual_ratio_select_kernel(DualRatioArgs a,
                                                                         DualSelectOut out,
                                                                         ScanState st) {
  __shared__ int lds_tile, lds_prefix;
  __shared__ int lds_waves[kScanThreads / kWave];
  const int n = *a.count;
  const int tile = scan_take_tile(st, &lds_tile);
  const int last_tile = n > 0 ? (n - 1) / kScanTile : 0;
  if (tile <= last_tile) {
    const unsigned long long best = *a.bound;
    const double bound = best == ~0ull ? HUGE_VAL
                                       : __longlong_as_double(static_cast<long long>(best)) *
                                             (1.0 + 1e-9);
    const int base = tile * kScanTile + threadIdx.x * kScanItems;
    unsigned keep = 0;
    for (int i = 0; i < kScanItems; ++i) {
      double ratio, harris;
      bool sets_bound;
      if (base + i < n && dual_breakpoint(a, base + i, &ratio, &harris, &sets_bound) &&
          ratio <= bound) {
        keep |= 1u << i;
      }
    }
    int total;
    const int excl = scan_block_exclusive(__popc(keep), &total, lds_waves);
    if (threadIdx.x == 0) lds_prefix = scan_look_back(st, tile, total);
    __syncthreads();
    int pos = lds_prefix + excl;
    while (keep != 0) {
      const int i = __ffs(keep) - 1;
      keep &= keep - 1;
      const int slot = base + i;
      const int col = a.list[slot];
      out.slots[pos] = slot;
      if (pos < out.host_cap) {
        out.cand_col[pos] = col;
        out.cand_coeff[pos] = a.list_coeff[slot];
        out.cand_rc[pos] = a.rc[col];
      }
      ++pos;
    }
    if (tile == last_tile && threadIdx.x == 0) {
      const int all = lds_prefix + total;
      *out.num_slots = all;
      out.counts[0] = all;
      out.counts[1] = n;
    }
  }
  scan_finish(st);
}

__device__ __forceinline__ unsigned long long order_bits(double x) {
  const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(x));
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__global__ void dual_ratio_keys_kernel(DualRatioArgs a, const int32_t* slots, int num_slots,
                                       unsigned long long* keys) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < num_slots;
       i += gridDim.x * blockDim.x) {
    double ratio = 0.0, harris;
    bool sets_bound;
    dual_breakpoint(a, slots[i], &ratio, &harris, &sets_bound);
    keys[i] = order_bits(ratio);
  }
}

// One thread: entering_variable.cc:163-207 in pop order (ratio ascending;
// a ratio tie would also order by magnitude and column, so it falls back).
__global__ void dual_flip_walk_kernel(DualRatioArgs a, const int32_t* sorted_slots,
                                      int num_slots, unsigned long long* bound2) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  double variation = a.variation_magnitude;
  double prev_ratio = 0.0;
  for (int i = 0; i < num_slots; ++i) {
    double ratio, harris, delta;
    bool sets_bound;
    dual_breakpoint(a, sorted_slots[i], &ratio, &harris, &sets_bound, &delta);
    if (i > 0 && ratio == prev_ratio) break;  // tie: keep the looser bound
    prev_ratio = ratio;
    if (variation > 0.0 && delta > 0.0) {
      variation -= delta;
      if (variation > 0.0) continue;  // flipped
    }
    // First accepted breakpoint: it caps harris_ratio at its Harris ratio.
    if (i + 1 < num_slots) {
      double next_ratio, h2, d2;
      bool s2;
      dual_breakpoint(a, sorted_slots[i + 1], &next_ratio, &h2, &s2, &d2);
      if (next_ratio == ratio) break;
    }
    // harris_ratio <= min(B, its Harris ratio) from here on (B: pass 1).
    const unsigned long long h = static_cast<unsigned long long>(__double_as_longlong(harris));
    *bound2 = h < *a.best ? h : *a.best;
    bound2[1] = static_cast<unsigned long long>(i + 1);  // walk length (statistics)
    return;
  }
  *bound2 = *a.best;
  bound2[1] = static_cast<unsigned long long>(num_slots) | (1ull << 40);
}

// ---------------------------------------------------------------------------
// Tightening by selection. The walk above pops only the smallest few hundred
// breakpoints (MILP_TIGHTEN_STATS on config 5: walks of 4-255 steps over
// k1 = 512-300 000 candidates), so instead of sorting all k1 keys, two
// histogram passes find a threshold T with at least min(target, k1)
// keys <= T, and one workgroup gathers those (at most kTightenCap), sorts
// them in LDS and walks them as dual_flip_walk_kernel walks the whole sorted
// list. Its first steps see the same keys in the same order (equal keys end
// both walks at the same step whatever their order), so the bound is the
// full walk's -- unless the walk runs off the gathered prefix or accepts its
// last element (whose successor it cannot compare): then the bound stays B,
// and the second pass hands the host every candidate, as without tightening.

// Keys of the pass-2 slots; the state's histograms, ticket and results zeroed.
__global__ __launch_bounds__(256) void dual_tighten_keys_kernel(DualRatioArgs a,
                                                                const int32_t* slots,
                                                                int num_slots,
                                                                unsigned long long* keys,
                                                                TightenState* st) {
  const int stride = gridDim.x * blockDim.x;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned int* words = reinterpret_cast<unsigned int*>(st);
  constexpr int kWords = static_cast<int>(sizeof(TightenState) / sizeof(unsigned int));
  for (int w = tid; w < kWords; w += stride) words[w] = 0u;
  for (int i = tid; i < num_slots; i += stride) {
    double ratio = 0.0, harris;
    bool sets_bound;
    dual_breakpoint(a, slots[i], &ratio, &harris, &sets_bound);
    keys[i] = order_bits(ratio);
  }
}

// Pass 0: histogram of the keys' top 12 bits; pass 1: of bits 40-51 of the
// keys in the bin pass 0 chose. The last workgroup finds the bin where the
// count from below reaches min(target_keys, n).
__global__ __launch_bounds__(256) void dual_tighten_hist_kernel(const unsigned long long* keys,
                                                                int n, TightenState* st,
                                                                int pass, int target_keys) {
  __shared__ unsigned int h[kTightenBins];
  __shared__ int lds_waves[256 / kWave];
  __shared__ bool last;
  for (int b = threadIdx.x; b < kTightenBins; b += blockDim.x) h[b] = 0u;
  __syncthreads();
  const unsigned long long bin0 = pass == 0 ? 0ull : st->bin0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned long long k = keys[i];
    if (pass == 0) {
      atomicAdd(&h[k >> 52], 1u);
    } else if ((k >> 52) == bin0) {
      atomicAdd(&h[(k >> 40) & 0xfffull], 1u);
    }
  }
  __syncthreads();
  unsigned int* global = st->hist[pass];
  for (int b = threadIdx.x; b < kTightenBins; b += blockDim.x) {
    if (h[b] != 0u) atomicAdd(global + b, h[b]);
  }
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&st->ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
  // Thread t owns bins [16t, 16t + 16).
  constexpr int kPer = kTightenBins / 256;
  unsigned int mine[kPer];
  int sum = 0;
  for (int j = 0; j < kPer; ++j) {
    mine[j] = __hip_atomic_load(global + threadIdx.x * kPer + j, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
    sum += static_cast<int>(mine[j]);
  }
  int total;
  const int excl = scan_block_exclusive(sum, &total, lds_waves);
  const int target = n < target_keys ? n : target_keys;
  const int base = pass == 0 ? 0 : static_cast<int>(st->below0);
  int cum = base + excl;
  if (cum < target && target <= cum + sum) {
    for (int j = 0; j < kPer; ++j) {
      const int before = cum;
      cum += static_cast<int>(mine[j]);
      if (cum >= target) {
        const unsigned int b = threadIdx.x * kPer + j;
        if (pass == 0) {
          st->bin0 = b;
          st->below0 = static_cast<unsigned int>(before);
        } else {
          st->threshold = (bin0 << 52) | (static_cast<unsigned long long>(b) << 40) |
                          ((1ull << 40) - 1ull);
          st->count = static_cast<unsigned int>(cum);
        }
        break;
      }
    }
  }
  if (threadIdx.x == 0) __hip_atomic_store(&st->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(1024) void dual_tighten_walk_kernel(DualRatioArgs a,
                                                                 const int32_t* slots,
                                                                 const unsigned long long* keys,
                                                                 int num_slots,
                                                                 const TightenState* st,
                                                                 unsigned long long* bound2) {
  __shared__ unsigned long long s_key[kTightenCap];
  __shared__ int s_slot[kTightenCap];
  __shared__ double s_ratio[1024], s_harris[1024], s_delta[1024];
  __shared__ int s_n, s_done;
  const int tid = threadIdx.x;
  const unsigned long long best = *a.best;
  const unsigned long long threshold = st->threshold;
  const int count = static_cast<int>(st->count);
  if (count > kTightenCap) {
    if (tid == 0) {
      bound2[0] = best;
      bound2[1] = static_cast<unsigned long long>(count) | (2ull << 40);
    }
    return;
  }
  if (tid == 0) {
    s_n = 0;
    s_done = 0;
  }
  __syncthreads();
  for (int i = tid; i < num_slots; i += blockDim.x) {
    const unsigned long long k = keys[i];
    if (k <= threshold) {
      const int p = atomicAdd(&s_n, 1);
      if (p < kTightenCap) {
        s_key[p] = k;
        s_slot[p] = slots[i];
      }
    }
  }
  __syncthreads();
  const int n = s_n;
  if (n > kTightenCap) {  // never expected: the histograms counted these keys
    if (tid == 0) {
      bound2[0] = best;
      bound2[1] = static_cast<unsigned long long>(n) | (2ull << 40);
    }
    return;
  }
  int size = 1;
  while (size < n) size <<= 1;
  for (int i = n + tid; i < size; i += blockDim.x) {
    s_key[i] = ~0ull;
    s_slot[i] = -1;
  }
  __syncthreads();
  // Bitonic sort by key (ascending).
  for (int k = 2; k <= size; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < size; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const unsigned long long ki = s_key[i], kj = s_key[ixj];
          if ((ki > kj) == up) {
            s_key[i] = kj;
            s_key[ixj] = ki;
            const int t = s_slot[i];
            s_slot[i] = s_slot[ixj];
            s_slot[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  // The walk (dual_flip_walk_kernel's loop), 1024 breakpoints per round.
  double variation = a.variation_magnitude;
  double prev_ratio = 0.0;
  unsigned long long result = best;
  int steps = 0;
  for (int c0 = 0; c0 < n; c0 += 1024) {
    if (c0 + tid < n) {
      double r = 0.0, h = 0.0, d = 0.0;
      bool sb;
      dual_breakpoint(a, s_slot[c0 + tid], &r, &h, &sb, &d);
      s_ratio[tid] = r;
      s_harris[tid] = h;
      s_delta[tid] = d;
    }
    __syncthreads();
    if (tid == 0) {
      for (int jj = 0; jj < 1024 && c0 + jj < n; ++jj) {
        const int i = c0 + jj;
        const double ratio = s_ratio[jj];
        steps = i + 1;
        if (i > 0 && ratio == prev_ratio) {  // tie: B, as the full walk
          s_done = 1;
          break;
        }
        prev_ratio = ratio;
        const double delta = s_delta[jj];
        if (variation > 0.0 && delta > 0.0) {
          variation -= delta;
          if (variation > 0.0) continue;  // flipped
        }
        // First accepted breakpoint.
        s_done = 1;
        if (i + 1 < n) {
          double next_ratio;
          if (jj + 1 < 1024) {
            next_ratio = s_ratio[jj + 1];
          } else {
            double h2, d2;
            bool s2;
            dual_breakpoint(a, s_slot[i + 1], &next_ratio, &h2, &s2, &d2);
          }
          if (next_ratio == ratio) break;  // tie: B
        } else if (n < num_slots) {
          break;  // its successor lies past the gathered keys: B
        }
        const unsigned long long h =
            static_cast<unsigned long long>(__double_as_longlong(s_harris[jj]));
        result = h < best ? h : best;
        break;
      }
    }
    __syncthreads();
    if (s_done) break;
  }
  // A walk through every gathered key without acceptance: B (the full walk
  // ends the same way when nothing lies past them, and is not known otherwise).
  if (tid == 0) {
    bound2[0] = result;
    bound2[1] = static_cast<unsigned long long>(steps) | (s_done ? 0ull : (1ull << 40));
  }
}

__global__ void update_reduced_costs_kernel(const int32_t* list, const double* list_coeff,
                                            const int* count, double mult, int leaving_col,
                                            double leaving_value, int entering_col,
                                            double* rc) {
  const int n = *count;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int col = list[i];
    if (col == entering_col) continue;  // set to 0 below
    rc[col] += mult * list_coeff[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // -1: the column lives on another column shard.
    if (leaving_col >= 0) rc[leaving_col] = leaving_value;  // basic before: never listed
    if (entering_col >= 0) rc[entering_col] = 0.0;
  }
}

__global__ void set_double_kernel(double* dst, double value) { *dst = value; }

__global__ void set_colbits_kernel(const int32_t* cols, const uint8_t* bits, int n,
                                   uint8_t* colbits) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    colbits[cols[i]] = bits[i];
}

// Changed words of a column mask: mask[idx[i]] = words[i] (inputs in mapped
// host memory: no copy-engine transfer for a mask that moved a few bits).
__global__ void set_mask_words_kernel(const int32_t* idx, const uint64_t* words, int n,
                                      uint64_t* mask) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    mask[idx[i]] = words[i];
}

// glop::VariableStatus values (lp_types.h:188-219).
constexpr int kAtLowerBound = 2;
constexpr int kAtUpperBound = 3;

__global__ void boxed_flips_kernel(const int32_t* cols, int n, const double* rc,
                                   const uint8_t* colbits, double threshold, uint8_t* flag) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int col = cols != nullptr ? cols[i] : i;
    const uint8_t bits = colbits[col];
    uint8_t f = 0;
    if (cols != nullptr || (bits & kColBoxed)) {
      const double reduced_cost = rc[col];
      const int status = ColStatus(bits);
      if (reduced_cost > threshold && status == kAtUpperBound) {
        f = 1;
      } else if (reduced_cost < -threshold && status == kAtLowerBound) {
        f = 1;
      }
    }
    flag[i] = f;
  }
}

// ---------------------------------------------------------------------------
// Row sums sum_j mult_j * A[r, j] in increasing j (the order the host scatter
// ColumnAddMultipleToDenseColumn produces), zero multipliers skipped
// (sparse.h:393). A workgroup owns kSumRows rows and walks them in chunks of
// kSumChunk entries: both waves load their rows' chunk (coalesced, one row
// per wave instruction) and write the products transposed into LDS, then lane
// i of wave 0 adds row i's chunk in entry order. A skipped entry is stored as
// -0.0, which leaves every sum unchanged (x + -0.0 == x, also for x = +-0.0).
// Chunk c + 1 is loaded while chunk c is added (double buffer).
constexpr int kSumRows = 32;
constexpr int kSumChunk = 64;
constexpr int kSumRowsPerWave = kSumRows / 2;

__device__ __forceinline__ void row_sum_load(const RowSumArgs& a, const int64_t* rs,
                                             const int64_t* re, int chunk, int wave, int lane,
                                             double* p) {
  int64_t idx[kSumRowsPerWave];
  int col[kSumRowsPerWave];
#pragma unroll
  for (int j = 0; j < kSumRowsPerWave; ++j) {
    const int i = wave * kSumRowsPerWave + j;
    idx[j] = rs[i] + int64_t(chunk) * kSumChunk + lane;
    col[j] = idx[j] < re[i] ? a.t_cols[idx[j]] : -1;
  }
#pragma unroll
  for (int j = 0; j < kSumRowsPerWave; ++j) {
    double m = 0.0;
    if (col[j] >= 0) {
      m = a.x[col[j]];
      if (a.skip != nullptr && bit_set(a.skip, col[j])) m = 0.0;
      m = a.sign * m;  // exact (sign is +-1)
    }
    p[j] = m != 0.0 ? m * a.t_vals[idx[j]] : -0.0;
  }
}

__global__ __launch_bounds__(128) void row_sum_kernel(RowSumArgs a) {
  __shared__ double tile[2][kSumChunk][kSumRows + 1];
  __shared__ int64_t rs[kSumRows];
  __shared__ int64_t re[kSumRows];
  __shared__ int num_chunks;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * kSumRows;
  if (wave == 0) {
    int chunks = 0;
    if (lane < kSumRows) {
      const int row = r0 + lane;
      int64_t s = 0;
      int64_t e = 0;
      if (row < a.num_rows) {
        s = a.t_starts[row];
        e = a.t_starts[row + 1];
      }
      rs[lane] = s;
      re[lane] = e;
      chunks = static_cast<int>((e - s + kSumChunk - 1) / kSumChunk);
    }
    for (int off = 32; off > 0; off >>= 1) chunks = max(chunks, __shfl_xor(chunks, off));
    if (lane == 0) num_chunks = chunks;
  }
  __syncthreads();
  const int nchunks = num_chunks;
  double p[kSumRowsPerWave];
  if (nchunks > 0) {
    row_sum_load(a, rs, re, 0, wave, lane, p);
#pragma unroll
    for (int j = 0; j < kSumRowsPerWave; ++j) tile[0][lane][wave * kSumRowsPerWave + j] = p[j];
  }
  __syncthreads();
  double acc = 0.0;
  for (int c = 0; c < nchunks; ++c) {
    const int b = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) row_sum_load(a, rs, re, c + 1, wave, lane, p);
    if (wave == 0 && lane < kSumRows) {
#pragma unroll 16
      for (int e = 0; e < kSumChunk; ++e) acc += tile[b][e][lane];
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < kSumRowsPerWave; ++j) {
        tile[b ^ 1][lane][wave * kSumRowsPerWave + j] = p[j];
      }
    }
    __syncthreads();
  }
  if (wave == 0 && lane < kSumRows && r0 + lane < a.num_rows) a.out[r0 + lane] = acc;
}

// ---------------------------------------------------------------------------
// 1 + SquaredNorm(column) for relevant columns (primal_edge_norms.cc:153-158
// with an identity basis: lu_factorization.cc:130 returns SquaredNorm(a), a
// plain in-order sum, lp_utils.cc:22-29).
__global__ __launch_bounds__(256) void column_squared_norm_kernel(
    const int64_t* starts, const double* vals, const uint64_t* relevant, int ncols,
    double* out) {
  const int lane = threadIdx.x & 63;
  const int col = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (col >= ncols) return;
  if (!bit_set(relevant, col)) return;
  const int64_t s = starts[col];
  const int64_t e = starts[col + 1];
  double acc = 0.0;
  for (int64_t base = s; base < e; base += kWave) {
    const int64_t i = base + lane;
    const double v = (i < e) ? vals[i] : 0.0;
    const double p = v * v;
    const int nvalid = (e - base) < kWave ? static_cast<int>(e - base) : kWave;
    for (int t = 0; t < kWave; ++t) {
      const double q = __shfl(p, t, kWave);
      if (t < nvalid) acc += q;
    }
  }
  if (lane == 0) out[col] = 1.0 + acc;
}

}  // namespace milp_kernels

// ---------------------------------------------------------------------------
// Host-side launchers (extern "C++" inside the engine library).
namespace milp_launch {
using namespace milp_kernels;

static inline int div_up(long a, long b) { return static_cast<int>((a + b - 1) / b); }

hipError_t column_dot(int mode, bool wave_per_col, const DotArgs& args, hipStream_t s) {
  if (args.ncols <= 0) return hipSuccess;
  const int threads = 256;
  const int per_block = wave_per_col ? threads / 64 : threads / 4;
  const int blocks = div_up(args.ncols, per_block);
  switch (mode * 2 + (wave_per_col ? 1 : 0)) {
    case 0: column_dot_kernel<0, false><<<blocks, threads, 0, s>>>(args); break;
    case 1: column_dot_kernel<0, true><<<blocks, threads, 0, s>>>(args); break;
    case 2: column_dot_kernel<1, false><<<blocks, threads, 0, s>>>(args); break;
    case 3: column_dot_kernel<1, true><<<blocks, threads, 0, s>>>(args); break;
    case 4: column_dot_kernel<2, false><<<blocks, threads, 0, s>>>(args); break;
    case 5: column_dot_kernel<2, true><<<blocks, threads, 0, s>>>(args); break;
    case 6: column_dot_kernel<3, false><<<blocks, threads, 0, s>>>(args); break;
    case 7: column_dot_kernel<3, true><<<blocks, threads, 0, s>>>(args); break;
    case 8: column_dot_kernel<4, false><<<blocks, threads, 0, s>>>(args); break;
    case 9: column_dot_kernel<4, true><<<blocks, threads, 0, s>>>(args); break;
    case 10: column_dot_kernel<5, false><<<blocks, threads, 0, s>>>(args); break;
    case 11: column_dot_kernel<5, true><<<blocks, threads, 0, s>>>(args); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int UNROLL>
static hipError_t launch_dense_dot(int mode, int blocks, const DenseArgs& args, hipStream_t s) {
  switch (mode) {
    case 0: dense_dot_kernel<0, UNROLL><<<blocks, 256, 0, s>>>(args); break;
    case 1: dense_dot_kernel<1, UNROLL><<<blocks, 256, 0, s>>>(args); break;
    case 2: dense_dot_kernel<2, UNROLL><<<blocks, 256, 0, s>>>(args); break;
    case 4: dense_dot_kernel<4, UNROLL><<<blocks, 256, 0, s>>>(args); break;
    case 5: dense_dot_kernel<5, UNROLL><<<blocks, 256, 0, s>>>(args); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t dense_dot(int mode, int unroll, const DenseArgs& args, hipStream_t s) {
  if (args.nd <= 0) return hipSuccess;
  const int blocks = div_up(args.nd, kDenseColsPerBlock);
  if (unroll >= 32) return launch_dense_dot<32>(mode, blocks, args, s);
  if (unroll >= 16) return launch_dense_dot<16>(mode, blocks, args, s);
  return launch_dense_dot<8>(mode, blocks, args, s);
}

hipError_t dense_pack(const int64_t* starts, const double* vals, const int32_t* dense_cols,
                      int nd, int m, double* body, double* tail, hipStream_t s) {
  if (nd <= 0 || m <= 0) return hipSuccess;
  dense_pack_kernel<<<4096, 256, 0, s>>>(starts, vals, dense_cols, nd, m, body, tail);
  return hipGetLastError();
}

hipError_t gather(const int32_t* list, int n, const double* src, double* dst, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  gather_kernel<<<std::min(2048, div_up(n, 256)), 256, 0, s>>>(list, n, src, dst);
  return hipGetLastError();
}

hipError_t compact_flags(const uint8_t* flags, int n, const double* coeff, int32_t* list,
                         double* vals, int* count, int32_t* host_list, double* host_vals,
                         int* host_count, const ScanState& st, hipStream_t s) {
  compact_flags_kernel<<<scan_tiles(n), kScanThreads, 0, s>>>(
      flags, n, coeff, list, vals, count, host_list, host_vals, host_count, st);
  return hipGetLastError();
}

hipError_t compact_small(const uint8_t* flags, int n, const double* coeff, int32_t* list,
                         double* vals, int* count, int32_t* host_list, double* host_vals,
                         int* host_count, hipStream_t s) {
  if (n > kSmallCompactMax) return hipErrorInvalidValue;
  compact_small_kernel<<<1, kCompactThreads, 0, s>>>(flags, n, coeff, list, vals, count,
                                                     host_list, host_vals, host_count);
  return hipGetLastError();
}

hipError_t row_wise_update(const RowWiseArgs& args, hipStream_t s) {
  const int blocks = div_up(args.num_cols, kChunk);
  row_wise_update_kernel<<<blocks, 256, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t row_wise_update_small(const RowWiseSmallArgs& args, int threads, hipStream_t s) {
  if (args.num_cols > kSmallLdsCols || args.num_filtered > kSmallRowsMax ||
      args.num_filtered < 0) {
    return hipErrorInvalidValue;
  }
  // 256 threads (4 waves: cheaper barriers between rows) when the rows fit.
  if (threads == 256 && args.num_filtered <= 256) {
    row_wise_small_kernel<256><<<1, 256, 0, s>>>(args);
  } else {
    row_wise_small_kernel<kCompactThreads><<<1, kCompactThreads, 0, s>>>(args);
  }
  return hipGetLastError();
}

hipError_t small_batch(int kind, const SmallBatchArgs& args, hipStream_t s) {
  if (args.count <= 0) return hipSuccess;
  if (args.count > kSmallBatchMax) return hipErrorInvalidValue;
  switch (kind) {
    case kSmallRowWise:
      small_batch_kernel<kSmallRowWise><<<args.count, kCompactThreads, 0, s>>>(args);
      break;
    case kSmallColWise:
      small_batch_kernel<kSmallColWise><<<args.count, kCompactThreads, 0, s>>>(args);
      break;
    case kSmallListDots:
      small_batch_kernel<kSmallListDots><<<args.count, kCompactThreads, 0, s>>>(args);
      break;
    case kSmallRowWiseByColumn:
      small_batch_kernel<kSmallRowWiseByColumn><<<args.count, kCompactThreads, 0, s>>>(args);
      break;
    case kMediumRowWise:
      small_batch_kernel<kMediumRowWise><<<args.count, kCompactThreads, 0, s>>>(args);
      break;
    case kMediumListDots:
      small_batch_kernel<kMediumListDots><<<args.count, kCompactThreads, 0, s>>>(args);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t row_wise_update_medium(const RowWiseSmallArgs& args, hipStream_t s) {
  if (args.num_cols > kMediumCols || args.num_filtered > kSmallRowsMax ||
      args.num_filtered < 0) {
    return hipErrorInvalidValue;
  }
  row_wise_medium_kernel<<<1, kCompactThreads, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t list_dots_small(const ListDotsSmallArgs& args, hipStream_t s) {
  if (args.m > kSmallLdsCols || args.n < 1) return hipErrorInvalidValue;
  list_dots_small_kernel<<<1, kCompactThreads, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t list_dots_medium(const ListDotsSmallArgs& args, hipStream_t s) {
  if (args.m > kMediumListRows || args.n < 1) return hipErrorInvalidValue;
  list_dots_medium_kernel<<<1, kCompactThreads, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t column_wise_update_small(const ColWiseSmallArgs& args, hipStream_t s) {
  if (args.m > kSmallColWiseRows || args.num_cols > kSmallLdsCols) return hipErrorInvalidValue;
  column_wise_small_kernel<<<1, kCompactThreads, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t row_wise_update_small_by_column(const RowWiseSmallColArgs& args, hipStream_t s) {
  if (args.num_cols > kSmallLdsCols || args.m > kSmallLdsCols || args.num_filtered < 0 ||
      args.num_filtered > args.m) {
    return hipErrorInvalidValue;
  }
  row_wise_small_by_column_kernel<<<1, kCompactThreads, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t tag_rows(const int32_t* filtered_rows, int num_filtered, uint32_t tag,
                    uint32_t* row_tag, int32_t* row_pos, hipStream_t s) {
  if (num_filtered <= 0) return hipSuccess;
  tag_rows_kernel<<<std::min(1024, div_up(num_filtered, 256)), 256, 0, s>>>(
      filtered_rows, num_filtered, tag, row_tag, row_pos);
  return hipGetLastError();
}

hipError_t row_wise_update_by_column(const RowWiseColArgs& args, hipStream_t s) {
  if (args.num_cols <= 0) return hipSuccess;
  row_wise_by_column_kernel<<<div_up(args.num_cols, 256), 256, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t row_wise_update_full_rows(const RowWiseFullArgs& args, hipStream_t s) {
  if (args.num_cols <= 0) return hipSuccess;
  row_wise_full_rows_kernel<<<div_up(args.num_cols, 256), 256, 0, s>>>(args);
  return hipGetLastError();
}

static inline int grid_for(int n) { return std::max(1, std::min(4096, div_up(n, 256))); }

hipError_t dual_ratio_bound(const DualRatioArgs& args, hipStream_t s) {
  dual_ratio_bound_kernel<<<grid_for(args.max_count), 256, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t dual_ratio_select(const DualRatioArgs& args, const DualSelectOut& out,
                             const ScanState& st, hipStream_t s) {
  dual_ratio_select_kernel<<<scan_tiles(args.max_count), kScanThreads, 0, s>>>(args, out, st);
  return hipGetLastError();
}

hipError_t dual_ratio_keys(const DualRatioArgs& args, const int32_t* slots, int num_slots,
                           unsigned long long* keys, hipStream_t s) {
  if (num_slots <= 0) return hipSuccess;
  dual_ratio_keys_kernel<<<grid_for(num_slots), 256, 0, s>>>(args, slots, num_slots, keys);
  return hipGetLastError();
}

hipError_t dual_flip_walk(const DualRatioArgs& args, const int32_t* sorted_slots,
                          int num_slots, unsigned long long* bound2, hipStream_t s) {
  dual_flip_walk_kernel<<<1, 64, 0, s>>>(args, sorted_slots, num_slots, bound2);
  return hipGetLastError();
}

hipError_t dual_tighten(const DualRatioArgs& args, const int32_t* slots, int num_slots,
                        unsigned long long* keys, TightenState* st, unsigned long long* bound2,
                        int target_keys, hipStream_t s) {
  if (num_slots <= 0) return hipSuccess;
  constexpr int kStateWords = static_cast<int>(sizeof(TightenState) / sizeof(unsigned int));
  const int key_blocks = std::max(grid_for(num_slots), div_up(kStateWords, 256));
  dual_tighten_keys_kernel<<<key_blocks, 256, 0, s>>>(args, slots, num_slots, keys, st);
  const int hist_blocks = std::max(1, std::min(256, div_up(num_slots, 256 * 8)));
  target_keys = std::max(1, std::min(target_keys, kTightenCap));
  dual_tighten_hist_kernel<<<hist_blocks, 256, 0, s>>>(keys, num_slots, st, 0, target_keys);
  dual_tighten_hist_kernel<<<hist_blocks, 256, 0, s>>>(keys, num_slots, st, 1, target_keys);
  dual_tighten_walk_kernel<<<1, 1024, 0, s>>>(args, slots, keys, num_slots, st, bound2);
  return hipGetLastError();
}

hipError_t update_reduced_costs(const int32_t* list, const double* list_coeff, const int* count,
                                int max_count, double mult, int leaving_col,
                                double leaving_value, int entering_col, double* rc,
                                hipStream_t s) {
  update_reduced_costs_kernel<<<grid_for(max_count), 256, 0, s>>>(
      list, list_coeff, count, mult, leaving_col, leaving_value, entering_col, rc);
  return hipGetLastError();
}

hipError_t set_double(double* dst, double value, hipStream_t s) {
  set_double_kernel<<<1, 1, 0, s>>>(dst, value);
  return hipGetLastError();
}

hipError_t set_colbits(const int32_t* cols, const uint8_t* bits, int n, uint8_t* colbits,
                       hipStream_t s) {
  if (n <= 0) return hipSuccess;
  set_colbits_kernel<<<grid_for(n), 256, 0, s>>>(cols, bits, n, colbits);
  return hipGetLastError();
}

hipError_t set_mask_words(const int32_t* idx, const uint64_t* words, int n, uint64_t* mask,
                          hipStream_t s) {
  if (n <= 0) return hipSuccess;
  set_mask_words_kernel<<<grid_for(n), 256, 0, s>>>(idx, words, n, mask);
  return hipGetLastError();
}

hipError_t boxed_flips(const int32_t* cols, int n, const double* rc, const uint8_t* colbits,
                       double threshold, uint8_t* flag, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  boxed_flips_kernel<<<grid_for(n), 256, 0, s>>>(cols, n, rc, colbits, threshold, flag);
  return hipGetLastError();
}

hipError_t row_sums(const RowSumArgs& args, hipStream_t s) {
  if (args.num_rows <= 0) return hipSuccess;
  row_sum_kernel<<<div_up(args.num_rows, kSumRows), 128, 0, s>>>(args);
  return hipGetLastError();
}

hipError_t column_squared_norms(const int64_t* starts, const double* vals,
                                const uint64_t* relevant, int ncols, double* out,
                                hipStream_t s) {
  if (ncols <= 0) return hipSuccess;
  column_squared_norm_kernel<<<div_up(ncols, 4), 256, 0, s>>>(starts, vals, relevant,
                                                              ncols, out);
  return hipGetLastError();
}

}  // namespace milp_launch
