// Argument blocks shared by the kernel launchers (simplex_kernels.hip) and
// the device layer (engine/device_lp.hip). Plain structs of device pointers.
#ifndef MILP_KERNEL_ARGS_H_
#define MILP_KERNEL_ARGS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace milp_kernels {

struct DotArgs {
  const int64_t* starts;
  const int32_t* rows;
  const double* vals;
  const double* y;
  int ncols;                // columns to visit (N, or list length)
  const int32_t* col_list;  // kListDots: the columns
  const uint64_t* mask;     // relevance / not-basic bitset (modes 0, 3)
  const double* c;          // kPricing: objective + perturbation
  double* out;              // result per column (or per list entry)
  uint8_t* flags;           // kUpdateRowColumnWise: |coeff| > drop; kListDots: listed
  double drop_tolerance;
  const uint8_t* skip;      // optional: columns handled by the dense block
  const double* y2;         // kUpdateRowWithDots / kPricingWithDots: w = B^-T d
  double* out2;             // w . a_j for listed columns
};

// Dense column block: the structural columns whose CSC column is full (all m
// rows). Values only, chain-major so that lane j of the wave for chain k
// streams chain k of column j (Glop's accumulator r_{k+1} in
// ColumnScalarProduct, sparse.h:514-542, since a full column's entry index
// equals its row index) with 16-byte loads that are contiguous across the
// wave. With steps = m / 4 chain elements per chain and pairs = steps / 2:
//   body[((t2 * 4 + k) * nd + j) * 2 + h] = A[4 (2 t2 + h) + k, col_j], t2 < pairs
//   body[pairs * nd * 8 + k * nd + j]     = A[4 (steps - 1) + k, col_j] if steps odd
//   tail[r * nd + j]                      = A[4 steps + r, col_j],       r < m % 4
struct DenseArgs {
  const double* body;
  const double* tail;
  const int32_t* dense_cols;  // nd ascending column ids
  int nd;
  int m;
  const double* y;        // dot vector (rho / y / w)
  const uint64_t* mask;   // kUpdateRowColumnWise: relevant columns
  const double* c;        // kPricing
  double* out;            // indexed by column id
  uint8_t* flags;         // kUpdateRowColumnWise: out; kListDots: in (listed)
  double drop_tolerance;
  const double* y2;       // kUpdateRowWithDots / kPricingWithDots
  double* out2;
};

struct RowWiseArgs {
  const int64_t* t_starts;  // CSR of [A | I] (transposed_matrix_)
  const int32_t* t_cols;
  const double* t_vals;
  const int32_t* filtered_rows;  // ascending
  const double* rho;             // rho value per filtered row
  int num_filtered;
  int num_cols;
  const uint64_t* relevant;
  double* coefficient;  // update row (device copy of UpdateRow::coefficient_)
  uint8_t* flags;       // listed positions
  double drop_tolerance;
  int algorithm;  // 0 single row, 1 hypersparse, 2 row-wise
};

// The whole row-wise update row of a small LP in ONE workgroup and one launch
// (row_wise_small_kernel): N <= kSmallLdsCols, 1 <= filtered rows <=
// kSmallRowsMax, their entries <= kSmallEntries (checked by the host). The
// filtered rows, their rho values and the relevant mask are read from mapped
// host memory; the list lands in mapped host memory (and the device copies).
constexpr int kSmallLdsCols = 8192;
// The column-wise update row of a small LP without a dense block (m <=
// kSmallColWiseRows) in one workgroup: rho (and w) staged from mapped host
// memory into LDS, one thread per relevant column in ColumnScalarProduct's chain
// order, column_dot_kernel's kUpdateRowColumnWise / kUpdateRowWithDots write
// rules, then the compaction; list, values (and the w dots, list order) land
// in mapped host memory.
constexpr int kSmallColWiseRows = 4096;
struct ColWiseSmallArgs {
  const int64_t* starts;
  const int32_t* rows;
  const double* vals;
  const double* rho;       // mapped host memory, m values
  const double* w;         // mapped host memory, m values, or nullptr
  int m;
  int num_cols;            // <= kSmallLdsCols
  const uint64_t* relevant;  // mapped host memory
  double* coefficient;
  uint8_t* flags;
  double* out2;            // w . a_j of kept columns (device, per column)
  double drop_tolerance;
  int32_t* list;  // device copies of the compacted list
  double* vals_out;
  int* count;
  int32_t* host_list;  // mapped host memory
  double* host_vals;
  int* host_count;
  double* host_dots;   // mapped host memory, list order (with w)
};

// The row-wise update row of a small LP with many filtered rows (or rows too
// long for kSmallEntries), one workgroup: thread per column over the CSC copy
// (row_wise_by_column_kernel's per-column order), row positions in LDS, then
// the compaction. m, N <= kSmallLdsCols; filtered rows <= m.
struct RowWiseSmallColArgs {
  const int64_t* starts;  // CSC of [A | I]
  const int32_t* rows;
  const double* vals;
  const int32_t* filtered_rows;  // mapped host memory, list order
  const double* rho;             // mapped host memory, rho per filtered row
  int num_filtered;
  int m;
  int num_cols;
  const uint64_t* relevant;      // mapped host memory
  double* coefficient;
  uint8_t* flags;
  double drop_tolerance;
  int algorithm;
  int32_t* list;
  double* list_vals;
  int* count;
  int32_t* host_list;
  double* host_vals;
  int* host_count;
};

// out[k] = a_{list[k]} . y for a small LP without a dense block, one
// workgroup: y (m <= kSmallLdsCols) staged from mapped host memory into LDS,
// one thread per column in ColumnScalarProduct's chain order, the results
// written straight to mapped host memory.
struct ListDotsSmallArgs {
  const int64_t* starts;
  const int32_t* rows;
  const double* vals;
  const double* y;  // mapped host memory, m values
  int m;
  const int32_t* list;  // device: compacted update-row list
  int n;
  double* out;  // mapped host memory
};
constexpr int kSmallRowsMax = 1024;
constexpr int kSmallEntries = 4096;
struct RowWiseSmallArgs {
  const int64_t* t_starts;
  const int32_t* t_cols;
  const double* t_vals;
  const int32_t* filtered_rows;  // mapped host memory, list order
  const double* rho;             // mapped host memory, rho per filtered row
  int num_filtered;
  int num_cols;
  const uint64_t* relevant;      // mapped host memory
  double* coefficient;
  uint8_t* flags;
  double drop_tolerance;
  int algorithm;  // 0 single row, 1 hypersparse, 2 row-wise
  int32_t* list;  // device copies of the compacted list
  double* vals;
  int* count;
  int32_t* host_list;  // mapped host memory
  double* host_vals;
  int* host_count;
};
constexpr int kMediumCols = 65536;

// The row-wise update row when every filtered row is full (all structural
// columns present): entry j < num_structural of CSR row r is column j and the
// row's last entry is its slack column. Slack outputs use the row tags.
struct RowWiseFullArgs {
  const int64_t* t_starts;  // CSR of [A | I]
  const double* t_vals;
  const int64_t* row_offsets;  // t_starts of each filtered row, list order k
  const double* rho;           // rho value per filtered row
  int num_filtered;
  int num_structural;
  int num_cols;
  const uint32_t* row_tag;
  const int32_t* row_pos;
  uint32_t tag;
  const uint64_t* relevant;
  double* coefficient;
  uint8_t* flags;
  double drop_tolerance;
  int algorithm;
};

// The same row-wise update row evaluated column by column from the CSC copy
// (for many filtered rows): row r of the filtered list sits at position
// row_pos[r] when row_tag[r] == tag.
struct RowWiseColArgs {
  const int64_t* starts;  // CSC of [A | I]
  const int32_t* rows;
  const double* vals;
  const uint32_t* row_tag;
  const int32_t* row_pos;
  uint32_t tag;
  const double* rho;  // rho value per filtered row, list order
  int num_cols;
  const uint64_t* relevant;
  double* coefficient;
  uint8_t* flags;
  double drop_tolerance;
  int algorithm;  // 0 single row, 1 hypersparse, 2 row-wise
};

// Dual simplex with device-resident reduced costs (engine/device_lp.h
// "dual device mode"). Per column one status byte:
//   bit 0 can_decrease, bit 1 can_increase, bit 2 non-basic boxed,
//   bits 3-5 glop::VariableStatus.
enum : uint8_t { kColCanDecrease = 1, kColCanIncrease = 2, kColBoxed = 4 };
__host__ __device__ inline int ColStatus(uint8_t b) { return (b >> 3) & 7; }

// Bound-flipping ratio test filter (entering_variable.cc:37-130) over the
// update-row list: pass 1 bounds the breakpoints that can matter, pass 2
// flags them.
struct DualRatioArgs {
  const int32_t* list;       // update-row positions (list order)
  const double* list_coeff;  // their coefficients
  const int* count;          // list length (device)
  int max_count;             // N (grid bound)
  const double* rc;
  const uint8_t* colbits;
  const double* bound_diff;  // upper - lower per column
  double sign;               // +1 if cost_variation > 0 else -1
  double threshold;          // minimum pivot magnitude
  double harris_tolerance;
  double minimum_delta;
  double variation_magnitude;
  unsigned long long* best;  // pass 1: min over H-setting breakpoints of the
                             // Harris ratio, as ordered bits (all values > 0)
  unsigned long long* best_next;  // pass 1 sets it to "none" for the next call
  const unsigned long long* bound;  // pass 2: the bound it filters with
};

// Single-pass ordered compaction (decoupled look-back): a launch takes tiles
// of kScanTile slots in ticket order; each tile publishes its count, then its
// inclusive prefix, tagged with the launch's epoch (no reset between
// launches); the last workgroup to finish rewinds the ticket counters.
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;
struct ScanState {
  unsigned long long* status;  // per tile: epoch << 32 | flag << 30 | count
  unsigned int* ticket;        // [0] tile ticket, [1] finished workgroups
  unsigned int epoch;          // distinct per launch, never 0
  int* fail;                   // host-visible: set if a look-back wait ran out
};

// The fused dual ratio filter + compaction writes here (mapped host memory).
struct DualSelectOut {
  int32_t* slots;      // device: kept list slots, in list order
  int* num_slots;      // device
  int32_t* cand_col;   // host-visible
  double* cand_coeff;  // host-visible
  double* cand_rc;     // host-visible
  int* counts;         // host-visible: [0] kept, [1] list length
  int host_cap;        // candidates at positions >= host_cap skip the host copy
};

// Tightening by selection (dual_tighten below): histogram passes over the
// sort keys' top 12 bits, then the next 12 within the chosen top bin, find a
// threshold with at least min(target, k1) keys at or below it (target
// kTightenTarget, MILP_TIGHTEN_TARGET in tests); one
// workgroup sorts those (at most kTightenCap) in LDS and walks them.
constexpr int kTightenTarget = 512;
constexpr int kTightenCap = 2048;
constexpr int kTightenBins = 4096;
struct TightenState {
  unsigned int hist[2][kTightenBins];
  unsigned int ticket;
  unsigned int bin0;       // pass 0: the top-12-bit bin the target falls in
  unsigned int below0;     // keys in the bins below it
  unsigned int count;      // pass 1: keys <= threshold
  unsigned long long threshold;
};

struct RowSumArgs {
  const int64_t* t_starts;
  const int32_t* t_cols;
  const double* t_vals;
  const double* x;       // multipliers per column
  const uint64_t* skip;  // optional: skip columns whose bit is set (basic)
  double sign;           // +1 (residual) or -1 (basic-value recompute)
  int num_rows;
  double* out;
};


// Batched small-LP launches (simplex_kernels.hip small_batch_kernel): one
// request per LP in a slot of mapped host memory.
enum SmallKind { kSmallRowWise = 0, kSmallColWise = 1, kSmallListDots = 2,
                 kSmallRowWiseByColumn = 3, kMediumRowWise = 4, kMediumListDots = 5,
                 kSmallKinds = 6 };
// The list dots of mid-size LPs (kMediumListDots): y (m <= kMediumListRows,
// 128 KB) staged in LDS as the small kind does.
constexpr int kMediumListRows = 16384;
struct SmallSlot {
  unsigned long long seq;  // published to done[slot] when the request is finished
  int kind;
  int pad;
  union {
    RowWiseSmallArgs rw;
    ColWiseSmallArgs cw;
    ListDotsSmallArgs ld;
    RowWiseSmallColArgs rc;
  };
};
constexpr int kSmallBatchMax = 128;  // requests per launch
struct SmallBatchArgs {
  const SmallSlot* slots;       // device view of the mapped slot table
  unsigned long long* done;     // device view of the mapped done words
  int count;
  int ids[kSmallBatchMax];
};

// Dense triangular solve (tri_solve.hip): TransposeLowerSolve of a
// TriangularMatrix with its outputs listed in dependency-level order and the
// values kept in that order on the device.
constexpr int kTriThreads = 1024;
constexpr int kTriPrefetch = 2;  // outputs per thread loaded ahead of their level
// Values a single-CU run of levels keeps in LDS (its own outputs): a run's
// positions never exceed this (the schedule builder cuts runs there).
constexpr int kTriLdsVals = 16384;
struct TriSolveArgs {
  const int32_t* level_start;  // [num_levels + 1] list positions of each level
  const int32_t* rec_row;      // [num_work] row (index into x) of each listed output
  const int32_t* rec_n;        // [num_work] its number of entries
  const int4* rec_entry;       // [num_work] entry positions (n <= 4) / overflow start
  const double2* rec_value;    // [2 * num_work] entry values (n <= 4)
  const double* diag;          // [num_work] diagonal, nullptr when all are 1
  const int32_t* ovf_pos;      // entries of the outputs with n > 4
  const double* ovf_value;
  const int32_t* pos_row;      // [num_pos] row of every position (listed first)
  double* x;                   // rows, in/out
  double* y;                   // [num_pos] values in position order (scratch)
  int num_work;
  int num_pos;
  int num_levels;
  int* top;                    // rows above *top are not computed (host: last non-zero)
  uint64_t* clock;             // debug (MILP_TRI_DEBUG): wall clock after each level, or null
  // Zero-copy staging (or null: the caller copies x and *top): host_x is
  // device-visible host memory holding x[first_col, num_rows) and, in the
  // int at host_x + num_rows, the top row; the plan starts by reading them
  // and ends by writing x[first_col, top] back.
  double* host_x;
  int first_col;
  int num_rows;
  int* fail;  // sync-free variant: set (host-visible) if a wait ran out
  // 0: grouped sums (TransposeLowerSolve); 1: LowerSolve's order -- one
  // subtraction per entry in list order, entries whose value is 0 skipped.
  int sequential;
  // Level plan: 1 when level 0 (outputs without entries, only a division)
  // is computed inside the gather kernel instead of a launch of its own.
  int fuse_level0;
  // Sync-free variants: a waiting lane's sleep between polls doubles from
  // one s_sleep unit up to this many (MILP_TRI_POLL_MAX; 1 = fixed).
  int poll_max;
  // A second right-hand side solved in the same launch (blockIdx.y == 1):
  // its own rows, positions, staging, top row and failure word.
  double* x2;
  double* y2;
  double* host_x2;
  int* top2;
  int* fail2;
  // Sync-free plans run the schedule as segments of consecutive levels, one
  // launch each, in order: this launch's positions are [seg_begin, seg_end).
  // A chip-wide segment (tri_syncfree_kernel) hands values between
  // workgroups through y; a narrow one (tri_chain_kernel, unpadded levels)
  // runs on one workgroup per right-hand side with its values in LDS.
  // Earlier segments are final in y when a launch starts.
  int seg_begin;
  int seg_end;
  // Sync-free plans: positions [0, level0_end) are level 0 (no entries, a
  // division at most), computed by tri_init_kernel; 0 = not fused.
  int level0_end;
};
// The argument set of right-hand side blockIdx.y (0 or 1).
__host__ __device__ inline TriSolveArgs TriRhs(const TriSolveArgs& a, int rhs) {
  TriSolveArgs b = a;
  if (rhs == 1) {
    b.x = a.x2;
    b.y = a.y2;
    b.host_x = a.host_x2;
    b.top = a.top2;
    b.fail = a.fail2;
  }
  return b;
}
// The sync-free variant needs every workgroup resident: at most this many
// outputs (512 workgroups of 256 threads, 2 per CU).
constexpr int kTriSyncFreeMaxWork = 512 * 256;
// Values the chain kernel keeps in LDS (96 KB): a tail never holds more.
constexpr int kTriChainVals = 12288;

// Dense tail of BTRAN's forward U^T solve (dense_tail.hip): upper_.
// TransposeUpperSolve (sparse.cc:848-897) when the last columns of U hold
// most of its entries (config 2's dense kernel). Columns [t, n) are the tail,
// solved by blocks of 64 columns (advance over the chip, finish on one wave).
constexpr int kTailMaxCols = 16384;
struct DenseTailArgs {
  const int64_t* starts;  // [T + 1] entry ranges of the tail columns (relative)
  const int32_t* rows;    // entries: rows (< the column)
  const double* vals;
  const double* diag;     // [T], nullptr when all are 1
  double* x;              // [n] the vector, in and out
  double* pre;            // [T] each column's running sum
  int64_t* cur;           // [T] each column's chain cursor (relative entry index)
  const double* host_x;   // device view of the pinned staging copy (n values)
  double* host_out;       // device view of the pinned output (x[t, n))
  int n;
  int t;
  int* fail;              // host-visible: a wait ran out
};
}  // namespace milp_kernels

namespace milp_launch {
hipError_t column_dot(int mode, bool wave_per_col, const milp_kernels::DotArgs& args,
                      hipStream_t s);
// unroll: 16-byte loads in flight per lane (8, 16 or 32).
hipError_t dense_dot(int mode, int unroll, const milp_kernels::DenseArgs& args, hipStream_t s);
hipError_t dense_pack(const int64_t* starts, const double* vals, const int32_t* dense_cols,
                      int nd, int m, double* body, double* tail, hipStream_t s);
hipError_t gather(const int32_t* list, int n, const double* src, double* dst, hipStream_t s);
// Flags -> ascending list + coefficient gather + count, one workgroup, for
// n <= kSmallCompactMax.
constexpr int kSmallCompactMax = 1 << 14;  // one workgroup writes the list to host memory
// host_* (optional, device-visible mapped host memory) receive a copy.
hipError_t compact_small(const uint8_t* flags, int n, const double* coeff, int32_t* list,
                         double* vals, int* count, int32_t* host_list, double* host_vals,
                         int* host_count, hipStream_t s);
// Any n: flags -> ascending list + coefficients + count in one launch
// (ordered single-pass compaction); host_* as above.
hipError_t compact_flags(const uint8_t* flags, int n, const double* coeff, int32_t* list,
                         double* vals, int* count, int32_t* host_list, double* host_vals,
                         int* host_count, const milp_kernels::ScanState& st, hipStream_t s);
// Tiles a compaction launch over n slots uses (ScanState::status length).
inline int scan_tiles(int n) {
  return n <= 0 ? 1 : (n + milp_kernels::kScanTile - 1) / milp_kernels::kScanTile;
}
hipError_t row_wise_update(const milp_kernels::RowWiseArgs& args, hipStream_t s);
// threads: 1024, or 256 (used when the filtered rows fit one per thread).
hipError_t row_wise_update_small(const milp_kernels::RowWiseSmallArgs& args, int threads,
                                 hipStream_t s);
hipError_t row_wise_update_medium(const milp_kernels::RowWiseSmallArgs& args, hipStream_t s);
hipError_t small_batch(int kind, const milp_kernels::SmallBatchArgs& args, hipStream_t s);
hipError_t list_dots_small(const milp_kernels::ListDotsSmallArgs& args, hipStream_t s);
hipError_t list_dots_medium(const milp_kernels::ListDotsSmallArgs& args, hipStream_t s);
hipError_t row_wise_update_small_by_column(const milp_kernels::RowWiseSmallColArgs& args,
                                           hipStream_t s);
hipError_t column_wise_update_small(const milp_kernels::ColWiseSmallArgs& args, hipStream_t s);
// Marks the filtered rows (row_tag[r] = tag, row_pos[r] = list position).
hipError_t tag_rows(const int32_t* filtered_rows, int num_filtered, uint32_t tag,
                    uint32_t* row_tag, int32_t* row_pos, hipStream_t s);
hipError_t row_wise_update_by_column(const milp_kernels::RowWiseColArgs& args, hipStream_t s);
hipError_t row_wise_update_full_rows(const milp_kernels::RowWiseFullArgs& args, hipStream_t s);
hipError_t row_sums(const milp_kernels::RowSumArgs& args, hipStream_t s);
// Dual device mode.
hipError_t dual_ratio_bound(const milp_kernels::DualRatioArgs& args, hipStream_t s);
// Pass 2 fused with its compaction and the candidate gather: the eligible
// slots with ratio <= *args.bound (1 + 1e-9), in list order, one launch.
hipError_t dual_ratio_select(const milp_kernels::DualRatioArgs& args,
                             const milp_kernels::DualSelectOut& out,
                             const milp_kernels::ScanState& st, hipStream_t s);
// Tighter bound: sort keys (ratio, order-preserving bits) of the pass-2 slots.
hipError_t dual_ratio_keys(const milp_kernels::DualRatioArgs& args, const int32_t* slots,
                           int num_slots, unsigned long long* keys, hipStream_t s);
// Walks the ratio-sorted breakpoints the way the second Glop loop pops them
// (flipping boxed ones while the variation stays positive) up to the first
// accepted breakpoint; *bound2 = min(B, its Harris ratio) (or B = *args.best
// on a ratio tie, where the pop order also depends on magnitudes).
hipError_t dual_flip_walk(const milp_kernels::DualRatioArgs& args, const int32_t* sorted_slots,
                          int num_slots, unsigned long long* bound2, hipStream_t s);
// The same bound from the smallest keys only (keys, two histogram passes,
// one sort-and-walk workgroup): bound2[0] is the full walk's result, or B
// when the walk leaves the gathered prefix; bound2[1] the walk length
// (statistics). Uses `keys` (num_slots entries) and `st` as scratch.
hipError_t dual_tighten(const milp_kernels::DualRatioArgs& args, const int32_t* slots,
                        int num_slots, unsigned long long* keys, milp_kernels::TightenState* st,
                        unsigned long long* bound2, int target_keys, hipStream_t s);
// rc[list[i]] += mult * list_coeff[i] (reduced_costs.cc:466-470), then
// rc[leaving] = leaving_value, rc[entering] = 0.
hipError_t update_reduced_costs(const int32_t* list, const double* list_coeff, const int* count,
                                int max_count, double mult, int leaving_col,
                                double leaving_value, int entering_col, double* rc,
                                hipStream_t s);
hipError_t set_double(double* dst, double value, hipStream_t s);
// colbits[cols[i]] = bits[i].
hipError_t set_colbits(const int32_t* cols, const uint8_t* bits, int n, uint8_t* colbits,
                       hipStream_t s);
// MakeBoxedVariableDualFeasible (revised_simplex.cc:2391-2437) decisions:
// flag[i] = new status (AT_LOWER/AT_UPPER) if cols[i] flips, else 0xff.
// cols == nullptr: every column whose bit 2 (non-basic boxed) is set.
hipError_t set_mask_words(const int32_t* idx, const uint64_t* words, int n, uint64_t* mask,
                          hipStream_t s);
hipError_t boxed_flips(const int32_t* cols, int n, const double* rc, const uint8_t* colbits,
                       double threshold, uint8_t* flag, hipStream_t s);
// segments: num_segments pairs; (lb, le) with lb >= 0 = levels [lb, le) on
// one CU; (-level - 1, blocks) = one wide level over `blocks` workgroups.
hipError_t tri_transpose_lower(const milp_kernels::TriSolveArgs& args, const int* segments,
                               int num_segments, hipStream_t s);
// The same solve driven by per-output readiness instead of levels
// (rec_row/x updated in place, no scatter): one launch per segment, segs =
// num_segs triples (first position, end position, 1 = narrow segment on one
// workgroup / 0 = chip-wide).
hipError_t tri_transpose_lower_syncfree(const milp_kernels::TriSolveArgs& args,
                                        const int* segs, int num_segs, hipStream_t s,
                                        int num_rhs = 1);
// The same, persistent: `groups` workgroups of kTriThreads threads walk the
// outputs in level order (thread t: t, t + T, ...); xcd_stride 8 keeps them
// on one XCD under round-robin dealing (speed only, any placement is correct).
hipError_t tri_transpose_lower_persistent(const milp_kernels::TriSolveArgs& args, int groups,
                                          int xcd_stride, hipStream_t s);
hipError_t column_squared_norms(const int64_t* starts, const double* vals,
                                const uint64_t* relevant, int ncols, double* out,
                                hipStream_t s);
// Dense-tail TransposeUpperSolve: copy-in of x from host_x, the blocks of
// 64 tail columns (advance + finish launches), copy-out of x[t, n) to host_out.
hipError_t dense_tail_upper_solve(const milp_kernels::DenseTailArgs& args, hipStream_t s);

}  // namespace milp_launch

#endif  // MILP_KERNEL_ARGS_H_
