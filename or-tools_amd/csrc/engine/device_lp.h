// Device state of one LP on one MI355X: the constraint matrix [A | I] in CSC
// and CSR (the compact_matrix_ and transposed_matrix_ of RevisedSimplex,
// revised_simplex.cc:989-1000), scratch vectors and the launchers of the
// kernels in csrc/kernels/simplex_kernels.hip. All launches go to the
// handle's own HIP stream. Results come back through pinned host buffers.
#ifndef MILP_DEVICE_LP_H_
#define MILP_DEVICE_LP_H_

#include <cstdint>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/mi_lp.h"
#include "device_solver.h"

namespace milp_kernels {
struct TriSolveArgs;
struct ScanState;
struct TightenState;
}
namespace sdual {
struct Mailbox;
}

namespace milp {
// Zeroes the MILP_SDUAL_PROFILE host counters (sdual_kernel.hip).
void SdualProfileReset();
// A batch call on `device` starts (begin) or ends using the device's segment
// pool; when the last one ends, the resident pool grid is told to stop.
void SdualPoolScope(int device, bool begin, int lps);
// Process teardown of the engine's long-lived device objects (sdual pool
// grids, LU server threads, small-batch launcher threads), before the HIP
// runtime's own: mi_lp_shutdown, and an atexit handler registered when the
// first such object is created (RegisterDeviceShutdown). Idempotent.
void ShutdownDevices();
void SdualShutdown();
void RegisterDeviceShutdown();

class CompactSparseMatrix;

// Records the device operation under way (MILP_WATCHDOG_S diagnostics).
void DeviceOp(const char* what);

struct DeviceError : public std::runtime_error {
  explicit DeviceError(const std::string& s) : std::runtime_error(s) {}
};

class DeviceLp : public DeviceSolver {
 public:
  DeviceLp() = default;
  ~DeviceLp() override;
  DeviceLp(const DeviceLp&) = delete;
  DeviceLp& operator=(const DeviceLp&) = delete;

  // Binds the handle to a GPU (hipSetDevice + stream). Throws DeviceError.
  void Init(int device);
  bool initialized() const { return stream_ != nullptr; }
  int device() const { return device_; }

  // Uploads [A | I] in CSC and CSR (transpose) and sizes every scratch buffer.
  void UploadMatrix(const CompactSparseMatrix& csc, const CompactSparseMatrix& csr);

  // Bit masks over the N columns; uploaded only when the words change.
  enum Mask { kRelevant = 0, kBasic = 1, kNotBasic = 2, kNumMasks = 3 };
  void SetMask(Mask which, const uint64_t* words, int num_words);

  // --- update row (update_row.cc:77-306) -------------------------------
  // Column-wise: coefficient_[j] = a_j . rho for relevant j.
  // With w != nullptr the same pass also computes a_j . w for the listed
  // columns, served by the next ListDotsOverUpdateRow(w) without a 2nd pass.
  void UpdateRowColumnWise(const std::vector<double>& rho, double drop_tolerance,
                           int64_t relevant_entries,
                           const std::vector<double>* w = nullptr);
  // algorithm 0 single row, 1 row-wise hypersparse, 2 row-wise.
  void UpdateRowRowWise(const std::vector<int>& filtered_rows,
                        const std::vector<double>& rho, int algorithm,
                        double drop_tolerance);
  // Fetches the listed positions (ascending) and their coefficients of the last
  // update row.
  void FetchUpdateRow(std::vector<int>* positions, std::vector<double>* values);
  // Reads coefficient_[col] of the last update row (non-listed positions).
  double ReadCoefficient(int col);

  // --- dots over the listed update-row columns ---------------------------
  // out[k] = a_{list[k]} . v (primal_edge_norms.cc:229-233).
  void ListDotsOverUpdateRow(const std::vector<double>& v, std::vector<double>* out);
  // out[k] = a_{cols[k]} . v for an arbitrary host column list.
  void ListDots(const std::vector<int>& cols, const std::vector<double>& v,
                std::vector<double>* out);

  // --- pricing (reduced_costs.cc:352-423) ------------------------------
  // With w != nullptr the same pass over A also computes a_j . w for the
  // columns listed by the last update row (the primal edge-norm dots of the
  // previous pivot, primal_edge_norms.cc:229-233), returned in list order.
  void Pricing(const std::vector<double>& c, const std::vector<double>& y,
               std::vector<double>* rc, const std::vector<double>* w = nullptr,
               std::vector<double>* list_dots = nullptr);
  // Changes whenever the device-side update-row list (and its flags) changes.
  uint64_t list_epoch() const;

  // --- 1 + ||a_j||^2 for relevant j (identity basis) -------------------
  void ColumnSquaredNorms(std::vector<double>* out);

  // --- row sums sign * sum_j x_j A[r, j] (increasing j), optionally skipping
  // basic columns (variable_values.cc:101-131).
  void RowSums(const std::vector<double>& x, bool skip_basic, double sign,
               std::vector<double>* out);

  // --- dual device mode: device-resident reduced costs ------------------
  // (see simplex.cc RevisedSimplex::DualDeviceMode). colbits: one byte per
  // column (kernel_args.h kCol*), bound_diff: upper - lower per column.
  void DualBegin(const std::vector<double>& rc, const std::vector<uint8_t>& colbits,
                 const std::vector<double>& bound_diff);
  void DualSetColBits(const std::vector<int32_t>& cols, const std::vector<uint8_t>& bits);
  // The reduced costs of the last Pricing() call become the device copy.
  void DualTakePricedReducedCosts();
  void DualDownloadReducedCosts(std::vector<double>* rc);
  void DualSetReducedCost(int col, double value);
  struct DualCandidates {
    std::vector<int> col;
    std::vector<double> coeff;  // update-row coefficient
    std::vector<double> rc;
    int list_count = 0;         // update-row positions
  };
  // entering_variable.cc:37-130 filter over the last update row.
  void DualRatioCandidates(double sign, double threshold, double harris_tolerance,
                           double minimum_delta, double variation_magnitude,
                           DualCandidates* out);
  // reduced_costs.cc:444-488 over the last update row.
  void DualUpdateReducedCosts(double mult, int leaving_col, double leaving_value,
                              int entering_col);
  // revised_simplex.cc:2391-2437 decisions; cols == nullptr: every non-basic
  // boxed column. flags[i] = 1 if (cols ? cols[i] : i) flips.
  void DualBoxedFlips(const std::vector<int>* cols, double threshold,
                      std::vector<uint8_t>* flags);
  // The listed DualBoxedFlips of the next loop top, launched early (engine:
  // right after this iteration's reduced-cost update, on the same stream, so
  // that the loop top reads the flags instead of a launch and a wait). The
  // next DualBoxedFlips takes them when it asks for the same columns and
  // threshold, no reduced cost was written since and none of those columns'
  // bits changed; otherwise it decides as usual. MILP_EARLY_FLIPS=0: off.
  void DualBoxedFlipsEarly(const std::vector<int>& cols, double threshold);

  // --- dense triangular solves of the LU (device_solve.hip) -------------
  struct TriBuffer {  // a device buffer of the triangular-solve state
    void* ptr = nullptr;
    size_t bytes = 0;
  };
  // Device buffers of a schedule (staged in this order).
  enum TriBuf {
    kTriLevels, kTriRecRow, kTriRecN, kTriRecEntry, kTriRecValue, kTriDiag, kTriOvfPos,
    kTriOvfValue, kTriPosRow, kTriNumStaged
  };
  // One triangular loop's level schedule and records (device_solver.h
  // TriKind), rebuilt when the factorization key changes.
  enum TriMatrix { kTriU = 0, kTriL = 1, kTriNumMatrices = kNumTriKinds };
  struct TriSchedule {
    uint64_t key = 0;
    bool ok = false;
    bool sequential = false;  // L: single subtractions, zero values skipped
    bool ones = true;
    int rows = 0, first_col = 0, work = 0, pos = 0, levels = 0;
    std::vector<int32_t> level_width;
    std::vector<int> segments;        // tri_transpose_lower launch plan
    TriBuffer buf[kTriNumStaged];
    std::vector<int32_t> rows_upto;   // listed outputs with row <= r
    std::vector<int64_t> entries_upto;  // their entries
    int max_entries = 0;
    int rows_over[3] = {0, 0, 0};     // outputs with > 4, 16, 64 entries
    int64_t late_entries = 0;         // long outputs: entries from the deepest input on
    // Sync-free launch segments: (first position, end position, narrow) triples.
    std::vector<int> runs;
    int chain_levels = 0;             // levels in narrow segments
    int max_wide_run = 0;             // positions of the largest chip-wide segment
    int level0_end = 0;               // positions of a chip-wide level 0 (the init fuses it)
  };
  struct TriContext {  // one solving thread's stream, values and graphs
    void* stream = nullptr;
    TriBuffer x, y, top;         // rows, positions, the solve's top row
    double* h_x = nullptr;       // pinned, mapped staging of x (+ the top row)
    double* m_x = nullptr;       // its device-visible address
    size_t h_x_elems = 0;
    int* h_top = nullptr;        // pinned
    void* graph_exec[kTriNumMatrices] = {};  // hipGraphExec_t per matrix
    uint64_t graph_key[kTriNumMatrices] = {};  // schedule captured for
    void* ev[2] = {nullptr, nullptr};
  };
  // TriangularMatrix::TransposeLowerSolve (sparse.cc:899-955) on one CU,
  // bit-identical. MILP_DEVICE_SOLVE=off|force|auto (auto: m >= 16384).
  bool TransposeLowerSolve(const TriangularMatrix& t, uint64_t key,
                           std::vector<double>* x) override;
  bool LowerSolve(const TriangularMatrix& lower, uint64_t key,
                  std::vector<double>* x) override;
  bool Solve(TriKind kind, const TriangularMatrix& t, uint64_t key, int start,
             std::vector<double>* x) override;
  bool SolvePair(TriKind kind, const TriangularMatrix& t, uint64_t key, std::vector<double>* x0,
                 std::vector<double>* x1) override;
  bool StartAsyncU(const TriangularMatrix& t, uint64_t key, const std::vector<double>& x) override;
  void FinishAsyncU(std::vector<double>* x) override;
  void DropAsyncU() override;
  bool SpecFlipEnabled() const { return spec_flip_ && tri_mapped_ && !tri_graph_; }

  // Accounting (roofline): launches, algorithmic bytes, HIP-event time.
  void SetTiming(bool on, uint32_t id_mask = ~0u);
  bool Timed(int id) const { return timing_ && (timing_ids_ >> (id & 31) & 1u) != 0; }
  const mi_lp_kernel_stats& stats();  // collects the pending event timings
  void ResetStats();
  void Synchronize();
  int dense_columns() const { return nd_; }
  // The U schedule in use (levels, listed outputs, entries; zeros if none).
  void TriScheduleShape(int64_t* levels, int64_t* outputs, int64_t* entries) const {
    const TriSchedule& s = tri_sched_[kTriU];
    *levels = s.ok ? s.levels : 0;
    *outputs = s.ok && !s.rows_upto.empty() ? s.rows_upto.back() : 0;
    *entries = s.ok && !s.entries_upto.empty() ? s.entries_upto.back() : 0;
  }

  // --- column shards ----------------------------------------
  // MILP_SHARDS=S > 1 splits the columns of [A | I] into S contiguous blocks
  // (64-column aligned, balanced by entries), each owned by a DeviceLp of its
  // own on MILP_SHARD_DEVICES (a comma list; default: this handle's device,
  // the "virtual" split). Every per-column operation (pricing, update row,
  // list dots, the dual device mode) runs shard by shard and the results are
  // joined in column order: the bound of the dual ratio test is a min over
  // shards, the candidates and update-row lists a concatenation. Row sums,
  // column norms and the triangular solves stay on this handle (full copy).
  int num_shards() const { return shards_.empty() ? 1 : static_cast<int>(shards_.size()); }
  // Cross-process split (include/mi_lp.h mi_lp_set_exchange): this process
  // owns block `rank` of `world`; fn all-gathers byte strings in rank order.
  using ExchangeFn = int (*)(void* ctx, const void* send, int64_t send_bytes, void* recv,
                             const int64_t* recv_bytes);
  void SetExchange(int rank, int world, void* ctx, ExchangeFn fn);
  bool IsLocalShard(int s) const { return shards_.empty() || shards_[s] != nullptr; }
  // Batched small-LP launches for this handle (the batch APIs turn it on for
  // their duration; MILP_SMALL_BATCH=1 turns it on everywhere, =0 nowhere).
  void SetSmallBatch(bool on);
  // A batch's few heaviest LPs take a high-priority stream, so their device
  // round trips do not queue behind the light LPs' kernels (the suite's wall
  // is their chain); applied now if the matrix is on the device, else at
  // its upload. false restores the process default (MILP_STREAM_PRIORITY).
  void SetBatchPriority(bool high);
  // Batched small LPs whose dual loop runs as a device segment (csrc/sdual):
  // the once-per-solve row sums and column dots outside the loop run on the
  // host thread that owns the LP (Glop's order, the kernels' bits) instead of
  // as single launches that queue behind hundreds of other LPs' work.
  void SetHostSmallOps(bool on) { host_small_ops_ = on; }
  // Whether a chip-wide update-row compaction also writes the list into
  // mapped host memory (off in dual device mode: the host reads the list
  // rarely, and then downloads it).
  void SetListMirror(bool on) { list_mirror_ = on; }
  bool host_small_ops() const { return host_small_ops_; }
  bool small_batch() const { return small_batch_; }
  int shard_begin(int s) const { return shard_begin_[s]; }

  // --- device dual simplex segment (csrc/sdual) ----------------------------
  // A device arena and a pinned staging image of at least `bytes`; the
  // RevisedSimplex side packs into sdual_staging() with pointers into
  // sdual_arena(), SdualRun moves [0, bytes) in, runs the segment on one
  // workgroup and moves it back (fiber-aware wait).
  // The mailbox (pinned, coherent, mapped) carries the segment's
  // factorization requests: rows basis entries and an LuImage of lu_cap.
  void SdualReserve(size_t bytes, int rows, int64_t lu_cap);
  void SdualFree();
  char* sdual_staging() const { return static_cast<char*>(sdual_staging_); }
  uintptr_t sdual_arena() const { return reinterpret_cast<uintptr_t>(sdual_arena_); }
  // serve(ctx) answers a request (the mailbox flag is 1) by writing an
  // LuImage into sdual_mailbox_image(); SdualRun then raises the flag to 2.
  void SdualRun(size_t bytes, const double* arena_coeff, int n, void (*serve)(void*), void* ctx);
  void SdualRunPooled(size_t bytes, const double* arena_coeff, int n, void (*serve)(void*),
                      void* ctx);
  sdual::Mailbox* sdual_mailbox() const { return sdual_mb_; }
  const int32_t* sdual_mailbox_basis() const { return sdual_mb_basis_; }
  char* sdual_mailbox_image() const { return sdual_mb_image_; }
  void SdualMailboxDevice(sdual::Mailbox** mb, int32_t** basis, char** image) const;
  void SdualMatrix(const int64_t** starts, const int32_t** rows, const double** vals,
                   const int64_t** t_starts, const int32_t** t_cols,
                   const double** t_vals) const;

 private:
  template <typename T>
  T* Alloc(size_t n);
  void Upload(void* dst, const void* src, size_t bytes);
  void Download(void* dst, const void* src, size_t bytes);
  void WaitStream();
  // Batched small-LP launches (MILP_SMALL_BATCH=1): the request goes into
  // this handle's slot of the device's SmallBatcher instead of a launch of
  // its own; WaitStream then waits for the slot's done word.
  template <typename Args>
  void LaunchSmall(int kind, const Args& args);
  void WaitSmallBatch();
  void RestoreDevice();  // after a fiber yield
  bool small_batch_ = false;
  bool host_small_ops_ = false;
  int batch_slot_ = -1;
  unsigned long long batch_seq_ = 0;
  bool batch_pending_ = false;
  void BeginKernel(int id);
  void EndKernel(int id, double bytes, bool count_launch = true);
  void* TakeEvent();
  void DrainTimings();
  milp_kernels::ScanState NextScan();
  void CheckScan();
  int* h_scan_fail_ = nullptr;  // mapped: a look-back wait ran out
  int* m_scan_fail_ = nullptr;
  int ShardOf(int col) const;
  void CreateShards();
  DeviceLp& Shard(int s);  // sets the shard's device current
  void ShardedUpload(const CompactSparseMatrix& csc);
  void ShardedSetMask(Mask which, const uint64_t* words, int num_words);
  void ShardedUpdateRowColumnWise(const std::vector<double>& rho, double drop,
                                  int64_t relevant_entries, const std::vector<double>* w);
  void ShardedUpdateRowRowWise(const std::vector<int>& filtered_rows,
                               const std::vector<double>& rho, int algorithm, double drop);
  void ShardedFetchUpdateRow(std::vector<int>* positions, std::vector<double>* values);
  double ShardedReadCoefficient(int col);
  void ShardedListDotsOverUpdateRow(const std::vector<double>& v, std::vector<double>* out);
  void ShardedListDots(const std::vector<int>& cols, const std::vector<double>& v,
                       std::vector<double>* out);
  void ShardedPricing(const std::vector<double>& c, const std::vector<double>& y,
                      std::vector<double>* rc, const std::vector<double>* w,
                      std::vector<double>* list_dots);
  void ShardedDualBegin(const std::vector<double>& rc, const std::vector<uint8_t>& colbits,
                        const std::vector<double>& bound_diff);
  void ShardedDualSetColBits(const std::vector<int32_t>& cols, const std::vector<uint8_t>& bits);
  void ShardedDualTakePricedReducedCosts();
  void ShardedDualDownloadReducedCosts(std::vector<double>* rc);
  void ShardedDualSetReducedCost(int col, double value);
  void ShardedDualRatioCandidates(double sign, double threshold, double harris_tolerance,
                                  double minimum_delta, double variation_magnitude,
                                  DualCandidates* out);
  void ShardedDualUpdateReducedCosts(double mult, int leaving_col, double leaving_value,
                                     int entering_col);
  void ShardedDualBoxedFlips(const std::vector<int>* cols, double threshold,
                             std::vector<uint8_t>* flags);
  void ShardedStats();
  void FlushOwnMasks();
  bool is_shard_ = false;
  std::vector<std::unique_ptr<DeviceLp>> shards_;  // null: a block owned by another process
  ExchangeFn exchange_fn_ = nullptr;
  void* exchange_ctx_ = nullptr;
  int exchange_rank_ = 0;
  int exchange_world_ = 1;
  void ExchangeParts(std::vector<std::string>* parts);
  std::vector<int> shard_begin_;
  bool own_mask_dirty_[kNumMasks] = {false, false, false};
  mi_lp_kernel_stats agg_stats_{};
  void Compact(int n);  // flags_ -> list_ (ascending) + coefficients, async
  void NextRowTag();
  void UpdateRowRowWiseSmall(const std::vector<int>& filtered_rows,
                             const std::vector<double>& rho, int algorithm, double drop,
                             double entries, bool serial);
  void UpdateRowColumnWiseSmall(const std::vector<double>& rho, double drop,
                                int64_t relevant_entries, const std::vector<double>* w);
  void UploadMask(Mask which);
  void FlushRelevantMask();
  void CopyHost(void* dst, const void* src, size_t bytes);
  void AccountList(const std::vector<int>& positions);
  void BuildDenseBlock();
  // Launches the CSC kernel over the sparse columns (all columns when there is
  // no dense block) and the dense-block kernel; mode as in column_dot.
  void LaunchColumnDots(int mode, const double* d_y, const double* d_c, double* d_out,
                        const double* d_y2 = nullptr, double* d_out2 = nullptr);
  void Check(int err, const char* what);
  // Gather lists of the outputs c in [fni, nc): entries (dependency row,
  // value) of output c at [st[c], st[c+1]) of idx/val, evaluated from the end
  // when `reverse`. Dependencies are rows > c (descending) or < c.
  void BuildTriSchedule(TriSchedule* s, int nc, int fni, bool ones, const double* diag,
                        const int64_t* st, const int32_t* idx, const double* val, bool reverse,
                        bool descending, bool sequential, uint64_t key, void* stream);
  bool TriSolve(int which, const TriangularMatrix& t, uint64_t key, std::vector<double>* x);
  bool TriPrepare(int which, const TriangularMatrix& t, uint64_t key, int slot,
                  const std::vector<double>& x);
  // Gather lists of a scatter loop: output r lists (column j, t[r, j]) for
  // the columns j >= fni holding row r, by ascending j (or descending).
  void TransposeColumns(const TriangularMatrix& t, bool descending);
  void TriReserve(TriBuffer* b, size_t bytes);
  void PrepareTriContext(int slot, int rows, int pos);
  milp_kernels::TriSolveArgs TriArgs(const TriSchedule& s, const TriContext& c) const;
  void TriCopyIn(const TriSchedule& s, const TriContext& c);
  void TriCopyOut(const TriSchedule& s, const TriContext& c);
  void EnqueueTriKernels(const TriSchedule& s, const milp_kernels::TriSolveArgs& a,
                         void* stream);
  void CaptureTriGraph(int which, TriContext* c);
  void FreeTriBuffers();

  void* sdual_arena_ = nullptr;
  void* sdual_staging_ = nullptr;
  void* sdual_staging_dev_ = nullptr;
  size_t sdual_cap_ = 0;
  void* sdual_mb_block_ = nullptr;  // pinned: Mailbox | basis | LuImage
  size_t sdual_mb_cap_ = 0;
  sdual::Mailbox* sdual_mb_ = nullptr;
  int32_t* sdual_mb_basis_ = nullptr;
  char* sdual_mb_image_ = nullptr;
  void* sdual_mb_device_ = nullptr;

  int device_ = -1;
  void* stream_ = nullptr;  // hipStream_t
  void* ev_start_ = nullptr;
  void* ev_stop_ = nullptr;
  bool timing_ = false;
  uint32_t timing_ids_ = ~0u;  // kernel ids bracketed with events while timing_
  struct PendingTiming {
    void* start;  // hipEvent_t
    void* stop;
    int id;
  };
  std::vector<PendingTiming> ev_pending_;
  std::vector<void*> ev_pool_;
  void* ev_open_ = nullptr;  // recorded by BeginKernel, closed by EndKernel
  double drop_ = 0.0;  // drop tolerance of the current update row
  mi_lp_kernel_stats stats_{};
  std::vector<void*> allocations_;

  int m_ = 0;
  int n_total_ = 0;  // N = n + m
  int64_t nnz_ = 0;
  double avg_col_len_ = 0.0;
  // CSC of [A | I]
  int64_t* d_starts_ = nullptr;
  int32_t* d_rows_ = nullptr;
  double* d_vals_ = nullptr;
  // CSR of [A | I]
  int64_t* d_t_starts_ = nullptr;
  int32_t* d_t_cols_ = nullptr;
  double* d_t_vals_ = nullptr;
  std::vector<int64_t> h_starts_;  // host copy for byte accounting
  // Dense column block (kernel_args.h DenseArgs): full structural columns.
  int nd_ = 0;
  int ns_ = 0;  // remaining (sparse) columns
  double* d_dense_body_ = nullptr;
  double* d_dense_tail_ = nullptr;
  int32_t* d_dense_cols_ = nullptr;
  int32_t* d_sparse_cols_ = nullptr;
  uint8_t* d_is_dense_ = nullptr;
  std::vector<uint8_t> h_is_dense_;
  std::vector<uint64_t> h_dense_words_;
  int64_t sparse_entries_ = 0;  // entries of the sparse columns
  std::vector<int64_t> h_t_starts_;

  // masks
  uint64_t* d_masks_[kNumMasks] = {nullptr, nullptr, nullptr};
  std::vector<uint64_t> h_masks_[kNumMasks];
  uint64_t* h_pin_mask_[kNumMasks] = {nullptr, nullptr, nullptr};
  // Changed-word updates of the masks: (index, word) pairs in mapped memory,
  // one slot per mask, guarded by ev_mask_ like the full-upload slot.
  static constexpr int kMaskDiffMax = 512;
  bool mask_on_device_[kNumMasks] = {false, false, false};  // device copy == h_masks_
  char* h_mask_diff_ = nullptr;
  char* m_mask_diff_ = nullptr;
  void* ev_mask_[kNumMasks] = {nullptr, nullptr, nullptr};  // hipEvent_t: slot reusable
  int mask_words_ = 0;

  // scratch
  double* d_vec_m_ = nullptr;    // rho / y / dli / ...
  double* d_vec_m2_ = nullptr;   // row-sum output
  double* d_vec_w_ = nullptr;    // second dot vector of the fused update row
  bool fused_ready_ = false;     // d_out_n_ holds w . a_j for the listed columns
  std::vector<double> fused_w_;  // the w those dots were computed with
  double* d_vec_n_ = nullptr;    // x / c
  double* d_coeff_ = nullptr;    // update row coefficients (persistent)
  uint8_t* d_flags_ = nullptr;
  int32_t* d_list_ = nullptr;    // compacted listed positions
  int* d_count_ = nullptr;
  double* d_out_n_ = nullptr;    // per-column results
  double* d_out_list_ = nullptr; // per-list-slot results
  int32_t* d_cols_ = nullptr;    // arbitrary column list / filtered rows
  void* d_upd_in_ = nullptr;     // row-wise inputs: rows, multipliers, CSR offsets
  void* h_upd_in_ = nullptr;     // pinned staging of d_upd_in_
  uint32_t* d_row_tag_ = nullptr; // filtered-row marks of the column-order row-wise kernel
  int32_t* d_row_pos_ = nullptr;
  uint32_t row_tag_ = 0;
  unsigned long long* d_scan_status_ = nullptr;  // ordered compactions (kernel_args.h)
  unsigned int* d_scan_ticket_ = nullptr;
  unsigned int scan_epoch_ = 0;
  uint64_t dual_calls_ = 0;  // alternates the pass-1 bound slots
  double* d_out_n2_ = nullptr;   // w . a_j of the fused pricing pass
  int list_count_ = 0;
  uint64_t list_epoch_ = 0;
  int64_t list_entries_ = 0;  // CSC entries over the listed sparse columns
  int64_t list_dense_ = 0;    // listed dense columns
  int dense_unroll_ = 8;      // MILP_DENSE_UNROLL: 16-B loads in flight per lane
  // Above this many filtered rows the row-wise update row runs column by
  // column (MILP_ROWWISE_CHUNK_MAX_ROWS); both kernels give identical bits.
  int rowwise_chunk_max_rows_ = 16;
  // Rows holding every structural column (MILP_FULL_ROWS=off disables the
  // full-row kernel).
  std::vector<uint8_t> h_row_full_;
  int num_structural_ = 0;
  bool full_rows_enabled_ = true;
  // The column-order kernel sorts a column's hits in registers: used only
  // when no column is longer than this (kernel kMaxColumnHits).
  static constexpr int kColumnKernelMaxColumnLength = 32;
  int64_t max_col_len_ = 0;

  // pinned staging
  int32_t* h_pin_i_ = nullptr;
  double* h_pin_d_ = nullptr;
  double* h_pin_d2_ = nullptr;
  double* h_pin_w_ = nullptr;
  int* h_pin_count_ = nullptr;
  int last_list_len_ = 0;
  // Mapped host memory written by the small-N compaction kernel.
  void* h_map_ = nullptr;
  int* h_map_count_ = nullptr;
  int32_t* h_map_list_ = nullptr;
  double* h_map_vals_ = nullptr;
  int* d_map_count_ = nullptr;
  int32_t* d_map_list_ = nullptr;
  double* d_map_vals_ = nullptr;
  bool list_mirror_ = true;
  bool mapped_result_ = false;  // the last Compact wrote to h_map_
  // Small LPs (N <= kSmallLdsCols): the row-wise update row is one launch
  // (row_wise_small_kernel) reading its inputs, including the relevant mask,
  // from mapped host memory (MILP_SMALL_FUSED=off disables).
  bool small_fused_enabled_ = true;
  // Up to this many filtered rows (and kSmallEntries entries) the small
  // row-wise update row applies rows in turn, above it column by column
  // (MILP_SMALL_SERIAL_ROWS). Measured on configs 3 and 4: rows in turn win
  // whenever they fit; the column pass reads all of A.
  int small_serial_rows_ = 1024;
  // Workgroup size of row_wise_small_kernel (MILP_SMALL_THREADS: 1024 or 256;
  // 256 measured 4-5 % slower on the config-4 probe).
  int small_threads_ = 1024;
  // Medium LPs (kSmallLdsCols < N <= kMediumCols, MILP_MEDIUM=off disables)
  // solved in a batch: the serial row-wise update row takes one batched launch
  // (accumulators in an LDS hash table); everything else is generic.
  bool medium_enabled_ = true;
  bool medium_ = false;
  void* h_small_in_ = nullptr;
  int32_t* h_small_rows_ = nullptr;
  double* h_small_rho_ = nullptr;
  uint64_t* h_small_mask_ = nullptr;
  const int32_t* d_small_rows_ = nullptr;
  const double* d_small_rho_ = nullptr;
  const uint64_t* d_small_mask_ = nullptr;
  double* h_small_y_ = nullptr;    // list-dots input (m)
  double* h_small_out_ = nullptr;  // list-dots output (N)
  const double* d_small_y_ = nullptr;
  double* d_small_out_ = nullptr;
  double* h_small_w_ = nullptr;     // column-wise update row: w (m)
  double* h_small_dots_ = nullptr;  // its w dots, list order (N)
  const double* d_small_w_ = nullptr;
  double* d_small_dots_ = nullptr;
  bool small_dots_mapped_ = false;  // fused_ready_ dots are in h_small_dots_
  bool mask_dirty_ = false;  // h_masks_[kRelevant] not yet uploaded
  bool small_inflight_ = false;  // a launch may still read h_small_in_
  // dual device mode
  bool dual_ready_ = false;
  double* d_rc_ = nullptr;
  uint8_t* d_colbits_ = nullptr;
  double* d_bound_diff_ = nullptr;
  unsigned long long* d_best_ = nullptr;
  uint8_t* d_slot_flags_ = nullptr;
  int32_t* d_slots_ = nullptr;
  int* d_num_slots_ = nullptr;
  int32_t* d_cand_col_ = nullptr;
  double* d_cand_coeff_ = nullptr;
  double* d_cand_rc_ = nullptr;
  int32_t* d_small_cols_ = nullptr;
  uint8_t* d_small_bits_ = nullptr;
  int32_t* h_cand_col_ = nullptr;
  double* h_cand_coeff_ = nullptr;
  double* h_cand_rc_ = nullptr;
  int* h_dual_counts_ = nullptr;  // [num candidates, list count] (mapped)
  int* m_dual_counts_ = nullptr;  // its device pointer
  int32_t* m_cand_col_ = nullptr;  // device pointers of the mapped h_cand_*
  double* m_cand_coeff_ = nullptr;
  double* m_cand_rc_ = nullptr;
  int32_t* h_cb_cols_ = nullptr;  // column-bit changes (pinned, event-guarded)
  uint8_t* h_cb_bits_ = nullptr;
  void* ev_cb_[2] = {nullptr, nullptr};  // column-bit slots (alternating)
  int cb_slot_ = 0;
  int32_t* m_cb_cols_ = nullptr;  // device pointers of the mapped h_cb_* / h_flip_*
  uint8_t* m_cb_bits_ = nullptr;
  int32_t* m_flip_cols_ = nullptr;
  uint8_t* m_flip_flags_ = nullptr;
  int32_t* h_flip_cols_ = nullptr;
  uint8_t* h_flip_flags_ = nullptr;
  // DualBoxedFlipsEarly's launch (its columns and flags in h_flip_*).
  struct EarlyFlips {
    bool pending = false;
    int n = 0;
    double threshold = 0.0;
    uint64_t rc_epoch = 0;
    std::vector<int32_t> cols_changed;  // column bits written since the launch
  };
  EarlyFlips early_flips_;
  bool early_flips_on_ = true;
  uint64_t rc_epoch_ = 0;  // counts the writes of d_rc_
  void* ev_flips_ = nullptr;
  void WaitEarlyFlips();
  int last_candidates_ = 0;
  int dual_list_count_ = 0;  // update-row length seen by the last ratio test
  // Above this many breakpoints under the first bound, the dual ratio test
  // tightens it on the device (MILP_DUAL_TIGHTEN_MIN).
  int tighten_min_candidates_ = 512;
  unsigned long long* d_best2_ = nullptr;
  milp_kernels::TightenState* d_tighten_ = nullptr;
  bool tighten_sort_ = false;  // MILP_DUAL_TIGHTEN_SORT=1: the full radix sort + walk
  int tighten_target_ = 512;   // MILP_TIGHTEN_TARGET: keys the selection keeps (tests go small)
  unsigned long long* d_keys_in_ = nullptr;
  unsigned long long* d_keys_out_ = nullptr;
  int32_t* d_sorted_slots_ = nullptr;
  void* d_sort_temp_ = nullptr;
  size_t sort_temp_bytes_ = 0;
  // dense triangular solves (device_solve.hip): the level-ordered schedules
  // of the last factorization's U and L, rebuilt when its key changes.
  int tri_mode_ = 0;  // 0 auto, 1 force, 2 off
  int tri_min_rows_ = 16384;
  int tri_wide_level_ = 600;  // MILP_TRI_WIDE: wider levels run over the chip
  int tri_debug_left_ = 0;
  bool tri_graph_ = false;    // MILP_TRI_GRAPH=1: replay a captured graph (measured 5-10 % slower on C5 than 4 direct launches)
  bool tri_tau_ = true;       // MILP_TRI_TAU
  bool tri_mapped_ = true;    // MILP_TRI_MAPPED: zero-copy staging inside the plan
  bool tri_syncfree_ = true;  // MILP_TRI_SYNCFREE: readiness-driven single launch
  int tri_syncfree_min_levels_ = 0;  // MILP_TRI_SYNCFREE_MIN_LEVELS: shallower -> level plan
  bool tri_fuse0_ = true;     // MILP_TRI_FUSE0: level 0 inside the gather kernel
  int tri_poll_max_ = 1;      // MILP_TRI_POLL_MAX: sync-free poll backoff cap (s_sleep units)
  int tri_persist_groups_ = 0;  // MILP_TRI_PERSIST: persistent sync-free workgroups (0: off)
  int tri_xcd_stride_ = 1;    // MILP_TRI_XCD=1: the persistent ones on one XCD (stride 8)
  bool stream_priority_ = false;  // MILP_STREAM_PRIORITY=1: solver stream high, tau stream low
  bool stream_priority_env_ = false;  // the process default above, for SetBatchPriority(false)
  bool stream_prioritized_ = false;  // stream_ was created at the highest priority
  void SetStreamPriority(bool high);
  bool tri_lower_ = true;     // MILP_TRI_LOWER: the L solves too
  // Off by default since round 4: with the host's dense loops faster (the
  // parallel non-zero appends), config 5's window runs 3 % faster without the
  // device BTRAN loops and 5 % faster without either (scripts/gpu_r04_ab2.sh).
  bool tri_btran_ = false;    // MILP_TRI_BTRAN=1: the other dense loops (BTRAN, UpperSolve) too
  // MILP_TRI_PAIR=0: the direction's and tau's U solves as two launches on
  // two streams. On by default since round 5 (config-5 window 724/759 ->
  // 773/827 it/s, profiles/r05_tri).
  bool tri_pair_ = true;
  // MILP_TRI_PAD=1: every chip-wide level starts on a wave boundary (empty
  // padding records). Needed while the sync-free stores sat below the wait
  // loop (a wave holding an output and its reader deadlocked); since the
  // loop exit is wave-uniform a reader may share its producer's wave.
  bool tri_pad_ = false;
  int tri_min_width_ = 128;   // MILP_TRI_MIN_WIDTH (auto mode)
  // MILP_TRI_CHAIN=1: single-workgroup segments; a narrow segment is a run
  // of at least MILP_TRI_CHAIN_MIN_LEVELS levels of at most
  // MILP_TRI_CHAIN_WIDTH outputs each (tri_chain_kernel). Off by default
  // since round 5: with the sync-free stores kept inside the wait loop one
  // chip-wide launch is faster (config-5 window 668 -> 713 it/s,
  // profiles/r05_tri).
  bool tri_chain_ = false;
  int tri_chain_width_ = 512;
  int tri_chain_min_levels_ = 4;
  uint64_t* d_tri_clock_ = nullptr;
  // Dense tail of BTRAN's forward U^T solve (dense_tail.hip): the last
  // factorization's tail columns on the device, rebuilt when its key changes.
  // Opt-in (MILP_DENSE_TAIL=1): on config 2's late bases each tail column's
  // entries are ~10 ascending runs of rows, so its chain stalls on the first
  // tail row of its order and most of it folds only after the previous
  // column -- a sequential chain the device runs slower than the host loop
  // (late window 17 vs 53 it/s). MILP_DENSE_TAIL_MIN_ENTRIES
  // (default 2^20) and MILP_DENSE_TAIL_MIN_COLS (default 128) gate it.
  struct DenseTail {
    uint64_t key = ~0ull;
    bool ok = false;
    int n = 0, fni = 0, t = 0;
    int64_t entries = 0;
    TriBuffer starts, cur, rows, vals, diag, x, pre;
    double* h_in = nullptr;    // pinned, mapped: x in (n values), then the fail word
    double* m_in = nullptr;
    double* h_out = nullptr;   // pinned, mapped: x[t, n) out
    double* m_out = nullptr;
    int cap_n = 0, cap_t = 0;
  };
  DenseTail dense_tail_;
  int dense_tail_mode_ = 0;
  int64_t dense_tail_min_entries_ = int64_t{1} << 20;
  int dense_tail_min_cols_ = 128;
  bool DenseTailSolve(const TriangularMatrix& t, uint64_t key, std::vector<double>* x);
  void FreeDenseTail();
  TriSchedule tri_sched_[kTriNumMatrices];
  // Per solving thread: 0 = the solver's thread (the handle's stream),
  // 1 = BasisFactorization's tau worker (its own stream), 2 = the second
  // vector of a pair solve (the solver's stream), 3 = the solver's
  // asynchronous U solve (StartAsyncU, its own stream).
  static constexpr int kTriSlots = 4;
  TriContext tri_ctx_[kTriSlots];
  // The one asynchronous U solve (slot 3): launched, or trivial (nothing to
  // compute: the input is the result).
  struct AsyncU {
    bool active = false;
    bool trivial = false;
    bool timed = false;  // events recorded around the launch
    int rows = 0;
    int first = 0;
    int top = 0;
    double bytes = 0.0;
  };
  AsyncU async_u_;
  // MILP_SPEC_FLIP=0 turns the speculative flip FTRAN (lu.h) off; read by the
  // dual loop through SpecFlipEnabled().
  bool spec_flip_ = true;
  std::mutex tri_mu_;  // schedule (re)builds and graph captures
  void* h_tri_stage_ = nullptr;  // pinned staging of the schedule upload
  size_t tri_stage_bytes_ = 0;
  std::vector<int64_t> tri_lt_starts_;  // L's rows (gather lists), built per factorization
  std::vector<int32_t> tri_lt_idx_;
  std::vector<double> tri_lt_val_;
};

}  // namespace milp

#endif  // MILP_DEVICE_LP_H_
