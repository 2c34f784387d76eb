// DeviceLp: dense triangular solves of the basis factorization (see
// device_solver.h and kernels/tri_solve.hip).
//
// Glop's FTRAN ends with U x = b (lu_factorization.cc:314-331). When the
// result is too dense for the hypersparse path it runs
// TriangularMatrix::TransposeLowerSolve (sparse.cc:899-955) on U's transpose:
// a gather over every row. On config 5 (m = 100 000) that is most of the
// host time of an iteration, twice per iteration (direction, bound flips).
// U changes only at refactorization, so its level schedule is built and
// uploaded once per factorization; each solve then moves the right-hand side
// in, replays the captured launch plan and moves the result out. The solver's
// thread and BasisFactorization's tau worker solve concurrently, each with
// its own stream, buffers and graph (TriContext); the schedule is shared.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "../kernels/kernel_args.h"
#include "device_lp.h"
#include "host_pool.h"
#include "lu.h"

namespace milp {

namespace {
inline hipStream_t Stream(void* p) { return reinterpret_cast<hipStream_t>(p); }

struct SolveCallTimer {
  mi_lp_kernel_stats* stats;
  int id;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  SolveCallTimer(mi_lp_kernel_stats* s, int i) : stats(s), id(i) {}
  ~SolveCallTimer() {
    stats->call_ms[id] +=
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
            .count();
  }
};

void FreeBuffer(DeviceLp::TriBuffer* b) {
  if (b->ptr != nullptr) (void)hipFree(b->ptr);
  *b = DeviceLp::TriBuffer();
}

}  // namespace

void DeviceLp::TriReserve(TriBuffer* b, size_t bytes) {
  if (b->ptr != nullptr && b->bytes >= bytes) return;
  FreeBuffer(b);
  const size_t n = std::max<size_t>(bytes, 16) + bytes / 4;
  Check(hipMalloc(&b->ptr, n), "hipMalloc (triangular solve)");
  b->bytes = n;
}

void DeviceLp::FreeTriBuffers() {
  for (TriBuffer& b : tri_buf_) FreeBuffer(&b);
  if (d_tri_clock_ != nullptr) (void)hipFree(d_tri_clock_);
  d_tri_clock_ = nullptr;
  for (int slot = 0; slot < 2; ++slot) {
    TriContext& c = tri_ctx_[slot];
    if (c.graph_exec != nullptr) {
      (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(c.graph_exec));
    }
    FreeBuffer(&c.x);
    FreeBuffer(&c.y);
    FreeBuffer(&c.top);
    if (c.h_x != nullptr) (void)hipHostFree(c.h_x);
    if (c.h_top != nullptr) (void)hipHostFree(c.h_top);
    for (void* e : c.ev) {
      if (e != nullptr) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e));
    }
    if (slot == 1 && c.stream != nullptr) {
      (void)hipStreamSynchronize(Stream(c.stream));
      (void)hipStreamDestroy(Stream(c.stream));
    }
    c = TriContext();
  }
  if (h_tri_stage_ != nullptr) (void)hipHostFree(h_tri_stage_);
  h_tri_stage_ = nullptr;
  tri_stage_bytes_ = 0;
  tri_key_ = 0;
  tri_ok_ = false;
}

// Level schedule of t's TransposeLowerSolve: output c (a column of t, rows
// first_non_identity .. num_cols-1) depends on the rows of its entries, all
// > c. level(c) = 0 without entries, else 1 + the deepest entry. Outputs
// with no entries and a unit diagonal are the identity and are not listed.
// Positions: the listed outputs by level (descending c inside a level, the
// host order), then the other rows >= first_non_identity (read, never
// written). Entries refer to positions.
void DeviceLp::BuildTriSchedule(const TriangularMatrix& t, uint64_t key, void* stream) {
  tri_key_ = key;
  tri_ok_ = false;
  const int nc = t.num_cols();
  const int fni = t.GetFirstNonIdentityColumn();
  tri_rows_ = nc;
  tri_first_col_ = fni;
  tri_ones_ = t.all_diagonal_coefficients_are_one_;
  const int64_t nnz = t.starts_[nc] - t.starts_[0];
  if (nnz >= (int64_t{1} << 31)) return;
  std::vector<int32_t> level(nc, 0);
  int depth = 0;
  int num_work = 0;
  for (int c = nc - 1; c >= fni; --c) {
    int l = 0;
    for (int64_t i = t.starts_[c]; i < t.starts_[c + 1]; ++i) {
      l = std::max(l, level[t.rows_[i]] + 1);
    }
    level[c] = l;
    depth = std::max(depth, l);
    if (l > 0 || !tri_ones_) ++num_work;
  }
  const int num_pos = nc - fni;
  // Counting sort by level.
  std::vector<int32_t> level_start(depth + 2, 0);
  for (int c = nc - 1; c >= fni; --c) {
    if (level[c] > 0 || !tri_ones_) ++level_start[level[c] + 1];
  }
  for (int l = 0; l <= depth; ++l) level_start[l + 1] += level_start[l];
  tri_work_ = num_work;
  tri_pos_ = num_pos;
  tri_levels_ = depth + 1;
  tri_level_width_.resize(depth + 1);
  for (int l = 0; l <= depth; ++l) tri_level_width_[l] = level_start[l + 1] - level_start[l];
  // Launch segments: each wide level alone over the chip, each run of narrow
  // levels as one single-CU launch (tri_solve.hip).
  tri_segments_.clear();
  for (int l = 0; l <= depth;) {
    const int w = tri_level_width_[l];
    if (w == 0) {
      ++l;
      continue;
    }
    if (w > tri_wide_level_) {
      tri_segments_.push_back(-l - 1);
      tri_segments_.push_back(std::min(1024, (w + 255) / 256));
      ++l;
      continue;
    }
    int e = l;
    while (e <= depth && tri_level_width_[e] <= tri_wide_level_) ++e;
    tri_segments_.push_back(l);
    tri_segments_.push_back(e);
    l = e;
  }
  if (const char* d = std::getenv("MILP_TRI_DEBUG")) tri_debug_left_ = std::atoi(d);
  // Positions.
  std::vector<int32_t> pos_row(num_pos);
  std::vector<int32_t> pos_of(nc, -1);
  {
    std::vector<int32_t> next(level_start.begin(), level_start.end() - 1);
    int tail = num_work;
    for (int c = nc - 1; c >= fni; --c) {
      const int k = (level[c] > 0 || !tri_ones_) ? next[level[c]]++ : tail++;
      pos_row[k] = c;
      pos_of[c] = k;
    }
  }
  int64_t num_ovf = 0;
  tri_max_entries_ = 0;
  tri_rows_over_[0] = tri_rows_over_[1] = tri_rows_over_[2] = 0;
  for (int k = 0; k < num_work; ++k) {
    const int c = pos_row[k];
    const int64_t n = t.starts_[c + 1] - t.starts_[c];
    if (n > 4) num_ovf += n;
    tri_max_entries_ = std::max<int>(tri_max_entries_, static_cast<int>(n));
    tri_rows_over_[0] += n > 4;
    tri_rows_over_[1] += n > 16;
    tri_rows_over_[2] += n > 64;
  }
  // Staging layout, 16-byte aligned pieces.
  auto al = [](size_t b) { return (b + 15) / 16 * 16; };
  const size_t b_levels = al(size_t(depth + 2) * 4);
  const size_t b_row = al(size_t(num_work) * 4);
  const size_t b_n = al(size_t(num_work) * 4);
  const size_t b_entry = size_t(num_work) * 16;
  const size_t b_value = size_t(num_work) * 32;
  const size_t b_diag = tri_ones_ ? 0 : al(size_t(num_work) * 8);
  const size_t b_ovf_pos = al(size_t(num_ovf) * 4);
  const size_t b_ovf_val = al(size_t(num_ovf) * 8);
  const size_t b_pos_row = al(size_t(num_pos) * 4);
  const size_t sizes[kTriNumStaged] = {b_levels, b_row,     b_n,       b_entry,  b_value,
                                       b_diag,   b_ovf_pos, b_ovf_val, b_pos_row};
  size_t offs[kTriNumStaged];
  size_t bytes = 0;
  for (int b = 0; b < kTriNumStaged; ++b) {
    offs[b] = bytes;
    bytes += sizes[b];
  }
  if (tri_stage_bytes_ < bytes) {
    if (h_tri_stage_ != nullptr) (void)hipHostFree(h_tri_stage_);
    h_tri_stage_ = nullptr;
    Check(hipHostMalloc(&h_tri_stage_, bytes + bytes / 4 + 16), "pin");
    tri_stage_bytes_ = bytes + bytes / 4 + 16;
  }
  char* st = static_cast<char*>(h_tri_stage_);
  int32_t* lstart = reinterpret_cast<int32_t*>(st + offs[kTriLevels]);
  int32_t* rec_row = reinterpret_cast<int32_t*>(st + offs[kTriRecRow]);
  int32_t* rec_n = reinterpret_cast<int32_t*>(st + offs[kTriRecN]);
  int32_t* rec_entry = reinterpret_cast<int32_t*>(st + offs[kTriRecEntry]);
  double* rec_value = reinterpret_cast<double*>(st + offs[kTriRecValue]);
  double* diag = reinterpret_cast<double*>(st + offs[kTriDiag]);
  int32_t* ovf_pos = reinterpret_cast<int32_t*>(st + offs[kTriOvfPos]);
  double* ovf_value = reinterpret_cast<double*>(st + offs[kTriOvfValue]);
  std::copy(level_start.begin(), level_start.end(), lstart);
  std::copy(pos_row.begin(), pos_row.end(), reinterpret_cast<int32_t*>(st + offs[kTriPosRow]));
  // Entries of each listed output in evaluation order: the host walks the
  // column from its last entry down (sparse.cc:908-955).
  int64_t o = 0;
  for (int k = 0; k < num_work; ++k) {
    const int c = pos_row[k];
    const int64_t b = t.starts_[c], e = t.starts_[c + 1];
    const int n = static_cast<int>(e - b);
    rec_row[k] = c;
    rec_n[k] = n;
    if (n <= 4) {
      for (int j = 0; j < 4; ++j) {
        rec_entry[4 * k + j] = j < n ? pos_of[t.rows_[e - 1 - j]] : 0;
        rec_value[4 * k + j] = j < n ? t.coefficients_[e - 1 - j] : 0.0;
      }
    } else {
      rec_entry[4 * k] = static_cast<int32_t>(o);
      rec_entry[4 * k + 1] = rec_entry[4 * k + 2] = rec_entry[4 * k + 3] = 0;
      for (int j = 0; j < 4; ++j) rec_value[4 * k + j] = 0.0;
      for (int64_t i = e - 1; i >= b; --i) {
        ovf_pos[o] = pos_of[t.rows_[i]];
        ovf_value[o] = t.coefficients_[i];
        ++o;
      }
    }
    if (!tri_ones_) diag[k] = t.diagonal_coefficients_[c];
  }
  // Prefix counts by output row, for the byte accounting of a solve that
  // stops at `top`.
  tri_rows_upto_.assign(nc + 1, 0);
  tri_entries_upto_.assign(nc + 1, 0);
  for (int c = 0; c < nc; ++c) {
    const bool listed = c >= fni && pos_of[c] < num_work;
    tri_rows_upto_[c + 1] = tri_rows_upto_[c] + (listed ? 1 : 0);
    tri_entries_upto_[c + 1] =
        tri_entries_upto_[c] + (listed ? t.starts_[c + 1] - t.starts_[c] : 0);
  }
  for (int b = 0; b < kTriNumStaged; ++b) {
    if (sizes[b] == 0) continue;
    TriReserve(&tri_buf_[b], sizes[b]);
    Check(hipMemcpyAsync(tri_buf_[b].ptr, st + offs[b], sizes[b], hipMemcpyHostToDevice,
                         Stream(stream)),
          "H2D");
  }
  // The staging buffer is reused by the next build: wait for the copies.
  Check(hipStreamSynchronize(Stream(stream)), "sync");
  tri_ok_ = true;  // each context recaptures its graph for the new key
}

void DeviceLp::PrepareTriContext(int slot, int rows) {
  TriContext& c = tri_ctx_[slot];
  if (c.stream == nullptr) {
    if (slot == 0) {
      c.stream = stream_;
    } else {
      hipStream_t st;
      Check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
      c.stream = st;
    }
    for (void*& e : c.ev) {
      hipEvent_t ev;
      Check(hipEventCreate(&ev), "hipEventCreate");
      e = ev;
    }
    Check(hipHostMalloc(reinterpret_cast<void**>(&c.h_top), 64), "pin");
    TriReserve(&c.top, 16);
  }
  const void* old_x = c.x.ptr;
  const void* old_y = c.y.ptr;
  TriReserve(&c.x, size_t(rows) * 8);
  TriReserve(&c.y, size_t(std::max(tri_pos_, 1)) * 8);
  if (c.x.ptr != old_x || c.y.ptr != old_y) c.graph_key = 0;  // buffers moved
  // rows values + the top row (an int in the slot after them), mapped.
  if (c.h_x_elems < size_t(rows) + 1) {
    if (c.h_x != nullptr) (void)hipHostFree(c.h_x);
    c.h_x = nullptr;
    c.h_x_elems = size_t(rows) + size_t(rows) / 4 + 1;
    Check(hipHostMalloc(reinterpret_cast<void**>(&c.h_x), c.h_x_elems * sizeof(double),
                        hipHostMallocMapped),
          "pin");
    void* dev = nullptr;
    Check(hipHostGetDevicePointer(&dev, c.h_x, 0), "mapped pointer");
    c.m_x = static_cast<double*>(dev);
    c.graph_key = 0;
  }
}

milp_kernels::TriSolveArgs DeviceLp::TriArgs(const TriContext& c) const {
  milp_kernels::TriSolveArgs a;
  a.level_start = static_cast<const int32_t*>(tri_buf_[kTriLevels].ptr);
  a.rec_row = static_cast<const int32_t*>(tri_buf_[kTriRecRow].ptr);
  a.rec_n = static_cast<const int32_t*>(tri_buf_[kTriRecN].ptr);
  a.rec_entry = static_cast<const int4*>(tri_buf_[kTriRecEntry].ptr);
  a.rec_value = static_cast<const double2*>(tri_buf_[kTriRecValue].ptr);
  a.diag = tri_ones_ ? nullptr : static_cast<const double*>(tri_buf_[kTriDiag].ptr);
  a.ovf_pos = static_cast<const int32_t*>(tri_buf_[kTriOvfPos].ptr);
  a.ovf_value = static_cast<const double*>(tri_buf_[kTriOvfValue].ptr);
  a.pos_row = static_cast<const int32_t*>(tri_buf_[kTriPosRow].ptr);
  a.x = static_cast<double*>(c.x.ptr);
  a.y = static_cast<double*>(c.y.ptr);
  a.top = static_cast<int*>(c.top.ptr);
  a.host_x = tri_mapped_ ? c.m_x : nullptr;
  a.first_col = tri_first_col_;
  a.num_rows = tri_rows_;
  a.fail = reinterpret_cast<int*>(c.m_x + tri_rows_) + 1;
  a.num_work = tri_work_;
  a.num_pos = tri_pos_;
  a.num_levels = tri_levels_;
  a.clock = nullptr;
  return a;
}

// One solve = copy in (x[fni..nc), top), the launches of the segment plan,
// copy out (x[fni..nc)). Without debugging the launches are captured once per
// factorization (and context) into a HIP graph and replayed with one launch:
// the plan has tens of kernels, whose individual launches would cost more
// host time than their GPU time.
// Without zero-copy staging (MILP_TRI_MAPPED=0): copy-engine transfers.
void DeviceLp::TriCopyIn(const TriContext& c) {
  if (tri_mapped_) return;
  const int fni = tri_first_col_;
  const size_t in = size_t(tri_rows_ - fni);
  double* d_x = static_cast<double*>(c.x.ptr);
  Check(hipMemcpyAsync(d_x + fni, c.h_x + fni, in * sizeof(double), hipMemcpyHostToDevice,
                       Stream(c.stream)),
        "H2D");
  Check(hipMemcpyAsync(c.top.ptr, c.h_top, sizeof(int), hipMemcpyHostToDevice, Stream(c.stream)),
        "H2D");
}

void DeviceLp::TriCopyOut(const TriContext& c) {
  if (tri_mapped_) return;
  const int fni = tri_first_col_;
  const size_t in = size_t(tri_rows_ - fni);
  const double* d_x = static_cast<const double*>(c.x.ptr);
  Check(hipMemcpyAsync(c.h_x + fni, d_x + fni, in * sizeof(double), hipMemcpyDeviceToHost,
                       Stream(c.stream)),
        "D2H");
}

void DeviceLp::EnqueueTriKernels(const milp_kernels::TriSolveArgs& a, void* stream) {
  if (tri_syncfree_ && a.clock == nullptr && a.num_work <= milp_kernels::kTriSyncFreeMaxWork) {
    Check(milp_launch::tri_transpose_lower_syncfree(a, Stream(stream)), "tri syncfree");
    return;
  }
  Check(milp_launch::tri_transpose_lower(a, tri_segments_.data(),
                                         static_cast<int>(tri_segments_.size() / 2),
                                         Stream(stream)),
        "tri_transpose_lower");
}

void DeviceLp::CaptureTriGraph(TriContext* c) {
  if (c->graph_exec != nullptr) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(c->graph_exec));
    c->graph_exec = nullptr;
  }
  hipGraph_t graph = nullptr;
  Check(hipStreamBeginCapture(Stream(c->stream), hipStreamCaptureModeThreadLocal), "capture");
  EnqueueTriKernels(TriArgs(*c), c->stream);
  Check(hipStreamEndCapture(Stream(c->stream), &graph), "capture end");
  hipGraphExec_t exec = nullptr;
  const hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  Check(e, "graph instantiate");
  c->graph_exec = exec;
  c->graph_key = tri_key_;
}

bool DeviceLp::TransposeLowerSolve(const TriangularMatrix& t, uint64_t key,
                                   std::vector<double>* x) {
  if (tri_mode_ == 2) return false;
  const int nc = t.num_cols();
  if (tri_mode_ == 0 && nc < tri_min_rows_) return false;
  if (static_cast<int>(x->size()) < nc) return false;
  // The solver's thread (slot 0) or the factorization's tau worker (slot 1).
  const int slot = g_lu_slot == 0 ? 0 : 1;
  if (slot != 0 && !tri_tau_) return false;
  const int id = slot == 0 ? MI_K_TRI_SOLVE : MI_K_TRI_SOLVE_TAU;
  SolveCallTimer timer(&stats_, id);
  if (slot != 0) Check(hipSetDevice(device_), "hipSetDevice");
  TriContext& c = tri_ctx_[slot];
  {
    // The schedule is shared: the first solve after a refactorization
    // builds it, the other thread waits. (No solve can be in flight with the
    // previous key: the tau worker is joined before every refactorization.)
    std::lock_guard<std::mutex> lock(tri_mu_);
    if (c.stream == nullptr) PrepareTriContext(slot, nc);
    if (tri_key_ != key) BuildTriSchedule(t, key, c.stream);
    if (!tri_ok_) return false;
    PrepareTriContext(slot, nc);
  }
  double* xv = x->data();
  const int fni = tri_first_col_;
  // sparse.cc:908-912: the host loop starts at the last non-zero.
  int top = nc - 1;
  while (top >= fni && xv[top] == 0.0) --top;
  if (top < fni) return true;
  if (tri_rows_upto_[top + 1] - tri_rows_upto_[fni] == 0) return true;  // identity part only
  // Outputs c >= fni read rows > c only: x[fni..nc) in and out.
  const size_t in = size_t(nc - fni);
  CopyHost(c.h_x + fni, xv + fni, in * sizeof(double));
  *c.h_top = top;
  int* h_words = reinterpret_cast<int*>(c.h_x + nc);
  h_words[0] = top;  // zero-copy plan reads it here
  h_words[1] = 0;    // the sync-free kernel's failure word
  const double rows = tri_rows_upto_[top + 1] - tri_rows_upto_[fni];
  const double entries =
      static_cast<double>(tri_entries_upto_[top + 1] - tri_entries_upto_[fni]);
  // Per computed output: its record (row, count: 8 B), its value in and out
  // (16 B), the diagonal (8 B) unless unit; per entry: position and value
  // (12 B) and the value it reads (8 B). The permutes in and out: 8 B in, 8 B
  // out and the 4-B row index per position, both ways.
  const double bytes = rows * (24.0 + (tri_ones_ ? 0.0 : 8.0)) + entries * 20.0 +
                       double(tri_pos_) * 20.0 + rows * 20.0;
  if (slot == 0 && tri_debug_left_ > 0) {
    // MILP_TRI_DEBUG=k: per-level wall clock of the first k solves after each
    // schedule build (single-CU segments), printed with the level widths.
    milp_kernels::TriSolveArgs a = TriArgs(c);
    if (d_tri_clock_ == nullptr) {
      Check(hipMalloc(reinterpret_cast<void**>(&d_tri_clock_), 65536 * sizeof(uint64_t)),
            "hipMalloc");
    }
    Check(hipMemsetAsync(d_tri_clock_, 0, 65536 * sizeof(uint64_t), Stream(c.stream)),
          "memset");
    if (tri_levels_ + 1 < 65536) a.clock = d_tri_clock_;
    TriCopyIn(c);
    BeginKernel(MI_K_TRI_SOLVE);
    EnqueueTriKernels(a, c.stream);
    EndKernel(MI_K_TRI_SOLVE, bytes);
    TriCopyOut(c);
    Synchronize();
    --tri_debug_left_;
    std::vector<uint64_t> clk(tri_levels_ + 1);
    Check(hipMemcpy(clk.data(), d_tri_clock_, clk.size() * sizeof(uint64_t),
                    hipMemcpyDeviceToHost), "D2H");
    std::fprintf(stderr,
                 "[tri] rows %d work %d levels %d segments %zu top %d entries/row max %d "
                 ">4 %d >16 %d >64 %d; per level (us/width):",
                 nc, tri_work_, tri_levels_, tri_segments_.size() / 2, top, tri_max_entries_,
                 tri_rows_over_[0], tri_rows_over_[1], tri_rows_over_[2]);
    for (int l = 0; l < tri_levels_; ++l) {
      const bool ok = clk[l] != 0 && clk[l + 1] >= clk[l];
      std::fprintf(stderr, " %.2f/%d", ok ? (clk[l + 1] - clk[l]) / 100.0 : -1.0,
                   tri_level_width_[l]);
    }
    std::fprintf(stderr, "\n");
  } else {
    if (tri_graph_ && (c.graph_key != tri_key_ || c.graph_exec == nullptr)) {
      std::lock_guard<std::mutex> lock(tri_mu_);  // one capture at a time
      CaptureTriGraph(&c);
    }
    TriCopyIn(c);
    if (slot == 0) {
      BeginKernel(MI_K_TRI_SOLVE);  // events around the graph: the kernels only
    } else if (timing_) {
      Check(hipEventRecord(reinterpret_cast<hipEvent_t>(c.ev[0]), Stream(c.stream)), "ev");
    }
    if (tri_graph_) {
      Check(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(c.graph_exec), Stream(c.stream)),
            "graph launch");
    } else {
      EnqueueTriKernels(TriArgs(c), c.stream);
    }
    if (slot == 0) {
      EndKernel(MI_K_TRI_SOLVE, bytes);
    } else if (timing_) {
      Check(hipEventRecord(reinterpret_cast<hipEvent_t>(c.ev[1]), Stream(c.stream)), "ev");
    }
    TriCopyOut(c);
    Check(hipStreamSynchronize(Stream(c.stream)), "sync");
    if (slot != 0) {
      // The worker's own counters (its id is written by this thread only).
      stats_.launches[id] += 1;
      stats_.algorithmic_bytes[id] += bytes;
      if (timing_) {
        float ms = 0.0f;
        Check(hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(c.ev[0]),
                                  reinterpret_cast<hipEvent_t>(c.ev[1])),
              "ev time");
        stats_.device_ms[id] += ms;
      }
    }
  }
  if (*static_cast<volatile int*>(h_words + 1) != 0) throw DeviceError("triangular solve: dependency wait timed out");
  CopyHost(xv + fni, c.h_x + fni, size_t(top - fni + 1) * sizeof(double));
  return true;
}

}  // namespace milp
