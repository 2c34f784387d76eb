// DeviceLp: dense triangular solves of the basis factorization (see
// device_solver.h and kernels/tri_solve.hip).
//
// Glop's FTRAN is L, then the rank-one (middle product form) updates, then U
// (lu_factorization.cc:214-331). When the vector is too dense for the
// hypersparse paths the two triangles run dense loops over every row:
//   U: TriangularMatrix::TransposeLowerSolve on U's transpose (sparse.cc:
//      899-955), a gather: output c reads rows > c in grouped order;
//   L: LowerSolveStartingAt (sparse.cc:793-812), a column scatter; output r
//      receives x[j] * v for the columns j < r of its row in ascending j, one
//      subtraction at a time, skipping x[j] == 0 -- so it is restated as a
//      gather over L's rows with that order and that skip.
// On config 5 (m = 100 000) these loops are most of an iteration's host time
// (direction, bound-flip and tau FTRANs). The matrices change only at
// refactorization, so each one's level schedule is built and uploaded once
// per factorization; a solve then stages the vector, replays the captured
// launch plan and takes the result back. The solver's thread and
// BasisFactorization's tau worker solve concurrently, each with its own
// stream, buffers and graphs (TriContext); the schedules are shared.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
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
  FreeDenseTail();
  for (TriSchedule& s : tri_sched_) {
    for (TriBuffer& b : s.buf) FreeBuffer(&b);
    s = TriSchedule();
  }
  if (d_tri_clock_ != nullptr) (void)hipFree(d_tri_clock_);
  d_tri_clock_ = nullptr;
  DropAsyncU();
  for (int slot = 0; slot < kTriSlots; ++slot) {
    TriContext& c = tri_ctx_[slot];
    for (void* g : c.graph_exec) {
      if (g != nullptr) (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(g));
    }
    FreeBuffer(&c.x);
    FreeBuffer(&c.y);
    FreeBuffer(&c.top);
    if (c.h_x != nullptr) (void)hipHostFree(c.h_x);
    if (c.h_top != nullptr) (void)hipHostFree(c.h_top);
    for (void* e : c.ev) {
      if (e != nullptr) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e));
    }
    if ((slot == 1 || slot == 3) && c.stream != nullptr) {
      (void)hipStreamSynchronize(Stream(c.stream));
      (void)hipStreamDestroy(Stream(c.stream));
    }
    c = TriContext();
  }
  if (h_tri_stage_ != nullptr) (void)hipHostFree(h_tri_stage_);
  h_tri_stage_ = nullptr;
  tri_stage_bytes_ = 0;
}

// Level schedule of one triangle. Output c in [fni, nc) depends on the rows
// of its gather list (all > c when `descending`, all < c otherwise);
// level(c) = 0 without entries, else 1 + the deepest entry. Outputs with no
// entries and a unit diagonal keep their input and are not listed.
// Positions: the listed outputs by level, then the other rows >= fni (read,
// never written). Entries refer to positions, in evaluation order.
// MILP_LU_TIMING=1: the device solve schedules built after refactorizations
// (host wall time, printed at exit with the factorization's stages).
namespace {
struct ScheduleBuildTotals {
  static inline const bool on = std::getenv("MILP_LU_TIMING") != nullptr;
  std::atomic<int64_t> ns{0}, builds{0};
  ~ScheduleBuildTotals() {
    if (!on || builds.load() == 0) return;
    std::fprintf(stderr, "[lu timing] tri schedule builds %lld, %.3f ms total, %.3f ms each\n",
                 static_cast<long long>(builds.load()), ns.load() / 1e6,
                 ns.load() / 1e6 / builds.load());
  }
};
ScheduleBuildTotals g_schedule_build;
}  // namespace
struct ScheduleBuildTimer {
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  ~ScheduleBuildTimer() {
    if (!ScheduleBuildTotals::on) return;
    g_schedule_build.ns += std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - t0).count();
    ++g_schedule_build.builds;
  }
};

void DeviceLp::BuildTriSchedule(TriSchedule* s, int nc, int fni, bool ones, const double* diag,
                                const int64_t* gst, const int32_t* gidx, const double* gval,
                                bool reverse, bool descending, bool sequential, uint64_t key,
                                void* stream) {
  s->key = key;
  s->ok = false;
  s->rows = nc;
  s->first_col = fni;
  s->ones = ones;
  s->sequential = sequential;
  const int64_t nnz = gst[nc] - gst[0];
  if (nnz >= (int64_t{1} << 31)) return;
  std::vector<int32_t> level(nc, 0);
  int depth = 0;
  int num_work = 0;
  auto visit = [&](int c) {
    int l = 0;
    for (int64_t i = gst[c]; i < gst[c + 1]; ++i) l = std::max(l, level[gidx[i]] + 1);
    level[c] = l;
    depth = std::max(depth, l);
    if (l > 0 || !ones) ++num_work;
  };
  if (descending) {
    for (int c = nc - 1; c >= fni; --c) visit(c);
  } else {
    for (int c = fni; c < nc; ++c) visit(c);
  }
  // Counting sort by level. With MILP_TRI_PAD each chip-wide level starts on
  // a wave boundary (empty padding records fill the gap), so that a wave of
  // the sync-free kernel never holds both an output and one of its readers;
  // the level plan's kernels always pad.
  std::vector<int32_t> level_count(depth + 1, 0);
  for (int c = fni; c < nc; ++c) {
    if (level[c] > 0 || !ones) ++level_count[level[c]];
  }
  // Narrow segments (sync-free plans only): runs of at least
  // tri_chain_min_levels_ levels of at most tri_chain_width_ outputs each,
  // cut where the chain kernel's LDS is full, solved by one workgroup; their
  // levels are not padded. The rest run chip-wide.
  std::vector<int> seg_level;  // (first level, end level, narrow) triples
  if (tri_chain_ && tri_syncfree_ && tri_persist_groups_ == 0) {
    int wide_from = 0;
    int l = 0;
    while (l <= depth) {
      if (level_count[l] > tri_chain_width_) {
        ++l;
        continue;
      }
      int e = l;
      int held = 0;
      while (e <= depth && level_count[e] <= tri_chain_width_ &&
             held + level_count[e] <= milp_kernels::kTriChainVals) {
        held += level_count[e];
        ++e;
      }
      if (e - l >= tri_chain_min_levels_) {
        if (l > wide_from) seg_level.insert(seg_level.end(), {wide_from, l, 0});
        seg_level.insert(seg_level.end(), {l, e, 1});
        wide_from = e;
      }
      l = std::max(e, l + 1);  // a level alone larger than the LDS stays wide
    }
    if (wide_from <= depth) seg_level.insert(seg_level.end(), {wide_from, depth + 1, 0});
  } else {
    seg_level = {0, depth + 1, 0};
  }
  std::vector<char> narrow(depth + 1, 0);
  s->chain_levels = 0;
  for (size_t i = 0; i < seg_level.size(); i += 3) {
    if (seg_level[i + 2] == 0) continue;
    for (int l = seg_level[i]; l < seg_level[i + 1]; ++l) narrow[l] = 1;
    s->chain_levels += seg_level[i + 1] - seg_level[i];
  }
  std::vector<int32_t> level_start(depth + 2, 0);
  for (int l = 0; l <= depth; ++l) {
    const bool pad = !narrow[l] && (tri_pad_ || !tri_syncfree_);
    level_start[l + 1] = level_start[l] + (pad ? (level_count[l] + 63) / 64 * 64 : level_count[l]);
  }
  s->runs.clear();
  s->max_wide_run = 0;
  for (size_t i = 0; i < seg_level.size(); i += 3) {
    const int b = level_start[seg_level[i]], e = level_start[seg_level[i + 1]];
    if (e <= b) continue;
    s->runs.insert(s->runs.end(), {b, e, seg_level[i + 2]});
    if (seg_level[i + 2] == 0) s->max_wide_run = std::max(s->max_wide_run, e - b);
  }
  // Level 0 on the chip (not in a narrow run): its outputs are a division of
  // their input, done by the init kernel of a sync-free solve.
  s->level0_end = (!narrow[0] && depth >= 0) ? level_start[1] : 0;
  num_work = level_start[depth + 1];  // listed outputs + padding
  const int num_pos = num_work + (nc - fni);  // + every row, read-only copies
  s->work = num_work;
  s->pos = num_pos;
  s->levels = depth + 1;
  s->level_width.assign(level_count.begin(), level_count.end());
  // Launch segments of the level plan: each wide level alone over the chip,
  // each run of narrow levels as one single-CU launch (tri_solve.hip).
  s->segments.clear();
  // Narrow = fits one CU and its LDS value store.
  const int wide_level = std::min(tri_wide_level_, milp_kernels::kTriLdsVals - 64);
  for (int l = 0; l <= depth;) {
    const int w = s->level_width[l];
    if (w == 0) {
      ++l;
      continue;
    }
    if (w > wide_level) {
      s->segments.push_back(-l - 1);
      s->segments.push_back(std::min(1024, (w + 255) / 256));
      ++l;
      continue;
    }
    // A run of narrow levels, cut where its padded positions would overflow
    // the CU kernel's LDS value store.
    int e = l;
    int run = 0;
    while (e <= depth && s->level_width[e] <= wide_level) {
      const int padded = (s->level_width[e] + 63) / 64 * 64;
      if (e > l && run + padded > milp_kernels::kTriLdsVals) break;
      run += padded;
      ++e;
    }
    s->segments.push_back(l);
    s->segments.push_back(e);
    l = e;
  }
  // Positions: the listed outputs by level (padding rows point at row fni and
  // are never computed), then the unlisted rows.
  std::vector<int32_t> pos_row(num_pos, fni);
  std::vector<int32_t> pos_of(nc, -1);
  std::vector<char> is_pad(num_work, 1);
  {
    std::vector<int32_t> next(level_start.begin(), level_start.end() - 1);
    int tail = num_work;
    for (int i = 0; i < nc - fni; ++i) {
      const int c = descending ? nc - 1 - i : fni + i;  // the host's order inside a level
      const bool listed = level[c] > 0 || !ones;
      const int k = listed ? next[level[c]]++ : tail++;
      if (listed) is_pad[k] = 0;
      pos_row[k] = c;
      pos_of[c] = k;
    }
    s->pos = tail;
  }
  int64_t num_ovf = 0;
  s->max_entries = 0;
  s->rows_over[0] = s->rows_over[1] = s->rows_over[2] = 0;
  s->late_entries = 0;
  for (int k = 0; k < num_work; ++k) {
    if (is_pad[k]) continue;
    const int c = pos_row[k];
    const int64_t n = gst[c + 1] - gst[c];
    if (n > 4) {
      // Entries evaluated at or after the first one of the deepest level:
      // what is left to fold once the last input arrives.
      int deepest = -1;
      int64_t first = 0;
      for (int64_t j = 0; j < n; ++j) {
        const int l = level[gidx[reverse ? gst[c + 1] - 1 - j : gst[c] + j]];
        if (l > deepest) {
          deepest = l;
          first = j;
        }
      }
      s->late_entries += n - first;
    }
    if (n > 4) num_ovf += n;
    s->max_entries = std::max<int>(s->max_entries, static_cast<int>(n));
    s->rows_over[0] += n > 4;
    s->rows_over[1] += n > 16;
    s->rows_over[2] += n > 64;
  }
  // Staging layout, 16-byte aligned pieces.
  auto al = [](size_t b) { return (b + 15) / 16 * 16; };
  const size_t b_levels = al(size_t(depth + 2) * 4);
  const size_t b_row = al(size_t(num_work) * 4);
  const size_t b_n = al(size_t(num_work) * 4);
  const size_t b_entry = size_t(num_work) * 16;
  const size_t b_value = size_t(num_work) * 32;
  const size_t b_diag = ones ? 0 : al(size_t(num_work) * 8);
  const size_t b_ovf_pos = al(size_t(num_ovf) * 4);
  const size_t b_ovf_val = al(size_t(num_ovf) * 8);
  const size_t b_pos_row = al(size_t(s->pos) * 4);
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
  double* rec_diag = reinterpret_cast<double*>(st + offs[kTriDiag]);
  int32_t* ovf_pos = reinterpret_cast<int32_t*>(st + offs[kTriOvfPos]);
  double* ovf_value = reinterpret_cast<double*>(st + offs[kTriOvfValue]);
  std::copy(level_start.begin(), level_start.end(), lstart);
  std::copy(pos_row.begin(), pos_row.begin() + s->pos,
            reinterpret_cast<int32_t*>(st + offs[kTriPosRow]));
  // Entries of each listed output in evaluation order (U: from the column's
  // last entry down, sparse.cc:908-955; L: ascending columns).
  int64_t o = 0;
  for (int k = 0; k < num_work; ++k) {
    if (is_pad[k]) {  // never computed: row beyond any top, no entries
      rec_row[k] = INT32_MAX;
      rec_n[k] = 0;
      for (int j = 0; j < 4; ++j) {
        rec_entry[4 * k + j] = 0;
        rec_value[4 * k + j] = 0.0;
      }
      if (!ones) rec_diag[k] = 1.0;
      continue;
    }
    const int c = pos_row[k];
    const int64_t b = gst[c], e = gst[c + 1];
    const int n = static_cast<int>(e - b);
    auto at = [&](int j) { return reverse ? e - 1 - j : b + j; };
    rec_row[k] = c;
    rec_n[k] = n;
    if (n <= 4) {
      for (int j = 0; j < 4; ++j) {
        rec_entry[4 * k + j] = j < n ? pos_of[gidx[at(j)]] : 0;
        rec_value[4 * k + j] = j < n ? gval[at(j)] : 0.0;
      }
    } else {
      rec_entry[4 * k] = static_cast<int32_t>(o);
      rec_entry[4 * k + 1] = rec_entry[4 * k + 2] = rec_entry[4 * k + 3] = 0;
      for (int j = 0; j < 4; ++j) rec_value[4 * k + j] = 0.0;
      for (int j = 0; j < n; ++j) {
        ovf_pos[o] = pos_of[gidx[at(j)]];
        ovf_value[o] = gval[at(j)];
        ++o;
      }
    }
    if (!ones) rec_diag[k] = diag[c];
  }
  // Prefix counts by output row, for the byte accounting of a solve that
  // stops at `top`.
  s->rows_upto.assign(nc + 1, 0);
  s->entries_upto.assign(nc + 1, 0);
  for (int c = 0; c < nc; ++c) {
    const bool listed = c >= fni && pos_of[c] < num_work;
    s->rows_upto[c + 1] = s->rows_upto[c] + (listed ? 1 : 0);
    s->entries_upto[c + 1] = s->entries_upto[c] + (listed ? gst[c + 1] - gst[c] : 0);
  }
  for (int b = 0; b < kTriNumStaged; ++b) {
    if (sizes[b] == 0) continue;
    TriReserve(&s->buf[b], sizes[b]);
    Check(hipMemcpyAsync(s->buf[b].ptr, st + offs[b], sizes[b], hipMemcpyHostToDevice,
                         Stream(stream)),
          "H2D");
  }
  // The staging buffer is reused by the next build: wait for the copies.
  Check(hipStreamSynchronize(Stream(stream)), "sync");
  s->ok = true;  // each context recaptures its graph for the new key
}

void DeviceLp::PrepareTriContext(int slot, int rows, int pos) {
  TriContext& c = tri_ctx_[slot];
  if (c.stream == nullptr) {
    if (slot == 0 || slot == 2) {  // the solver's thread: its own vector (0) or a pair's second (2)
      c.stream = stream_;
    } else {
      hipStream_t st;
      if (stream_prioritized_) {
        int least = 0, greatest = 0;
        Check(hipDeviceGetStreamPriorityRange(&least, &greatest), "priority range");
        Check(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, least), "hipStreamCreate");
      } else {
        Check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
      }
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
  TriReserve(&c.x, size_t(std::max(rows, 1)) * 8);
  TriReserve(&c.y, size_t(std::max(pos, 1)) * 8);
  bool moved = c.x.ptr != old_x || c.y.ptr != old_y;
  // rows values + the top row and the failure word (ints after them), mapped.
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
    moved = true;
  }
  if (moved) c.graph_key[0] = c.graph_key[1] = 0;  // captured addresses are stale
}

milp_kernels::TriSolveArgs DeviceLp::TriArgs(const TriSchedule& s, const TriContext& c) const {
  milp_kernels::TriSolveArgs a;
  a.level_start = static_cast<const int32_t*>(s.buf[kTriLevels].ptr);
  a.rec_row = static_cast<const int32_t*>(s.buf[kTriRecRow].ptr);
  a.rec_n = static_cast<const int32_t*>(s.buf[kTriRecN].ptr);
  a.rec_entry = static_cast<const int4*>(s.buf[kTriRecEntry].ptr);
  a.rec_value = static_cast<const double2*>(s.buf[kTriRecValue].ptr);
  a.diag = s.ones ? nullptr : static_cast<const double*>(s.buf[kTriDiag].ptr);
  a.ovf_pos = static_cast<const int32_t*>(s.buf[kTriOvfPos].ptr);
  a.ovf_value = static_cast<const double*>(s.buf[kTriOvfValue].ptr);
  a.pos_row = static_cast<const int32_t*>(s.buf[kTriPosRow].ptr);
  a.x = static_cast<double*>(c.x.ptr);
  a.y = static_cast<double*>(c.y.ptr);
  a.top = static_cast<int*>(c.top.ptr);
  a.host_x = tri_mapped_ ? c.m_x : nullptr;
  a.first_col = s.first_col;
  a.num_rows = s.rows;
  a.fail = reinterpret_cast<int*>(c.m_x + s.rows) + 1;
  a.num_work = s.work;
  a.num_pos = s.pos;
  a.num_levels = s.levels;
  a.sequential = s.sequential ? 1 : 0;
  a.fuse_level0 = tri_fuse0_ ? 1 : 0;
  a.poll_max = tri_poll_max_;
  a.clock = nullptr;
  a.x2 = nullptr;
  a.y2 = nullptr;
  a.host_x2 = nullptr;
  a.top2 = nullptr;
  a.fail2 = nullptr;
  a.seg_begin = 0;
  a.seg_end = s.work;
  a.level0_end = tri_fuse0_ ? s.level0_end : 0;
  return a;
}

// One solve = stage x[fni..nc) and the top row, the launch plan, take x back.
// Without debugging the plan is captured once per factorization, matrix and
// context into a HIP graph and replayed with one launch. Staging is
// zero-copy inside the plan (kernels read and write mapped host memory);
// MILP_TRI_MAPPED=0 uses copy-engine transfers instead.
void DeviceLp::TriCopyIn(const TriSchedule& s, const TriContext& c) {
  if (tri_mapped_) return;
  const int fni = s.first_col;
  const size_t in = size_t(s.rows - fni);
  double* d_x = static_cast<double*>(c.x.ptr);
  Check(hipMemcpyAsync(d_x + fni, c.h_x + fni, in * sizeof(double), hipMemcpyHostToDevice,
                       Stream(c.stream)),
        "H2D");
  Check(hipMemcpyAsync(c.top.ptr, c.h_top, sizeof(int), hipMemcpyHostToDevice, Stream(c.stream)),
        "H2D");
}

void DeviceLp::TriCopyOut(const TriSchedule& s, const TriContext& c) {
  if (tri_mapped_) return;
  const int fni = s.first_col;
  const size_t in = size_t(s.rows - fni);
  const double* d_x = static_cast<const double*>(c.x.ptr);
  Check(hipMemcpyAsync(c.h_x + fni, d_x + fni, in * sizeof(double), hipMemcpyDeviceToHost,
                       Stream(c.stream)),
        "D2H");
}

void DeviceLp::EnqueueTriKernels(const TriSchedule& s, const milp_kernels::TriSolveArgs& a,
                                 void* stream) {
  // The single-launch kernel pays a cross-workgroup hand-off per level; a
  // shallow schedule runs faster as a few level launches.
  if (tri_persist_groups_ > 0 && tri_syncfree_ && a.clock == nullptr &&
      s.levels >= tri_syncfree_min_levels_) {
    Check(milp_launch::tri_transpose_lower_persistent(a, tri_persist_groups_, tri_xcd_stride_,
                                                      Stream(stream)),
          "tri persistent");
    return;
  }
  if (tri_syncfree_ && a.clock == nullptr && s.max_wide_run <= milp_kernels::kTriSyncFreeMaxWork &&
      s.levels >= tri_syncfree_min_levels_) {
    Check(milp_launch::tri_transpose_lower_syncfree(a, s.runs.data(),
                                                    static_cast<int>(s.runs.size() / 3),
                                                    Stream(stream)),
          "tri syncfree");
    return;
  }
  Check(milp_launch::tri_transpose_lower(a, s.segments.data(),
                                         static_cast<int>(s.segments.size() / 2),
                                         Stream(stream)),
        "tri_transpose_lower");
}

void DeviceLp::CaptureTriGraph(int which, TriContext* c) {
  if (c->graph_exec[which] != nullptr) {
    (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(c->graph_exec[which]));
    c->graph_exec[which] = nullptr;
  }
  const TriSchedule& s = tri_sched_[which];
  hipGraph_t graph = nullptr;
  Check(hipStreamBeginCapture(Stream(c->stream), hipStreamCaptureModeThreadLocal), "capture");
  EnqueueTriKernels(s, TriArgs(s, *c), c->stream);
  Check(hipStreamEndCapture(Stream(c->stream), &graph), "capture end");
  hipGraphExec_t exec = nullptr;
  const hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  Check(e, "graph instantiate");
  c->graph_exec[which] = exec;
  c->graph_key[which] = s.key;
}

bool DeviceLp::TransposeLowerSolve(const TriangularMatrix& t, uint64_t key,
                                   std::vector<double>* x) {
  return TriSolve(kTriU, t, key, x);
}

bool DeviceLp::LowerSolve(const TriangularMatrix& lower, uint64_t key, std::vector<double>* x) {
  if (!tri_lower_) return false;
  return TriSolve(kTriL, lower, key, x);
}

void DeviceLp::FreeDenseTail() {
  DenseTail& d = dense_tail_;
  for (TriBuffer* b : {&d.starts, &d.cur, &d.rows, &d.vals, &d.diag, &d.x, &d.pre}) {
    FreeBuffer(b);
  }
  if (d.h_in != nullptr) (void)hipHostFree(d.h_in);
  if (d.h_out != nullptr) (void)hipHostFree(d.h_out);
  d = DenseTail();
}

// BTRAN's forward U^T solve (TriangularMatrix::TransposeUpperSolve,
// sparse.cc:848-897) with its dense tail on the device (dense_tail.hip).
// Columns [fni, t) run the host loop here, unchanged; columns [t, n) -- the
// trailing columns holding at least n / 8 entries each -- on the device: the
// leading groups of four that read rows < t only, for all tail columns at
// once, then the tail's own dependency walk on one workgroup. Every output
// is evaluated with the loop's operations in the loop's order (same bits).
// False: the host loop runs the whole solve.
bool DeviceLp::DenseTailSolve(const TriangularMatrix& u, uint64_t key, std::vector<double>* xv) {
  if (dense_tail_mode_ == 0 || g_lu_slot != 0) return false;
  const int n = u.num_cols();
  if (static_cast<int>(xv->size()) < n) return false;
  DenseTail& d = dense_tail_;
  const int64_t* st = u.starts_.data();
  if (d.key != key) {
    DeviceOp("dense tail build");
    d.key = key;
    d.ok = false;
    d.n = n;
    d.fni = u.GetFirstNonIdentityColumn();
    int t = n;
    const int64_t dense = std::max<int64_t>(16, n / 8);
    while (t > d.fni && st[t] - st[t - 1] >= dense) --t;
    const int T = n - t;
    const int64_t entries = st[n] - st[t];
    if (T < dense_tail_min_cols_ || T > milp_kernels::kTailMaxCols ||
        entries < dense_tail_min_entries_) {
      return false;
    }
    d.t = t;
    d.entries = entries;
    // Per tail column: the end of its leading groups of four whose rows are
    // all below t (final when the tail starts).
    std::vector<int64_t> rel(T + 1), split(T);
    const int32_t* rows = u.rows_.data();
    for (int c = t; c < n; ++c) {
      const int64_t i0 = st[c], i1 = st[c + 1];
      int64_t i = i0;
      while (i + 3 < i1 && rows[i] < t && rows[i + 1] < t && rows[i + 2] < t && rows[i + 3] < t) {
        i += 4;
      }
      rel[c - t] = i0 - st[t];
      split[c - t] = i - st[t];
    }
    rel[T] = entries;
    if (std::getenv("MILP_DENSE_TAIL_DEBUG") != nullptr) {
      int64_t prefix = 0, unsorted = 0;
      for (int c = t; c < n; ++c) {
        prefix += split[c - t] - rel[c - t];
        for (int64_t i = st[c]; i + 1 < st[c + 1]; ++i) unsorted += rows[i] > rows[i + 1];
      }
      std::fprintf(stderr,
                   "[dense tail] n %d fni %d t %d T %d entries %lld prefix %lld triangle %lld "
                   "unsorted pairs %lld, columns [fni, t) entries %lld\n",
                   n, d.fni, t, T, static_cast<long long>(entries), static_cast<long long>(prefix),
                   static_cast<long long>(entries - prefix), static_cast<long long>(unsorted),
                   static_cast<long long>(st[t] - st[d.fni]));
    }
    TriReserve(&d.starts, sizeof(int64_t) * (T + 1));
    TriReserve(&d.cur, sizeof(int64_t) * T);
    TriReserve(&d.rows, sizeof(int32_t) * entries);
    TriReserve(&d.vals, sizeof(double) * entries);
    TriReserve(&d.x, sizeof(double) * n);
    TriReserve(&d.pre, sizeof(double) * T);
    hipStream_t s = Stream(stream_);
    Check(hipMemcpyAsync(d.starts.ptr, rel.data(), sizeof(int64_t) * (T + 1),
                         hipMemcpyHostToDevice, s), "dense tail upload");
    Check(hipMemcpyAsync(d.rows.ptr, rows + st[t], sizeof(int32_t) * entries,
                         hipMemcpyHostToDevice, s), "dense tail upload");
    Check(hipMemcpyAsync(d.vals.ptr, u.coefficients_.data() + st[t], sizeof(double) * entries,
                         hipMemcpyHostToDevice, s), "dense tail upload");
    if (!u.all_diagonal_coefficients_are_one_) {
      TriReserve(&d.diag, sizeof(double) * T);
      Check(hipMemcpyAsync(d.diag.ptr, u.diagonal_coefficients_.data() + t, sizeof(double) * T,
                           hipMemcpyHostToDevice, s), "dense tail upload");
    }
    if (d.cap_n < n) {
      if (d.h_in != nullptr) (void)hipHostFree(d.h_in);
      Check(hipHostMalloc(reinterpret_cast<void**>(&d.h_in), sizeof(double) * (n + 1),
                          hipHostMallocMapped), "dense tail staging");
      Check(hipHostGetDevicePointer(reinterpret_cast<void**>(&d.m_in), d.h_in, 0), "mapped");
      d.cap_n = n;
    }
    if (d.cap_t < T) {
      if (d.h_out != nullptr) (void)hipHostFree(d.h_out);
      Check(hipHostMalloc(reinterpret_cast<void**>(&d.h_out), sizeof(double) * T,
                          hipHostMallocMapped), "dense tail staging");
      Check(hipHostGetDevicePointer(reinterpret_cast<void**>(&d.m_out), d.h_out, 0), "mapped");
      d.cap_t = T;
    }
    Check(hipStreamSynchronize(s), "dense tail upload");  // rel/split are freed below
    d.ok = true;
  }
  if (!d.ok) return false;
  SolveCallTimer timer(&stats_, MI_K_TRI_SOLVE_T);
  const int t = d.t;
  const int T = n - t;
  double* x = xv->data();
  // Columns [fni, t): the host loop (sparse.cc:848-897), as it runs them.
  {
    const int32_t* rows = u.rows_.data();
    const double* coefs = u.coefficients_.data();
    const bool ones = u.all_diagonal_coefficients_are_one_;
    int64_t i = st[d.fni];
    for (int col = d.fni; col < t; ++col) {
      double sum = x[col];
      const int64_t i_end = st[col + 1];
      const int64_t shifted_end = i_end - 3;
      for (; i < shifted_end; i += 4) {
        sum -= coefs[i] * x[rows[i]] + coefs[i + 1] * x[rows[i + 1]] +
               coefs[i + 2] * x[rows[i + 2]] + coefs[i + 3] * x[rows[i + 3]];
      }
      if (i < i_end) {
        sum -= coefs[i] * x[rows[i]];
        if (i + 1 < i_end) {
          sum -= coefs[i + 1] * x[rows[i + 1]];
          if (i + 2 < i_end) sum -= coefs[i + 2] * x[rows[i + 2]];
        }
        i = i_end;
      }
      x[col] = ones ? sum : sum / u.diagonal_coefficients_[col];
    }
  }
  DeviceOp("dense tail solve");
  CopyHost(d.h_in, x, sizeof(double) * n);
  int* fail = reinterpret_cast<int*>(d.h_in + n);
  *fail = 0;
  milp_kernels::DenseTailArgs a{};
  a.starts = static_cast<const int64_t*>(d.starts.ptr);
  a.cur = static_cast<int64_t*>(d.cur.ptr);
  a.rows = static_cast<const int32_t*>(d.rows.ptr);
  a.vals = static_cast<const double*>(d.vals.ptr);
  a.diag = u.all_diagonal_coefficients_are_one_ ? nullptr : static_cast<const double*>(d.diag.ptr);
  a.x = static_cast<double*>(d.x.ptr);
  a.pre = static_cast<double*>(d.pre.ptr);
  a.host_x = d.m_in;
  a.host_out = d.m_out;
  a.n = n;
  a.t = t;
  a.fail = reinterpret_cast<int*>(d.m_in + n);
  // Algorithmic bytes: per entry its row and value (12 B) and the value it
  // reads (8 B); per tail output its running sum, cursor, diagonal, value in
  // and out.
  const double bytes = 20.0 * static_cast<double>(d.entries) + 40.0 * T + 16.0 * n;
  BeginKernel(MI_K_TRI_SOLVE_T);
  Check(milp_launch::dense_tail_upper_solve(a, Stream(stream_)), "dense tail solve");
  EndKernel(MI_K_TRI_SOLVE_T, bytes);
  Check(hipStreamSynchronize(Stream(stream_)), "dense tail sync");
  if (*static_cast<volatile int*>(fail) != 0) {
    throw DeviceError("dense tail solve: dependency wait timed out");
  }
  CopyHost(x + t, d.h_out, sizeof(double) * T);
  return true;
}

bool DeviceLp::Solve(TriKind kind, const TriangularMatrix& t, uint64_t key, int /*start*/,
                     std::vector<double>* x) {
  if (kind == TriKind::kUpperTUp && DenseTailSolve(t, key, x)) return true;
  // LowerSolveStartingAt(start): the loops below `start` only meet zeros in
  // every caller (a unit row, or L's input below its first non-zero), which
  // the gather computes as the loop leaves them.
  if (kind != TriKind::kUpperT && !tri_btran_) return false;
  if (kind == TriKind::kLower && !tri_lower_) return false;
  return TriSolve(static_cast<int>(kind), t, key, x);
}

// Gather lists of a scatter loop over t's columns (LowerSolveStartingAt,
// UpperSolve): output r lists the columns j >= fni whose column holds row r,
// with t[r, j], by ascending j (LowerSolve's column order) or descending
// (UpperSolve's). Built into tri_lt_* (a counting transpose).
void DeviceLp::TransposeColumns(const TriangularMatrix& t, bool descending) {
  const int nc = t.num_cols();
  const int fni = t.GetFirstNonIdentityColumn();
  tri_lt_starts_.assign(nc + 1, 0);
  for (int j = fni; j < nc; ++j) {
    for (int64_t i = t.starts_[j]; i < t.starts_[j + 1]; ++i) ++tri_lt_starts_[t.rows_[i] + 1];
  }
  for (int r = 0; r < nc; ++r) tri_lt_starts_[r + 1] += tri_lt_starts_[r];
  tri_lt_idx_.resize(tri_lt_starts_[nc]);
  tri_lt_val_.resize(tri_lt_starts_[nc]);
  std::vector<int64_t> fill(tri_lt_starts_.begin(), tri_lt_starts_.end() - 1);
  auto put = [&](int j) {
    for (int64_t i = t.starts_[j]; i < t.starts_[j + 1]; ++i) {
      const int64_t at = fill[t.rows_[i]]++;
      tri_lt_idx_[at] = j;
      tri_lt_val_[at] = t.coefficients_[i];
    }
  };
  if (descending) {
    for (int j = nc - 1; j >= fni; --j) put(j);
  } else {
    for (int j = fni; j < nc; ++j) put(j);
  }
}

// The schedule of `which` for this factorization and the solving context
// (built and sized on first use). False: the solve should run on the host.
bool DeviceLp::TriPrepare(int which, const TriangularMatrix& t, uint64_t key, int slot,
                          const std::vector<double>& x) {
  if (tri_mode_ == 2) return false;
  const int nc = t.num_cols();
  if (tri_mode_ == 0 && nc < tri_min_rows_) return false;
  // Medium LPs solved in a batch keep the host triangles: many LPs' level
  // chains contend for the device queues, each hop pays the contended launch
  // latency (ta041-shaped batch of 64, 16 in flight: 15.7 LPs/s with the
  // device solves, 37.7 with the host's).
  if (tri_mode_ == 0 && small_batch_ && medium_) return false;
  if (static_cast<int>(x.size()) < nc) return false;
  const TriKind kind = static_cast<TriKind>(which);
  if (slot == 1) Check(hipSetDevice(device_), "hipSetDevice");
  TriContext& c = tri_ctx_[slot];
  TriSchedule& s = tri_sched_[which];
  {
    // The schedules are shared: the first solve after a refactorization
    // builds one, the other thread waits. (No solve can be in flight with the
    // previous key: the tau worker is joined before every refactorization.)
    std::lock_guard<std::mutex> lock(tri_mu_);
    DeviceOp("tri lock held");
    if (c.stream == nullptr) PrepareTriContext(slot, nc, 1);
    if (s.key != key) {
      // An asynchronous U solve reads the schedule being replaced.
      if (which == kTriU && async_u_.active && !async_u_.trivial) {
        (void)hipStreamSynchronize(Stream(tri_ctx_[3].stream));
      }
      DeviceOp("tri build");
      ScheduleBuildTimer build_timer;
      const int fni = t.GetFirstNonIdentityColumn();
      const bool ones = t.all_diagonal_coefficients_are_one_;
      const double* diag = t.diagonal_coefficients_.data();
      switch (kind) {
        case TriKind::kUpperT:
        case TriKind::kLowerT:
          // TransposeLowerSolve (sparse.cc:899-955): gather lists = t's
          // columns, evaluated from their ends; reads rows > c.
          BuildTriSchedule(&s, nc, fni, ones, diag, t.starts_.data(), t.rows_.data(),
                           t.coefficients_.data(), /*reverse=*/true, /*descending=*/true,
                           /*sequential=*/false, key, c.stream);
          break;
        case TriKind::kUpperTUp:
          // TransposeUpperSolve (sparse.cc:848-897): t's columns forward;
          // reads rows < c, also rows below the first non-identity column
          // (positions from row 0).
          BuildTriSchedule(&s, nc, 0, ones, diag, t.starts_.data(), t.rows_.data(),
                           t.coefficients_.data(), /*reverse=*/false, /*descending=*/false,
                           /*sequential=*/false, key, c.stream);
          break;
        case TriKind::kLower:
        case TriKind::kUnitRow:
          // LowerSolveStartingAt (sparse.cc:792-812): a scatter by ascending
          // columns, restated as a gather over t's rows in that order.
          TransposeColumns(t, /*descending=*/false);
          BuildTriSchedule(&s, nc, fni, ones, diag, tri_lt_starts_.data(), tri_lt_idx_.data(),
                           tri_lt_val_.data(), /*reverse=*/false, /*descending=*/false,
                           /*sequential=*/true, key, c.stream);
          break;
        case TriKind::kUpper:
          // UpperSolve (sparse.cc:814-846): the scatter by descending columns;
          // rows below the first non-identity column receive too (outputs
          // from row 0; their own columns are identity, never divided).
          TransposeColumns(t, /*descending=*/true);
          BuildTriSchedule(&s, nc, 0, ones, diag, tri_lt_starts_.data(), tri_lt_idx_.data(),
                           tri_lt_val_.data(), /*reverse=*/false, /*descending=*/true,
                           /*sequential=*/true, key, c.stream);
          break;
      }
      if (which == kTriU) {
        if (const char* d = std::getenv("MILP_TRI_DEBUG")) tri_debug_left_ = std::atoi(d);
      }
      if (s.ok && std::getenv("MILP_TRI_SCHED") != nullptr) {
        // Shape of each schedule as built: how many levels are narrow, and
        // how much of the long outputs' work waits for their deepest input.
        int narrow64 = 0, narrow1024 = 0;
        for (int w : s.level_width) {
          narrow64 += w <= 64;
          narrow1024 += w <= 1024;
        }
        int64_t long_entries = 0;
        for (int c = 0; c < nc; ++c) {
          const int64_t n = s.entries_upto[c + 1] - s.entries_upto[c];
          if (n > 4) long_entries += n;
        }
        std::fprintf(stderr,
                     "[tri sched] kind %d rows %d first %d work %d levels %d (<=64: %d, "
                     "<=1024: %d) long outputs %d entries %lld late %lld; segments %zu, "
                     "%d levels narrow\n",
                     which, nc, s.first_col, s.work, s.levels, narrow64, narrow1024,
                     s.rows_over[0], static_cast<long long>(long_entries),
                     static_cast<long long>(s.late_entries), s.runs.size() / 3,
                     s.chain_levels);
      }
    }
    if (!s.ok) return false;
    // Auto mode: the device pays a dependency hop per level, the host loop a
    // few ns per entry; a triangle without enough outputs per level stays on
    // the host (MILP_TRI_MIN_WIDTH, outputs per level on average).
    // The narrow segments' levels cost an LDS hand-off each, not a trip
    // between XCDs: only the chip-wide levels count.
    if (tri_mode_ == 0 && s.work < int64_t(s.levels - s.chain_levels) * tri_min_width_) {
      return false;
    }
    PrepareTriContext(slot, nc, s.pos);
  }
  return true;
}

bool DeviceLp::TriSolve(int which, const TriangularMatrix& t, uint64_t key,
                        std::vector<double>* x) {
  // The solver's thread (slot 0) or the factorization's tau worker (slot 1).
  const int slot = g_lu_slot == 0 ? 0 : 1;
  if (slot != 0 && !tri_tau_) return false;
  const TriKind kind = static_cast<TriKind>(which);
  const int id = slot != 0                       ? MI_K_TRI_SOLVE_TAU
                 : kind == TriKind::kUpperT      ? MI_K_TRI_SOLVE
                 : kind == TriKind::kLower       ? MI_K_TRI_SOLVE_L
                 : kind == TriKind::kUpper       ? MI_K_TRI_SOLVE_UPPER
                                                 : MI_K_TRI_SOLVE_T;
  SolveCallTimer timer(&stats_, id);
  DeviceOp(which == kTriU ? (slot == 0 ? "tri U enter" : "tri U enter (slot 1)")
                          : (slot == 0 ? "tri L enter" : "tri L enter (slot 1)"));
  if (!TriPrepare(which, t, key, slot, *x)) return false;
  const int nc = t.num_cols();
  TriContext& c = tri_ctx_[slot];
  TriSchedule& s = tri_sched_[which];
  double* xv = x->data();
  const int fni = s.first_col;
  // U (sparse.cc:908-912): the host loop starts at the last non-zero; the
  // L loop runs over every column (outputs below its start receive nothing).
  int top = nc - 1;
  if (kind == TriKind::kUpperT || kind == TriKind::kLowerT) {
    while (top >= fni && xv[top] == 0.0) --top;
    if (top < fni) return true;
  }
  if (s.rows_upto[top + 1] - s.rows_upto[fni] == 0) return true;  // identity part only
  // Outputs c >= fni read rows >= fni only: x[fni..nc) in and out.
  const size_t in = size_t(nc - fni);
  FtranTimer ft(kFtDevCopyIn);
  CopyHost(c.h_x + fni, xv + fni, in * sizeof(double));
  ft.Lap(kFtDevRun);
  *c.h_top = top;
  int* h_words = reinterpret_cast<int*>(c.h_x + nc);
  h_words[0] = top;  // zero-copy plan reads it here
  h_words[1] = 0;    // the sync-free kernel's failure word
  const double rows = s.rows_upto[top + 1] - s.rows_upto[fni];
  const double entries = static_cast<double>(s.entries_upto[top + 1] - s.entries_upto[fni]);
  // Per computed output: its record (row, count: 8 B), its value in and out
  // (16 B), the diagonal (8 B) unless unit; per entry: position and value
  // (12 B) and the value it reads (8 B). The permutes in and out: 8 B in, 8 B
  // out and the 4-B row index per position, both ways.
  const double bytes = rows * (24.0 + (s.ones ? 0.0 : 8.0)) + entries * 20.0 +
                       double(s.pos) * 20.0 + rows * 20.0;
  if (slot == 0 && which == kTriU && tri_debug_left_ > 0) {
    // MILP_TRI_DEBUG=k: per-level wall clock of the first k U solves after
    // each schedule build (level plan), printed with the level widths.
    milp_kernels::TriSolveArgs a = TriArgs(s, c);
    if (d_tri_clock_ == nullptr) {
      Check(hipMalloc(reinterpret_cast<void**>(&d_tri_clock_), 65536 * sizeof(uint64_t)),
            "hipMalloc");
    }
    Check(hipMemsetAsync(d_tri_clock_, 0, 65536 * sizeof(uint64_t), Stream(c.stream)),
          "memset");
    if (s.levels + 1 < 65536) a.clock = d_tri_clock_;
    TriCopyIn(s, c);
    BeginKernel(id);
    EnqueueTriKernels(s, a, c.stream);
    EndKernel(id, bytes);
    TriCopyOut(s, c);
    // The armed MPF right-pool append reads the FTRAN vector before it is
    // overwritten below, as on the normal path.
    g_overlap.Run();
    Synchronize();
    --tri_debug_left_;
    std::vector<uint64_t> clk(s.levels + 1);
    Check(hipMemcpy(clk.data(), d_tri_clock_, clk.size() * sizeof(uint64_t),
                    hipMemcpyDeviceToHost),
          "D2H");
    const TriSchedule& l = tri_sched_[kTriL];
    std::fprintf(stderr,
                 "[tri] U: rows %d work %d levels %d segments %zu top %d entries/row max %d "
                 ">4 %d >16 %d >64 %d | L: work %d levels %d entries/row max %d >4 %d >16 %d "
                 ">64 %d; U per level (us/width):",
                 nc, s.work, s.levels, s.segments.size() / 2, top, s.max_entries,
                 s.rows_over[0], s.rows_over[1], s.rows_over[2], l.work, l.levels,
                 l.max_entries, l.rows_over[0], l.rows_over[1], l.rows_over[2]);
    for (int lv = 0; lv < s.levels; ++lv) {
      const bool ok = clk[lv] != 0 && clk[lv + 1] >= clk[lv];
      std::fprintf(stderr, " %.2f/%d", ok ? (clk[lv + 1] - clk[lv]) / 100.0 : -1.0,
                   s.level_width[lv]);
    }
    std::fprintf(stderr, "\n");
  } else {
    if (tri_graph_ && (c.graph_key[which] != s.key || c.graph_exec[which] == nullptr)) {
      DeviceOp("tri capture");
      std::lock_guard<std::mutex> lock(tri_mu_);  // one capture at a time
      CaptureTriGraph(which, &c);
      DeviceOp("tri capture done");
    }
    TriCopyIn(s, c);
    if (slot == 0) {
      BeginKernel(id);  // events around the graph: the kernels only
    } else if (Timed(id)) {
      Check(hipEventRecord(reinterpret_cast<hipEvent_t>(c.ev[0]), Stream(c.stream)), "ev");
    }
    if (tri_graph_) {
      Check(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(c.graph_exec[which]),
                           Stream(c.stream)),
            "graph launch");
    } else {
      EnqueueTriKernels(s, TriArgs(s, c), c.stream);
    }
    if (slot == 0) {
      EndKernel(id, bytes);
    } else if (Timed(id)) {
      Check(hipEventRecord(reinterpret_cast<hipEvent_t>(c.ev[1]), Stream(c.stream)), "ev");
    }
    TriCopyOut(s, c);
    if (slot == 0) g_overlap.Run();  // host work behind the device's
    DeviceOp("tri sync");
    Check(hipStreamSynchronize(Stream(c.stream)), "sync");
    DeviceOp("tri sync done");
    if (slot != 0) {
      // The worker's own counters (its id is written by this thread only).
      stats_.launches[id] += 1;
      stats_.algorithmic_bytes[id] += bytes;
      if (Timed(id)) {
        float ms = 0.0f;
        Check(hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(c.ev[0]),
                                  reinterpret_cast<hipEvent_t>(c.ev[1])),
              "ev time");
        stats_.device_ms[id] += ms;
      }
    }
  }
  if (*static_cast<volatile int*>(h_words + 1) != 0) {
    throw DeviceError("triangular solve: dependency wait timed out");
  }
  ft.Lap(kFtDevCopyOut);
  CopyHost(xv + fni, c.h_x + fni, size_t(top - fni + 1) * sizeof(double));
  return true;
}

// Two right-hand sides of the FTRAN's U solve in one launch (the direction
// and the dual steepest-edge tau, dual_edge_norms.cc:134-141, both against
// the same factorization): blockIdx.y picks the vector, each has its own
// rows, positions, staging and top row, the schedule is shared. Each vector's
// outputs are computed exactly as a single solve computes them.
bool DeviceLp::SolvePair(TriKind kind, const TriangularMatrix& t, uint64_t key,
                         std::vector<double>* x0, std::vector<double>* x1) {
  if (kind != TriKind::kUpperT || !tri_pair_ || g_lu_slot != 0) return false;
  if (!tri_syncfree_ || !tri_mapped_ || tri_graph_ || tri_persist_groups_ > 0) return false;
  if (tri_debug_left_ > 0) return false;
  SolveCallTimer timer(&stats_, MI_K_TRI_SOLVE);
  DeviceOp("tri U pair enter");
  if (!TriPrepare(kTriU, t, key, 0, *x0)) return false;
  if (static_cast<int>(x1->size()) < t.num_cols()) return false;
  TriSchedule& s = tri_sched_[kTriU];
  // Both vectors' workgroups resident at once: 2 x 512 workgroups of 256
  // at most, 4 per CU of the 8 the kernel's registers allow.
  if (s.max_wide_run > milp_kernels::kTriSyncFreeMaxWork || s.levels < tri_syncfree_min_levels_) {
    return false;
  }
  const int nc = t.num_cols();
  const int fni = s.first_col;
  {
    std::lock_guard<std::mutex> lock(tri_mu_);
    PrepareTriContext(2, nc, s.pos);
  }
  TriContext& c0 = tri_ctx_[0];
  TriContext& c1 = tri_ctx_[2];
  std::vector<double>* xs[2] = {x0, x1};
  TriContext* cs[2] = {&c0, &c1};
  int tops[2];
  double bytes = 0.0;
  for (int v = 0; v < 2; ++v) {
    const double* xv = xs[v]->data();
    int top = nc - 1;
    while (top >= fni && xv[top] == 0.0) --top;
    // A vector with nothing to compute (only the identity part) is solved
    // alone by the caller's single path.
    if (top < fni || s.rows_upto[top + 1] - s.rows_upto[fni] == 0) return false;
    tops[v] = top;
    const double rows = s.rows_upto[top + 1] - s.rows_upto[fni];
    const double entries = static_cast<double>(s.entries_upto[top + 1] - s.entries_upto[fni]);
    bytes += rows * (24.0 + (s.ones ? 0.0 : 8.0)) + entries * 20.0 + double(s.pos) * 20.0 +
             rows * 20.0;
  }
  const size_t in = size_t(nc - fni);
  for (int v = 0; v < 2; ++v) {
    TriContext& c = *cs[v];
    CopyHost(c.h_x + fni, xs[v]->data() + fni, in * sizeof(double));
    int* words = reinterpret_cast<int*>(c.h_x + nc);
    words[0] = tops[v];
    words[1] = 0;
  }
  milp_kernels::TriSolveArgs a = TriArgs(s, c0);
  a.x2 = static_cast<double*>(c1.x.ptr);
  a.y2 = static_cast<double*>(c1.y.ptr);
  a.host_x2 = c1.m_x;
  a.top2 = static_cast<int*>(c1.top.ptr);
  a.fail2 = reinterpret_cast<int*>(c1.m_x + s.rows) + 1;
  BeginKernel(MI_K_TRI_SOLVE);
  Check(milp_launch::tri_transpose_lower_syncfree(a, s.runs.data(),
                                                  static_cast<int>(s.runs.size() / 3),
                                                  Stream(c0.stream), 2),
        "tri pair");
  EndKernel(MI_K_TRI_SOLVE, bytes);
  g_overlap.Run();  // host work behind the device's
  DeviceOp("tri pair sync");
  Check(hipStreamSynchronize(Stream(c0.stream)), "sync");
  for (int v = 0; v < 2; ++v) {
    const int* words = reinterpret_cast<const int*>(cs[v]->h_x + nc);
    if (*static_cast<const volatile int*>(words + 1) != 0) {
      throw DeviceError("triangular solve: dependency wait timed out");
    }
  }
  for (int v = 0; v < 2; ++v) {
    CopyHost(xs[v]->data() + fni, cs[v]->h_x + fni, size_t(tops[v] - fni + 1) * sizeof(double));
  }
  return true;
}

// The dense U solve of the speculative flip FTRAN (device_solver.h
// StartAsyncU): TriSolve's staging and launch plan on slot 3's stream, with
// no wait; FinishAsyncU waits and copies the result back as TriSolve does.
bool DeviceLp::StartAsyncU(const TriangularMatrix& t, uint64_t key, const std::vector<double>& x) {
  if (g_lu_slot != 0 || !spec_flip_ || !tri_mapped_ || tri_graph_ || tri_debug_left_ > 0) {
    return false;
  }
  DropAsyncU();
  if (!TriPrepare(kTriU, t, key, 3, x)) return false;
  const int nc = t.num_cols();
  TriContext& c = tri_ctx_[3];
  TriSchedule& s = tri_sched_[kTriU];
  const int fni = s.first_col;
  int top = nc - 1;
  while (top >= fni && x[top] == 0.0) --top;
  async_u_.active = true;
  async_u_.trivial = top < fni || s.rows_upto[top + 1] - s.rows_upto[fni] == 0;
  if (async_u_.trivial) return true;
  DeviceOp("tri U async enter");
  CopyHost(c.h_x + fni, x.data() + fni, size_t(nc - fni) * sizeof(double));
  int* h_words = reinterpret_cast<int*>(c.h_x + nc);
  h_words[0] = top;
  h_words[1] = 0;
  const double rows = s.rows_upto[top + 1] - s.rows_upto[fni];
  const double entries = static_cast<double>(s.entries_upto[top + 1] - s.entries_upto[fni]);
  async_u_.bytes = rows * (24.0 + (s.ones ? 0.0 : 8.0)) + entries * 20.0 +
                   double(s.pos) * 20.0 + rows * 20.0;
  async_u_.rows = nc;
  async_u_.first = fni;
  async_u_.top = top;
  async_u_.timed = Timed(MI_K_TRI_SOLVE);
  if (async_u_.timed) {
    Check(hipEventRecord(reinterpret_cast<hipEvent_t>(c.ev[0]), Stream(c.stream)), "ev");
  }
  EnqueueTriKernels(s, TriArgs(s, c), c.stream);
  if (async_u_.timed) {
    Check(hipEventRecord(reinterpret_cast<hipEvent_t>(c.ev[1]), Stream(c.stream)), "ev");
  }
  return true;
}

void DeviceLp::FinishAsyncU(std::vector<double>* x) {
  if (!async_u_.active) throw DeviceError("asynchronous U solve: none in flight");
  async_u_.active = false;
  if (async_u_.trivial) return;
  TriContext& c = tri_ctx_[3];
  DeviceOp("tri U async sync");
  Check(hipStreamSynchronize(Stream(c.stream)), "sync");
  stats_.launches[MI_K_TRI_SOLVE] += 1;
  stats_.algorithmic_bytes[MI_K_TRI_SOLVE] += async_u_.bytes;
  if (async_u_.timed && Timed(MI_K_TRI_SOLVE)) {
    float ms = 0.0f;
    Check(hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(c.ev[0]),
                              reinterpret_cast<hipEvent_t>(c.ev[1])),
          "ev time");
    stats_.device_ms[MI_K_TRI_SOLVE] += ms;
  }
  const int nc = async_u_.rows;
  if (*reinterpret_cast<volatile int*>(reinterpret_cast<int*>(c.h_x + nc) + 1) != 0) {
    throw DeviceError("triangular solve: dependency wait timed out");
  }
  const int fni = async_u_.first;
  CopyHost(x->data() + fni, c.h_x + fni, size_t(async_u_.top - fni + 1) * sizeof(double));
}

void DeviceLp::DropAsyncU() {
  if (!async_u_.active) return;
  async_u_.active = false;
  if (!async_u_.trivial && tri_ctx_[3].stream != nullptr) {
    (void)hipStreamSynchronize(Stream(tri_ctx_[3].stream));
  }
}

}  // namespace milp
