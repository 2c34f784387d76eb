// DeviceLp over column shards (the single-LP split).
//
// Every per-iteration operation of the simplex on [A | I] is per column:
// pricing rc_j = c_j - a_j.y (reduced_costs.cc:352-423), the update row
// coefficient a_j.rho (update_row.cc:77-306, every algorithm accumulates one
// column's terms in rho order), the list dots, the device reduced-cost
// update, the boxed flips. Split the columns into contiguous blocks and each
// block's results are exactly the unsplit results for those columns; joined
// in column order they are the unsplit vectors, bit for bit.
//
// The one cross-column decision is the dual ratio test's filter
// (entering_variable.cc:37-130, DeviceLp::DualRatioCandidates): shard s keeps
// the breakpoints with ratio <= B_s (1 + 1e-9), B_s its own bound. B_s is a
// min over a subset, so B_s >= B (the unsplit bound) and every shard returns
// a superset of what the unsplit filter keeps from its columns; the tightened
// bound of a shard's pop-order walk is likewise >= the unsplit one (a walk
// over fewer boxed breakpoints consumes less of the variation). Glop's two
// loops then run on the host over the concatenation, in list order: the
// extra breakpoints are ones the unfiltered loops would see anyway, so the
// choice, the flips and the ties are the unsplit ones. On separate GPUs this
// join is the all-reduce(min) + all-gather of the reference's sharded
// design; here the host is the one consumer, so it is a concatenation in
// host memory.
#include <hip/hip_runtime.h>

#include <chrono>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../kernels/kernel_args.h"
#include "device_lp.h"
#include "lp_data.h"

namespace milp {

namespace {
// Restores the handle's device when a sharded call returns (the shards may
// live on other GPUs; kernels launch on the calling thread's device).
struct DeviceGuard {
  int device;
  ~DeviceGuard() { (void)hipSetDevice(device); }
};
// Shard results travel between processes as byte strings: vectors with a
// count prefix, appended and read back in the same order.
struct PartWriter {
  std::string b;
  template <typename T>
  void Put(const std::vector<T>& v) {
    const int64_t n = static_cast<int64_t>(v.size());
    b.append(reinterpret_cast<const char*>(&n), sizeof(n));
    if (n > 0) b.append(reinterpret_cast<const char*>(v.data()), size_t(n) * sizeof(T));
  }
  template <typename T>
  void Put(T x) {
    b.append(reinterpret_cast<const char*>(&x), sizeof(x));
  }
};
struct PartReader {
  const std::string& b;
  size_t at = 0;
  template <typename T>
  void Get(std::vector<T>* v) {
    int64_t n = 0;
    Raw(&n, sizeof(n));
    v->resize(size_t(n));
    if (n > 0) Raw(v->data(), size_t(n) * sizeof(T));
  }
  template <typename T>
  T Get() {
    T x{};
    Raw(&x, sizeof(x));
    return x;
  }
  void Raw(void* dst, size_t bytes) {
    if (at + bytes > b.size()) throw DeviceError("column split: short exchange message");
    std::memcpy(dst, b.data() + at, bytes);
    at += bytes;
  }
};
}  // namespace

// Cross-process split: `world` processes solve the same LP,
// each with the same host control flow; process `rank` owns column block
// `rank` on its own GPU. Every per-column operation runs on the owned block
// only, and a join gathers the blocks' results in block order through the
// caller's all-gather, so every process sees the joined vectors the
// single-process split (and the unsplit engine) computes.
void DeviceLp::SetExchange(int rank, int world, void* ctx, ExchangeFn fn) {
  if (world <= 1 || fn == nullptr) {
    exchange_fn_ = nullptr;
    exchange_rank_ = 0;
    exchange_world_ = 1;
    return;
  }
  if (rank < 0 || rank >= world) throw DeviceError("column split: bad rank");
  if (m_ > 0) throw DeviceError("column split: set the exchange before loading the LP");
  exchange_fn_ = fn;
  exchange_ctx_ = ctx;
  exchange_rank_ = rank;
  exchange_world_ = world;
  DeviceGuard guard{device_};
  shards_.clear();
  shards_.resize(world);
  auto shard = std::make_unique<DeviceLp>();
  shard->is_shard_ = true;
  shard->Init(device_);
  shard->timing_ = timing_;
  shards_[rank] = std::move(shard);
}

// Local shard results in, every shard's results out (block order).
void DeviceLp::ExchangeParts(std::vector<std::string>* parts) {
  if (exchange_fn_ == nullptr) return;
  const auto t0 = std::chrono::steady_clock::now();
  struct Account {
    mi_lp_kernel_stats& st;
    std::chrono::steady_clock::time_point t0;
    int64_t bytes = 0;
    ~Account() {
      st.launches[MI_K_EXCHANGE] += 2;  // sizes, then the messages
      st.algorithmic_bytes[MI_K_EXCHANGE] += static_cast<double>(bytes);
      st.call_ms[MI_K_EXCHANGE] += std::chrono::duration<double, std::milli>(
                                       std::chrono::steady_clock::now() - t0).count();
    }
  } account{stats_, t0};
  const int world = exchange_world_;
  const std::string& mine = (*parts)[exchange_rank_];
  int64_t n = static_cast<int64_t>(mine.size());
  std::vector<int64_t> sizes(world, 0);
  std::vector<int64_t> eight(world, int64_t{sizeof(int64_t)});
  if (exchange_fn_(exchange_ctx_, &n, sizeof(n), sizes.data(), eight.data()) != 0) {
    throw DeviceError("column split: exchange of sizes failed");
  }
  int64_t total = 0;
  for (int64_t z : sizes) total += z;
  account.bytes = total;
  std::string all(size_t(total), '\0');
  if (exchange_fn_(exchange_ctx_, mine.data(), n, all.data(), sizes.data()) != 0) {
    throw DeviceError("column split: exchange failed");
  }
  int64_t at = 0;
  for (int r = 0; r < world; ++r) {
    (*parts)[r].assign(all.data() + at, size_t(sizes[r]));
    at += sizes[r];
  }
}

void DeviceLp::CreateShards() {
  if (is_shard_) return;
  const char* v = std::getenv("MILP_SHARDS");
  const int count = v != nullptr ? std::atoi(v) : 1;
  if (count <= 1) return;
  std::vector<int> devices;
  if (const char* d = std::getenv("MILP_SHARD_DEVICES")) {
    std::string list(d);
    size_t at = 0;
    while (at <= list.size()) {
      const size_t comma = list.find(',', at);
      const std::string item = list.substr(at, comma == std::string::npos ? std::string::npos
                                                                           : comma - at);
      if (!item.empty()) devices.push_back(std::atoi(item.c_str()));
      if (comma == std::string::npos) break;
      at = comma + 1;
    }
  }
  DeviceGuard guard{device_};
  for (int s = 0; s < count; ++s) {
    auto shard = std::make_unique<DeviceLp>();
    shard->is_shard_ = true;
    shard->Init(devices.empty() ? device_ : devices[s % devices.size()]);
    shard->timing_ = timing_;
    shards_.push_back(std::move(shard));
  }
}

DeviceLp& DeviceLp::Shard(int s) {
  DeviceLp& d = *shards_[s];
  if (d.device_ != device_) Check(hipSetDevice(d.device_), "hipSetDevice");
  return d;
}

int DeviceLp::ShardOf(int col) const {
  return static_cast<int>(std::upper_bound(shard_begin_.begin(), shard_begin_.end(), col) -
                          shard_begin_.begin()) - 1;
}

// Column blocks balanced by entries, each starting on a 64-column boundary
// (so a block's mask bits are whole words of the full mask).
void DeviceLp::ShardedUpload(const CompactSparseMatrix& csc) {
  DeviceGuard guard{device_};
  const int ns = static_cast<int>(shards_.size());
  const int n = csc.num_cols();
  const int64_t total = csc.num_entries();
  shard_begin_.assign(ns + 1, n);
  shard_begin_[0] = 0;
  int64_t seen = 0;
  int s = 1;
  for (int c = 0; c < n && s < ns; ++c) {
    seen += csc.ColumnNumEntries(c);
    if (seen * ns >= total * s && (c + 1) % 64 == 0) shard_begin_[s++] = c + 1;
  }
  for (; s < ns; ++s) shard_begin_[s] = n;  // tiny LPs: empty trailing shards
  for (int k = 0; k < ns; ++k) {
    if (!IsLocalShard(k)) continue;
    CompactSparseMatrix slice, slice_t;
    slice.PopulateColumnSlice(csc, shard_begin_[k], shard_begin_[k + 1]);
    slice_t.PopulateFromTranspose(slice);
    Shard(k).UploadMatrix(slice, slice_t);
  }
}

uint64_t DeviceLp::list_epoch() const {
  if (shards_.empty()) return list_epoch_;
  uint64_t e = 0;
  for (const auto& d : shards_) {
    if (d) e += d->list_epoch_;
  }
  return e;
}

void DeviceLp::SetTiming(bool on, uint32_t id_mask) {
  timing_ = on;
  timing_ids_ = id_mask;
  for (auto& d : shards_) {
    if (d) {
      d->timing_ = on;
      d->timing_ids_ = id_mask;
    }
  }
}

void DeviceLp::FlushOwnMasks() {
  for (int k = 0; k < kNumMasks; ++k) {
    if (own_mask_dirty_[k]) {
      UploadMask(static_cast<Mask>(k));
      own_mask_dirty_[k] = false;
    }
  }
}

void DeviceLp::ShardedSetMask(Mask which, const uint64_t* words, int num_words) {
  if (num_words != mask_words_) throw DeviceError("mask size mismatch");
  // This handle's copy (row sums, column norms) is uploaded when next used.
  std::memcpy(h_masks_[which].data(), words, num_words * sizeof(uint64_t));
  own_mask_dirty_[which] = true;
  DeviceGuard guard{device_};
  for (int s = 0; s < num_shards(); ++s) {
    const int b = shard_begin_[s], e = shard_begin_[s + 1];
    if (e == b || !IsLocalShard(s)) continue;
    Shard(s).SetMask(which, words + b / 64, (e - b + 63) / 64);
  }
}

void DeviceLp::ShardedUpdateRowColumnWise(const std::vector<double>& rho, double drop,
                                          int64_t relevant_entries,
                                          const std::vector<double>* w) {
  DeviceGuard guard{device_};
  for (int s = 0; s < num_shards(); ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    if (d.n_total_ == 0) continue;
    // (byte accounting only) the shard's share of the relevant entries
    const double share = double(d.nnz_) / double(std::max<int64_t>(1, nnz_));
    d.UpdateRowColumnWise(rho, drop, static_cast<int64_t>(share * relevant_entries), w);
  }
}

void DeviceLp::ShardedUpdateRowRowWise(const std::vector<int>& filtered_rows,
                                       const std::vector<double>& rho, int algorithm,
                                       double drop) {
  DeviceGuard guard{device_};
  for (int s = 0; s < num_shards(); ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    if (d.n_total_ > 0) d.UpdateRowRowWise(filtered_rows, rho, algorithm, drop);
  }
}

void DeviceLp::ShardedFetchUpdateRow(std::vector<int>* positions, std::vector<double>* values) {
  DeviceGuard guard{device_};
  positions->clear();
  values->clear();
  const int ns = num_shards();
  std::vector<std::string> parts(ns);
  for (int s = 0; s < ns; ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    std::vector<int> p;
    std::vector<double> v;
    if (d.n_total_ > 0) d.FetchUpdateRow(&p, &v);
    PartWriter w;
    w.Put(p);
    w.Put(v);
    parts[s] = std::move(w.b);
  }
  ExchangeParts(&parts);
  std::vector<int> p;
  std::vector<double> v;
  for (int s = 0; s < ns; ++s) {
    PartReader r{parts[s]};
    r.Get(&p);
    r.Get(&v);
    for (int& c : p) c += shard_begin_[s];
    positions->insert(positions->end(), p.begin(), p.end());
    values->insert(values->end(), v.begin(), v.end());
  }
  list_count_ = static_cast<int>(positions->size());
}

double DeviceLp::ShardedReadCoefficient(int col) {
  DeviceGuard guard{device_};
  const int s = ShardOf(col);
  if (exchange_fn_ == nullptr) return Shard(s).ReadCoefficient(col - shard_begin_[s]);
  // The owner reads, everyone receives (a broadcast as an all-gather).
  std::vector<std::string> parts(num_shards());
  PartWriter w;
  w.Put(IsLocalShard(s) ? Shard(s).ReadCoefficient(col - shard_begin_[s]) : 0.0);
  parts[exchange_rank_] = std::move(w.b);
  ExchangeParts(&parts);
  PartReader r{parts[s]};
  return r.Get<double>();
}

void DeviceLp::ShardedListDotsOverUpdateRow(const std::vector<double>& v,
                                            std::vector<double>* out) {
  DeviceGuard guard{device_};
  out->clear();
  const int ns = num_shards();
  std::vector<std::string> parts(ns);
  std::vector<double> part;
  for (int s = 0; s < ns; ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    part.clear();
    if (d.n_total_ > 0) d.ListDotsOverUpdateRow(v, &part);
    PartWriter w;
    w.Put(part);
    parts[s] = std::move(w.b);
  }
  ExchangeParts(&parts);
  for (int s = 0; s < ns; ++s) {
    PartReader r{parts[s]};
    r.Get(&part);
    out->insert(out->end(), part.begin(), part.end());
  }
}

void DeviceLp::ShardedListDots(const std::vector<int>& cols, const std::vector<double>& v,
                               std::vector<double>* out) {
  DeviceGuard guard{device_};
  const int ns = num_shards();
  std::vector<std::vector<int>> sub(ns), where(ns);
  for (int i = 0; i < static_cast<int>(cols.size()); ++i) {
    const int s = ShardOf(cols[i]);
    sub[s].push_back(cols[i] - shard_begin_[s]);
    where[s].push_back(i);
  }
  out->assign(cols.size(), 0.0);
  std::vector<std::string> parts(ns);
  std::vector<double> part;
  for (int s = 0; s < ns; ++s) {
    if (!IsLocalShard(s)) continue;
    part.clear();
    if (!sub[s].empty()) Shard(s).ListDots(sub[s], v, &part);
    PartWriter w;
    w.Put(part);
    parts[s] = std::move(w.b);
  }
  ExchangeParts(&parts);
  for (int s = 0; s < ns; ++s) {
    PartReader r{parts[s]};
    r.Get(&part);
    for (size_t k = 0; k < part.size() && k < where[s].size(); ++k) (*out)[where[s][k]] = part[k];
  }
}

void DeviceLp::ShardedPricing(const std::vector<double>& c, const std::vector<double>& y,
                              std::vector<double>* rc, const std::vector<double>* w,
                              std::vector<double>* list_dots) {
  DeviceGuard guard{device_};
  rc->resize(n_total_);
  if (list_dots != nullptr) list_dots->clear();
  const int ns = num_shards();
  std::vector<std::string> parts(ns);
  std::vector<double> cs, part, dots;
  for (int s = 0; s < ns; ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    part.clear();
    dots.clear();
    if (d.n_total_ > 0) {
      const int b = shard_begin_[s];
      cs.assign(c.begin() + b, c.begin() + shard_begin_[s + 1]);
      d.Pricing(cs, y, &part, w, w != nullptr ? &dots : nullptr);
    }
    PartWriter pw;
    pw.Put(part);
    pw.Put(dots);
    parts[s] = std::move(pw.b);
  }
  ExchangeParts(&parts);
  for (int s = 0; s < ns; ++s) {
    PartReader r{parts[s]};
    r.Get(&part);
    r.Get(&dots);
    std::copy(part.begin(), part.end(), rc->begin() + shard_begin_[s]);
    if (w != nullptr) list_dots->insert(list_dots->end(), dots.begin(), dots.end());
  }
}

void DeviceLp::ShardedDualBegin(const std::vector<double>& rc,
                                const std::vector<uint8_t>& colbits,
                                const std::vector<double>& bound_diff) {
  DeviceGuard guard{device_};
  for (int s = 0; s < num_shards(); ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    if (d.n_total_ == 0) continue;
    const int b = shard_begin_[s], e = shard_begin_[s + 1];
    d.DualBegin(std::vector<double>(rc.begin() + b, rc.begin() + e),
                std::vector<uint8_t>(colbits.begin() + b, colbits.begin() + e),
                std::vector<double>(bound_diff.begin() + b, bound_diff.begin() + e));
  }
}

void DeviceLp::ShardedDualSetColBits(const std::vector<int32_t>& cols,
                                     const std::vector<uint8_t>& bits) {
  DeviceGuard guard{device_};
  const int ns = num_shards();
  std::vector<std::vector<int32_t>> sc(ns);
  std::vector<std::vector<uint8_t>> sb(ns);
  for (size_t i = 0; i < cols.size(); ++i) {
    const int s = ShardOf(cols[i]);
    sc[s].push_back(cols[i] - shard_begin_[s]);
    sb[s].push_back(bits[i]);
  }
  for (int s = 0; s < ns; ++s) {
    if (!sc[s].empty() && IsLocalShard(s)) Shard(s).DualSetColBits(sc[s], sb[s]);
  }
}

void DeviceLp::ShardedDualTakePricedReducedCosts() {
  DeviceGuard guard{device_};
  for (int s = 0; s < num_shards(); ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    if (d.n_total_ > 0) d.DualTakePricedReducedCosts();
  }
}

void DeviceLp::ShardedDualDownloadReducedCosts(std::vector<double>* rc) {
  DeviceGuard guard{device_};
  rc->resize(n_total_);
  const int ns = num_shards();
  std::vector<std::string> parts(ns);
  std::vector<double> part;
  for (int s = 0; s < ns; ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    part.clear();
    if (d.n_total_ > 0) d.DualDownloadReducedCosts(&part);
    PartWriter w;
    w.Put(part);
    parts[s] = std::move(w.b);
  }
  ExchangeParts(&parts);
  for (int s = 0; s < ns; ++s) {
    PartReader r{parts[s]};
    r.Get(&part);
    std::copy(part.begin(), part.end(), rc->begin() + shard_begin_[s]);
  }
}

void DeviceLp::ShardedDualSetReducedCost(int col, double value) {
  DeviceGuard guard{device_};
  const int s = ShardOf(col);
  if (IsLocalShard(s)) Shard(s).DualSetReducedCost(col - shard_begin_[s], value);
}

void DeviceLp::ShardedDualRatioCandidates(double sign, double threshold,
                                          double harris_tolerance, double minimum_delta,
                                          double variation_magnitude, DualCandidates* out) {
  DeviceGuard guard{device_};
  out->col.clear();
  out->coeff.clear();
  out->rc.clear();
  out->list_count = 0;
  const int ns = num_shards();
  std::vector<std::string> parts(ns);
  DualCandidates part;
  for (int s = 0; s < ns; ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    part = DualCandidates();
    if (d.n_total_ > 0) {
      d.DualRatioCandidates(sign, threshold, harris_tolerance, minimum_delta,
                            variation_magnitude, &part);
    }
    PartWriter w;
    w.Put(part.col);
    w.Put(part.coeff);
    w.Put(part.rc);
    w.Put(static_cast<int64_t>(part.list_count));
    parts[s] = std::move(w.b);
  }
  // Across processes this is the reference's exchange: the blocks' filtered
  // breakpoints (each a superset under its own bound, see the top of this
  // file) gathered in block order.
  ExchangeParts(&parts);
  for (int s = 0; s < ns; ++s) {
    PartReader r{parts[s]};
    r.Get(&part.col);
    r.Get(&part.coeff);
    r.Get(&part.rc);
    part.list_count = static_cast<int>(r.Get<int64_t>());
    for (int& c : part.col) c += shard_begin_[s];
    out->col.insert(out->col.end(), part.col.begin(), part.col.end());
    out->coeff.insert(out->coeff.end(), part.coeff.begin(), part.coeff.end());
    out->rc.insert(out->rc.end(), part.rc.begin(), part.rc.end());
    out->list_count += part.list_count;
  }
  last_candidates_ = static_cast<int>(out->col.size());
}

void DeviceLp::ShardedDualUpdateReducedCosts(double mult, int leaving_col,
                                             double leaving_value, int entering_col) {
  DeviceGuard guard{device_};
  for (int s = 0; s < num_shards(); ++s) {
    if (!IsLocalShard(s)) continue;
    DeviceLp& d = Shard(s);
    if (d.n_total_ == 0) continue;
    const int b = shard_begin_[s], e = shard_begin_[s + 1];
    const int lc = leaving_col >= b && leaving_col < e ? leaving_col - b : -1;
    const int ec = entering_col >= b && entering_col < e ? entering_col - b : -1;
    d.DualUpdateReducedCosts(mult, lc, leaving_value, ec);
  }
}

void DeviceLp::ShardedDualBoxedFlips(const std::vector<int>* cols, double threshold,
                                     std::vector<uint8_t>* flags) {
  DeviceGuard guard{device_};
  const int ns = num_shards();
  std::vector<uint8_t> part;
  std::vector<std::string> parts(ns);
  if (cols == nullptr) {
    flags->assign(n_total_, 0);
    for (int s = 0; s < ns; ++s) {
      if (!IsLocalShard(s)) continue;
      DeviceLp& d = Shard(s);
      part.clear();
      if (d.n_total_ > 0) d.DualBoxedFlips(nullptr, threshold, &part);
      PartWriter w;
      w.Put(part);
      parts[s] = std::move(w.b);
    }
    ExchangeParts(&parts);
    for (int s = 0; s < ns; ++s) {
      PartReader r{parts[s]};
      r.Get(&part);
      std::copy(part.begin(), part.end(), flags->begin() + shard_begin_[s]);
    }
    return;
  }
  std::vector<std::vector<int>> sub(ns), where(ns);
  for (int i = 0; i < static_cast<int>(cols->size()); ++i) {
    const int s = ShardOf((*cols)[i]);
    sub[s].push_back((*cols)[i] - shard_begin_[s]);
    where[s].push_back(i);
  }
  flags->assign(cols->size(), 0);
  for (int s = 0; s < ns; ++s) {
    if (!IsLocalShard(s)) continue;
    part.clear();
    if (!sub[s].empty()) Shard(s).DualBoxedFlips(&sub[s], threshold, &part);
    PartWriter w;
    w.Put(part);
    parts[s] = std::move(w.b);
  }
  ExchangeParts(&parts);
  for (int s = 0; s < ns; ++s) {
    PartReader r{parts[s]};
    r.Get(&part);
    for (size_t k = 0; k < part.size() && k < where[s].size(); ++k) (*flags)[where[s][k]] = part[k];
  }
}

void DeviceLp::ShardedStats() {
  agg_stats_ = stats_;
  for (auto& d : shards_) {
    if (!d) continue;  // another process's block
    const mi_lp_kernel_stats& st = d->stats();
    for (int k = 0; k < MI_K_COUNT; ++k) {
      agg_stats_.launches[k] += st.launches[k];
      agg_stats_.algorithmic_bytes[k] += st.algorithmic_bytes[k];
      agg_stats_.device_ms[k] += st.device_ms[k];
      agg_stats_.call_ms[k] += st.call_ms[k];
    }
  }
}

}  // namespace milp
