// Device-resident primal simplex segment: Glop's PrimalMinimize loop
// (revised_simplex.cc:2751-3045) on the segment machinery of sdual_core.h
// (same arena, the same factorization service through the mailbox, the same
// solves, update row and reduced-cost code). Compiled twice like
// sdual_core.h: one lane on the host (the CPU checks run it inside the
// oracle's own primal loop), the 64 lanes of a wave on gfx950.
//
// Supported: the MPF basis representation, steepest-edge pricing (the
// default primal feasibility and optimization rules), phase I with Glop's
// piecewise-linear costs and phase II. The segment starts after the loop-top
// block and runs until the loop needs the host (SdExit): a final status, an
// unbounded ray, a limit, or a capacity.
#ifndef MILP_SPRIMAL_CORE_H_
#define MILP_SPRIMAL_CORE_H_

namespace sdual {

// Segment-local final statuses (kExitStatus; the host maps them).
constexpr int32_t kStOptimal = 0, kStPrimalFeasible = 1, kStPrimalInfeasible = 2;

// ---- ScalarProduct(dense u, ScatteredVector v) (lp_utils.h:54-103) ----
SD_INLINE f64 vec_scalar_product(const f64* u, const Vec& v, f64* lds_scratch) {
#if defined(__HIP_DEVICE_COMPILE__)
  // Up to 256 terms (a block's ((a + b) + c) + d of the dense form, or one
  // product of the sparse form) on the lanes, summed in order by lane 0.
  l_f64* red = SD_L(f64, reinterpret_cast<SdScratch*>(lds_scratch)->red);
  const int lane = sd_lane();
  const bool dense = vec_dense(v, 0.8);
  const f64* c = v.values;
  const int n = dense ? v.size / 4 : v.nnz;
  f64 sum = 0.0;
  for (int base = 0; base < n; base += 256) {
    const int cnt = n - base < 256 ? n - base : 256;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = base + 64 * q + lane;
      f64 term = 0.0;
      if (64 * q + lane < cnt) {
        if (dense) {
          const int i = 4 * j;
          term = (u[i] * c[i]) + (u[i + 1] * c[i + 1]) + (u[i + 2] * c[i + 2]) +
                 (u[i + 3] * c[i + 3]);
        } else {
          const int i = v.nz[j];
          term = u[i] * c[i];
        }
      }
      red[64 * q + lane] = term;
    }
    sd_sync();
    if (lane == 0) {
      for (int j = 0; j < cnt; ++j) sum += red[j];
    }
    sd_sync();
  }
  if (lane == 0) {
    if (dense) {
      for (int i = 4 * n; i < v.size; ++i) sum += u[i] * c[i];
    }
    red[0] = sum;
  }
  sd_sync();
  const f64 result = red[0];
  sd_sync();
  return result;
#else
  (void)lds_scratch;
  f64 sum = 0.0;
  if (vec_dense(v, 0.8)) {
    int i = 0;
    const int blocks = v.size / 4;
    for (int b = 0; b < blocks; ++b) {
      sum += (u[i] * v.values[i]) + (u[i + 1] * v.values[i + 1]) +
             (u[i + 2] * v.values[i + 2]) + (u[i + 3] * v.values[i + 3]);
      i += 4;
    }
    for (; i < v.size; ++i) sum += u[i] * v.values[i];
    return sum;
  }
  for (int k = 0; k < v.nnz; ++k) sum += u[v.nz[k]] * v.values[v.nz[k]];
  return sum;
#endif
}
SD_INLINE f64 sp_vec_squared_norm(Lp& s, const Vec& v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return vec_squared_norm_dev(v, s.lds_scratch);
#else
  (void)s;
  return vec_squared_norm(v);
#endif
}

// ---- ReducedCosts, primal side (reduced_costs.cc:53-94, 226-311, 490-497) ----
SD_INLINE void rc_reset_for_new_objective(Lp& s) {
  s.recompute_bo = 1;
  s.recompute_bo_left_inverse = 1;
  s.rc_precise = 0;
  rc_set_recompute_and_notify(s);
}
SD_INLINE f64 rc_test_entering_precision(Lp& s, int col) {
  if (s.recompute_bo) rc_compute_basic_objective(s);
  const f64 old_rc = s.rc[col];
  const f64 precise = s.objective[col] + s.cost_pert[col] -
                      vec_scalar_product(s.basic_obj, s.dir, s.lds_scratch);
  s.rc[col] = precise;
  if (!s.recompute_rc) {
    const f64 acc = old_rc - precise;
    const f64 scale = (sd_fabs(precise) <= 1.0) ? 1.0 : precise;
    if (sd_fabs(acc) / scale > s.recompute_reduced_costs_threshold) rc_make_precise(s);
  }
  return precise;
}
SD_INLINE bool rc_is_valid_primal_entering(const Lp& s, int col) {
  const f64 rc = s.rc[col];
  const f64 tol = s.dual_tol;
  return (bit_get(s.can_inc, col) && (rc < -tol)) || (bit_get(s.can_dec, col) && (rc > tol));
}
SD_INLINE void rc_set_nonbasic_cost_to_zero(Lp& s, int col) {
  s.rc[col] -= s.objective[col];
  s.objective[col] = 0.0;
}

// ---- PrimalEdgeNorms, steepest edge (primal_edge_norms.cc) ----
// LuFactorization::RightSolveSquaredNorm (lu_factorization.cc:128-156) of
// matrix column `col`, after BasisFactorization's bump.
SD_INLINE f64 bf_right_solve_squared_norm(Lp& s, int col) {
  const int64_t b = s.A.starts[col], e = s.A.starts[col + 1];
  bf_bump(s, e - b);
  if (s.is_identity) {  // SquaredNorm(ColumnView), in entry order
    f64 sum = 0.0;
    for (int64_t i = b; i < e; ++i) sum += sq(s.A.coefs[i]);
    return sum;
  }
  int32_t* nz = s.dp.equiv;  // non_zero_rows_ scratch (m + 1)
  f64* z = s.zero_scratch;
  const int n0 = static_cast<int>(e - b);
  for (int k = sd_lane(); k < n0; k += sd_lanes()) {  // a column's rows are distinct
    const int pr = s.row_perm[s.A.rows[b + k]];
    z[pr] = s.A.coefs[b + k];
    nz[k] = pr;
  }
  sd_sync();
  int nnz = n0;
  { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.lower, nz, &nnz, s.stored); }
  if (nnz == 0) {
    SdSubTimer t_(&s.phase_ticks[9]);
    tri_lower_solve_from(s.lower, 0, z);
  } else {
    { SdSubTimer t_x_(&s.phase_ticks[17]); tri_hyper_solve(s.lower, z, nz, &nnz); }
    { SdSubTimer t_x_(&s.phase_ticks[16]); tri_rows_to_consider(s.upper, nz, &nnz, s.stored); }
  }
  if (nnz == 0) {
    SdSubTimer t_(&s.phase_ticks[9]);
    tri_upper_solve(s.upper, z);
  } else {
    SdSubTimer t_x_(&s.phase_ticks[17]);
    tri_hyper_solve_rev(s.upper, z, nz, &nnz);
  }
  f64 sum = 0.0;
  if (nnz == 0) {
    sum = dense_squared_norm(z, s.m);
    sd_sync();
    for (int i = sd_lane(); i < s.m; i += sd_lanes()) z[i] = 0.0;
  } else {
    for (int k = 0; k < nnz; ++k) sum += sq(z[nz[k]]);
    sd_sync();
    for (int k = sd_lane(); k < nnz; k += sd_lanes()) z[nz[k]] = 0.0;
  }
  sd_sync();
  return sum;
}
SD_INLINE void pen_set_recompute(Lp& s) {
  s.pen_recompute = 1;
  s.pp_recompute = 1;  // the watcher (PrimalPrices::recompute_)
}
// ComputeEdgeSquaredNorms (:147-161): the relevant columns in order.
SD_INLINE const f64* pen_get(Lp& s) {
  if (s.pen_recompute) {
    for (int w = 0; w < s.nwords; ++w) {
      uint64_t word = s.relevant[w];
      while (word) {
        const int col = w * 64 + sd_ctz(word);
        word &= word - 1;
        if (col >= s.N) break;
        s.pen_norms[col] = 1.0 + bf_right_solve_squared_norm(s, col);
      }
    }
    s.pen_recompute = 0;
  }
  return s.pen_norms;
}
// TestEnteringEdgeNormPrecision (:79-108)
SD_INLINE bool pen_test_entering_precision(Lp& s, int col) {
  if (s.pen_recompute) return true;
  const f64 old_sq = s.pen_norms[col];
  const f64 precise_sq = 1.0 + sp_vec_squared_norm(s, s.dir);
  s.pen_norms[col] = precise_sq;
  const f64 precise = sd_sqrt(precise_sq);
  const f64 acc = (precise - sd_sqrt(old_sq)) / precise;
  if (sd_fabs(acc) > s.recompute_edges_norm_threshold) pen_set_recompute(s);
  return !(old_sq < 0.25 * precise_sq);
}
// ComputeDirectionLeftInverse (:166-199)
SD_INLINE void pen_direction_left_inverse(Lp& s) {
  Vec& w = s.dli;
  const Vec& d = s.dir;
  const int size = d.size;
  const f64 threshold = 0.05 * static_cast<f64>(size);
  if (w.nnz != 0 && static_cast<f64>(w.nnz + d.nnz) < 2.0 * threshold) {
    vec_clear_and_resize(w, size);
    for (int k = sd_lane(); k < d.nnz; k += sd_lanes()) {  // distinct rows
      w.values[d.nz[k]] = d.values[d.nz[k]];
    }
    sd_sync();
  } else {
    for (int i = sd_lane(); i < size; i += sd_lanes()) w.values[i] = d.values[i];
    sd_sync();
    w.size = size;
    w.nnz = 0;
  }
  if (static_cast<f64>(d.nnz) < threshold) {
    for (int k = sd_lane(); k < d.nnz; k += sd_lanes()) w.nz[k] = d.nz[k];
    sd_sync();
    w.nnz = d.nnz;
  }
  bf_left_solve(s, w);
}
// UpdateEdgeSquaredNorms (:208-258): every listed column writes its own norm.
SD_INLINE void pen_update_edge_squared_norms(Lp& s, int entering_col, int leaving_col,
                                             int leaving_row) {
  const f64 pivot = -s.dir.values[leaving_row];
  const f64 entering_sq = s.pen_norms[entering_col];
  const f64 leaving_sq = sd_max(1.0, entering_sq / sq(pivot));
  const f64 factor = 2.0 / pivot;
  const f64* w = s.dli.values;
  SdSubTimer t_x_(&s.phase_ticks[24]);
  int64_t ops = 0;
  for (int k = sd_lane(); k < s.n_nzpos; k += sd_lanes()) {
    const int col = s.nzpos[k];
    const f64 coeff = s.coeff[col];
    const f64 scalar_product = col_dot(s.A, col, w);
    ops += col_entries(s.A, col);
    s.pen_norms[col] += coeff * (coeff * leaving_sq + factor * scalar_product);
    const f64 lower_bound = 1.0 + sq(coeff / pivot);
    if (s.pen_norms[col] < lower_bound) s.pen_norms[col] = lower_bound;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  ops = sd_wave_sum_i64(ops);
#endif
  sd_sync();
  s.pen_ops += ops;
  s.pen_norms[leaving_col] = leaving_sq;
}
// UpdateBeforeBasisPivot (:110-136), steepest edge (Devex weights stay reset).
SD_INLINE void pen_update_before_pivot(Lp& s, int entering_col, int leaving_col,
                                       int leaving_row) {
  if (s.pen_recompute) return;
  ur_compute_update_row(s, leaving_row);
  pen_direction_left_inverse(s);
  pen_update_edge_squared_norms(s, entering_col, leaving_col, leaving_row);
}

// ---- PrimalPrices (reduced_costs.cc:512-600) ----
SD_INLINE f64 pp_price(const Lp& s, int col, const f64* sn) {
  return sq(s.rc[col]) / sn[col];
}
SD_INLINE bool pp_dual_infeasible(const Lp& s, int col, f64 tol) {
  const f64 rc = s.rc[col];
  return ((rc > tol) && bit_get(s.can_dec, col)) != ((rc < -tol) && bit_get(s.can_inc, col));
}
// UpdateEntering candidates over the listed columns (`cols`, n) or, with
// cols == nullptr, over the relevant columns in increasing order
// (from_clean_state: nothing is removed).
SD_INLINE void pp_update_candidates(Lp& s, const int32_t* cols, int n, bool from_clean) {
  const f64 tol = s.dual_tol;
  const f64* sn = pen_get(s);
  rc_get(s);
#if defined(__HIP_DEVICE_COMPILE__)
  // 64 columns at a time: values and candidate bits on the lanes (distinct
  // columns; shared words take atomic or/and), then the columns that can
  // enter the top-k (price >= the threshold at the chunk's start: the
  // threshold never decreases) replay dp_update_top_k in order.
  const int lane = sd_lane();
  const int total = cols != nullptr ? n : s.N;
  for (int base = 0; base < total; base += 64) {
    const int k = base + lane;
    int col = 0;
    bool have = false;
    if (k < total) {
      col = cols != nullptr ? cols[k] : k;
      have = cols != nullptr || bit_get(s.relevant, col);
    }
    f64 price = 0.0;
    bool cand = false;
    if (have) {
      unsigned long long* word = reinterpret_cast<unsigned long long*>(s.pp.cand + (col >> 6));
      const unsigned long long bit = 1ull << (col & 63);
      if (pp_dual_infeasible(s, col, tol)) {
        price = pp_price(s, col, sn);
        s.pp.values[col] = price;
        atomicOr(word, bit);
        cand = price >= s.pp.threshold;
      } else if (!from_clean) {
        atomicAnd(word, ~bit);
      }
    }
    uint64_t mask = __ballot(cand);
    while (mask != 0) {
      const int l = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int c = __shfl(col, l, 64);
      const f64 p = __shfl(price, l, 64);
      if (p >= s.pp.threshold) dp_update_top_k(s, s.pp, c, p);
    }
  }
  sd_sync();
#else
  auto one = [&](int col) {
    if (pp_dual_infeasible(s, col, tol)) {
      dp_add_or_update(s, s.pp, col, pp_price(s, col, sn));
    } else if (!from_clean) {
      dp_remove(s, s.pp, col);
    }
  };
  if (cols != nullptr) {
    for (int k = 0; k < n; ++k) one(cols[k]);
  } else {
    for (int w = 0; w < s.nwords; ++w) {
      uint64_t word = s.relevant[w];
      while (word) {
        const int col = w * 64 + sd_ctz(word);
        word &= word - 1;
        if (col >= s.N) break;
        one(col);
      }
    }
  }
#endif
}
// GetBestEnteringColumn (:534-545)
SD_INLINE int pp_get_best_entering_column(Lp& s) {
  if (s.pp_recompute) {
    rc_get(s);
    dp_clear_and_resize(s, s.pp, s.N);
    pp_update_candidates(s, nullptr, 0, true);
    s.pp_recompute = 0;
  }
  return dp_get_maximum(s, s.pp);
}
// RecomputePriceAt (:556-567)
SD_INLINE void pp_recompute_price_at(Lp& s, int col) {
  if (s.pp_recompute) return;
  if (rc_is_valid_primal_entering(s, col)) {
    const f64* sn = pen_get(s);
    rc_get(s);
    dp_add_or_update(s, s.pp, col, pp_price(s, col, sn));
  } else {
    dp_remove(s, s.pp, col);
  }
}

// ---- VariableValues, primal side (variable_values.cc) ----
SD_INLINE void vv_update_on_pivoting(Lp& s, int entering_col, f64 step) {
  for (int k = sd_lane(); k < s.dir.nnz; k += sd_lanes()) {  // distinct basic columns
    const int row = s.dir.nz[k];
    s.x[s.basis[row]] -= s.dir.values[row] * step;
  }
  sd_sync();
  s.x[entering_col] += step;
}
// ComputeMaximumPrimalResidual (:120-131): A x over every column, in column
// order per row (the row sums of the transpose keep that order), then the
// infinity norm.
SD_INLINE f64 vv_max_primal_residual(Lp& s) {
  f64 err = 0.0;
  for (int r = sd_lane(); r < s.m; r += sd_lanes()) {
    f64 acc = 0.0;
    for (int64_t i = s.At.starts[r]; i < s.At.starts[r + 1]; ++i) {
      const int col = s.At.rows[i];
      const f64 mult = s.x[col];
      if (mult == 0.0) continue;  // ColumnAddMultipleToDenseColumn skips zero multipliers
      acc += mult * s.At.coefs[i];
    }
    err = sd_max(err, sd_fabs(acc));
  }
  return sd_wave_max(err);
}
// ComputeMaximumPrimalInfeasibility (:133-143)
SD_INLINE f64 vv_max_primal_infeasibility(Lp& s) {
  f64 pi = 0.0;
  for (int col = sd_lane(); col < s.N; col += sd_lanes()) {
    pi = sd_max(pi, sd_max(s.x[col] - s.ub[col], s.lb[col] - s.x[col]));
  }
  return sd_wave_max(pi);
}
// UpdatePrimalPhaseICosts (variable_values.h): over the listed rows (or all).
SD_INLINE bool vv_update_phase1_costs(Lp& s, const int32_t* rows, int n) {
  const f64 tol = s.primal_feasibility_tolerance;
  bool changed = false;
  const int total = rows != nullptr ? n : s.m;
  for (int k = sd_lane(); k < total; k += sd_lanes()) {  // distinct basic columns
    const int row = rows != nullptr ? rows[k] : k;
    const int col = s.basis[row];
    f64 cost = 0.0;
    if (s.x[col] - s.ub[col] > tol) {
      cost = 1.0;
    } else if (s.lb[col] - s.x[col] > tol) {
      cost = -1.0;
    }
    if (cost != s.objective[col]) {
      changed = true;
      s.objective[col] = cost;
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  changed = __ballot(changed) != 0;
#endif
  sd_sync();
  return changed;
}

// ---- ratio tests ----
// ChooseLeavingVariableRow (revised_simplex.cc:1829-2003) with
// ComputeHarrisRatioAndLeavingCandidates (:1756-1806). Returns false when
// the caller must refactorize.
SD_INLINE bool sp_harris_ratio(Lp& s, int entering_col, f64 reduced_cost, int* leaving_row,
                               f64* step_length, f64* target_bound) {
  const bool positive = reduced_cost > 0.0;
  const f64 entering_value = s.x[entering_col];
  f64 current_ratio = positive ? entering_value - s.lb[entering_col]
                               : s.ub[entering_col] - entering_value;
  const f64 harris_tolerance = s.harris_tolerance_ratio * s.primal_feasibility_tolerance;
  const f64 minimum_delta = s.degenerate_ministep_factor * s.primal_feasibility_tolerance;
  const f64 threshold =
      s.num_updates == 0 ? s.minimum_acceptable_pivot : s.ratio_test_zero_threshold;
  f64 harris_ratio = current_ratio;
  int nc = 0;
  for (int k = 0; k < s.dir.nnz; ++k) {
    const int row = s.dir.nz[k];
    const f64 direction = s.dir.values[row];
    const f64 magnitude = sd_fabs(direction);
    if (magnitude <= threshold) continue;
    const int col = s.basis[row];
    const f64 value = s.x[col];
    f64 ratio;
    if (positive) {
      ratio = direction > 0.0 ? (s.ub[col] - value) / direction : (s.lb[col] - value) / direction;
    } else {
      ratio = direction > 0.0 ? (value - s.lb[col]) / direction : (value - s.ub[col]) / direction;
    }
    if (ratio <= harris_ratio) {
      s.lc_row[nc] = row;
      s.lc_ratio[nc] = ratio;
      ++nc;
      harris_ratio =
          sd_min(harris_ratio, sd_max(minimum_delta / magnitude, ratio + harris_tolerance / magnitude));
    }
  }
  if (current_ratio <= harris_ratio) {
    *leaving_row = kInvalid;
    *step_length = current_ratio;
    return true;
  }
  f64 pivot_magnitude = 0.0;
  *leaving_row = kInvalid;
  int n_equiv = 0;
  for (int k = 0; k < nc; ++k) {
    const f64 ratio = s.lc_ratio[k];
    if (ratio > harris_ratio) continue;
    const int row = s.lc_row[k];
    const f64 candidate_magnitude = sd_fabs(s.dir.values[row]);
    if (candidate_magnitude < pivot_magnitude) continue;
    if (candidate_magnitude == pivot_magnitude) {
      // IsRatioMoreOrEquallyStable(ratio, current_ratio)
      const bool stable = current_ratio >= 0.0 ? (ratio >= 0.0 && ratio <= current_ratio)
                                               : (ratio >= current_ratio);
      if (!stable) continue;
      if (ratio == current_ratio) {
        s.ent_equiv[n_equiv++] = row;
        continue;
      }
    }
    n_equiv = 0;
    current_ratio = ratio;
    pivot_magnitude = candidate_magnitude;
    *leaving_row = row;
  }
  if (n_equiv != 0) {
    s.ent_equiv[n_equiv++] = *leaving_row;
    *leaving_row = s.ent_equiv[uniform_int(s, n_equiv - 1)];
  }
  *step_length = current_ratio <= 0.0 ? minimum_delta / pivot_magnitude : current_ratio;
  if (pivot_magnitude < s.small_pivot_threshold * s.dir_inf_norm && s.num_updates != 0) {
    return false;
  }
  if (*leaving_row != kInvalid) {
    const bool leaving_coeff_positive = s.dir.values[*leaving_row] > 0.0;
    const int col = s.basis[*leaving_row];
    *target_bound = (positive == leaving_coeff_positive) ? s.ub[col] : s.lb[col];
  }
  return true;
}
// BreakPoint order (revised_simplex.cc:2010-2035): the heap's top is the
// smallest ratio, then the largest magnitude, then the smallest row.
SD_INLINE bool bp1_less(const Lp& s, int a, int b) {
  if (s.bp1_ratio[a] == s.bp1_ratio[b]) {
    if (s.bp1_mag[a] == s.bp1_mag[b]) return s.bp1_row[a] > s.bp1_row[b];
    return s.bp1_mag[a] < s.bp1_mag[b];
  }
  return s.bp1_ratio[a] > s.bp1_ratio[b];
}
SD_INLINE void bp1_move(Lp& s, int dst, int src) {
  s.bp1_row[dst] = s.bp1_row[src];
  s.bp1_ratio[dst] = s.bp1_ratio[src];
  s.bp1_mag[dst] = s.bp1_mag[src];
  s.bp1_target[dst] = s.bp1_target[src];
}
// libstdc++ __push_heap / __adjust_heap with the element held in slot `tmp`.
SD_INLINE void bp1_push_heap(Lp& s, int hole, int top, int tmp) {
  int parent = (hole - 1) / 2;
  while (hole > top && bp1_less(s, parent, tmp)) {
    bp1_move(s, hole, parent);
    hole = parent;
    parent = (hole - 1) / 2;
  }
  bp1_move(s, hole, tmp);
}
SD_INLINE void bp1_adjust_heap(Lp& s, int hole, int len, int tmp) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (bp1_less(s, second, second - 1)) second--;
    bp1_move(s, hole, second);
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    bp1_move(s, hole, second - 1);
    hole = second - 1;
  }
  bp1_push_heap(s, hole, top, tmp);
}
// PrimalPhaseIChooseLeavingVariableRow (revised_simplex.cc:2039-2145).
// Returns false when the caller must refactorize.
SD_INLINE bool sp_phase1_ratio(Lp& s, int entering_col, f64 reduced_cost, int* leaving_row,
                               f64* step_length, f64* target_bound) {
  const f64 entering_value = s.x[entering_col];
  f64 current_ratio = (reduced_cost > 0.0) ? entering_value - s.lb[entering_col]
                                           : s.ub[entering_col] - entering_value;
  const f64 tolerance = s.primal_feasibility_tolerance;
  const int tmp = 2 * s.m + 1;  // the heap's spare slot
  int len = 0;
  for (int k = 0; k < s.dir.nnz; ++k) {
    const int row = s.dir.nz[k];
    const f64 direction = reduced_cost > 0.0 ? s.dir.values[row] : -s.dir.values[row];
    const f64 magnitude = sd_fabs(direction);
    if (magnitude < tolerance) continue;
    const int col = s.basis[row];
    const f64 value = s.x[col];
    const f64 lower_bound = s.lb[col];
    const f64 upper_bound = s.ub[col];
    const f64 to_lower = (lower_bound - tolerance - value) / direction;
    const f64 to_upper = (upper_bound + tolerance - value) / direction;
    if (to_lower >= 0.0 && to_lower < current_ratio) {
      s.bp1_row[len] = row;
      s.bp1_ratio[len] = to_lower;
      s.bp1_mag[len] = magnitude;
      s.bp1_target[len] = lower_bound;
      ++len;
    }
    if (to_upper >= 0.0 && to_upper < current_ratio) {
      s.bp1_row[len] = row;
      s.bp1_ratio[len] = to_upper;
      s.bp1_mag[len] = magnitude;
      s.bp1_target[len] = upper_bound;
      ++len;
    }
  }
  // std::make_heap
  if (len >= 2) {
    int parent = (len - 2) / 2;
    while (true) {
      bp1_move(s, tmp, parent);
      bp1_adjust_heap(s, parent, len, tmp);
      if (parent == 0) break;
      parent--;
    }
  }
  f64 improvement = sd_fabs(reduced_cost);
  f64 best_magnitude = 0.0;
  *leaving_row = kInvalid;
  while (len > 0) {
    if (s.bp1_mag[0] > best_magnitude) {
      *leaving_row = s.bp1_row[0];
      current_ratio = s.bp1_ratio[0];
      best_magnitude = s.bp1_mag[0];
      *target_bound = s.bp1_target[0];
    }
    improvement -= s.bp1_mag[0];
    if (improvement <= 0.0) break;
    // std::pop_heap then pop_back
    if (len > 1) {
      bp1_move(s, tmp, len - 1);
      bp1_move(s, len - 1, 0);
      bp1_adjust_heap(s, 0, len - 1, tmp);
    }
    --len;
  }
  if (*leaving_row != kInvalid) {
    const f64 threshold = s.small_pivot_threshold * s.dir_inf_norm;
    if (best_magnitude < threshold && s.num_updates != 0) return false;
  }
  *step_length = current_ratio;
  return true;
}

// The primal phase-I / phase-II loop (revised_simplex.cc:2751-3045), entered
// after the loop-top block. Phases as sd_run: 0 loop top, 1 entering column,
// 5 FTRAN, 4 ratio test, 6 norms / rc / prices, 7 pivot, 8 factorization.
SD_INLINE int32_t sp_run(Lp& s) {
  s.exit_code = kExitNone;
  s.iterations_done = 0;
  bool at_top = false;
  uint64_t mark_ = sd_now();
  int phase_ = 0;
  struct Flush {
    Lp& s;
    uint64_t& mark;
    int& phase;
    SD_HD ~Flush() { s.phase_ticks[phase] += sd_now() - mark; }
  } flush_{s, mark_, phase_};
  while (true) {
    SD_PHASE(0);
    if (at_top) {
      if ((s.iteration_cap > 0 && s.iterations_done >= s.iteration_cap) ||
          !sd_room_for_iteration(s)) {
        return s.exit_code = kExitLoopTop;
      }
      if (!s.refactorize && s.must_refactorize) s.refactorize = 1;
      if (!s.refactorize && s.pen_recompute) s.refactorize = 1;
      // RefactorizeBasisIfNeeded
      if (s.refactorize && s.num_updates != 0) {
        SD_PHASE(8);
        const int st = sd_refactorize(s, 0);
        SD_PHASE(0);
        if (st == 1) return s.exit_code = kExitLuError;
        if (st == 2) {
          s.refactorize = 0;
          return s.exit_code = kExitResumeTop;
        }
        ur_invalidate(s);
        rs_permute_basis(s);
      }
      s.refactorize = 0;
      if (s.num_updates == 0) {
        SdSubTimer t_x_(&s.phase_ticks[20]);
        // CorrectErrorsOnVariableValues
        if (vv_max_primal_residual(s) >= s.harris_tolerance_ratio * s.primal_feasibility_tolerance) {
          vv_recompute_basic_values(s);
        }
        if (s.phase_feasibility && vv_update_phase1_costs(s, nullptr, 0)) {
          rc_reset_for_new_objective(s);
        }
        if (!s.phase_feasibility && rs_objective_value(s) < s.primal_objective_limit) {
          s.objective_limit_reached = 1;
          return s.exit_code = kExitObjectiveLimit;
        }
      } else if (s.phase_feasibility) {
        if (vv_update_phase1_costs(s, s.dir.nz, s.dir.nnz)) rc_reset_for_new_objective(s);
      }
    }
    at_top = true;
    SD_PHASE(1);
    const int entering_col = pp_get_best_entering_column(s);
    if (entering_col == kInvalid) {
      if (s.rc_precise && s.num_updates == 0) {
        if (s.phase_feasibility) {
          s.exit_status = vv_max_primal_infeasibility(s) < s.primal_feasibility_tolerance
                              ? kStPrimalFeasible
                              : kStPrimalInfeasible;
        } else {
          s.exit_status = kStOptimal;
        }
        return s.exit_code = kExitStatus;
      }
      rc_make_precise(s);
      s.refactorize = 1;
      continue;
    }
    SD_PHASE(5);
    rs_compute_direction(s, entering_col);
    if (!pen_test_entering_precision(s, entering_col)) {
      pp_recompute_price_at(s, entering_col);
      continue;
    }
    const f64 reduced_cost = rc_test_entering_precision(s, entering_col);
    pp_recompute_price_at(s, entering_col);
    if (!rc_is_valid_primal_entering(s, entering_col)) {
      rc_make_precise(s);
      continue;
    }
    rs_advance_deterministic_time(s);
    if (s.num_iterations == s.max_number_of_iterations || s.tl_det_elapsed > s.tl_det_max) {
      return s.exit_code = kExitReturnOk;
    }
    SD_PHASE(4);
    f64 step_length = 0.0;
    int leaving_row = kInvalid;
    f64 target_bound = 0.0;
    const bool ok = s.phase_feasibility
                        ? sp_phase1_ratio(s, entering_col, reduced_cost, &leaving_row,
                                          &step_length, &target_bound)
                        : sp_harris_ratio(s, entering_col, reduced_cost, &leaving_row,
                                          &step_length, &target_bound);
    if (!ok) {
      s.refactorize = 1;
      continue;
    }
    if (step_length == sd_inf() || step_length == -sd_inf()) {
      if (s.num_updates != 0 || !s.rc_precise) {
        rc_make_precise(s);
        s.refactorize = 1;
        continue;
      }
      s.exit_entering = entering_col;
      s.exit_reduced_cost = reduced_cost;
      return s.exit_code = kExitUnbounded;
    }
    f64 step = (reduced_cost > 0.0) ? -step_length : step_length;
    if (s.phase_feasibility && leaving_row != kInvalid) {
      step = (s.x[s.basis[leaving_row]] - target_bound) / s.dir.values[leaving_row];
    }
    const int leaving_col = leaving_row == kInvalid ? kInvalid : s.basis[leaving_row];
    bool is_degenerate = false;
    if (leaving_row != kInvalid) {
      const f64 dir = -s.dir.values[leaving_row] * step;
      is_degenerate = (dir == 0.0) || (dir > 0.0 && s.x[leaving_col] >= target_bound) ||
                      (dir < 0.0 && s.x[leaving_col] <= target_bound);
    }
    SD_PHASE(7);
    {
      SdSubTimer t_x_(&s.phase_ticks[25]);
      vv_update_on_pivoting(s, entering_col, step);
    }
    if (leaving_row != kInvalid) {
      SD_PHASE(6);
      pen_update_before_pivot(s, entering_col, leaving_col, leaving_row);
      rc_update_before_pivot(s, entering_col, leaving_row);
      if (!s.pp_recompute) pp_update_candidates(s, s.nzpos, s.n_nzpos, false);
      SD_PHASE(7);
      if (!is_degenerate) s.x[leaving_col] = target_bound;
      int refactor = 0;
      if (sd_pivot(s, entering_col, leaving_row, target_bound, &refactor) != kExitNone) {
        return s.exit_code = kExitLuError;
      }
      if (refactor != 0) {
        SD_PHASE(8);
        const int st = sd_refactorize(s, refactor == 2 ? 1 : 0);
        if (st == 1) return s.exit_code = kExitLuError;
        if (st == 2) return s.exit_code = kExitResumePivot;
        rs_permute_basis(s);  // IsRefactorized() holds after a factorization
      }
    } else {
      if (step > 0.0) {
        vi_to_nonbasic(s, entering_col, kAtUpper);
        vv_set_nonbasic_from_status(s, entering_col);
      } else if (step < 0.0) {
        vi_to_nonbasic(s, entering_col, kAtLower);
        vv_set_nonbasic_from_status(s, entering_col);
      }
      if (!s.pp_recompute) dp_remove(s, s.pp, entering_col);
    }
    if (s.phase_feasibility && leaving_row != kInvalid) {
      vv_set_nonbasic_from_status(s, leaving_col);
      rc_set_nonbasic_cost_to_zero(s, leaving_col);
      pp_recompute_price_at(s, leaving_col);
    }
#if !defined(__HIP_DEVICE_COMPILE__)
    if (s.trace != nullptr) s.trace(&s);
#endif
    ++s.num_iterations;  // OnIterationDone
    ++s.iterations_done;
  }
}

}  // namespace sdual

#endif  // MILP_SPRIMAL_CORE_H_
