// LPSolver layer of the Glop drop-in: what glop::LPSolver does around
// RevisedSimplex::Solve (ortools/glop/lp_solver.cc:150-262) for the
// MPSolver path (linear_solver/glop_interface.cc:104-169):
//
//   validity checks (lp_solver.cc:185-202)
//   -> ScalingPreprocessor::Run (preprocessor.cc:3855-3876):
//        SparseMatrixScaler::Scale (lp_data/matrix_scaler.cc: geometric
//        passes + equilibration), ScaleObjective, ScaleBounds (lp_data.cc:
//        1178-1258)
//   -> the MI355X engine (mi_lp_load / mi_lp_solve on the caller's handle)
//   -> ScalingPreprocessor::RecoverSolution (preprocessor.cc:3878-3912)
//   -> LoadAndVerifySolution's value part (lp_solver.cc:334-367):
//        reduced costs c - y.A_j, Kahan objective, strong-optimal moves of
//        primal and dual values into their bounds, constraint activities.
//
// Host code only: the scaling is O(nnz) once per solve and runs before the
// LP reaches HBM. The arithmetic follows the cited loops one operation at a
// time, so the LP the engine receives is the one Glop's simplex would see
// with presolve off and scaling on (use_preprocessing = false).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <exception>
#include <limits>
#include <string>
#include <vector>

#include "../../../include/mi_lp.h"

namespace milp {
namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

// The LP as LPSolver holds it (LinearProgram fields touched by the scaling).
struct ScaledLp {
  int32_t m = 0, n = 0;
  std::vector<int64_t> starts;
  std::vector<int32_t> rows;
  std::vector<double> vals;
  std::vector<double> col_lb, col_ub, row_lb, row_ub, obj;
  double offset = 0.0, scale = 1.0;
};

// SparseMatrixScaler (lp_data/matrix_scaler.h:79-111, matrix_scaler.cc).
// row_scale / col_scale are the "unscaling" factors: A' = R^-1 A C^-1.
struct MatrixScaler {
  std::vector<double> row_scale, col_scale;
  ScaledLp* lp = nullptr;

  void Init(ScaledLp* p) {
    lp = p;
    row_scale.assign(p->m, 1.0);
    col_scale.assign(p->n, 1.0);
  }

  // SparseMatrix::ComputeMinAndMaxMagnitudes (sparse.cc:375-393).
  void MinMax(double* mn, double* mx) const {
    *mn = kInf;
    *mx = 0.0;
    for (double v : lp->vals) {
      const double a = std::fabs(v);
      if (a != 0.0) {
        *mn = std::min(*mn, a);
        *mx = std::max(*mx, a);
      }
    }
    if (*mx == 0.0) *mn = 0.0;
  }

  // matrix_scaler.cc VarianceOfAbsoluteValueOfNonZeros: column order.
  double Variance() const {
    double sq = 0.0, ab = 0.0, cnt = 0.0;
    for (double v : lp->vals) {
      const double a = std::fabs(v);
      if (a != 0.0) {
        sq += a * a;
        ab += a;
        ++cnt;
      }
    }
    if (cnt == 0.0) return 0.0;
    return (sq - ab * ab / cnt) / cnt;
  }

  // ScaleMatrixRows: counts factors != 1, then divides every entry by its
  // row's factor (SparseColumn::ComponentWiseDivide, sparse_vector.h:793-798).
  int ScaleRows(const std::vector<double>& f) {
    int scaled = 0;
    for (int r = 0; r < lp->m; ++r) {
      if (f[r] != 1.0) {
        ++scaled;
        row_scale[r] *= f[r];
      }
    }
    const int64_t nnz = lp->starts[lp->n];
    for (int64_t k = 0; k < nnz; ++k) lp->vals[k] /= f[lp->rows[k]];
    return scaled;
  }

  // ScaleMatrixColumn: DivideByConstant (sparse_vector.h:785-790).
  void ScaleColumn(int c, double f) {
    col_scale[c] *= f;
    for (int64_t k = lp->starts[c]; k < lp->starts[c + 1]; ++k) lp->vals[k] /= f;
  }

  int ScaleRowsGeometrically() {
    std::vector<double> mx(lp->m, 0.0), mn(lp->m, kInf);
    const int64_t nnz = lp->starts[lp->n];
    for (int64_t k = 0; k < nnz; ++k) {
      const double a = std::fabs(lp->vals[k]);
      const int r = lp->rows[k];
      if (a != 0.0) {
        mx[r] = std::max(mx[r], a);
        mn[r] = std::min(mn[r], a);
      }
    }
    std::vector<double> f(lp->m, 0.0);
    for (int r = 0; r < lp->m; ++r) f[r] = mx[r] == 0.0 ? 1.0 : std::sqrt(mx[r] * mn[r]);
    return ScaleRows(f);
  }

  int ScaleColumnsGeometrically() {
    int scaled = 0;
    for (int c = 0; c < lp->n; ++c) {
      double mx = 0.0, mn = kInf;
      for (int64_t k = lp->starts[c]; k < lp->starts[c + 1]; ++k) {
        const double a = std::fabs(lp->vals[k]);
        if (a != 0.0) {
          mx = std::max(mx, a);
          mn = std::min(mn, a);
        }
      }
      if (mx != 0.0) {
        ScaleColumn(c, std::sqrt(mx * mn));
        ++scaled;
      }
    }
    return scaled;
  }

  int EquilibrateRows() {
    std::vector<double> mx(lp->m, 0.0);
    const int64_t nnz = lp->starts[lp->n];
    for (int64_t k = 0; k < nnz; ++k) {
      const double a = std::fabs(lp->vals[k]);
      if (a != 0.0) mx[lp->rows[k]] = std::max(mx[lp->rows[k]], a);
    }
    for (int r = 0; r < lp->m; ++r) {
      if (mx[r] == 0.0) mx[r] = 1.0;
    }
    return ScaleRows(mx);
  }

  int EquilibrateColumns() {
    int scaled = 0;
    for (int c = 0; c < lp->n; ++c) {
      double mx = 0.0;  // InfinityNorm (lp_utils.cc:103-109)
      for (int64_t k = lp->starts[c]; k < lp->starts[c + 1]; ++k) {
        mx = std::max(mx, std::fabs(lp->vals[k]));
      }
      if (mx != 0.0) {
        ScaleColumn(c, mx);
        ++scaled;
      }
    }
    return scaled;
  }

  // SparseMatrixScaler::Scale (matrix_scaler.cc). LINEAR_PROGRAM scaling
  // (an auxiliary LP solved by Glop) is not restated; like upstream when
  // that LP fails, it falls through to the geometric + equilibration path.
  void Scale() {
    double mn, mx;
    MinMax(&mn, &mx);
    if (mn == 0.0) return;  // null matrix
    if (mx / mn < 1e20) {   // kMaxDynamicRangeForGeometricScaling
      for (int it = 0; it < 4; ++it) {  // kScalingIterations
        const int rows = ScaleRowsGeometrically();
        const int cols = ScaleColumnsGeometrically();
        if (Variance() < 10.0 || (cols == 0 && rows == 0)) break;
      }
    }
    EquilibrateRows();
    EquilibrateColumns();
  }
};

// lp_data.cc:1144-1153.
void UpdateMinMax(const std::vector<double>& v, double* mn, double* mx) {
  for (double x : v) {
    const double a = std::fabs(x);
    if (a == 0 || a == kInf) continue;
    *mn = std::min(*mn, a);
    *mx = std::max(*mx, a);
  }
}

// lp_data.cc:1178-1186.
double DivisorSoThatRangeContainsOne(double mn, double mx) {
  if (mn > 1.0 && mn < kInf) return mn;
  if (mx > 0.0 && mx < 1.0) return mx;
  return 1.0;
}

// LinearProgram::ScaleObjective (lp_data.cc:1190-1223).
double ScaleObjective(ScaledLp* lp, int method) {
  double mn = kInf, mx = 0.0;
  UpdateMinMax(lp->obj, &mn, &mx);
  double f = 1.0;
  switch (method) {
    case MI_LP_NO_COST_SCALING:
      break;
    case MI_LP_CONTAIN_ONE_COST_SCALING:
      f = DivisorSoThatRangeContainsOne(mn, mx);
      break;
    case MI_LP_MEAN_COST_SCALING: {  // GetMeanScalingFactor (lp_data.cc:1166-1176)
      double mean = 0.0;
      int count = 0;
      for (double v : lp->obj) {
        if (v == 0.0) continue;
        ++count;
        mean += std::fabs(v);
      }
      f = count == 0 ? 1.0 : mean / static_cast<double>(count);
      break;
    }
    case MI_LP_MEDIAN_COST_SCALING: {  // GetMedianScalingFactor (lp_data.cc:1155-1164)
      std::vector<double> med;
      for (double v : lp->obj) {
        if (v != 0.0) med.push_back(std::fabs(v));
      }
      if (!med.empty()) {
        std::sort(med.begin(), med.end());
        f = med[med.size() / 2];
      }
      break;
    }
    default:
      break;
  }
  if (f != 1.0) {
    for (double& c : lp->obj) {
      if (c == 0.0) continue;
      c = c / f;
    }
    lp->scale = lp->scale * f;
    lp->offset = lp->offset / f;
  }
  return f;
}

// LinearProgram::ScaleBounds (lp_data.cc:1225-1258).
double ScaleBounds(ScaledLp* lp) {
  double mn = kInf, mx = 0.0;
  UpdateMinMax(lp->col_lb, &mn, &mx);
  UpdateMinMax(lp->col_ub, &mn, &mx);
  UpdateMinMax(lp->row_lb, &mn, &mx);
  UpdateMinMax(lp->row_ub, &mn, &mx);
  const double f = DivisorSoThatRangeContainsOne(mn, mx);
  if (f != 1.0) {
    lp->scale = lp->scale * f;
    lp->offset = lp->offset / f;
    for (int c = 0; c < lp->n; ++c) {
      lp->col_lb[c] = lp->col_lb[c] / f;
      lp->col_ub[c] = lp->col_ub[c] / f;
    }
    for (int r = 0; r < lp->m; ++r) {
      lp->row_lb[r] = lp->row_lb[r] / f;
      lp->row_ub[r] = lp->row_ub[r] / f;
    }
  }
  return f;
}

// lp_data_utils.cc Scale(): matrix, then c /= C, bounds *= C, rows /= R.
void ScaleLp(ScaledLp* lp, MatrixScaler* s) {
  s->Init(lp);
  s->Scale();
  for (int c = 0; c < lp->n; ++c) lp->obj[c] /= s->col_scale[c];
  for (int c = 0; c < lp->n; ++c) lp->col_ub[c] *= s->col_scale[c];
  for (int c = 0; c < lp->n; ++c) lp->col_lb[c] *= s->col_scale[c];
  for (int r = 0; r < lp->m; ++r) lp->row_ub[r] /= s->row_scale[r];
  for (int r = 0; r < lp->m; ++r) lp->row_lb[r] /= s->row_scale[r];
}

// base/accurate_sum.h AccurateSum::Add.
struct KahanSum {
  double sum = 0.0, err = 0.0;
  void Add(double v) {
    err += v;
    const double t = sum + err;
    err += sum - t;
    sum = t;
  }
};

// LinearProgram::IsValid (lp_data.cc:1307-1345) with AreBoundsValid
// (lp_data.h:697-704), as LPSolver checks it (lp_solver.cc:193-199).
bool IsValid(const ScaledLp& lp, double max_magnitude) {
  auto ok_value = [&](double v) { return std::isfinite(v) && std::fabs(v) <= max_magnitude; };
  if (!ok_value(lp.offset)) return false;
  if (!ok_value(lp.scale) || lp.scale == 0.0) return false;
  auto ok_bounds = [&](double lb, double ub) {
    if (std::isnan(lb) || std::isnan(ub)) return false;
    if (lb == kInf && ub == kInf) return false;
    if (lb == -kInf && ub == -kInf) return false;
    if (lb > ub) return false;
    if (std::isfinite(lb) && std::fabs(lb) > max_magnitude) return false;
    if (std::isfinite(ub) && std::fabs(ub) > max_magnitude) return false;
    return true;
  };
  for (int c = 0; c < lp.n; ++c) {
    if (!ok_bounds(lp.col_lb[c], lp.col_ub[c])) return false;
    if (!ok_value(lp.obj[c])) return false;
  }
  for (double v : lp.vals) {
    if (!ok_value(v)) return false;
  }
  for (int r = 0; r < lp.m; ++r) {
    if (!ok_bounds(lp.row_lb[r], lp.row_ub[r])) return false;
  }
  return true;
}

}  // namespace
}  // namespace milp

extern "C" {

void mi_lp_solver_params_default(mi_lp_solver_params* p) {
  if (p == nullptr) return;
  std::memset(p, 0, sizeof(*p));
  p->use_scaling = 1;                       // parameters.proto:187
  p->scaling_method = MI_LP_EQUILIBRATION;  // :95
  p->cost_scaling = MI_LP_CONTAIN_ONE_COST_SCALING;  // :209-210
  p->provide_strong_optimal_guarantee = 1;  // :271
  p->max_valid_magnitude = 1e30;            // max_valid_magnitude default
}

}  // extern "C"

namespace {
// mi_lp_load's argument rule: every array an LP of this shape reads is given.
bool LpArraysPresent(int32_t m, int32_t n, const int64_t* cs, const int32_t* ri,
                     const double* vals, const double* clb, const double* cub, const double* rlb,
                     const double* rub, const double* obj) {
  if (cs[n] > 0 && (ri == nullptr || vals == nullptr)) return false;
  if (n > 0 && (clb == nullptr || cub == nullptr || obj == nullptr)) return false;
  if (m > 0 && (rlb == nullptr || rub == nullptr)) return false;
  return true;
}
}  // namespace

extern "C" {

int mi_lp_scale(const mi_lp_solver_params* sp, int32_t m, int32_t n, const int64_t* cs,
                const int32_t* ri, double* vals, double* clb, double* cub, double* rlb,
                double* rub, double* obj, double* obj_offset, double* obj_scale,
                double* row_scale, double* col_scale, double* cost_factor,
                double* bound_factor) {
  if (sp == nullptr || cs == nullptr || obj_offset == nullptr || obj_scale == nullptr ||
      cost_factor == nullptr || bound_factor == nullptr) {
    return MI_LP_ERROR_NULL;
  }
  if (m < 0 || n < 0 || cs[0] != 0 || cs[n] < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  if (!LpArraysPresent(m, n, cs, ri, vals, clb, cub, rlb, rub, obj)) return MI_LP_ERROR_NULL;
  try {
    milp::ScaledLp lp;
    lp.m = m;
    lp.n = n;
    lp.starts.assign(cs, cs + n + 1);
    lp.rows.assign(ri, ri + cs[n]);
    for (int32_t r : lp.rows) {
      if (r < 0 || r >= m) return MI_LP_ERROR_INVALID_PROBLEM;
    }
    lp.vals.assign(vals, vals + cs[n]);
    lp.col_lb.assign(clb, clb + n);
    lp.col_ub.assign(cub, cub + n);
    lp.row_lb.assign(rlb, rlb + m);
    lp.row_ub.assign(rub, rub + m);
    lp.obj.assign(obj, obj + n);
    lp.offset = *obj_offset;
    lp.scale = *obj_scale;
    milp::MatrixScaler scaler;
    scaler.Init(&lp);
    *cost_factor = 1.0;
    *bound_factor = 1.0;
    if (sp->use_scaling) {
      milp::ScaleLp(&lp, &scaler);
      *cost_factor = milp::ScaleObjective(&lp, sp->cost_scaling);
      *bound_factor = milp::ScaleBounds(&lp);
    }
    std::copy(lp.vals.begin(), lp.vals.end(), vals);
    std::copy(lp.col_lb.begin(), lp.col_lb.end(), clb);
    std::copy(lp.col_ub.begin(), lp.col_ub.end(), cub);
    std::copy(lp.row_lb.begin(), lp.row_lb.end(), rlb);
    std::copy(lp.row_ub.begin(), lp.row_ub.end(), rub);
    std::copy(lp.obj.begin(), lp.obj.end(), obj);
    *obj_offset = lp.offset;
    *obj_scale = lp.scale;
    if (row_scale != nullptr) std::copy(scaler.row_scale.begin(), scaler.row_scale.end(), row_scale);
    if (col_scale != nullptr) std::copy(scaler.col_scale.begin(), scaler.col_scale.end(), col_scale);
    return MI_LP_OK;
  } catch (const std::exception&) {
    return MI_LP_ERROR_INTERNAL;
  }
}

int mi_lp_solver_solve(mi_lp* h, const mi_lp_solver_params* sp, int32_t m, int32_t n,
                       const int64_t* cs, const int32_t* ri, const double* vals,
                       const double* clb, const double* cub, const double* rlb,
                       const double* rub, const double* obj, double obj_offset,
                       double obj_scale, int32_t maximize, const volatile int32_t* interrupt,
                       mi_lp_result* out, double* primal, double* duals, double* rc,
                       double* act, int8_t* vstat, int8_t* cstat) {
  using milp::ScaledLp;
  if (h == nullptr || sp == nullptr || out == nullptr || cs == nullptr) return MI_LP_ERROR_NULL;
  if (m < 0 || n < 0 || cs[0] != 0 || cs[n] < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  if (!LpArraysPresent(m, n, cs, ri, vals, clb, cub, rlb, rub, obj)) return MI_LP_ERROR_NULL;
  std::memset(out, 0, sizeof(*out));
  try {
    const ScaledLp orig = [&] {
      ScaledLp lp;
      lp.m = m;
      lp.n = n;
      lp.starts.assign(cs, cs + n + 1);
      lp.rows.assign(ri, ri + cs[n]);
      lp.vals.assign(vals, vals + cs[n]);
      lp.col_lb.assign(clb, clb + n);
      lp.col_ub.assign(cub, cub + n);
      lp.row_lb.assign(rlb, rlb + m);
      lp.row_ub.assign(rub, rub + m);
      lp.obj.assign(obj, obj + n);
      lp.offset = obj_offset;
      lp.scale = obj_scale;
      return lp;
    }();
    // IsCleanedUp (lp_solver.cc:185-191): rows strictly increasing per
    // column, no explicit zeros, rows in range.
    for (int c = 0; c < n; ++c) {
      if (orig.starts[c + 1] < orig.starts[c]) return MI_LP_ERROR_INVALID_PROBLEM;
      for (int64_t k = orig.starts[c]; k < orig.starts[c + 1]; ++k) {
        const int r = orig.rows[k];
        if (r < 0 || r >= m || orig.vals[k] == 0.0) return MI_LP_ERROR_INVALID_PROBLEM;
        if (k > orig.starts[c] && orig.rows[k - 1] >= r) return MI_LP_ERROR_INVALID_PROBLEM;
      }
    }
    if (!milp::IsValid(orig, sp->max_valid_magnitude)) {
      out->problem_status = MI_LP_INVALID_PROBLEM;
      return MI_LP_OK;
    }
    ScaledLp lp = orig;
    milp::MatrixScaler scaler;
    double cost_factor = 1.0, bound_factor = 1.0;
    if (sp->use_scaling) {
      milp::ScaleLp(&lp, &scaler);
      cost_factor = milp::ScaleObjective(&lp, sp->cost_scaling);
      bound_factor = milp::ScaleBounds(&lp);
    }
    int rc_load = mi_lp_load(h, m, n, lp.starts.data(), lp.rows.data(), lp.vals.data(),
                             lp.col_lb.data(), lp.col_ub.data(), lp.row_lb.data(),
                             lp.row_ub.data(), lp.obj.data(), lp.offset, lp.scale, maximize);
    if (rc_load != MI_LP_OK) return rc_load;
    mi_lp_result r;
    const int rc_solve = mi_lp_solve(h, interrupt, &r);
    if (rc_solve != MI_LP_OK) return rc_solve;
    *out = r;
    std::vector<double> x(n), y(m);
    std::vector<int8_t> vs(n), cstats(m);
    if (r.error_code != MI_LP_OK) return MI_LP_OK;
    mi_lp_get_primal(h, x.data());
    mi_lp_get_duals(h, y.data());
    mi_lp_get_statuses(h, vs.data(), cstats.data());
    // ScalingPreprocessor::RecoverSolution (preprocessor.cc:3878-3912).
    if (sp->use_scaling) {
      for (int c = 0; c < n; ++c) x[c] /= scaler.col_scale[c];
      for (int c = 0; c < n; ++c) x[c] *= bound_factor;
      for (int row = 0; row < m; ++row) y[row] /= scaler.row_scale[row];
      for (int row = 0; row < m; ++row) y[row] *= cost_factor;
      for (int c = 0; c < n; ++c) {
        switch (vs[c]) {
          case MI_LP_AT_UPPER_BOUND:
          case MI_LP_FIXED_VALUE:
            x[c] = orig.col_ub[c];
            break;
          case MI_LP_AT_LOWER_BOUND:
            x[c] = orig.col_lb[c];
            break;
          default:
            break;
        }
      }
    }
    // LoadAndVerifySolution (lp_solver.cc:334-367), value part.
    const bool strong = sp->provide_strong_optimal_guarantee && r.problem_status == MI_LP_OPTIMAL;
    if (strong) {
      for (int c = 0; c < n; ++c) {  // MovePrimalValuesWithinBounds (:540-555)
        x[c] = std::min(x[c], orig.col_ub[c]);
        x[c] = std::max(x[c], orig.col_lb[c]);
      }
      const double sign = maximize ? -1.0 : 1.0;  // MoveDualValuesWithinBounds (:557-579)
      for (int row = 0; row < m; ++row) {
        double d = sign * y[row];
        if (orig.row_lb[row] == -milp::kInf && d > 0.0) d = 0.0;
        if (orig.row_ub[row] == milp::kInf && d < 0.0) d = 0.0;
        y[row] = sign * d;
      }
    }
    milp::KahanSum sum;  // ComputeObjective (:888-896)
    for (int c = 0; c < n; ++c) sum.Add(orig.obj[c] * x[c]);
    out->objective = orig.scale * (sum.sum + orig.offset);  // ProblemObjectiveValue (:306-308)
    if (rc != nullptr) {  // ComputeReducedCosts (:877-886)
      for (int c = 0; c < n; ++c) {
        double dot = 0.0;
        for (int64_t k = orig.starts[c]; k < orig.starts[c + 1]; ++k) {
          dot += y[orig.rows[k]] * orig.vals[k];
        }
        rc[c] = orig.obj[c] - dot;
      }
    }
    if (act != nullptr) {  // ComputeConstraintActivities (:866-875)
      std::fill(act, act + m, 0.0);
      for (int c = 0; c < n; ++c) {
        if (x[c] == 0.0) continue;
        for (int64_t k = orig.starts[c]; k < orig.starts[c + 1]; ++k) {
          act[orig.rows[k]] += x[c] * orig.vals[k];
        }
      }
    }
    if (primal != nullptr) std::copy(x.begin(), x.end(), primal);
    if (duals != nullptr) std::copy(y.begin(), y.end(), duals);
    if (vstat != nullptr) std::copy(vs.begin(), vs.end(), vstat);
    if (cstat != nullptr) std::copy(cstats.begin(), cstats.end(), cstat);
    return MI_LP_OK;
  } catch (const std::exception&) {
    return MI_LP_ERROR_INTERNAL;
  }
}

}  // extern "C"
