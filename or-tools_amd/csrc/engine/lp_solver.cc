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
#include <memory>
#include <string>
#include <vector>

#include "../../../include/mi_lp.h"
#include "presolve.h"

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

// LPSolver::IsProblemSolutionConsistent (lp_solver.cc:679-790).
bool IsSolutionConsistent(const ScaledLp& lp, const presolve::Solution& s) {
  // The size checks come first (:683-686): a postsolve or a caller-supplied
  // simplex that returned a wrong-sized solution is ABNORMAL, never indexed.
  const size_t n = static_cast<size_t>(lp.n), m = static_cast<size_t>(lp.m);
  if (s.vstat.size() != n || s.cstat.size() != m) return false;
  if (s.primal.size() != n || s.dual.size() != m) return false;
  if (s.status != MI_LP_OPTIMAL && s.status != MI_LP_PRIMAL_FEASIBLE &&
      s.status != MI_LP_DUAL_FEASIBLE) {
    return true;
  }
  auto within = [](double x, double y, double tol) {  // AreWithinAbsoluteTolerance
    if (std::isinf(x) || std::isinf(y)) return x == y;
    return std::fabs(x - y) <= tol;
  };
  int64_t num_basic = 0;
  for (int c = 0; c < lp.n; ++c) {
    const double value = s.primal[c];
    const double lb = lp.col_lb[c];
    const double ub = lp.col_ub[c];
    switch (s.vstat[c]) {
      case MI_LP_BASIC:
        ++num_basic;
        break;
      case MI_LP_FIXED_VALUE:
        if (value != ub && value != lb) return false;
        break;
      case MI_LP_AT_LOWER_BOUND:
        if (value != lb || lb == ub) return false;
        break;
      case MI_LP_AT_UPPER_BOUND:
        if (!within(value, ub, 1e-7) || lb == ub) return false;
        break;
      case MI_LP_FREE:
        if (lb != -kInf || ub != kInf || value != 0.0) return false;
        break;
      default:
        return false;
    }
  }
  for (int r = 0; r < lp.m; ++r) {
    const double dual = s.dual[r];
    const double lb = lp.row_lb[r];
    const double ub = lp.row_ub[r];
    switch (s.cstat[r]) {
      case MI_LP_BASIC:
        if (dual != 0.0) return false;
        ++num_basic;
        break;
      case MI_LP_FIXED_VALUE:
        if (ub - lb > 1e-12) return false;
        break;
      case MI_LP_AT_LOWER_BOUND:
        if (lb == -kInf) return false;
        break;
      case MI_LP_AT_UPPER_BOUND:
        if (ub == kInf) return false;
        break;
      case MI_LP_FREE:
        if (dual != 0.0) return false;
        if (lb != -kInf || ub != kInf) return false;
        break;
      default:
        return false;
    }
  }
  return num_basic == lp.m;
}

presolve::Params PresolveParamsOf(const mi_lp_solver_params& sp) {
  presolve::Params p;
  p.use_preprocessing = sp.use_preprocessing != 0;
  p.use_implied_free_preprocessor = sp.use_implied_free_preprocessor != 0;
  p.solve_dual_problem = sp.solve_dual_problem;
  p.dualizer_threshold = sp.dualizer_threshold;
  p.preprocessor_zero_tolerance = sp.preprocessor_zero_tolerance;
  p.solution_feasibility_tolerance = sp.solution_feasibility_tolerance;
  p.drop_tolerance = sp.drop_tolerance;
  return p;
}

presolve::Lp ToPresolveLp(const ScaledLp& s, bool maximize) {
  presolve::Lp lp;
  lp.num_rows = s.m;
  lp.cols.resize(s.n);
  for (int c = 0; c < s.n; ++c) {
    for (int64_t k = s.starts[c]; k < s.starts[c + 1]; ++k) {
      lp.cols[c].push_back({s.rows[k], s.vals[k]});
    }
  }
  lp.col_lb = s.col_lb;
  lp.col_ub = s.col_ub;
  lp.obj = s.obj;
  lp.row_lb = s.row_lb;
  lp.row_ub = s.row_ub;
  lp.offset = s.offset;
  lp.scale = s.scale;
  lp.maximize = maximize;
  return lp;
}

ScaledLp FromPresolveLp(const presolve::Lp& p) {
  ScaledLp s;
  s.m = p.num_rows;
  s.n = p.num_cols();
  s.starts.assign(s.n + 1, 0);
  for (int c = 0; c < s.n; ++c) {
    s.starts[c + 1] = s.starts[c] + static_cast<int64_t>(p.cols[c].size());
    for (const presolve::Entry& e : p.cols[c]) {
      s.rows.push_back(e.index);
      s.vals.push_back(e.coeff);
    }
  }
  s.col_lb = p.col_lb;
  s.col_ub = p.col_ub;
  s.obj = p.obj;
  s.row_lb = p.row_lb;
  s.row_ub = p.row_ub;
  s.offset = p.offset;
  s.scale = p.scale;
  return s;
}

ScaledLp CopyLp(int32_t m, int32_t n, const int64_t* cs, const int32_t* ri, const double* vals,
                const double* clb, const double* cub, const double* rlb, const double* rub,
                const double* obj, double obj_offset, double obj_scale) {
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
}

// IsCleanedUp (lp_solver.cc:185-191): rows strictly increasing per column, no
// explicit zeros, rows in range.
bool IsCleanedUp(const ScaledLp& lp) {
  for (int c = 0; c < lp.n; ++c) {
    if (lp.starts[c + 1] < lp.starts[c]) return false;
    for (int64_t k = lp.starts[c]; k < lp.starts[c + 1]; ++k) {
      const int r = lp.rows[k];
      if (r < 0 || r >= lp.m || lp.vals[k] == 0.0) return false;
      if (k > lp.starts[c] && lp.rows[k - 1] >= r) return false;
    }
  }
  return true;
}

// The engine as the LPSolver's simplex (RunRevisedSimplexIfNeeded,
// lp_solver.cc:591-658): load, solve, and read back the solution.
struct EngineSimplex {
  mi_lp* h;
  const volatile int32_t* interrupt;
};

int EngineSimplexSolve(void* user, int32_t m, int32_t n, const int64_t* cs, const int32_t* ri,
                       const double* vals, const double* clb, const double* cub,
                       const double* rlb, const double* rub, const double* obj, double offset,
                       double scale, int32_t maximize, mi_lp_result* out, double* primal,
                       double* duals, int8_t* vstat, int8_t* cstat) {
  const EngineSimplex* e = static_cast<const EngineSimplex*>(user);
  const int rc_load =
      mi_lp_load(e->h, m, n, cs, ri, vals, clb, cub, rlb, rub, obj, offset, scale, maximize);
  if (rc_load != MI_LP_OK) return rc_load;
  const int rc_solve = mi_lp_solve(e->h, e->interrupt, out);
  if (rc_solve != MI_LP_OK) return rc_solve;
  if (out->error_code != MI_LP_OK) return MI_LP_OK;
  mi_lp_get_primal(e->h, primal);
  mi_lp_get_duals(e->h, duals);
  mi_lp_get_statuses(e->h, vstat, cstat);
  return MI_LP_OK;
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
  p->use_preprocessing = 1;                 // :326
  p->change_status_to_imprecise = 1;        // :275
  p->use_implied_free_preprocessor = 1;     // :473
  p->solve_dual_problem = 2;                // :236, LET_SOLVER_DECIDE
  p->dualizer_threshold = 1.5;              // :241
  p->preprocessor_zero_tolerance = 1e-9;    // :356
  p->solution_feasibility_tolerance = 1e-6; // :251
  p->drop_tolerance = 1e-14;                // :183
}

// Test hook (tests/native/lp_solver_asan.cc): IsProblemSolutionConsistent
// on an m x n LP with no constraints on its values and a solution whose
// vectors have the given lengths: free columns at 0, basic slacks (the slack
// basis, consistent when the sizes are right). Returns 1 when
// consistent; a wrong-sized solution must be 0 (and must not be indexed).
int milp_test_solution_consistent(int32_t m, int32_t n, int32_t status, int64_t primal_len,
                                  int64_t dual_len, int64_t vstat_len, int64_t cstat_len) {
  milp::ScaledLp lp;
  lp.m = m;
  lp.n = n;
  lp.starts.assign(static_cast<size_t>(n) + 1, 0);
  lp.col_lb.assign(n, -milp::kInf);
  lp.col_ub.assign(n, milp::kInf);
  lp.obj.assign(n, 0.0);
  lp.row_lb.assign(m, -milp::kInf);
  lp.row_ub.assign(m, milp::kInf);
  milp::presolve::Solution s;
  s.status = status;
  s.primal.assign(primal_len, 0.0);
  s.dual.assign(dual_len, 0.0);
  s.vstat.assign(vstat_len, static_cast<int8_t>(MI_LP_FREE));
  s.cstat.assign(cstat_len, static_cast<int8_t>(MI_LP_BASIC));
  return milp::IsSolutionConsistent(lp, s) ? 1 : 0;
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

// Opaque presolve object of the C ABI.
struct mi_presolve {
  std::unique_ptr<milp::presolve::MainPresolve> pre;
  milp::presolve::Lp lp;
  int32_t m0 = 0, n0 = 0;
  bool ran = false, recovered = false, post = false;
};

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
    milp::ScaledLp lp = milp::CopyLp(m, n, cs, ri, vals, clb, cub, rlb, rub, obj, *obj_offset,
                                     *obj_scale);
    for (int32_t r : lp.rows) {
      if (r < 0 || r >= m) return MI_LP_ERROR_INVALID_PROBLEM;
    }
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

int mi_lp_solver_solve_with(mi_lp_simplex_fn fn, void* user, const mi_lp_solver_params* sp,
                            int32_t m, int32_t n, const int64_t* cs, const int32_t* ri,
                            const double* vals, const double* clb, const double* cub,
                            const double* rlb, const double* rub, const double* obj,
                            double obj_offset, double obj_scale, int32_t maximize,
                            mi_lp_result* out, double* primal, double* duals, double* rc,
                            double* act, int8_t* vstat, int8_t* cstat) {
  using milp::ScaledLp;
  namespace ps = milp::presolve;
  if (fn == nullptr || sp == nullptr || out == nullptr || cs == nullptr) return MI_LP_ERROR_NULL;
  if (m < 0 || n < 0 || cs[0] != 0 || cs[n] < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  if (!LpArraysPresent(m, n, cs, ri, vals, clb, cub, rlb, rub, obj)) return MI_LP_ERROR_NULL;
  std::memset(out, 0, sizeof(*out));
  try {
    const ScaledLp orig =
        milp::CopyLp(m, n, cs, ri, vals, clb, cub, rlb, rub, obj, obj_offset, obj_scale);
    if (!milp::IsCleanedUp(orig)) return MI_LP_ERROR_INVALID_PROBLEM;
    if (!milp::IsValid(orig, sp->max_valid_magnitude)) {
      out->problem_status = MI_LP_INVALID_PROBLEM;
      return MI_LP_OK;
    }
    // MainLpPreprocessor::Run (preprocessor.cc:76-147): the presolve passes,
    // then the ScalingPreprocessor through RunAndPushIfRelevant (:152-194).
    ps::MainPresolve pre(milp::PresolveParamsOf(*sp));
    ps::Lp plp = milp::ToPresolveLp(orig, maximize != 0);
    const bool postsolve = pre.Run(&plp);
    int32_t status = pre.status();
    const bool inner_max = plp.maximize;
    const ScaledLp inner = milp::FromPresolveLp(plp);
    plp = ps::Lp();
    ScaledLp lp = inner;
    milp::MatrixScaler scaler;
    double cost_factor = 1.0, bound_factor = 1.0;
    bool scaled = false;
    if (status == MI_LP_INIT) {
      if (lp.m == 0 && lp.n == 0) {
        status = MI_LP_OPTIMAL;
      } else if (sp->use_scaling) {
        milp::ScaleLp(&lp, &scaler);
        cost_factor = milp::ScaleObjective(&lp, sp->cost_scaling);
        bound_factor = milp::ScaleBounds(&lp);
        scaled = true;
      }
    }
    // LPSolver::SolveWithTimeLimit (lp_solver.cc:226-247).
    ps::Solution sol(lp.m, lp.n);
    sol.status = status;
    mi_lp_result r;
    std::memset(&r, 0, sizeof(r));
    if (status == MI_LP_INIT) {
      const int rc_fn = fn(user, lp.m, lp.n, lp.starts.data(), lp.rows.data(), lp.vals.data(),
                           lp.col_lb.data(), lp.col_ub.data(), lp.row_lb.data(),
                           lp.row_ub.data(), lp.obj.data(), lp.offset, lp.scale,
                           inner_max ? 1 : 0, &r, sol.primal.data(), sol.dual.data(),
                           sol.vstat.data(), sol.cstat.data());
      if (rc_fn != MI_LP_OK) return rc_fn;
      if (r.error_code != MI_LP_OK) {
        *out = r;
        return MI_LP_OK;
      }
      sol.status = r.problem_status;
    }
    // ScalingPreprocessor::RecoverSolution (preprocessor.cc:3878-3912).
    if (scaled) {
      for (int c = 0; c < lp.n; ++c) sol.primal[c] /= scaler.col_scale[c];
      for (int c = 0; c < lp.n; ++c) sol.primal[c] *= bound_factor;
      for (int row = 0; row < lp.m; ++row) sol.dual[row] /= scaler.row_scale[row];
      for (int row = 0; row < lp.m; ++row) sol.dual[row] *= cost_factor;
      for (int c = 0; c < lp.n; ++c) {
        switch (sol.vstat[c]) {
          case MI_LP_AT_UPPER_BOUND:
          case MI_LP_FIXED_VALUE:
            sol.primal[c] = inner.col_ub[c];
            break;
          case MI_LP_AT_LOWER_BOUND:
            sol.primal[c] = inner.col_lb[c];
            break;
          default:
            break;
        }
      }
    }
    // MainLpPreprocessor::DestructiveRecoverSolution (preprocessor.cc:203-209).
    if (postsolve) pre.Recover(&sol);
    *out = r;
    // LoadAndVerifySolution (lp_solver.cc:323-367).
    if (!milp::IsSolutionConsistent(orig, sol)) {
      out->problem_status = MI_LP_ABNORMAL;
      out->objective = 0.0;
      if (primal != nullptr) std::fill(primal, primal + n, 0.0);
      if (duals != nullptr) std::fill(duals, duals + m, 0.0);
      if (rc != nullptr) std::fill(rc, rc + n, 0.0);
      if (act != nullptr) std::fill(act, act + m, 0.0);
      if (vstat != nullptr) std::fill(vstat, vstat + n, static_cast<int8_t>(MI_LP_FREE));
      if (cstat != nullptr) std::fill(cstat, cstat + m, static_cast<int8_t>(MI_LP_FREE));
      return MI_LP_OK;
    }
    int32_t verified = sol.status;
    std::vector<double>& x = sol.primal;
    std::vector<double>& y = sol.dual;
    const double optimization_sign = maximize ? -1.0 : 1.0;
    const double tolerance = sp->solution_feasibility_tolerance;
    auto allowed_error = [tolerance](double value) {  // AllowedError (:316-318)
      return tolerance * std::max(1.0, std::fabs(value));
    };
    std::vector<double> reduced(n, 0.0);
    auto compute_reduced_costs = [&]() {  // ComputeReducedCosts (:877-886)
      for (int c = 0; c < n; ++c) {
        double dot = 0.0;
        for (int64_t k = orig.starts[c]; k < orig.starts[c + 1]; ++k) {
          dot += y[orig.rows[k]] * orig.vals[k];
        }
        reduced[c] = orig.obj[c] - dot;
      }
    };
    auto compute_objective = [&]() {  // ComputeObjective (:888-896)
      milp::KahanSum sum;
      for (int c = 0; c < n; ++c) sum.Add(orig.obj[c] * x[c]);
      return sum.sum;
    };
    compute_reduced_costs();
    const double primal_objective = compute_objective();
    double dual_objective;
    {  // ComputeDualObjective (:914-975)
      milp::KahanSum sum;
      for (int row = 0; row < m; ++row) {
        const double corrected = optimization_sign * y[row];
        if (corrected > 0.0 && orig.row_lb[row] != -milp::kInf) sum.Add(y[row] * orig.row_lb[row]);
        if (corrected < 0.0 && orig.row_ub[row] != milp::kInf) sum.Add(y[row] * orig.row_ub[row]);
      }
      for (int c = 0; c < n; ++c) {
        const double rcm = optimization_sign * reduced[c];
        double correction = 0.0;
        if (sol.vstat[c] == MI_LP_AT_LOWER_BOUND && rcm > 0.0) {
          correction = rcm * orig.col_lb[c];
        } else if (sol.vstat[c] == MI_LP_AT_UPPER_BOUND && rcm < 0.0) {
          correction = rcm * orig.col_ub[c];
        } else if (sol.vstat[c] == MI_LP_FIXED_VALUE) {
          correction = rcm * orig.col_ub[c];
        }
        sum.Add(optimization_sign * correction);
      }
      dual_objective = sum.sum;
    }
    const bool strong = sp->provide_strong_optimal_guarantee && verified == MI_LP_OPTIMAL;
    if (strong) {
      for (int c = 0; c < n; ++c) {  // MovePrimalValuesWithinBounds (:540-555)
        x[c] = std::min(x[c], orig.col_ub[c]);
        x[c] = std::max(x[c], orig.col_lb[c]);
      }
      for (int row = 0; row < m; ++row) {  // MoveDualValuesWithinBounds (:557-579)
        double d = optimization_sign * y[row];
        if (orig.row_lb[row] == -milp::kInf && d > 0.0) d = 0.0;
        if (orig.row_ub[row] == milp::kInf && d < 0.0) d = 0.0;
        y[row] = optimization_sign * d;
      }
    }
    // ProblemObjectiveValue (:306-312).
    out->objective = orig.scale * (compute_objective() + orig.offset);
    compute_reduced_costs();
    std::vector<double> activity(m, 0.0);  // ComputeConstraintActivities (:866-875)
    for (int c = 0; c < n; ++c) {
      if (x[c] == 0.0) continue;
      for (int64_t k = orig.starts[c]; k < orig.starts[c + 1]; ++k) {
        activity[orig.rows[k]] += x[c] * orig.vals[k];
      }
    }
    // The precision checks of LoadAndVerifySolution (:369-472).
    bool rhs_too_large = false, cost_too_large = false, primal_inf_too_large = false,
         dual_inf_too_large = false, primal_res_too_large = false, dual_res_too_large = false;
    for (int row = 0; row < m; ++row) {  // ComputeMaxRhsPerturbation... (:838-864)
      const double lb = orig.row_lb[row], ub = orig.row_ub[row], a = activity[row];
      double err = 0.0, ok = 0.0;
      if (sol.cstat[row] == MI_LP_AT_LOWER_BOUND || a < lb) {
        err = std::fabs(a - lb);
        ok = allowed_error(lb);
      } else if (sol.cstat[row] == MI_LP_AT_UPPER_BOUND || a > ub) {
        err = std::fabs(a - ub);
        ok = allowed_error(ub);
      }
      rhs_too_large |= err > ok;
    }
    for (int c = 0; c < n; ++c) {  // ComputeMaxCostPerturbation... (:810-834)
      const double rcm = optimization_sign * reduced[c];
      const int8_t st = sol.vstat[c];
      if (st == MI_LP_BASIC || st == MI_LP_FREE || (st == MI_LP_AT_UPPER_BOUND && rcm > 0.0) ||
          (st == MI_LP_AT_LOWER_BOUND && rcm < 0.0)) {
        cost_too_large |= std::fabs(rcm) > allowed_error(orig.obj[c]);
      }
    }
    for (int c = 0; c < n; ++c) {  // ComputePrimalValueInfeasibility (:992-1020)
      const double lb = orig.col_lb[c], ub = orig.col_ub[c];
      if (lb == ub) {
        primal_inf_too_large |= std::fabs(x[c] - ub) > allowed_error(ub);
        continue;
      }
      if (x[c] > ub) primal_inf_too_large |= x[c] - ub > allowed_error(ub);
      if (x[c] < lb) primal_inf_too_large |= lb - x[c] > allowed_error(lb);
    }
    for (int row = 0; row < m; ++row) {  // ComputeDualValueInfeasibility (:1073-1095)
      const double d = optimization_sign * y[row];
      if (orig.row_lb[row] == -milp::kInf) dual_inf_too_large |= d > tolerance;
      if (orig.row_ub[row] == milp::kInf) dual_inf_too_large |= -d > tolerance;
    }
    for (int row = 0; row < m; ++row) {  // ComputeActivityInfeasibility (:1022-1071)
      const double lb = orig.row_lb[row], ub = orig.row_ub[row], a = activity[row];
      if (lb == ub) {
        primal_res_too_large |= std::fabs(a - ub) > allowed_error(ub);
        continue;
      }
      if (a > ub) primal_res_too_large |= a - ub > allowed_error(ub);
      if (a < lb) primal_res_too_large |= lb - a > allowed_error(lb);
    }
    for (int c = 0; c < n; ++c) {  // ComputeReducedCostInfeasibility (:1097-1122)
      const double rcm = optimization_sign * reduced[c];
      const double ok = allowed_error(orig.obj[c]);
      if (orig.col_lb[c] == -milp::kInf) dual_res_too_large |= rcm > ok;
      if (orig.col_ub[c] == milp::kInf) dual_res_too_large |= -rcm > ok;
    }
    double objective_error_ub = 0.0;  // ComputeMaxExpectedObjectiveError (:977-990)
    for (int c = 0; c < n; ++c) {
      objective_error_ub += std::fabs(orig.obj[c]) * allowed_error(x[c]);
    }
    if (sp->change_status_to_imprecise) {
      if (strong && (rhs_too_large || cost_too_large)) verified = MI_LP_IMPRECISE;
      if (verified == MI_LP_OPTIMAL &&
          std::fabs(primal_objective - dual_objective) > objective_error_ub) {
        verified = MI_LP_IMPRECISE;
      }
      if ((verified == MI_LP_OPTIMAL || verified == MI_LP_PRIMAL_FEASIBLE) &&
          (primal_res_too_large || primal_inf_too_large)) {
        verified = MI_LP_IMPRECISE;
      }
      if ((verified == MI_LP_OPTIMAL || verified == MI_LP_DUAL_FEASIBLE) &&
          (dual_res_too_large || dual_inf_too_large)) {
        verified = MI_LP_IMPRECISE;
      }
    }
    out->problem_status = verified;
    if (rc != nullptr) std::copy(reduced.begin(), reduced.end(), rc);
    if (act != nullptr) std::copy(activity.begin(), activity.end(), act);
    if (primal != nullptr) std::copy(x.begin(), x.end(), primal);
    if (duals != nullptr) std::copy(y.begin(), y.end(), duals);
    if (vstat != nullptr) std::copy(sol.vstat.begin(), sol.vstat.end(), vstat);
    if (cstat != nullptr) std::copy(sol.cstat.begin(), sol.cstat.end(), cstat);
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
  if (h == nullptr) return MI_LP_ERROR_NULL;
  milp::EngineSimplex engine{h, interrupt};
  return mi_lp_solver_solve_with(milp::EngineSimplexSolve, &engine, sp, m, n, cs, ri, vals, clb,
                                 cub, rlb, rub, obj, obj_offset, obj_scale, maximize, out,
                                 primal, duals, rc, act, vstat, cstat);
}

// --- presolve alone -------------------------------------------------------------
mi_presolve* mi_presolve_create(void) {
  try {
    return new mi_presolve();
  } catch (const std::exception&) {
    return nullptr;
  }
}

void mi_presolve_destroy(mi_presolve* ps) { delete ps; }

int mi_presolve_run(mi_presolve* ps, const mi_lp_solver_params* sp, int32_t m, int32_t n,
                    const int64_t* cs, const int32_t* ri, const double* vals, const double* clb,
                    const double* cub, const double* rlb, const double* rub, const double* obj,
                    double obj_offset, double obj_scale, int32_t maximize, int32_t* status) {
  if (ps == nullptr || sp == nullptr || cs == nullptr || status == nullptr) {
    return MI_LP_ERROR_NULL;
  }
  if (ps->ran) return MI_LP_ERROR_STATE;
  if (m < 0 || n < 0 || cs[0] != 0 || cs[n] < 0) return MI_LP_ERROR_INVALID_PROBLEM;
  if (!LpArraysPresent(m, n, cs, ri, vals, clb, cub, rlb, rub, obj)) return MI_LP_ERROR_NULL;
  try {
    const milp::ScaledLp orig =
        milp::CopyLp(m, n, cs, ri, vals, clb, cub, rlb, rub, obj, obj_offset, obj_scale);
    if (!milp::IsCleanedUp(orig)) return MI_LP_ERROR_INVALID_PROBLEM;
    ps->pre = std::make_unique<milp::presolve::MainPresolve>(milp::PresolveParamsOf(*sp));
    ps->lp = milp::ToPresolveLp(orig, maximize != 0);
    ps->m0 = m;
    ps->n0 = n;
    ps->ran = true;
    if (!milp::IsValid(orig, sp->max_valid_magnitude)) {  // lp_solver.cc:196-202
      *status = MI_LP_INVALID_PROBLEM;
      return MI_LP_OK;
    }
    ps->post = ps->pre->Run(&ps->lp);
    *status = ps->pre->status();
    return MI_LP_OK;
  } catch (const std::exception&) {
    return MI_LP_ERROR_INTERNAL;
  }
}

int mi_presolve_dims(const mi_presolve* ps, int32_t* m, int32_t* n, int64_t* nnz,
                     int32_t* maximize) {
  if (ps == nullptr) return MI_LP_ERROR_NULL;
  if (!ps->ran) return MI_LP_ERROR_STATE;
  if (m != nullptr) *m = ps->lp.num_rows;
  if (n != nullptr) *n = ps->lp.num_cols();
  if (nnz != nullptr) *nnz = ps->lp.num_entries();
  if (maximize != nullptr) *maximize = ps->lp.maximize ? 1 : 0;
  return MI_LP_OK;
}

int mi_presolve_get(const mi_presolve* ps, int64_t* cs, int32_t* ri, double* vals, double* clb,
                    double* cub, double* rlb, double* rub, double* obj, double* obj_offset,
                    double* obj_scale) {
  if (ps == nullptr) return MI_LP_ERROR_NULL;
  if (!ps->ran) return MI_LP_ERROR_STATE;
  const milp::ScaledLp s = milp::FromPresolveLp(ps->lp);
  if (cs != nullptr) std::copy(s.starts.begin(), s.starts.end(), cs);
  if (ri != nullptr) std::copy(s.rows.begin(), s.rows.end(), ri);
  if (vals != nullptr) std::copy(s.vals.begin(), s.vals.end(), vals);
  if (clb != nullptr) std::copy(s.col_lb.begin(), s.col_lb.end(), clb);
  if (cub != nullptr) std::copy(s.col_ub.begin(), s.col_ub.end(), cub);
  if (rlb != nullptr) std::copy(s.row_lb.begin(), s.row_lb.end(), rlb);
  if (rub != nullptr) std::copy(s.row_ub.begin(), s.row_ub.end(), rub);
  if (obj != nullptr) std::copy(s.obj.begin(), s.obj.end(), obj);
  if (obj_offset != nullptr) *obj_offset = s.offset;
  if (obj_scale != nullptr) *obj_scale = s.scale;
  return MI_LP_OK;
}

int mi_presolve_recover(mi_presolve* ps, int32_t* status, const double* primal,
                        const double* duals, const int8_t* vstat, const int8_t* cstat,
                        double* primal_out, double* duals_out, int8_t* vstat_out,
                        int8_t* cstat_out) {
  if (ps == nullptr || status == nullptr) return MI_LP_ERROR_NULL;
  if (!ps->ran || ps->recovered) return MI_LP_ERROR_STATE;
  const int32_t m = ps->lp.num_rows;
  const int32_t n = ps->lp.num_cols();
  if ((n > 0 && (primal == nullptr || vstat == nullptr)) ||
      (m > 0 && (duals == nullptr || cstat == nullptr))) {
    return MI_LP_ERROR_NULL;
  }
  try {
    milp::presolve::Solution s(m, n);
    s.status = *status;
    if (n > 0) {
      std::copy(primal, primal + n, s.primal.begin());
      std::copy(vstat, vstat + n, s.vstat.begin());
    }
    if (m > 0) {
      std::copy(duals, duals + m, s.dual.begin());
      std::copy(cstat, cstat + m, s.cstat.begin());
    }
    if (ps->post) ps->pre->Recover(&s);
    ps->recovered = true;
    if (static_cast<int32_t>(s.primal.size()) != ps->n0 ||
        static_cast<int32_t>(s.dual.size()) != ps->m0 ||
        static_cast<int32_t>(s.vstat.size()) != ps->n0 ||
        static_cast<int32_t>(s.cstat.size()) != ps->m0) {
      return MI_LP_ERROR_INTERNAL;
    }
    *status = s.status;
    if (primal_out != nullptr) std::copy(s.primal.begin(), s.primal.end(), primal_out);
    if (duals_out != nullptr) std::copy(s.dual.begin(), s.dual.end(), duals_out);
    if (vstat_out != nullptr) std::copy(s.vstat.begin(), s.vstat.end(), vstat_out);
    if (cstat_out != nullptr) std::copy(s.cstat.begin(), s.cstat.end(), cstat_out);
    return MI_LP_OK;
  } catch (const std::exception&) {
    return MI_LP_ERROR_INTERNAL;
  }
}

int32_t mi_presolve_num_passes(const mi_presolve* ps) {
  if (ps == nullptr || !ps->ran) return 0;
  return static_cast<int32_t>(ps->pre->applied().size());
}

const char* mi_presolve_pass_name(const mi_presolve* ps, int32_t i) {
  if (ps == nullptr || !ps->ran || i < 0 ||
      i >= static_cast<int32_t>(ps->pre->applied().size())) {
    return nullptr;
  }
  return ps->pre->applied()[i].c_str();
}

}  // extern "C"
