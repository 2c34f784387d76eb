// Glop's presolve (glop/preprocessor.cc, MainLpPreprocessor) for the LPSolver
// layer: the LP the caller gives is reduced by the same sequence of passes
// Glop runs before the simplex, and the simplex solution of the reduced LP is
// mapped back ("postsolve") pass by pass in reverse order.
//
// Host code, O(nnz) per pass, run once per LPSolver solve before the reduced
// LP goes to HBM. Each pass cites the reference loop it restates; the
// floating-point operations follow those loops one at a time (g++ with
// -ffp-contract=off, as the rest of the host engine).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace milp {
namespace presolve {

// glop::ProblemStatus / VariableStatus / ConstraintStatus numbering (the
// values of include/mi_lp.h).
enum Status : int32_t {
  kOptimal = 0,
  kPrimalInfeasible = 1,
  kDualInfeasible = 2,
  kInfeasibleOrUnbounded = 3,
  kPrimalUnbounded = 4,
  kDualUnbounded = 5,
  kInit = 6,
  kPrimalFeasible = 7,
  kDualFeasible = 8,
  kAbnormal = 9,
  kInvalidProblem = 10,
  kImprecise = 11,
};
enum BasisStatus : int8_t {
  kBasic = 0,
  kFixedValue = 1,
  kAtLowerBound = 2,
  kAtUpperBound = 3,
  kFree = 4,
};

// The GlopParameters fields the passes read (parameters.proto).
struct Params {
  bool use_preprocessing = true;        // 34
  bool use_implied_free_preprocessor = true;  // 67
  int solve_dual_problem = 2;           // 20: ALWAYS_DO 0, NEVER_DO 1, LET_SOLVER_DECIDE 2
  double dualizer_threshold = 1.5;      // 21
  double preprocessor_zero_tolerance = 1e-9;      // 39
  double solution_feasibility_tolerance = 1e-6;   // 22
  double drop_tolerance = 1e-14;        // 52
};

// One sparse column (or a row of the transpose): entries sorted by index,
// no zeros, as SparseColumn is after CleanUp().
struct Entry {
  int32_t index;
  double coeff;
};
using SparseVec = std::vector<Entry>;

// glop::LinearProgram, the fields the passes touch.
struct Lp {
  int32_t num_rows = 0;
  std::vector<SparseVec> cols;
  std::vector<double> col_lb, col_ub, obj, row_lb, row_ub;
  double offset = 0.0, scale = 1.0;
  bool maximize = false;

  int32_t num_cols() const { return static_cast<int32_t>(cols.size()); }
  int64_t num_entries() const;
  double MinCost(int32_t col) const { return maximize ? -obj[col] : obj[col]; }
  // SparseMatrix::PopulateFromTranspose: row r lists (col, coeff) in
  // increasing column order.
  std::vector<SparseVec> Transpose() const;
  void DeleteColumns(const std::vector<bool>& del);  // lp_data.cc:1067-1114
  void DeleteRows(const std::vector<bool>& del);     // lp_data.cc:1260-1305
  int32_t AddColumn(double lb, double ub, double cost);  // CreateNewVariable
};

// glop::ProblemSolution.
struct Solution {
  int32_t status = kOptimal;
  std::vector<double> primal, dual;
  std::vector<int8_t> vstat, cstat;
  Solution() = default;
  Solution(int32_t m, int32_t n)
      : primal(n, 0.0), dual(m, 0.0), vstat(n, kFree), cstat(m, kFree) {}
};

class Pass;

// MainLpPreprocessor (preprocessor.cc:76-209) minus the scaling, which the
// LPSolver layer runs on the presolved LP (engine/lp_solver.cc).
class MainPresolve {
 public:
  explicit MainPresolve(const Params& p);
  ~MainPresolve();
  // Runs the passes on *lp. Returns true when a postsolve is needed.
  bool Run(Lp* lp);
  // Glop's status after presolve: kInit when the simplex must run.
  int32_t status() const { return status_; }
  // DestructiveRecoverSolution (preprocessor.cc:203-209).
  void Recover(Solution* s);
  // Names of the passes that changed the LP, in order (the postsolve stack).
  const std::vector<std::string>& applied() const { return applied_; }

 private:
  void RunPass(std::unique_ptr<Pass> pass, const char* name, Lp* lp);
  Params params_;
  int32_t status_ = kInit;
  std::vector<std::unique_ptr<Pass>> stack_;
  std::vector<std::string> applied_;
};

}  // namespace presolve
}  // namespace milp
