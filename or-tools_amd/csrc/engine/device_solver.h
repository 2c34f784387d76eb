// Device substitutes for the dense triangular solves of the basis
// factorization's FTRAN (lu_factorization.cc:214-331): the U solve
// (lp_data/sparse.cc:899-955 TriangularMatrix::TransposeLowerSolve, a gather
// over U's rows) and the L solve (sparse.cc:793-812 LowerSolveStartingAt, a
// column scatter, restated as a gather over L's rows). Implemented by DeviceLp; the LU code only
// sees this interface so that lu.h stays free of HIP types.
#ifndef MILP_DEVICE_SOLVER_H_
#define MILP_DEVICE_SOLVER_H_

#include <cstdint>
#include <functional>
#include <vector>

namespace milp {

class TriangularMatrix;

// The dense loops of TriangularMatrix (sparse.cc:776-955) the device
// replaces, by the matrix of the LU they run on:
enum class TriKind {
  kUpperT = 0,     // transpose_upper_.TransposeLowerSolve: FTRAN's U (gather from the end)
  kLower = 1,      // lower_.LowerSolveStartingAt: FTRAN's L (column scatter)
  kUpperTUp = 2,   // upper_.TransposeUpperSolve: BTRAN's U^T (forward gather)
  kLowerT = 3,     // lower_.TransposeLowerSolve: BTRAN's L^T (gather from the end)
  kUnitRow = 4,    // transpose_upper_.LowerSolveStartingAt: the unit-row BTRAN's U^T
  kUpper = 5,      // upper_.UpperSolve: the product-form FTRAN's U (backward scatter)
};
constexpr int kNumTriKinds = 6;

// Host work the solving thread may do while a device triangular solve is in
// flight: set by the caller, run once -- by the device solve between its
// launch and its wait, or else by the caller before any host loop touches
// the vector the work reads. (The MPF right-pool append of a dense FTRAN
// column, basis_representation.cc:468-501, reads the vector the U solve then
// overwrites; the device solve has copied it by then.)
struct OverlapWork {
  std::function<void()> f;
  void Run();
};
extern thread_local OverlapWork g_overlap;
// Set while overlap work runs inside a device solve: that work's own dense
// loops stay on the host (the solving thread's device context is busy).
extern thread_local bool g_in_overlap;

class DeviceSolver {
 public:
  virtual ~DeviceSolver() = default;
  // x <- the result of the host loop `kind` on t, bit for bit (start: the
  // first column of LowerSolveStartingAt; ignored by the other loops).
  // Returns false, leaving x untouched, when the solve should run on the
  // host (MILP_DEVICE_SOLVE and the size threshold decide).
  virtual bool Solve(TriKind kind, const TriangularMatrix& t, uint64_t key, int start,
                     std::vector<double>* x) = 0;
  // Two right-hand sides of the same dense loop in one device launch (each
  // vector's bits as its own Solve); false: solve them one by one.
  virtual bool SolvePair(TriKind kind, const TriangularMatrix& t, uint64_t key,
                         std::vector<double>* x0, std::vector<double>* x1) {
    (void)kind, (void)t, (void)key, (void)x0, (void)x1;
    return false;
  }
  // The dense U solve (TransposeLowerSolve) of a vector needed later: staged
  // now and launched on a stream of its own, so it runs behind the caller's
  // other work (engine: the speculative flip FTRAN, lu.h). FinishAsyncU
  // waits and writes the result into x (the vector given to StartAsyncU,
  // kept by the caller); DropAsyncU waits and discards it. One at a time.
  virtual bool StartAsyncU(const TriangularMatrix& t, uint64_t key, const std::vector<double>& x) {
    (void)t, (void)key, (void)x;
    return false;
  }
  virtual void FinishAsyncU(std::vector<double>* x) { (void)x; }
  virtual void DropAsyncU() {}
  // x <- the result of t.TransposeLowerSolve(x), bit for bit. `key`
  // identifies the matrix (its LU and the factorization that built it): the
  // device copy and its dependency schedule are rebuilt when it changes.
  // Returns false, leaving x untouched, when the solve should run on the
  // host (MILP_DEVICE_SOLVE and the size threshold decide).
  virtual bool TransposeLowerSolve(const TriangularMatrix& t, uint64_t key,
                                   std::vector<double>* x) = 0;
  // x <- the result of lower.LowerSolveStartingAt(start, x) (sparse.cc:
  // 793-812, the L solve of every dense FTRAN), bit for bit. Outputs below
  // `start` receive nothing in that loop, so the device computes them all.
  virtual bool LowerSolve(const TriangularMatrix& lower, uint64_t key,
                          std::vector<double>* x) = 0;
};

}  // namespace milp

#endif  // MILP_DEVICE_SOLVER_H_
