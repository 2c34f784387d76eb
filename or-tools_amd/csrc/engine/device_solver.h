// Device substitutes for the dense triangular solves of the basis
// factorization's FTRAN (lu_factorization.cc:214-331): the U solve
// (lp_data/sparse.cc:899-955 TriangularMatrix::TransposeLowerSolve, a gather
// over U's rows) and the L solve (sparse.cc:793-812 LowerSolveStartingAt, a
// column scatter, restated as a gather over L's rows). Implemented by DeviceLp; the LU code only
// sees this interface so that lu.h stays free of HIP types.
#ifndef MILP_DEVICE_SOLVER_H_
#define MILP_DEVICE_SOLVER_H_

#include <cstdint>
#include <vector>

namespace milp {

class TriangularMatrix;

class DeviceSolver {
 public:
  virtual ~DeviceSolver() = default;
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
