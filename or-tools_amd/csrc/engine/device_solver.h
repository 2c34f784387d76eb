// Device substitutes for the dense triangular solves of the basis
// factorization (lp_data/sparse.cc:899-955 TriangularMatrix::TransposeLowerSolve,
// the row-oriented form Glop uses for the U solve of every FTRAN,
// lu_factorization.cc:314-331). Implemented by DeviceLp; the LU code only
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
};

}  // namespace milp

#endif  // MILP_DEVICE_SOLVER_H_
