// Argument blocks shared by the kernel launchers (simplex_kernels.hip) and
// the device layer (engine/device_lp.hip). Plain structs of device pointers.
#ifndef MILP_KERNEL_ARGS_H_
#define MILP_KERNEL_ARGS_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace milp_kernels {

struct DotArgs {
  const int64_t* starts;
  const int32_t* rows;
  const double* vals;
  const double* y;
  int ncols;                // columns to visit (N, or list length)
  const int32_t* col_list;  // kListDots: the columns
  const uint64_t* mask;     // relevance / not-basic bitset (modes 0, 3)
  const double* c;          // kPricing: objective + perturbation
  double* out;              // result per column (or per list entry)
  uint8_t* flags;           // kUpdateRowColumnWise: |coeff| > drop
  double drop_tolerance;
};

struct RowWiseArgs {
  const int64_t* t_starts;  // CSR of [A | I] (transposed_matrix_)
  const int32_t* t_cols;
  const double* t_vals;
  const int32_t* filtered_rows;  // ascending
  const double* rho;             // rho value per filtered row
  int num_filtered;
  int num_cols;
  const uint64_t* relevant;
  double* coefficient;  // update row (device copy of UpdateRow::coefficient_)
  uint8_t* flags;       // listed positions
  double drop_tolerance;
  int algorithm;  // 0 single row, 1 hypersparse, 2 row-wise
};

struct RowSumArgs {
  const int64_t* t_starts;
  const int32_t* t_cols;
  const double* t_vals;
  const double* x;       // multipliers per column
  const uint64_t* skip;  // optional: skip columns whose bit is set (basic)
  double sign;           // +1 (residual) or -1 (basic-value recompute)
  int num_rows;
  double* out;
};

}  // namespace milp_kernels

namespace milp_launch {
hipError_t column_dot(int mode, bool wave_per_col, const milp_kernels::DotArgs& args,
                      hipStream_t s);
hipError_t row_wise_update(const milp_kernels::RowWiseArgs& args, hipStream_t s);
hipError_t row_sums(const milp_kernels::RowSumArgs& args, hipStream_t s);
hipError_t column_squared_norms(const int64_t* starts, const double* vals,
                                const uint64_t* relevant, int ncols, double* out,
                                hipStream_t s);
}  // namespace milp_launch

#endif  // MILP_KERNEL_ARGS_H_
