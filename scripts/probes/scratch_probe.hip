// Development aid: one kernel that needs private (scratch) memory, nothing
// else. Run under `rocprofv3 --pmc` to tell a profiler teardown crash that
// scratch-using kernels trigger from one of the engine's (the device dual
// segment kernels use 784 B of scratch per lane).
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void scratch_kernel(const int* idx, double* out) {
  double a[96];  // indexed by a runtime value: lives in scratch
  for (int i = 0; i < 96; ++i) a[i] = i * 0.5 + threadIdx.x;
  out[blockIdx.x * blockDim.x + threadIdx.x] = a[idx[threadIdx.x] % 96];
}

int main() {
  int* idx;
  double* out;
  (void)hipMalloc(&idx, 64 * sizeof(int));
  (void)hipMalloc(&out, 64 * 64 * sizeof(double));
  (void)hipMemset(idx, 7, 64 * sizeof(int));
  scratch_kernel<<<64, 64>>>(idx, out);
  double h = 0;
  (void)hipMemcpy(&h, out, sizeof(double), hipMemcpyDeviceToHost);
  std::printf("scratch probe %g\n", h);
  (void)hipFree(idx);
  (void)hipFree(out);
  return 0;
}
