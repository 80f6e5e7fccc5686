// ort_k_pupil.hip -- device pupil sampling (ort_generate_pupil; math in ort_pupil.h)

#include "ort_kernels.h"
#include "ort_pupil.h"

namespace ortk {

__global__ __launch_bounds__(kBlock) void pupil_kernel(const ort_pupil d, double* px,
                                                       double* py) {
  const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= d.n_points) return;
  double x, y;
  ort::pupil_point(d, k, x, y);
  px[k] = x;
  py[k] = y;
}

int launch_pupil(const ort_pupil& d, double* px, double* py, hipStream_t stream) {
  const int64_t blocks = (d.n_points + kBlock - 1) / kBlock;
  if (blocks == 0) return ORT_OK;
  if (blocks > 0x7fffffff) return ORT_ERR_ARG;
  hipLaunchKernelGGL(pupil_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, d, px, py);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

}  // namespace ortk
