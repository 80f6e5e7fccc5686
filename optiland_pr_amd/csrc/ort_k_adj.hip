// ort_k_adj.hip -- adjoint VJP: slot flags, wave-partial reduction, contraction with the
// tangent tables, and the launch sequence (kernel templates: ort_adjoint.h)

#include "ort_adjoint.h"

namespace ortk {

// need[slot]: some parameter depends on the slot (skips its wave sums)
__global__ void adj_need_kernel(const AArgs j) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= j.n_slot) return;
  int need = 0;
  for (int p = 0; p < j.n_param && !need; ++p) need = slot_weight(j, slot, p) != 0.0;
  j.need[slot] = need;
}

// slot_sum[slot] = sum over waves, in a fixed order
__global__ __launch_bounds__(kBlock) void adj_reduce_kernel(const AArgs j) {
  const int slot = blockIdx.x;
  double v = 0.0;
  if (j.need[slot]) {
    const double* src = j.partial + (int64_t)slot * j.n_wave;
    for (int64_t w = threadIdx.x; w < j.n_wave; w += kBlock) v += src[w];
  }
  __shared__ double ws[kBlock / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < kBlock / 64; ++w) s += ws[w];
    j.slot_sum[slot] = s;
  }
}

// grad[p] += sum_slot slot_sum[slot] * d slot / d p
__global__ __launch_bounds__(kBlock) void adj_contract_kernel(const AArgs j) {
  for (int p = threadIdx.x; p < j.n_param; p += kBlock) {
    double g = 0.0;
    for (int slot = 0; slot < j.n_slot; ++slot) {
      if (!j.need[slot]) continue;
      const double w = slot_weight(j, slot, p);
      if (w != 0.0) g += j.slot_sum[slot] * w;
    }
    j.grad[p] += g;
  }
}

int adj_run(const KArgs& a, const AArgs& j, int tangents, uint32_t km, bool resident,
            int64_t blocks, hipStream_t stream) {
  AdjFn fn = resident ? (tangents == 4 ? select_adj4r(km) : select_adj2r(km))
                      : (tangents == 4 ? select_adj4(km) : select_adj2(km));
  if (!fn) return ORT_ERR_ARG;
  if (hipMemsetAsync(j.partial, 0, (size_t)j.n_slot * (size_t)j.n_wave * sizeof(double),
                     stream) != hipSuccess)
    return ORT_ERR_LAUNCH;
  hipLaunchKernelGGL(adj_need_kernel, dim3((unsigned)((j.n_slot + kBlock - 1) / kBlock)),
                     dim3(kBlock), 0, stream, j);
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(kBlock), 0, stream, a, j);
  hipLaunchKernelGGL(adj_reduce_kernel, dim3((unsigned)j.n_slot), dim3(kBlock), 0, stream, j);
  hipLaunchKernelGGL(adj_contract_kernel, dim3(1), dim3(kBlock), 0, stream, j);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

}  // namespace ortk
