// ort_k_trace_mono.hip -- Newton-lens trace kernels on generated rays whose wavelength row
// is wave-uniform (F_MONO: the optical tables through scalar loads), 15 specialisations
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {

KernelFn select_trace_mono(uint32_t feat) {
  switch (feat) {
#define ORT_CASE(K) \
  case (F_GEN | F_MONO | (K)): \
    return trace_kernel<F_GEN | F_MONO | (K)>;
    ORT_CASE(1) ORT_CASE(2) ORT_CASE(3) ORT_CASE(4) ORT_CASE(5) ORT_CASE(6) ORT_CASE(7)
    ORT_CASE(8) ORT_CASE(9) ORT_CASE(10) ORT_CASE(11) ORT_CASE(12) ORT_CASE(13) ORT_CASE(14)
    ORT_CASE(15)
#undef ORT_CASE
    default:
      return nullptr;
  }
}

}  // namespace ortk
