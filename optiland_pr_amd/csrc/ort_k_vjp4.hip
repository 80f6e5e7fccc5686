// ort_k_vjp4.hip -- autograd VJP kernels (16 Newton-kind specialisations) with 4 tangent(s) per launch
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {
VjpFn select_vjp4(uint32_t km) {
  constexpr int P = 4;
  switch (km) {
#define ORT_V(K) \
  case (K):      \
    return vjp_kernel<P, (K)>;
    ORT_V(0) ORT_V(1) ORT_V(2) ORT_V(3) ORT_V(4) ORT_V(5) ORT_V(6) ORT_V(7)
    ORT_V(8) ORT_V(9) ORT_V(10) ORT_V(11) ORT_V(12) ORT_V(13) ORT_V(14) ORT_V(15)
#undef ORT_V
    default: return nullptr;
  }
}

}  // namespace ortk
