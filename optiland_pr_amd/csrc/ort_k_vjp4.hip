// ort_k_vjp4.hip -- autograd VJP kernels with 4 tangent(s) per launch
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {
VjpFn select_vjp4(uint32_t km) {
  constexpr int P = 4;
  using namespace ort;
  switch (km) {
#define ORT_V(K) \
  case (K):      \
    return vjp_kernel<P, (K)>;
    ORT_V(KM_ZERN) ORT_V(KM_ZERN | KM_EVEN) ORT_V(KM_ZERN | KM_ODD)
    ORT_V(KM_ZERN | KM_EVEN | KM_ODD) ORT_V(KM_ZERN | KM_FREE)
    ORT_V(KM_ZERN | KM_FREE | KM_EVEN) ORT_V(KM_ZERN | KM_FREE | KM_ODD)
    ORT_V(KM_ZERN | KM_FREE | KM_EVEN | KM_ODD)
#undef ORT_V
    default: return nullptr;
  }
}

}  // namespace ortk
