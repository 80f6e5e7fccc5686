// ort_k_adj4r.hip -- adjoint VJP kernels of resident-ray traces (ort_trace_sequential_vjp), 4-tangent local duals
// (16 Newton-kind specialisations; kernel template: ort_adjoint.h)

#include "ort_adjoint.h"

namespace ortk {
AdjFn select_adj4r(uint32_t km) {
  switch (km) {
#define ORT_A(K) \
  case (K):      \
    return adj_kernel<(K), 4, true>;
    ORT_A(0) ORT_A(1) ORT_A(2) ORT_A(3) ORT_A(4) ORT_A(5) ORT_A(6) ORT_A(7)
    ORT_A(8) ORT_A(9) ORT_A(10) ORT_A(11) ORT_A(12) ORT_A(13) ORT_A(14) ORT_A(15)
#undef ORT_A
    default: return nullptr;
  }
}

}  // namespace ortk
