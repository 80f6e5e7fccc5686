// ort_k_geom.hip -- per-geometry primitive kernels (16 Newton-kind specialisations, and
// one with every kind and the NURBS solves)
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {
GeomFn select_geom(uint32_t km) {
  if (km & ort::KM_NURBS) return geom_kernel<15u | ort::KM_NURBS>;  // NURBS: every kind
  switch (km) {
#define ORT_G(K) \
  case (K):      \
    return geom_kernel<(K)>;
    ORT_G(0) ORT_G(1) ORT_G(2) ORT_G(3) ORT_G(4) ORT_G(5) ORT_G(6) ORT_G(7)
    ORT_G(8) ORT_G(9) ORT_G(10) ORT_G(11) ORT_G(12) ORT_G(13) ORT_G(14)
#undef ORT_G
    default: return geom_kernel<15>;
  }
}

}  // namespace ortk
