// ort_k_vjp.hip -- VJP kernel selection by tangent count
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {
VjpFn select_vjp1(uint32_t km);
VjpFn select_vjp2(uint32_t km);
VjpFn select_vjp4(uint32_t km);

VjpFn select_vjp(int tangents, uint32_t km) {
  switch (tangents) {
    case 1: return select_vjp1(km);
    case 2: return select_vjp2(km);
    case 4: return select_vjp4(km);
    default: return nullptr;
  }
}

VjpReduceFn select_vjp_reduce(int tangents) {
  switch (tangents) {
    case 1: return vjp_reduce_kernel<1>;
    case 2: return vjp_reduce_kernel<2>;
    case 4: return vjp_reduce_kernel<4>;
    default: return nullptr;
  }
}

}  // namespace ortk
