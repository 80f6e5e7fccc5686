// ort_k_trace_ia.hip -- trace kernels for lenses with thin-lens, phase or grating
// surfaces (F_IA; every Newton kind compiled in, 6 specialisations), and the same six with
// the NURBS solves (KM_NURBS) for lenses that have NURBS surfaces
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {

KernelFn select_trace_ia(uint32_t feat) {
  constexpr uint32_t kAll = 15u;  // every Newton kind
  if (feat & ort::KM_NURBS) {  // lenses with NURBS surfaces (ort_sweep.h fill_args)
    switch (feat & (F_GEN | F_REC | F_WRAY)) {
#define ORT_C(F) \
  case (F):      \
    return trace_kernel<F_IA | kAll | ort::KM_NURBS | (F)>;
      ORT_C(0) ORT_C(F_GEN) ORT_C(F_REC) ORT_C(F_GEN | F_REC) ORT_C(F_WRAY) ORT_C(F_WRAY | F_REC)
#undef ORT_C
      default:
        return nullptr;
    }
  }
  switch (feat & (F_GEN | F_REC | F_WRAY)) {
#define ORT_C(F) \
  case (F):      \
    return trace_kernel<F_IA | kAll | (F)>;
    ORT_C(0) ORT_C(F_GEN) ORT_C(F_REC) ORT_C(F_GEN | F_REC) ORT_C(F_WRAY) ORT_C(F_WRAY | F_REC)
#undef ORT_C
    default:
      return nullptr;
  }
}

}  // namespace ortk
