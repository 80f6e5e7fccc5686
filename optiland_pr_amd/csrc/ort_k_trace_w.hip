// ort_k_trace_w.hip -- Newton-lens trace kernels for rays with per-ray wavelengths
// (F_WRAY: n and k from lens.materials per ray; 30 specialisations)
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {
template <uint32_t FEAT>
KernelFn pick_w() {
  return trace_kernel<FEAT>;
}

KernelFn select_trace_w(uint32_t feat) {
  switch (feat) {
#define ORT_CASE(F) \
  case (F):         \
    return pick_w<(F)>();
#define ORT_CASES(G) ORT_CASE(G | 1) ORT_CASE(G | 2) ORT_CASE(G | 3) \
    ORT_CASE(G | 4) ORT_CASE(G | 5) ORT_CASE(G | 6) ORT_CASE(G | 7) ORT_CASE(G | 8)  \
    ORT_CASE(G | 9) ORT_CASE(G | 10) ORT_CASE(G | 11) ORT_CASE(G | 12) ORT_CASE(G | 13) \
    ORT_CASE(G | 14) ORT_CASE(G | 15)
    ORT_CASES(F_WRAY)
    ORT_CASES(F_WRAY | F_REC)
#undef ORT_CASES
#undef ORT_CASE
    default:
      return nullptr;
  }
}

}  // namespace ortk
