// ort_k_trace.hip -- Newton-lens trace kernels without per-surface records (32 specialisations)
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_kernels.h"

namespace ortk {
template <uint32_t FEAT>
KernelFn pick() {
  return trace_kernel<FEAT>;
}

KernelFn select_trace_rec(uint32_t feat);  // ort_k_trace_rec.hip

KernelFn select_trace(uint32_t feat) {
  if (feat & F_TAPE) return select_trace_tape(feat);
  if (feat & F_WRAY) return select_trace_w(feat);
  if (feat & F_MONO) {
    // scalar optics loads: instantiated for generated rays without records (the pupil
    // traces); other combinations read the rows per lane
    if ((feat & ~(F_KM | F_MONO)) == F_GEN) return select_trace_mono(feat);
    feat &= ~F_MONO;
  }
  if (feat & F_REC) return select_trace_rec(feat);
  switch (feat) {
#define ORT_CASE(F) \
  case (F):         \
    return pick<(F)>();
#define ORT_CASES(G) ORT_CASE(G | 0) ORT_CASE(G | 1) ORT_CASE(G | 2) ORT_CASE(G | 3) \
    ORT_CASE(G | 4) ORT_CASE(G | 5) ORT_CASE(G | 6) ORT_CASE(G | 7) ORT_CASE(G | 8)  \
    ORT_CASE(G | 9) ORT_CASE(G | 10) ORT_CASE(G | 11) ORT_CASE(G | 12) ORT_CASE(G | 13) \
    ORT_CASE(G | 14) ORT_CASE(G | 15)
    ORT_CASES(0)
    ORT_CASES(F_GEN)
#undef ORT_CASES
#undef ORT_CASE
    default:
      return nullptr;
  }
}

}  // namespace ortk
