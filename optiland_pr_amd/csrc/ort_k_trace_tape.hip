// ort_k_trace_tape.hip -- Newton-lens trace kernels on generated rays that write the
// adjoint tape as they trace (F_TAPE, ort_options.tape): the forward of a differentiable
// trace, whose backward (ort_trace_pupil_vjp with ort_vjp_params.tape) then runs the
// reverse sweep only. 30 specialisations (kernel templates: ort_kernels.h), plus the
// single-wavelength ones with the rms spot size's rows in the epilogue (F_RMS, ort_reduce.h)
// and their verify-round forms (F_STRIDE: a grid of kVerifyGrid workgroups).

#include "ort_reduce.h"

namespace ortk {

KernelFn select_trace_tape(uint32_t feat) {
  switch (feat) {
#define ORT_CASE(K) \
  case (F_TAPE | F_GEN | F_MONO | (K)): \
    return trace_kernel<F_TAPE | F_GEN | F_MONO | (K)>; \
  case (F_TAPE | F_GEN | (K)): \
    return trace_kernel<F_TAPE | F_GEN | (K)>; \
  case (F_TAPE | F_GEN | F_MONO | F_RMS | (K)): \
    return trace_kernel<F_TAPE | F_GEN | F_MONO | F_RMS | (K)>; \
  case (F_STRIDE | F_TAPE | F_GEN | F_MONO | (K)): \
    return trace_kernel<F_STRIDE | F_TAPE | F_GEN | F_MONO | (K)>; \
  case (F_STRIDE | F_TAPE | F_GEN | F_MONO | F_RMS | (K)): \
    return trace_kernel<F_STRIDE | F_TAPE | F_GEN | F_MONO | F_RMS | (K)>;
    ORT_CASE(1) ORT_CASE(2) ORT_CASE(3) ORT_CASE(4) ORT_CASE(5) ORT_CASE(6) ORT_CASE(7)
    ORT_CASE(8) ORT_CASE(9) ORT_CASE(10) ORT_CASE(11) ORT_CASE(12) ORT_CASE(13) ORT_CASE(14)
    ORT_CASE(15)
#undef ORT_CASE
    default:
      return nullptr;
  }
}

}  // namespace ortk
