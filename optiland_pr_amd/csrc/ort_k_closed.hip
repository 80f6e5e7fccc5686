// ort_k_closed.hip -- closed-form-lens kernels and the generation-only kernel
// (kernel templates: ort_kernels.h; compiled as its own translation unit)

#include "ort_reduce.h"

namespace ortk {
__global__ __launch_bounds__(kBlock) void generate_kernel(const KArgs a) {
  const int64_t rid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (rid >= a.n_rays) return;
  const int64_t sidx = rid / a.seg_len;
  const ort_segment sg = a.seg[sidx];
  const int64_t p = a.pupil_per_ray ? rid : (rid - sidx * a.seg_len);
  const ort::Ray r = ort::generate_ray(sg, a.px[p], a.py[p], a.apod);
  a.out.x[rid] = r.x;
  a.out.y[rid] = r.y;
  a.out.z[rid] = r.z;
  a.out.L[rid] = r.L;
  a.out.M[rid] = r.M;
  a.out.N[rid] = r.N;
  a.out.i[rid] = r.i;
  a.out.opd[rid] = r.opd;
}

KernelFn select_generate() { return generate_kernel; }

__global__ __launch_bounds__(kBlock) void material_nk_kernel(const ort_material* mats,
                                                             const double* coef, int32_t mat,
                                                             const double* w, int64_t n,
                                                             double* n_out, double* k_out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const ort_material m = mats[mat];
  const double wi = w[i];
  if (n_out) n_out[i] = ort::material_n(m, coef, wi);
  if (k_out) k_out[i] = ort::material_k(m, coef, wi);
}

void launch_material_nk(const ort_material* mats, const double* coef, int32_t mat,
                        const double* w, int64_t n, double* n_out, double* k_out,
                        hipStream_t stream) {
  const int64_t blocks = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(material_nk_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     mats, coef, mat, w, n, n_out, k_out);
}

int closed_block() { return kClosedBlock; }

KernelFn select_closed(uint32_t feat) {
#ifdef ORT_NO_AXIAL  // A/B timing only
  feat &= ~F_AXIAL;
#endif
  switch (feat & (F_GEN | F_REC | F_MONO | F_WRAY | F_AXIAL | F_SPOT)) {
#define ORT_C(F) \
  case (F):      \
    return trace_closed_kernel<(F)>;        \
  case (F) | F_AXIAL:                       \
    return trace_closed_kernel<(F) | F_AXIAL>;
    ORT_C(0) ORT_C(F_GEN) ORT_C(F_REC) ORT_C(F_GEN | F_REC)
    ORT_C(F_MONO) ORT_C(F_MONO | F_GEN) ORT_C(F_MONO | F_REC) ORT_C(F_MONO | F_GEN | F_REC)
    ORT_C(F_WRAY) ORT_C(F_WRAY | F_REC)
    ORT_C(F_GEN | F_SPOT) ORT_C(F_MONO | F_GEN | F_SPOT)
#undef ORT_C
    default: return nullptr;
  }
}

}  // namespace ortk
