// ort_k_wavefront.hip -- the chief-ray wavefront of one (field, wavelength) on the device
// (wavefront/strategy.py:68-239 ChiefRayStrategy, wavefront/opd.py:143-157 rms,
// wavefront/wavefront.py:97-143 fit_and_remove_tilt's normal equations).
//
// wavefront_opd_kernel, one ray per thread, the reference's elementwise chain in its
// operation order (-ffp-contract=off):
//   ray -> reference-sphere distance from the image plane (_opd_image_to_xp, :68-116:
//   the quadratic with L, M, N reversed, d < 0 clamped to 0, the far root when the near
//   one is negative) -> opd = ray opd - n_image t -> + the launch-plane tilt for angle
//   fields (_correct_tilt, :118-166) -> opd_wv = (opd_ref - opd) / (lambda 1e-3) and the
//   exit-pupil point (x, y, z) - t (L, M, N) (:226-234);
// plus per-block partials of the OPD rms over i > 0 and of the tilt fit's weighted sums,
// reduced in index order by wavefront_final_kernel (deterministic, no atomics).

#include "ort_reduce.h"

namespace ortk {
namespace {

constexpr int kWfSums = 11;  // count(i > 0), sum opd^2 (i > 0), sum w, wx, wy, wxx, wxy,
                             // wyy, w opd, wx opd, wy opd (w = intensity)

struct WfArgs {
  ort_rays rays;
  const double* px;
  const double* py;
  int64_t n;
  ort_wavefront_ref ref;
  double* opd_wv;
  double* pupil_x;
  double* pupil_y;
  double* pupil_z;
  double* part;  // [n_blocks][kWfSums]
  int32_t n_blocks;
  double* sums;  // [kWfSums]
};

__global__ __launch_bounds__(kRedThreads) void wavefront_opd_kernel(const WfArgs a) {
  const int64_t r = (int64_t)blockIdx.x * kRedThreads + threadIdx.x;
  double v[kWfSums];
#pragma unroll
  for (int k = 0; k < kWfSums; ++k) v[k] = 0.0;
  if (r < a.n) {
    const ort_wavefront_ref& q = a.ref;
    const double xr = a.rays.x[r], yr = a.rays.y[r], zr = a.rays.z[r];
    const double L = -a.rays.L[r], M = -a.rays.M[r], N = -a.rays.N[r];
    // strategy.py:94-116
    const double aa = L * L + M * M + N * N;
    const double b = 2.0 * (L * (xr - q.xc) + M * (yr - q.yc) + N * (zr - q.zc));
    const double c = xr * xr + yr * yr + zr * zr - 2.0 * (xr * q.xc + yr * q.yc + zr * q.zc) +
                     q.xc2 + q.yc2 + q.zc2 - q.r2;
    double d = b * b - 4.0 * aa * c;
    d = d < 0.0 ? 0.0 : d;
    double t = (-b - ::sqrt(d)) / (2.0 * aa);
    if (t < 0.0) t = (-b + ::sqrt(d)) / (2.0 * aa);
    const double opd_img = q.n_image * t;
    double opd = a.rays.opd[r] - opd_img;
    if (q.tilt) {  // strategy.py:150-166 (angle fields)
      const double X = a.px[r] * q.epd / 2.0;
      const double Y = a.py[r] * q.epd / 2.0;
      opd = opd + (q.ux * X + q.uy * Y);
    }
    const double wv = (q.opd_ref - opd) / q.wl_mm;  // strategy.py:226
    const double tp = opd_img / q.n_image;           // :227-230
    const double xp = xr - tp * a.rays.L[r];
    const double yp = yr - tp * a.rays.M[r];
    a.opd_wv[r] = wv;
    if (a.pupil_x) a.pupil_x[r] = xp;
    if (a.pupil_y) a.pupil_y[r] = yp;
    if (a.pupil_z) a.pupil_z[r] = zr - tp * a.rays.N[r];
    const double w = a.rays.i[r];
    if (w > 0.0) {  // opd.py:151-157
      v[0] = 1.0;
      v[1] = wv * wv;
    }
    v[2] = w;  // wavefront.py:116-131 (the reference weights every ray, i = 0 ones by 0)
    v[3] = w * xp;
    v[4] = w * yp;
    v[5] = w * xp * xp;
    v[6] = w * xp * yp;
    v[7] = w * yp * yp;
    v[8] = w * wv;
    v[9] = w * xp * wv;
    v[10] = w * yp * wv;
  }
  __shared__ double lds[4 * kWfSums];
  block_sum<kWfSums>(v, lds);
  if (threadIdx.x == 0) {
    double* p = a.part + (int64_t)blockIdx.x * kWfSums;
#pragma unroll
    for (int k = 0; k < kWfSums; ++k) p[k] = v[k];
  }
}

__global__ __launch_bounds__(kRedThreads) void wavefront_final_kernel(const WfArgs a) {
  __shared__ double lds[4 * kWfSums];
  double v[kWfSums];
  reduce_rows_n<kWfSums>(a.part, a.n_blocks, v, lds);
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < kWfSums; ++k) a.sums[k] = v[k];
}

}  // namespace
}  // namespace ortk

using namespace ortk;

extern "C" {

int64_t ort_wavefront_workspace_size(int64_t n) {
  if (n < 0) return ORT_ERR_ARG;
  const int64_t blocks = n > 0 ? (n + kRedThreads - 1) / kRedThreads : 1;
  return blocks * kWfSums * (int64_t)sizeof(double);
}

int ort_wavefront_opd(const ort_rays* rays, const double* px, const double* py, int64_t n,
                      const ort_wavefront_ref* ref, double* opd_wv, double* pupil_x,
                      double* pupil_y, double* pupil_z, void* workspace,
                      int64_t workspace_size, double* sums, void* stream) {
  if (!rays || !ref || !sums || n < 0) return ORT_ERR_ARG;
  const int64_t need = ort_wavefront_workspace_size(n);
  if (!workspace || workspace_size < need) return ORT_ERR_ARG;
  if (n > 0 && (!rays->x || !rays->y || !rays->z || !rays->L || !rays->M || !rays->N ||
                !rays->i || !rays->opd || !opd_wv))
    return ORT_ERR_ARG;
  if (n > 0 && ref->tilt && (!px || !py)) return ORT_ERR_ARG;
  const int64_t blocks = n > 0 ? (n + kRedThreads - 1) / kRedThreads : 1;
  if (blocks > 0x7fffffff) return ORT_ERR_ARG;
  WfArgs a{};
  a.rays = *rays;
  a.px = px;
  a.py = py;
  a.n = n;
  a.ref = *ref;
  a.opd_wv = opd_wv;
  a.pupil_x = pupil_x;
  a.pupil_y = pupil_y;
  a.pupil_z = pupil_z;
  a.part = (double*)workspace;
  a.n_blocks = (int32_t)blocks;
  a.sums = sums;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(wavefront_opd_kernel, dim3((unsigned)blocks), dim3(kRedThreads), 0, s, a);
  hipLaunchKernelGGL(wavefront_final_kernel, dim3(1), dim3(kRedThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

}  // extern "C"
