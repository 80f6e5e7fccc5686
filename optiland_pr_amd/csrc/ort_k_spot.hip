// ort_k_spot.hip -- spot-diagram statistics on the device (analysis/spot_diagram.py:
// 317-357 centroid / geometric / rms radius, over the i > 0 points of :425-437 taken into
// the image surface frame), so a SpotDiagram's numbers leave HBM as a few doubles per
// (field, wavelength) pair instead of as masked ray arrays.
//
// Two passes, each a partial-sum kernel over fixed 2048-ray chunks of one pair followed
// by a one-block-per-pair kernel that reduces the chunk partials in index order: the
// result is deterministic (bit-identical run to run). Pass 1: count, sum x, sum y ->
// centroids; pass 2: sum and max of (x - cx)^2 + (y - cy)^2 about the centroid of the
// field's reference-wavelength pair. NaN points propagate as in NumPy (the sums carry
// them; the max takes an explicit NaN flag, since fmax would drop it).

#include "ort_kernels.h"

namespace ortk {
namespace {

constexpr int kSpotThreads = 256;
constexpr int kSpotPerThread = 8;
constexpr int64_t kSpotChunk = (int64_t)kSpotThreads * kSpotPerThread;

struct SpotArgs {
  const double* x;
  const double* y;
  const double* z;
  const double* i;
  int64_t n_pupil;
  int32_t n_wl;
  int32_t ref_wl;
  int32_t n_ops;
  const ort_cs_op* ops;
  int32_t n_chunks;  // chunks per pair
  double* part;      // [n_pairs][n_chunks][3]
  double* cent;      // [n_pairs][2]
  double* out;       // [n_pairs][5]
};

// one image point in the surface frame (visualization/system/utils.py:16-46: the point
// as a ray with zero direction, localized by the surface's coordinate system)
__device__ inline void local_point(const SpotArgs& a, int64_t r, double& x, double& y) {
  ort::Ray p;
  p.x = a.x[r];
  p.y = a.y[r];
  p.z = a.z[r];
  p.L = 0.0; p.M = 0.0; p.N = 0.0;
  for (int k = 0; k < a.n_ops; ++k) ort::apply_cs_op(p, cst(a.ops)[k]);
  x = p.x;
  y = p.y;
}

template <int NV>
__device__ inline void block_sum(double (&v)[NV], double* lds) {
#pragma unroll
  for (int k = 0; k < NV; ++k)
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0.0;
    for (int ww = 0; ww < kSpotThreads / 64; ++ww) s += lds[ww * NV + k];
    v[k] = s;
  }
}

// pass 1 / 2 partials of one chunk
template <int PASS>
__global__ __launch_bounds__(kSpotThreads) void spot_partial_kernel(const SpotArgs a) {
  const int64_t pair = blockIdx.y;
  const int64_t c0 = (int64_t)blockIdx.x * kSpotChunk;
  const int64_t base = pair * a.n_pupil;
  double v[3] = {0.0, 0.0, 0.0};
  double cx = 0.0, cy = 0.0;
  if (PASS == 2) {
    const int64_t ref = (pair / a.n_wl) * a.n_wl + a.ref_wl;
    cx = a.cent[ref * 2 + 0];
    cy = a.cent[ref * 2 + 1];
  }
  for (int k = 0; k < kSpotPerThread; ++k) {
    const int64_t j = c0 + (int64_t)k * kSpotThreads + threadIdx.x;
    if (j >= a.n_pupil) break;
    const int64_t r = base + j;
    if (!(a.i[r] > 0.0)) continue;  // spot_diagram.py:425-427
    double x, y;
    local_point(a, r, x, y);
    if (PASS == 1) {
      v[0] += 1.0;
      v[1] += x;
      v[2] += y;
    } else {
      const double dx = x - cx, dy = y - cy;
      const double r2 = dx * dx + dy * dy;  // x**2 + y**2 of the centred spot
      v[0] += r2;
      const double rad = ::sqrt(r2);
      if (rad != rad) v[2] = 1.0;  // NaN seen
      else if (rad > v[1]) v[1] = rad;
    }
  }
  __shared__ double lds[(kSpotThreads / 64) * 3];
  if (PASS == 1) {
    block_sum<3>(v, lds);
  } else {
    double s[1] = {v[0]};
    block_sum<1>(s, lds);
    __syncthreads();
    // max and NaN flag: wave then block maximum (order-independent)
    double m = v[1], f = v[2];
    for (int o = 32; o > 0; o >>= 1) {
      m = ::fmax(m, __shfl_xor(m, o, 64));
      f = ::fmax(f, __shfl_xor(f, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      lds[w * 2 + 0] = m;
      lds[w * 2 + 1] = f;
    }
    __syncthreads();
    m = 0.0;
    f = 0.0;
    for (int ww = 0; ww < kSpotThreads / 64; ++ww) {
      m = ::fmax(m, lds[ww * 2 + 0]);
      f = ::fmax(f, lds[ww * 2 + 1]);
    }
    v[0] = s[0];
    v[1] = m;
    v[2] = f;
  }
  if (threadIdx.x == 0) {
    double* p = a.part + (pair * a.n_chunks + blockIdx.x) * 3;
    p[0] = v[0];
    p[1] = v[1];
    p[2] = v[2];
  }
}

// reduce the chunk partials of one pair in index order
template <int PASS>
__global__ __launch_bounds__(kSpotThreads) void spot_final_kernel(const SpotArgs a) {
  const int64_t pair = blockIdx.x;
  const double* p = a.part + pair * a.n_chunks * 3;
  __shared__ double lds[(kSpotThreads / 64) * 3];
  if (PASS == 1) {
    double v[3] = {0.0, 0.0, 0.0};
    for (int c = threadIdx.x; c < a.n_chunks; c += kSpotThreads) {
      v[0] += p[c * 3 + 0];
      v[1] += p[c * 3 + 1];
      v[2] += p[c * 3 + 2];
    }
    block_sum<3>(v, lds);
    if (threadIdx.x == 0) {
      const double n = v[0];
      const double cx = v[1] / n, cy = v[2] / n;  // be.mean: sum / count (0 / 0 = NaN)
      a.cent[pair * 2 + 0] = cx;
      a.cent[pair * 2 + 1] = cy;
      a.out[pair * 5 + 0] = n;
      a.out[pair * 5 + 1] = cx;
      a.out[pair * 5 + 2] = cy;
    }
  } else {
    double s[1] = {0.0};
    double m = 0.0, f = 0.0;
    for (int c = threadIdx.x; c < a.n_chunks; c += kSpotThreads) {
      s[0] += p[c * 3 + 0];
      m = ::fmax(m, p[c * 3 + 1]);
      f = ::fmax(f, p[c * 3 + 2]);
    }
    block_sum<1>(s, lds);
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) {
      m = ::fmax(m, __shfl_xor(m, o, 64));
      f = ::fmax(f, __shfl_xor(f, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      lds[w * 2 + 0] = m;
      lds[w * 2 + 1] = f;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int ww = 0; ww < kSpotThreads / 64; ++ww) {
        m = ::fmax(m, lds[ww * 2 + 0]);
        f = ::fmax(f, lds[ww * 2 + 1]);
      }
      const double n = a.out[pair * 5 + 0];
      const bool nan = f != 0.0 || s[0] != s[0];
      a.out[pair * 5 + 3] = ::sqrt(s[0] / n);  // be.sqrt(be.mean(x**2 + y**2))
      a.out[pair * 5 + 4] = (nan || n == 0.0) ? __builtin_nan("") : m;  // be.max
    }
  }
}

}  // namespace
}  // namespace ortk

using namespace ortk;

extern "C" {

int64_t ort_spot_workspace_size(const ort_spot_layout* lay) {
  if (!lay || lay->n_pupil < 0 || lay->n_fields < 0 || lay->n_wl < 1) return ORT_ERR_ARG;
  const int64_t pairs = (int64_t)lay->n_fields * lay->n_wl;
  const int64_t chunks = lay->n_pupil > 0 ? (lay->n_pupil + kSpotChunk - 1) / kSpotChunk : 1;
  return (pairs * chunks * 3 + pairs * 2) * (int64_t)sizeof(double);
}

int ort_spot_stats(const ort_rays* rays, const ort_spot_layout* lay, void* workspace,
                   int64_t workspace_size, double* out, void* stream) {
  if (!rays || !lay || !out) return ORT_ERR_ARG;
  const int64_t need = ort_spot_workspace_size(lay);
  if (need < 0) return (int)need;
  if (lay->ref_wl < 0 || lay->ref_wl >= lay->n_wl) return ORT_ERR_ARG;
  if (lay->n_local_ops < 0 || (lay->n_local_ops > 0 && !lay->local_ops)) return ORT_ERR_ARG;
  const int64_t pairs = (int64_t)lay->n_fields * lay->n_wl;
  if (pairs == 0) return ORT_OK;
  if (!workspace || workspace_size < need) return ORT_ERR_ARG;
  if (lay->n_pupil > 0 && (!rays->x || !rays->y || !rays->z || !rays->i)) return ORT_ERR_ARG;
  const int64_t chunks = lay->n_pupil > 0 ? (lay->n_pupil + kSpotChunk - 1) / kSpotChunk : 1;
  if (chunks > 0x7fffffff || pairs > 65535) return ORT_ERR_ARG;
  SpotArgs a{};
  a.x = rays->x;
  a.y = rays->y;
  a.z = rays->z;
  a.i = rays->i;
  a.n_pupil = lay->n_pupil;
  a.n_wl = lay->n_wl;
  a.ref_wl = lay->ref_wl;
  a.n_ops = lay->n_local_ops;
  a.ops = lay->local_ops;
  a.n_chunks = (int32_t)chunks;
  a.part = (double*)workspace;
  a.cent = a.part + pairs * chunks * 3;
  a.out = out;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)chunks, (unsigned)pairs);
  hipLaunchKernelGGL(spot_partial_kernel<1>, grid, dim3(kSpotThreads), 0, s, a);
  hipLaunchKernelGGL(spot_final_kernel<1>, dim3((unsigned)pairs), dim3(kSpotThreads), 0, s, a);
  hipLaunchKernelGGL(spot_partial_kernel<2>, grid, dim3(kSpotThreads), 0, s, a);
  hipLaunchKernelGGL(spot_final_kernel<2>, dim3((unsigned)pairs), dim3(kSpotThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

}  // extern "C"
