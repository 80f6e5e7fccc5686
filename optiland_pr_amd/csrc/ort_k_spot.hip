// ort_k_spot.hip -- spot-diagram statistics on the device (analysis/spot_diagram.py:
// 317-357 centroid / geometric / rms radius, over the i > 0 points of :425-437 taken into
// the image surface frame), so a SpotDiagram's numbers leave HBM as a few doubles per
// (field, wavelength) pair instead of as masked ray arrays.
//
// Two kernels over fixed chunks of one pair (<= 256 chunks per pair: one ray per thread
// for a small spot diagram, so it still spreads over many CUs, several for a large one):
//   spot_sum_kernel    count, sum x, sum y of the chunk -> part1[pair][chunk]
//   spot_dev_kernel    the centroid of the field's reference-wavelength pair, reduced by
//                      every block from part1 in index order (<= 768 doubles,
//                      L2-resident), then sum and max of (x - cx)^2 + (y - cy)^2 over the
//                      chunk -> part2[pair][chunk]
//   spot_final_kernel  one block per pair: the pair's partials in index order -> out[pair]
// Every reduction runs in a fixed order, so the result is bit-identical run to run (no
// atomics: kernel boundaries order the passes, no cross-block fence). NaN points
// propagate as in NumPy (the sums carry them; the max keeps an explicit NaN flag, since
// fmax would drop it). Measured and dropped: spot_final as the last block of
// spot_dev_kernel to arrive (a per-pair atomic count with agent-scope release / acquire):
// 8.8 us for that kernel vs 4.5 + 3.9 us for the two -- every block's release writes back
// its L2 and the final reduction still runs after the last arrival.
//
// Each pass issues its per-ray loads before the reduction of the previous pass's
// partials, so the two memory round trips overlap.

#include "ort_reduce.h"

namespace ortk {
namespace {

constexpr int kSpotThreads = kRedThreads;
constexpr int64_t kSpotMaxChunks = 256;  // chunks per pair at most: a chunk is 256 rays
                                         // times ceil(n_pupil / (256 * 256)) per thread
// ort_rms_spot (one pair, 1M points in config 5): more, shorter chunks -- 256 blocks of 16
// points per thread leave the two passes latency-bound; every pass-2 block re-reduces the
// pass-1 rows (24 B per chunk), so the count stays moderate. ORT_RMS_CHUNKS: A/B builds.
#ifndef ORT_RMS_CHUNKS
#define ORT_RMS_CHUNKS 1024
#endif
constexpr int64_t kRmsMaxChunks = ORT_RMS_CHUNKS;

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
  int32_t n_chunks;     // chunks per pair
  int32_t per_thread;   // rays per thread (chunk = per_thread * 256 rays)
  double* part1;        // [n_pairs][n_chunks][3]: count, sum x, sum y
  double* part2;        // [n_pairs][n_chunks][3]: sum r^2, max r, NaN flag
  double* out;          // [n_pairs][5] (ort_spot_partials: [n_pairs][3])
  // ort_spot_partials phase 2: the pairs' (count, sum x, sum y) reduced over every rank;
  // the centroids come from these instead of this rank's part1
  const double* gsum;
  double* rms_out;      // ort_rms_spot: the rms radius of pair 0 again, as its own scalar
};

// one image point in the surface frame (visualization/system/utils.py:16-46: the point
// as a ray with zero direction, localized by the surface's coordinate system)
__device__ inline void local_point(const SpotArgs& a, int64_t r, double& x, double& y) {
  ort::Ray p;
  p.x = a.x[r];
  p.y = a.y[r];
  p.z = a.n_ops ? a.z[r] : 0.0;
  p.L = 0.0; p.M = 0.0; p.N = 0.0;
  for (int k = 0; k < a.n_ops; ++k) ort::apply_cs_op(p, cst(a.ops)[k]);
  x = p.x;
  y = p.y;
}

// the same for a point already loaded (x, y, z)
__device__ inline void local_xyz(const SpotArgs& a, double x, double y, double z, double& ox,
                                 double& oy) {
  ort::Ray p;
  p.x = x;
  p.y = y;
  p.z = a.n_ops ? z : 0.0;
  p.L = 0.0; p.M = 0.0; p.N = 0.0;
  for (int k = 0; k < a.n_ops; ++k) ort::apply_cs_op(p, cst(a.ops)[k]);
  ox = p.x;
  oy = p.y;
}

// A thread's rays j0 + k * 256 (k < per_thread, j < n_pupil) of a chunk, visited in k
// order, their loads issued four rays at a time ahead of the use (the intensity test no
// longer gates the coordinate loads): fn(x, y) for each point with i > 0 (every point
// when i is NULL), in the same order as the one-ray-at-a-time loop.
template <class F>
__device__ inline void chunk_points(const SpotArgs& a, int64_t pair, int64_t j0, F&& fn) {
  for (int k0 = 0; k0 < a.per_thread; k0 += 4) {
    double xs[4], ys[4], zs[4], is[4];
    bool in[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = j0 + (int64_t)(k0 + u) * kSpotThreads;
      in[u] = k0 + u < a.per_thread && j < a.n_pupil;
      const int64_t r = pair * a.n_pupil + (in[u] ? j : 0);
      is[u] = (in[u] && a.i) ? a.i[r] : 1.0;
      xs[u] = in[u] ? a.x[r] : 0.0;
      ys[u] = in[u] ? a.y[r] : 0.0;
      zs[u] = (in[u] && a.n_ops) ? a.z[r] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (in[u] && is[u] > 0.0) {  // spot_diagram.py:425-427
        double x, y;
        local_xyz(a, xs[u], ys[u], zs[u], x, y);
        fn(x, y);
      }
    }
  }
}

// sums of the 3 columns of part[0 .. n) (index-strided per thread, then block_sum)
__device__ inline void reduce_rows(const double* part, int n, double (&v)[3], double* lds) {
  v[0] = v[1] = v[2] = 0.0;
  for (int c = threadIdx.x; c < n; c += kSpotThreads) {
    v[0] += part[c * 3 + 0];
    v[1] += part[c * 3 + 1];
    v[2] += part[c * 3 + 2];
  }
  block_sum<3>(v, lds);
}

__global__ __launch_bounds__(kSpotThreads) void spot_sum_kernel(const SpotArgs a) {
  const int64_t pair = blockIdx.y;
  const int64_t j0 = (int64_t)blockIdx.x * a.per_thread * kSpotThreads + threadIdx.x;
  double v[3] = {0.0, 0.0, 0.0};
  chunk_points(a, pair, j0, [&](double x, double y) {
    v[0] += 1.0;
    v[1] += x;
    v[2] += y;
  });
  __shared__ double lds[4 * 3];
  block_sum<3>(v, lds);
  if (threadIdx.x == 0) {
    double* p = a.part1 + (pair * a.n_chunks + blockIdx.x) * 3;
    p[0] = v[0];
    p[1] = v[1];
    p[2] = v[2];
  }
}

__global__ __launch_bounds__(kSpotThreads) void spot_dev_kernel(const SpotArgs a) {
  const int64_t pair = blockIdx.y;
  __shared__ double lds[4 * 3];
  // one ray per thread: its point is loaded before the centroid's reduction below, so the
  // two memory round trips overlap (same arithmetic as the loop further down)
  bool on = false;
  double px = 0.0, py = 0.0;
  if (a.per_thread == 1) {
    const int64_t j = (int64_t)blockIdx.x * kSpotThreads + threadIdx.x;
    if (j < a.n_pupil) {
      const int64_t r = pair * a.n_pupil + j;
      on = !a.i || a.i[r] > 0.0;
      if (on) local_point(a, r, px, py);
    }
  }
  // centroid of the field's reference-wavelength spot (spot_diagram.py:317-328)
  const int64_t ref = (pair / a.n_wl) * a.n_wl + a.ref_wl;
  double c[3];
  if (a.gsum) {
    c[0] = a.gsum[ref * 3 + 0];
    c[1] = a.gsum[ref * 3 + 1];
    c[2] = a.gsum[ref * 3 + 2];
  } else {
    reduce_rows(a.part1 + ref * a.n_chunks * 3, a.n_chunks, c, lds);
  }
  const double cx = c[1] / c[0], cy = c[2] / c[0];

  const int64_t j0 = (int64_t)blockIdx.x * a.per_thread * kSpotThreads + threadIdx.x;
  double s = 0.0, m = 0.0, f = 0.0;
  auto add = [&](double x, double y) {
    const double dx = x - cx, dy = y - cy;
    const double r2 = dx * dx + dy * dy;  // x**2 + y**2 of the centred spot
    s += r2;
    const double rad = ::sqrt(r2);
    if (rad != rad) f = 1.0;  // NaN seen
    else m = ::fmax(m, rad);
  };
  if (a.per_thread == 1) {
    if (on) add(px, py);
  } else {
    chunk_points(a, pair, j0, add);
  }
  double v[1] = {s};
  block_sum<1>(v, lds);
  m = wave_max(m);
  f = wave_max(f);
  __shared__ double mx[4][2];
  if ((threadIdx.x & 63) == 0) {
    mx[threadIdx.x >> 6][0] = m;
    mx[threadIdx.x >> 6][1] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kSpotThreads / 64; ++w) {
      m = ::fmax(m, mx[w][0]);
      f = ::fmax(f, mx[w][1]);
    }
    double* p = a.part2 + (pair * a.n_chunks + blockIdx.x) * 3;
    p[0] = v[0];
    p[1] = m;
    p[2] = f;
  }
}

// one block per pair: the pair's totals, every reduction in index order
__global__ __launch_bounds__(kSpotThreads) void spot_final_kernel(const SpotArgs a) {
  const int64_t pair = blockIdx.x;
  __shared__ double lds[4 * 3];
  __shared__ double mx[4][2];
  double own[3];
  const double* p2 = a.part2 + pair * a.n_chunks * 3;
  double t[1] = {0.0};
  double m = 0.0, f = 0.0;
  // pass-2 partials read before pass 1's reduction (overlapping round trips)
  for (int k = threadIdx.x; k < a.n_chunks; k += kSpotThreads) {
    t[0] += p2[k * 3 + 0];
    m = ::fmax(m, p2[k * 3 + 1]);
    f = ::fmax(f, p2[k * 3 + 2]);
  }
  reduce_rows(a.part1 + pair * a.n_chunks * 3, a.n_chunks, own, lds);
  block_sum<1>(t, lds);
  m = wave_max(m);
  f = wave_max(f);
  if ((threadIdx.x & 63) == 0) {
    mx[threadIdx.x >> 6][0] = m;
    mx[threadIdx.x >> 6][1] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kSpotThreads / 64; ++w) {
      m = ::fmax(m, mx[w][0]);
      f = ::fmax(f, mx[w][1]);
    }
    const double n = own[0];
    double* o = a.out + pair * 5;
    o[0] = n;
    o[1] = own[1] / n;  // be.mean: sum / count (0 / 0 = NaN)
    o[2] = own[2] / n;
    o[3] = ::sqrt(t[0] / n);  // be.sqrt(be.mean(x**2 + y**2))
    o[4] = (f != 0.0 || t[0] != t[0] || n == 0.0) ? __builtin_nan("") : m;  // be.max
    if (a.rms_out && pair == 0) *a.rms_out = o[3];
  }
}

// pass 2 + totals. Measured and dropped: both in one workgroup per pair for small pairs
// (each wave forming its chunks' four 64-lane sub-chunk sums in block_sum's order,
// bit-identical to these two kernels): 4 waves with one load round trip per sub-chunk
// 46.9 us, 16 waves with eight sub-chunks' loads in flight per wave 17.3 us, against
// 4.6 + 4.0 us -- three workgroups (three CUs) move and reduce the 38K points slower than
// 150 chunk workgroups plus one extra launch.
void launch_pass2(const SpotArgs& a, int64_t pairs, int64_t chunks, hipStream_t s) {
  hipLaunchKernelGGL(spot_dev_kernel, dim3((unsigned)chunks, (unsigned)pairs), dim3(kSpotThreads),
                     0, s, a);
  hipLaunchKernelGGL(spot_final_kernel, dim3((unsigned)pairs), dim3(kSpotThreads), 0, s, a);
}

// ort_spot_partials: one block per pair, the pair's chunk partials in index order ->
// out[pair][3] (PASS 1: count, sum x, sum y; PASS 2: sum r^2, max r, NaN flag)
template <int PASS>
__global__ __launch_bounds__(kSpotThreads) void spot_pair_kernel(const SpotArgs a) {
  const int64_t pair = blockIdx.x;
  __shared__ double lds[4 * 3];
  __shared__ double mx[4][2];
  double* o = a.out + pair * 3;
  if constexpr (PASS == 1) {
    double v[3];
    reduce_rows(a.part1 + pair * a.n_chunks * 3, a.n_chunks, v, lds);
    if (threadIdx.x == 0) {
      o[0] = v[0];
      o[1] = v[1];
      o[2] = v[2];
    }
  } else {
    const double* p2 = a.part2 + pair * a.n_chunks * 3;
    double t[1] = {0.0};
    double m = 0.0, f = 0.0;
    for (int k = threadIdx.x; k < a.n_chunks; k += kSpotThreads) {
      t[0] += p2[k * 3 + 0];
      m = ::fmax(m, p2[k * 3 + 1]);
      f = ::fmax(f, p2[k * 3 + 2]);
    }
    block_sum<1>(t, lds);
    m = wave_max(m);
    f = wave_max(f);
    if ((threadIdx.x & 63) == 0) {
      mx[threadIdx.x >> 6][0] = m;
      mx[threadIdx.x >> 6][1] = f;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < kSpotThreads / 64; ++w) {
        m = ::fmax(m, mx[w][0]);
        f = ::fmax(f, mx[w][1]);
      }
      o[0] = t[0];
      o[1] = m;
      o[2] = f;
    }
  }
}

// d rms / d (x_i, y_i) = (x_i - mean x, y_i - mean y) / (n rms) times the upstream
// gradient (torch's chain through sqrt, mean and the squares; the mean's own share,
// sum_k (x_k - mean x) / n, is zero up to rounding and dropped)
__global__ __launch_bounds__(kSpotThreads) void rms_spot_vjp_kernel(
    const double* x, const double* y, int64_t n, const double* stats, const double* grad_out,
    double* gx, double* gy) {
  const int64_t i = (int64_t)blockIdx.x * kSpotThreads + threadIdx.x;
  if (i >= n) return;
  const double cx = stats[1], cy = stats[2];
  const double w = *grad_out / (stats[0] * stats[3]);
#ifndef ORT_TEMPORAL_STORE  // written once, read by the trace's VJP launch (ORT_ST's rule)
  __builtin_nontemporal_store((x[i] - cx) * w, &gx[i]);
  __builtin_nontemporal_store((y[i] - cy) * w, &gy[i]);
#else
  gx[i] = (x[i] - cx) * w;
  gy[i] = (y[i] - cy) * w;
#endif
}

// ort_rms_finish: the taped forward's F_RMS rows -> the rms spot size (ort_reduce.h
// rms_finish_block), one workgroup of 256 threads holding up to 16 rows each in registers
// (config 5: 4096 rows, one load round trip) -- the same workgroup shape and order as
// ort_newton_finish_rms's second workgroup, so both give the same bits
constexpr int kFinThreads = kRmsFinThreads;

__global__ __launch_bounds__(kFinThreads) void rms_finish_kernel(const double* part,
                                                                 int n_rows, double* stats,
                                                                 double* rms) {
  __shared__ double lds[kFinThreads / 64 * 3];
  rms_finish_block<kFinThreads, kRmsFinRows>(part, n_rows, stats, rms, lds);
}

}  // namespace
}  // namespace ortk

using namespace ortk;

extern "C" {

// max_chunks: chunks per pair at most (kSpotMaxChunks for the spot diagram's statistics,
// kRmsMaxChunks for ort_rms_spot's one pair of up to millions of points)
static int64_t spot_per_thread(const ort_spot_layout* lay, int64_t max_chunks = kSpotMaxChunks) {
  const int64_t cap = max_chunks * kSpotThreads;
  return lay->n_pupil > cap ? (lay->n_pupil + cap - 1) / cap : 1;
}
static int64_t spot_chunks(const ort_spot_layout* lay, int64_t max_chunks = kSpotMaxChunks) {
  const int64_t chunk = spot_per_thread(lay, max_chunks) * kSpotThreads;
  return lay->n_pupil > 0 ? (lay->n_pupil + chunk - 1) / chunk : 1;
}

static int64_t spot_workspace_size(const ort_spot_layout* lay, int64_t max_chunks) {
  if (!lay || lay->n_pupil < 0 || lay->n_fields < 0 || lay->n_wl < 1) return ORT_ERR_ARG;
  const int64_t pairs = (int64_t)lay->n_fields * lay->n_wl;
  return pairs * spot_chunks(lay, max_chunks) * 3 * 2 * (int64_t)sizeof(double);
}

int64_t ort_spot_workspace_size(const ort_spot_layout* lay) {
  return spot_workspace_size(lay, kSpotMaxChunks);
}

static int spot_args(const ort_rays* rays, const ort_spot_layout* lay, void* workspace,
                     int64_t workspace_size, double* out, SpotArgs& a, int64_t& pairs,
                     int64_t& chunks, int64_t max_chunks = kSpotMaxChunks) {
  if (!rays || !lay || !out) return ORT_ERR_ARG;
  const int64_t need = spot_workspace_size(lay, max_chunks);
  if (need < 0) return (int)need;
  if (lay->ref_wl < 0 || lay->ref_wl >= lay->n_wl) return ORT_ERR_ARG;
  if (lay->n_local_ops < 0 || (lay->n_local_ops > 0 && !lay->local_ops)) return ORT_ERR_ARG;
  pairs = (int64_t)lay->n_fields * lay->n_wl;
  if (pairs == 0) return ORT_OK;
  if (!workspace || workspace_size < need) return ORT_ERR_ARG;
  if (lay->n_pupil > 0 && (!rays->x || !rays->y || !rays->i)) return ORT_ERR_ARG;
  if (lay->n_pupil > 0 && lay->n_local_ops > 0 && !rays->z) return ORT_ERR_ARG;
  chunks = spot_chunks(lay, max_chunks);
  if (spot_per_thread(lay, max_chunks) > 0x7fffffff || pairs > 65535) return ORT_ERR_ARG;
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
  a.per_thread = (int32_t)spot_per_thread(lay, max_chunks);
  a.part1 = (double*)workspace;
  a.part2 = a.part1 + pairs * chunks * 3;
  a.out = out;
  return ORT_OK;
}

int ort_trace_spot(const ort_lens* lens, const double* px, const double* py,
                   ort_rays* rays_out, const ort_batch* batch, const ort_options* opt,
                   int32_t* status, const ort_spot_layout* lay, void* workspace,
                   int64_t workspace_size, double* out, void* stream) {
  if (!batch || !lay || !rays_out) return ORT_ERR_ARG;
  if (batch->n_rays != (int64_t)lay->n_fields * lay->n_wl * lay->n_pupil) return ORT_ERR_ARG;
  if (batch->n_rays == 0) return ORT_OK;
  SpotArgs a{};
  int64_t pairs = 0, chunks = 0;
  int rc = spot_args(rays_out, lay, workspace, workspace_size, out, a, pairs, chunks);
  if (rc) return rc;
  SpotFuse f{a.part1, lay->local_ops, lay->n_local_ops, (int32_t)chunks, pairs, false};
  if (a.per_thread != 1) f.pairs = -1;  // a chunk spans several rays per thread: unfused
  rc = trace_pupil_impl(lens, px, py, rays_out, batch, opt, nullptr, nullptr, status, stream,
                        &f);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)chunks, (unsigned)pairs);
  if (!f.fused) hipLaunchKernelGGL(spot_sum_kernel, grid, dim3(kSpotThreads), 0, s, a);
  launch_pass2(a, pairs, chunks, s);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

int ort_spot_stats(const ort_rays* rays, const ort_spot_layout* lay, void* workspace,
                   int64_t workspace_size, double* out, void* stream) {
  SpotArgs a{};
  int64_t pairs = 0, chunks = 0;
  const int rc = spot_args(rays, lay, workspace, workspace_size, out, a, pairs, chunks);
  if (rc || pairs == 0) return rc;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)chunks, (unsigned)pairs);  // n_pupil == 0: one empty chunk
  hipLaunchKernelGGL(spot_sum_kernel, grid, dim3(kSpotThreads), 0, s, a);
  launch_pass2(a, pairs, chunks, s);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

// ---- RayOperand.rms_spot_size (optimization/operand/ray.py:300-340) -----------------
// rms = sqrt(mean((x - mean x)^2 + (y - mean y)^2)) over ALL n points (no intensity mask),
// by the spot-statistics passes above with one pair: stats[5] as ort_spot_stats' row.
int64_t ort_rms_spot_workspace_size(int64_t n) {
  ort_spot_layout lay{};
  lay.n_pupil = n;
  lay.n_fields = 1;
  lay.n_wl = 1;
  return spot_workspace_size(&lay, kRmsMaxChunks);
}

int ort_rms_spot(const double* x, const double* y, int64_t n, void* workspace,
                 int64_t workspace_size, double* stats, double* rms, void* stream) {
  if (n < 0 || !stats || (n > 0 && (!x || !y))) return ORT_ERR_ARG;
  ort_spot_layout lay{};
  lay.n_pupil = n;
  lay.n_fields = 1;
  lay.n_wl = 1;
  ort_rays r{};
  r.x = (double*)x;
  r.y = (double*)y;
  r.i = (double*)x;  // validated as present, then replaced by "no mask" below
  SpotArgs a{};
  int64_t pairs = 0, chunks = 0;
  int rc = spot_args(&r, &lay, workspace, workspace_size, stats, a, pairs, chunks,
                     kRmsMaxChunks);
  if (rc) return rc;
  a.i = nullptr;  // every point counts (the operand does not mask vignetted rays)
  a.rms_out = rms;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)chunks, 1u);
  hipLaunchKernelGGL(spot_sum_kernel, grid, dim3(kSpotThreads), 0, s, a);
  launch_pass2(a, pairs, chunks, s);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

int ort_rms_spot_vjp(const double* x, const double* y, int64_t n, const double* stats,
                     const double* grad_out, double* gx, double* gy, void* stream) {
  if (n < 0 || !stats || !grad_out || (n > 0 && (!x || !y || !gx || !gy))) return ORT_ERR_ARG;
  if (n == 0) return ORT_OK;
  const int64_t blocks = (n + kSpotThreads - 1) / kSpotThreads;
  if (blocks > 0x7fffffff) return ORT_ERR_ARG;
  hipLaunchKernelGGL(rms_spot_vjp_kernel, dim3((unsigned)blocks), dim3(kSpotThreads), 0,
                     (hipStream_t)stream, x, y, n, stats, grad_out, gx, gy);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

int ort_rms_finish(const double* part, int64_t n_rows, double* stats, double* rms,
                   void* stream) {
  if (!part || !stats || n_rows < 1 || n_rows > ((int64_t)1 << 28)) return ORT_ERR_ARG;
  hipLaunchKernelGGL(rms_finish_kernel, dim3(1), dim3(kFinThreads), 0, (hipStream_t)stream,
                     part, (int)n_rows, stats, rms);
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

int ort_spot_partials(const ort_rays* rays, const ort_spot_layout* lay, int32_t phase,
                      const double* sums1, void* workspace, int64_t workspace_size,
                      double* out, void* stream) {
  if (phase != 1 && phase != 2) return ORT_ERR_ARG;
  if (phase == 2 && !sums1) return ORT_ERR_ARG;
  SpotArgs a{};
  int64_t pairs = 0, chunks = 0;
  const int rc = spot_args(rays, lay, workspace, workspace_size, out, a, pairs, chunks);
  if (rc || pairs == 0) return rc;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)chunks, (unsigned)pairs);
  if (phase == 1) {
    hipLaunchKernelGGL(spot_sum_kernel, grid, dim3(kSpotThreads), 0, s, a);
    hipLaunchKernelGGL(spot_pair_kernel<1>, dim3((unsigned)pairs), dim3(kSpotThreads), 0, s, a);
  } else {
    a.gsum = sums1;
    hipLaunchKernelGGL(spot_dev_kernel, grid, dim3(kSpotThreads), 0, s, a);
    hipLaunchKernelGGL(spot_pair_kernel<2>, dim3((unsigned)pairs), dim3(kSpotThreads), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? ORT_OK : ORT_ERR_LAUNCH;
}

}  // extern "C"
