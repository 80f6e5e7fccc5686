// ort_reduce.h -- deterministic block reductions for the analysis kernels
// (ort_k_spot.hip, ort_k_wavefront.hip): wave sums (DPP), then the block's waves
// in index order, so a reduction over fixed chunks is bit-identical run to run.
#pragma once

#include "ort_kernels.h"

namespace ortk {

constexpr int kRedThreads = 256;  // threads per block of the analysis kernels

// wave sums: ort_kernels.h wave_sum (DPP row operations with the whole wave active,
// the xor butterfly otherwise; a fixed order either way)
__device__ inline double wave_sum_xor(double v) { return wave_sum(v); }
__device__ inline double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = ::fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sums of NV values (lanes by xor butterfly, then waves 0..NT/64-1 in order);
// every thread gets the totals. lds: >= NT / 64 * NV doubles; safe to call back to back.
template <int NV, int NT = kRedThreads>
__device__ inline void block_sum(double (&v)[NV], double* lds) {
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = wave_sum_xor(v[k]);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[w * NV + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double s = 0.0;
    for (int ww = 0; ww < NT / 64; ++ww) s += lds[ww * NV + k];
    v[k] = s;
  }
}

// column sums of rows part[0 .. n) of NV doubles, each thread striding over rows in
// index order, then block_sum
template <int NV>
__device__ inline void reduce_rows_n(const double* part, int n, double (&v)[NV], double* lds) {
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.0;
  for (int c = threadIdx.x; c < n; c += kRedThreads)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += part[c * NV + k];
  block_sum<NV>(v, lds);
}

// F_SPOT epilogue of trace_closed_kernel: spot_sum_kernel's pass over one chunk
// (ort_k_spot.hip, one ray per thread), on the rays still in registers -- the same
// per-thread values (the point localized by the same ops, masked by i > 0) and the same
// block_sum, so the partial rows are bit-identical to that kernel's
template <uint32_t FEAT>
__device__ void spot_epilogue(const KArgs& a, const ort::Ray& r, double inten, bool active) {
  static_assert(kClosedBlock == kRedThreads, "one chunk per trace block");
  double v[3] = {0.0, 0.0, 0.0};
  if (active && inten > 0.0) {  // spot_diagram.py:425-427
    ort::Ray p;
    p.x = r.x;
    p.y = r.y;
    p.z = a.spot_n_ops ? r.z : 0.0;
    p.L = 0.0; p.M = 0.0; p.N = 0.0;
    for (int k = 0; k < a.spot_n_ops; ++k) ort::apply_cs_op(p, cst(a.spot_ops)[k]);
    v[0] = 1.0;
    v[1] = 0.0 + p.x;  // as spot_sum_kernel's 0.0 += x (-0.0 -> +0.0)
    v[2] = 0.0 + p.y;
  }
  __shared__ double lds[4 * 3];
  block_sum<3>(v, lds);
  if (threadIdx.x == 0) {
    double* o = a.spot_part1 + (int64_t)blockIdx.x * 3;
    o[0] = v[0];
    o[1] = v[1];
    o[2] = v[2];
  }
}

// F_RMS epilogue of the taped Newton kernel (RayOperand.rms_spot_size on the traced
// points, optimization/operand/ray.py:300-340): block vb's row {count, sum x, sum y,
// sum of (x - mx)^2 + (y - my)^2 about the block's own centroid (mx, my)}, each by
// block_sum in its fixed order; rms_finish_kernel (ort_k_spot.hip) combines the rows
// (Chan et al.'s pairwise update: the second moments re-centred on the total centroid),
// so the rms leaves the forward without a second read of the points
__device__ inline void rms_epilogue(const KArgs& a, const ort::Ray& r, bool active,
                                    int64_t vb) {
  static_assert(kBlock == kRedThreads, "one row per trace workgroup");
  double v[3] = {0.0, 0.0, 0.0};
  if (active) {
    v[0] = 1.0;
    v[1] = r.x;
    v[2] = r.y;
  }
  __shared__ double lds[4 * 3];
  block_sum<3>(v, lds);
  double d[1] = {0.0};
  if (active) {
    const double dx = r.x - v[1] / v[0], dy = r.y - v[2] / v[0];
    d[0] = dx * dx + dy * dy;
  }
  block_sum<1>(d, lds);
  if (threadIdx.x == 0) {
    double* o = a.rms_part + vb * 4;
    o[0] = v[0];
    o[1] = v[1];
    o[2] = v[2];
    o[3] = d[0];
  }
}

// The rms spot size from the F_RMS rows (ort_rms_finish, and the second workgroup of
// ort_newton_finish_rms): one workgroup of NT threads, each holding up to ROWS rows in
// registers (rows past NT * ROWS re-read in the second sum). The counts and sums in index
// order give the centroid (mx, my); then M2 = sum over rows of [M2_b + n_b ((sx_b / n_b -
// mx)^2 + (sy_b / n_b - my)^2)] (a row with n_b = 0 adds nothing: Chan et al.'s pairwise
// update), rms = sqrt(M2 / n); stats as ort_rms_spot's row (n, mean x, mean y, rms) with the
// geometric radius, which this pass has no data for, NaN. lds: >= NT / 64 * 3 doubles.
__device__ inline double rms_row_m2(const double* p, double mx, double my) {
  const double nb = p[0];
  if (!(nb > 0.0)) return 0.0;
  const double dx = p[1] / nb - mx, dy = p[2] / nb - my;
  return p[3] + nb * (dx * dx + dy * dy);
}

constexpr int kRmsFinThreads = 256;  // the one workgroup shape of both finish launches
constexpr int kRmsFinRows = 16;

template <int NT, int ROWS>
__device__ inline void rms_finish_block(const double* part, int n_rows, double* stats,
                                        double* rms, double* lds) {
  double row[ROWS][4];
#pragma unroll
  for (int k = 0; k < ROWS; ++k) {
    const int c = threadIdx.x + k * NT;
#pragma unroll
    for (int f = 0; f < 4; ++f) row[k][f] = c < n_rows ? part[(int64_t)c * 4 + f] : 0.0;
  }
  double v[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < ROWS; ++k) {
    v[0] += row[k][0];
    v[1] += row[k][1];
    v[2] += row[k][2];
  }
  for (int c = threadIdx.x + ROWS * NT; c < n_rows; c += NT) {
    v[0] += part[(int64_t)c * 4 + 0];
    v[1] += part[(int64_t)c * 4 + 1];
    v[2] += part[(int64_t)c * 4 + 2];
  }
  block_sum<3, NT>(v, lds);
  const double mx = v[1] / v[0], my = v[2] / v[0];
  double m[1] = {0.0};
#pragma unroll
  for (int k = 0; k < ROWS; ++k) m[0] += rms_row_m2(row[k], mx, my);
  for (int c = threadIdx.x + ROWS * NT; c < n_rows; c += NT)
    m[0] += rms_row_m2(part + (int64_t)c * 4, mx, my);
  block_sum<1, NT>(m, lds);
  if (threadIdx.x == 0) {
    const double r = ::sqrt(m[0] / v[0]);
    stats[0] = v[0];
    stats[1] = mx;
    stats[2] = my;
    stats[3] = r;
    stats[4] = __builtin_nan("");
    if (rms) *rms = r;
  }
}

}  // namespace ortk
