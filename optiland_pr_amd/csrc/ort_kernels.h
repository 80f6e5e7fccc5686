// ort_kernels.h -- MI355X (gfx950) kernels of the sequential real-ray trace (templates).
//
// Shared by the kernel translation units (ort_k_*.hip, compiled in parallel, each
// instantiating one family of specialisations) and the C ABI (ort_api.hip), which only
// reaches kernels through the select_* functions declared at the end.
//
// One ray per lane, all surfaces fused in one launch. The ray state
// (x, y, z, L, M, N, i, opd) stays in VGPRs from the first surface to the image; the
// surface table is wave-uniform (indexed by the loop counter) so every surface
// parameter is fetched with scalar loads into SGPRs. Per-ray HBM traffic is one read of
// the inputs (64 B of rays, or 16 B of pupil coordinates) and one 64 B write.
//
// Newton surfaces (even/odd asphere, Zernike) follow the reference's GLOBAL stopping
// rule (newton_raphson.py:148: break when max|f| < tol over all rays of the trace call)
// by speculate-and-verify: every ray performs exactly sched[group][s] updates and
// reports, per group and surface, the AND of its "converged at update j" bits and the
// last update index at which it was not converged; the host checks the schedule
// against those and re-launches on a mismatch (rare). ORT_NEWTON_WAVE instead stops a
// wave as soon as its 64 lanes have converged (approximate, faster).
//
// Compiled with -ffp-contract=off: see ort_core.h.

#pragma once

#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "ort_core.h"
#include "ort_fastpath.h"
#include "ort_interact.h"
#include "ort_material.h"
#include "ort_sweep.h"  // KArgs, fill_args, localize / globalize, the derivative sweeps

namespace ortk {

// Streaming stores of the ray outputs, records and the adjoint tape (written once, read by
// a later launch) are issued non-temporal: A/B on the MI355X (rocprofv3 / bench, two
// repetitions each) DoubleGauss 1M-ray launch 68.7 / 69.0 -> 66.2 / 65.7 us, config 5 step
// 0.716 / 0.713 -> 0.686 / 0.693 ms (the taped forward). ORT_TEMPORAL_STORE (A/B builds)
// restores plain stores.
#ifndef ORT_TEMPORAL_STORE
#define ORT_ST(lhs, v) __builtin_nontemporal_store((v), &(lhs))
#else
#define ORT_ST(lhs, v) ((lhs) = (v))
#endif


constexpr int kBlock = 256;
// workgroups of a verify-and-re-trace round of trace_kernel (a multiple of 8, so the
// grid-stride loop keeps each block on its XCD): 4 per CU, the taped kernel's full
// occupancy at 4 waves per SIMD. ORT_VERIFY_GRID: A/B builds.
#ifndef ORT_VERIFY_GRID
#define ORT_VERIFY_GRID 1024
#endif
constexpr int64_t kVerifyGrid = ORT_VERIFY_GRID;
static_assert(kVerifyGrid % 8 == 0, "XCD-preserving stride");
// trace_closed_kernel's block size (ort_k_closed.hip; its launch asks closed_block()):
// a per-TU constant so A/B builds of that TU alone can change it
#ifndef ORT_CLOSED_BLOCK
#define ORT_CLOSED_BLOCK 256
#endif
constexpr int kClosedBlock = ORT_CLOSED_BLOCK;

// ort_trace_spot -> trace_pupil_impl (ort_api.hip): where the fused spot pass 1 writes;
// fused reports whether the launch took it
struct SpotFuse {
  double* part1;
  const ort_cs_op* ops;
  int32_t n_ops;
  int32_t chunks;
  int64_t pairs;
  bool fused;
};
int trace_pupil_impl(const ort_lens* lens, const double* px, const double* py,
                     ort_rays* rays_out, const ort_batch* batch, const ort_options* opt,
                     double* rec, ort_newton_stat* newton_stat, int32_t* status, void* stream,
                     SpotFuse* fuse);

// the F_SPOT epilogue (ort_reduce.h): every thread of the block calls it
template <uint32_t FEAT>
__device__ void spot_epilogue(const KArgs& a, const ort::Ray& r, double inten, bool active);
// the F_RMS epilogue (ort_reduce.h): every thread of the block calls it
__device__ inline void rms_epilogue(const KArgs& a, const ort::Ray& r, bool active,
                                    int64_t vb);

// Ray of this thread when every (field, lambda) segment traces the SAME pupil samples
// (real_ray_tracer.py:74-77 field-major layout: ray = segment * seg_len + p): block b
// would read pupil chunk b % chunks once per segment, i.e. n_seg times from HBM (the
// chunks of a 4M-ray pupil do not stay in a 4 MB L2). Blocks are dealt round-robin over
// the 8 XCDs (MI355X_MICROARCH.md, dispatch), so the blocks sharing an XCD (b % 8) get a
// contiguous range of the chunk-major order L = chunk * n_seg + segment: every XCD reads
// each of its pupil chunks once and serves all segments from its L2. Any dispatch order
// gives the same results (a bijection over blocks); only the traffic depends on it.
// Requires n_rays == n_seg * seg_len and seg_len % kBlock == 0 (host-checked).
// vb / nb: the workgroup's (virtual) block of the launch's nb blocks (trace_kernel's
// grid-stride loop keeps vb % 8 == blockIdx.x % 8: its grids are multiples of 8 or nb)
__device__ inline int64_t pair_major_ray(const KArgs& a, int64_t vb, int64_t nb) {
  const int64_t B = nb;
  const int64_t b = vb;
  const int64_t x = b & 7, local = b >> 3;
  int64_t start = 0;
  for (int64_t y = 0; y < x; ++y) start += (B - y + 7) >> 3;  // blocks of the lower XCD slots
  const int64_t L = start + local;
  const int64_t seg = L % a.n_seg, chunk = L / a.n_seg;
  return seg * a.seg_len + chunk * kBlock + threadIdx.x;
}

__device__ inline uint64_t wave_and_u64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v &= __shfl_xor(v, o, 64);
  return v;
}
__device__ inline int wave_max_i32(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// Same-address atomics from every wave of a large grid serialise in L2, and almost every
// wave would leave the value unchanged (the Newton statistics of one group agree across
// its waves): read first (relaxed) and issue the atomic only when it changes something.
__device__ inline void and_if_changes(uint64_t* p, uint64_t v) {
  const uint64_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((cur & v) != cur) atomicAnd((unsigned long long*)p, (unsigned long long)v);
}
__device__ inline void max_if_changes(int32_t* p, int32_t v) {
  const int32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (v > cur) atomicMax(p, v);
}

// Optical constants of surface si at the ray's wavelength (same scalar-load batch as the
// surface record when the row is wave-uniform). F_MONO makes that a compile-time fact:
// with a run-time test the compiler merges both loads into one per-lane vector load
// through a selected address, a dependent round trip per surface. Under F_MONO the host
// guarantees every lane of a wave has the same wavelength row (one row, or (field, lambda)
// segments whose boundaries are multiples of 64 rays), so the row index is read from the
// first active lane into an SGPR.
__device__ inline int uniform_row(int lam) { return __builtin_amdgcn_readfirstlane(lam); }

template <uint32_t FEAT = 0>
__device__ inline ort_surface_optics optics_at(const KArgs& a, int lam, int si) {
  if constexpr ((FEAT & F_MONO) != 0) return cst(a.optics)[uniform_row(lam) * a.n_surf + si];
  return optics_row(a, lam, si);
}

template <uint32_t FEAT>
__device__ inline ort_surface_optics surface_optics(const KArgs& a, const ort_surface& s,
                                                    int lam, int si, double w) {
  if constexpr ((FEAT & F_WRAY) != 0) return optics_ray(a, s, w);
  return optics_at<FEAT>(a, lam, si);
}

// absorption of the image-space medium (final propagate)
template <uint32_t FEAT>
__device__ inline double final_alpha(const KArgs& a, int lam, double w) {
  if constexpr ((FEAT & F_WRAY) != 0)
    return ort::absorption_alpha(ort::material_k(cst(a.mats)[a.final_mat], a.coef, w), w);
  if constexpr ((FEAT & F_MONO) != 0) return cst(a.alpha_tab)[uniform_row(lam) * a.n_mat + a.final_mat];
  return tab(a.alpha_tab, a.n_lambda, a.n_mat, lam, a.final_mat);
}

// geometry ids this library implements (enum ort_geometry); the kernels turn any other
// id into NaN rays plus ORT_STATUS_BAD_GEOMETRY
__device__ inline bool known_geometry(int g) { return g >= ORT_GEOM_PLANE && g <= ORT_GEOM_NURBS; }
// surfaces of the Newton schedule / statistics machinery (not plane, conic or NURBS)
__device__ inline bool scheduled_geometry(int g) {
  return g != ORT_GEOM_PLANE && g != ORT_GEOM_STANDARD && g != ORT_GEOM_NURBS;
}

// status bit of a normalisation-range error at surface s (zernike.py:234-246,
// chebyshev.py:203-215: both raise ValueError in the reference)
__device__ inline int range_bit(const ort_surface& s) {
  return s.geometry == ORT_GEOM_CHEBYSHEV ? (int)ORT_STATUS_CHEBYSHEV_RANGE
                                          : (int)ORT_STATUS_ZERNIKE_RANGE;
}

// Per-lane "the stop test passed at stop index k" bits over the 128-index window
// [conv_base, conv_base + 128) of ort_newton_stat.conv_mask
struct ConvBits {
  uint64_t w0 = 0, w1 = 0;
  __device__ inline void set(int k, int base) {
    const int b = k - base;
    if (b >= 0 && b < 64) w0 |= 1ull << b;
    else if (b >= 64 && b < 128) w1 |= 1ull << (b - 64);
  }
};

// Newton statistics of one (group, surface): AND of the per-update convergence bits and
// the max non-converged index (see ort_newton_stat), read-before-atomic. The lane's
// evaluated stop indices are j_lo .. U (its bits outside stay 0, last_bad is the largest
// of them that did not converge). A group-uniform wave whose indices all fall in the
// mask window (conv_base 0, U < 128) forms the wave's AND and max from one ballot per
// index -- bit j of the AND is set iff no reporting lane missed j, and the max is the
// last j some reporting lane missed: the same values as the shuffle reductions (six
// dependent cross-lane steps each, three reductions per Newton surface) at a fraction of
// the instructions and latency (#ifndef ORT_SHFL_REPORT, A/B builds)
__device__ inline void report_newton(const KArgs& a, int si, bool active, int64_t group,
                                     bool group_uniform, ConvBits m, int last_bad, int U = -1,
                                     int j_lo = 0) {
  if (!a.stats) return;
#ifndef ORT_SHFL_REPORT
  if (group_uniform && a.conv_base == 0) {
    const int Uw = __builtin_amdgcn_readfirstlane(U);
    if (Uw >= 0 && Uw < 128) {
      if (__ballot(active) == 0) return;  // no reporting lane: nothing changes
      uint64_t w0 = 0, w1 = 0;
      int lb = -1;
      for (int j = j_lo; j <= Uw; ++j) {
        const bool bit = ((j < 64 ? m.w0 >> j : m.w1 >> (j - 64)) & 1) != 0;
        if (__ballot(active && !bit) == 0) {
          if (j < 64)
            w0 |= 1ull << j;
          else
            w1 |= 1ull << (j - 64);
        } else {
          lb = j;
        }
      }
      if ((threadIdx.x & 63) != 0) return;
      ort_newton_stat* st = &a.stats[group * a.n_surf + si];
      if (w0 != ~0ull) and_if_changes(&st->conv_mask[0], w0);
      if (w1 != ~0ull) and_if_changes(&st->conv_mask[1], w1);
      if (lb >= 0) max_if_changes(&st->last_bad, lb);
      return;
    }
  }
#endif
  if (!active) {
    m.w0 = m.w1 = ~0ull;
    last_bad = -1;
  }
  ort_newton_stat* st = &a.stats[group * a.n_surf + si];
  if (group_uniform) {
    m.w0 = wave_and_u64(m.w0);
    m.w1 = wave_and_u64(m.w1);
    last_bad = wave_max_i32(last_bad);
    if ((threadIdx.x & 63) != 0) return;
  } else if (!active) {
    return;
  }
  if (m.w0 != ~0ull) and_if_changes(&st->conv_mask[0], m.w0);
  if (m.w1 != ~0ull) and_if_changes(&st->conv_mask[1], m.w1);
  if (last_bad >= 0) max_if_changes(&st->last_bad, last_bad);
}

// Grid-sag intersection (grid_sag.py:108-140): Newton from t = 0, the reference stops
// after the first update whose max |dt| over the call is < tol. Under the schedule every
// ray makes exactly U updates and reports bit j = "|dt| < tol after update j" (j >= 1),
// so the host's verify reads the stopping count exactly as for the other Newton kinds.
template <uint32_t FEAT>
__device__ inline double grid_distance(const KArgs& a, const ort_surface& s, int si,
                                       const ort::Ray& r, bool active, int64_t group,
                                       bool group_uniform, const int32_t* sched) {
  const ort::GridView g = ort::grid_view(a.coef + s.coef_off);
  const double tol = s.tol;
  const int max_iter = s.max_iter;
  double t = 0.0;
  if (a.newton_mode == ORT_NEWTON_WAVE) {
    int j = 0;
    while (j < max_iter) {
      const double dt = ort::grid_step(g, r, t);
      t = t + dt;
      ++j;
      if (__all(!active || fabs(dt) < tol)) break;
    }
    if (a.stats && (threadIdx.x & 63) == 0)
      max_if_changes(&a.stats[(group_uniform ? group : 0) * a.n_surf + si].max_updates, j);
    return ort::grid_final(g, r, t);
  }
  const int U = sched ? sched[group * a.n_surf + si] : max_iter;
  ConvBits mask;
  int last_bad = -1;
  for (int j = 0;; ++j) {
    const bool lane_on = active && j < U;
    if (!__any(lane_on)) break;
    if (lane_on) {
      const double dt = ort::grid_step(g, r, t);
      t = t + dt;
      const bool conv = fabs(dt) < tol;  // NaN never converges
      if (conv) mask.set(j + 1, a.conv_base);  // stop index j + 1: the test after update j
      if (!conv) last_bad = j + 1;
    }
  }
  report_newton(a, si, active, group, group_uniform, mask, last_bad, U, 1);
  return ort::grid_final(g, r, t);
}

// Newton refinement of t at surface s for one lane (newton_raphson.py:119-168).
// hn: set when (nnx, nny, nnz) hold the normal at the returned t -- the last evaluation
// is at P(t) itself (the stop test), and the point r + t D it evaluates is, operation
// for operation, the propagated point Surface.trace takes the normal at
// (standard_surface.py:215-225, homogeneous.py:45-47), so that normal is the
// interaction's normal: one sag + normal evaluation per Newton surface saved.
// F_TAPE: tape (this ray's tape rows of surface si, nullptr for inactive lanes) gets row
// 7 + m = the iterate before the m-th last update (t_{U-1-m}) for m < min(U, kHist), as
// the adjoint's replay_distance tapes it.
// FAST (trace_kernel's deferred-check pass): the initial conic guess, the even / odd
// asphere evaluations and the updates on ort_fastpath.h's sequences, range failures ORed
// into `bad` (plus a non-finite f: such a lane's statistics come from the exact pass);
// a lane reports its Newton statistics here only while it is not bad -- the values up to
// then are bit-identical to the exact path's, and the exact pass reports the bad lanes
template <uint32_t FEAT, bool FAST>
__device__ inline __attribute__((always_inline)) double newton_eval_fast(const KArgs& a, const ort_surface& s,
                                          const ort::Ray& r, double t, int mode, bool& rerr,
                                          double& nx, double& ny, double& nz, bool& bad) {
  constexpr uint32_t KM = FEAT & F_KM;
  if constexpr (FAST && (KM & (ort::KM_EVEN | ort::KM_ODD)) != 0) {
    const double xi = r.x + t * r.L;
    const double yi = r.y + t * r.M;
    const double zi = r.z + t * r.N;
    double sag;
    if ((KM & ort::KM_EVEN) != 0 && (KM == ort::KM_EVEN || s.geometry == ORT_GEOM_EVEN_ASPHERE))
      sag = ort::fast::sagnorm_even(xi, yi, s, cst(a.coef) + s.coef_off, s.n_coef, mode, nx, ny,
                                    nz, bad);
    else if ((KM & ort::KM_ODD) != 0 && ((KM & ~ort::KM_ODD) == 0 || s.geometry == ORT_GEOM_ODD_ASPHERE))
      sag = ort::fast::sagnorm_odd(xi, yi, s, cst(a.coef) + s.coef_off, s.n_coef, mode, nx, ny,
                                   nz, bad);
    else
      sag = ort::newton_sagnorm<KM>(s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed, xi,
                                    yi, mode, rerr, nx, ny, nz);
    const double f = sag - zi;
    ORT_CHK(bad, !(::fabs(f) < 0x1p1000));
    return f;
  } else {
    return ort::newton_eval<KM>(s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed, r, t,
                                mode, rerr, nx, ny, nz);
  }
}

template <uint32_t FEAT, bool FAST = false>
__device__ inline __attribute__((always_inline)) double newton_distance(const KArgs& a, const ort_surface& s, int si,
                                         const ort::Ray& r, bool active, int64_t group,
                                         bool group_uniform, int& range_bits, bool& hn,
                                         double& nnx, double& nny, double& nnz,
                                         double* tape, const int32_t* sched,
                                         bool& bad) {
  hn = false;
  if constexpr ((FEAT & ort::KM_FREE) != 0) {
    if (s.geometry == ORT_GEOM_GRID_SAG)
      return grid_distance<FEAT>(a, s, si, r, active, group, group_uniform, sched);
  }
  if constexpr ((FEAT & ort::KM_NURBS) != 0) {
    if (s.geometry == ORT_GEOM_NURBS)  // its own per-ray (u, v) solve (ort_nurbs.h)
      return ort::nurbs_distance(ort::nurbs_view(a.coef + s.coef_off), s.tol, s.max_iter, r);
  }
  const bool rinf = (s.flags & ORT_SURF_RADIUS_INF) != 0;
  double t;
  if constexpr (FAST)
    t = ort::fast::distance_conic(r, s, rinf, bad);
  else
    t = ort::distance_conic(r, s.radius, s.conic, rinf);
  const double tol = s.tol;
  const int max_iter = s.max_iter;
  if (a.newton_mode == ORT_NEWTON_WAVE) {
    // Per-wave global rule: every lane of the wave does the same number of updates,
    // the wave stops at the first j where all its (non-NaN) lanes have |f| < tol.
    // (the evaluations give the update's slopes; the unit normal once at the stop)
    int j = 0;
    for (; j < max_iter; ++j) {
      bool rerr = false;
      double nx, ny, nz;
      const double f = ort::newton_eval<(FEAT & F_KM)>(s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed, r,
                                                      t, ort::kSlope, rerr, nx, ny, nz);
      if (active && rerr) range_bits |= range_bit(s);
      const bool conv = !active || !(fabs(f) >= tol);
      if (__all(conv)) {
        bool rerr2 = false;
        (void)ort::newton_eval<(FEAT & F_KM)>(s, s.radius, s.conic, cst(a.coef), cst(a.zern),
                                              kNoSeed, r, t, ort::kNormal, rerr2, nnx, nny, nnz);
        hn = true;
        break;
      }
      t = ort::newton_step_any(r, t, f, nx, ny, nz);
    }
    if (a.stats && (threadIdx.x & 63) == 0)
      max_if_changes(&a.stats[(group_uniform ? group : 0) * a.n_surf + si].max_updates, j);
    return t;
  }
  // ORT_NEWTON_SCHEDULE: exactly U updates, plus the check evaluation at j = U.
  const int U = sched ? sched[group * a.n_surf + si] : max_iter;
  ConvBits mask;
  int last_bad = -1;
  // Every evaluation is one call site (the kernel's code size is its hot loop): at j < U
  // sag + the update's slopes at P(t) (kSlope) and the update; at j = U (the stop test)
  // the same evaluation, the interaction's unit normal formed from those slopes -- for the
  // even / odd / Zernike kinds (n = (dz/dx, dz/dy, -1) / norm, the same operations as their
  // kNormal evaluation). Kernels with freeform kinds, and ORT_NO_SLOPE A/B builds, evaluate
  // the unit normal and update with the reference's -n / nz_safe.
#ifdef ORT_NO_SLOPE
  constexpr bool kSl = false;
#else
  constexpr bool kSl = ((FEAT & F_KM) & ~(ort::KM_EVEN | ort::KM_ODD | ort::KM_ZERN)) == 0;
#endif
  for (int j = 0;; ++j) {
    const bool lane_on = active && j <= U;
    if (!__any(lane_on)) break;
    if (lane_on) {
      bool rerr = false;
      double nx, ny, nz;
      const bool upd = j < U;
      const double f = newton_eval_fast<FEAT, FAST>(a, s, r, t, kSl ? ort::kSlope : ort::kNormal,
                                                    rerr, nx, ny, nz, bad);
      // the reference evaluates sag at j = 0..U-1 always, and at j = U only when the
      // loop broke there (U < max_iter)
      if (rerr && (j < U || U < max_iter) && !(FAST && bad)) range_bits |= range_bit(s);
      const bool conv = fabs(f) < tol;  // NaN never converges (np.max propagates NaN)
      if (conv) mask.set(j, a.conv_base);
      if (!conv) last_bad = j;
      if (upd) {
        if constexpr ((FEAT & F_TAPE) != 0) {
          // the iterate before the m-th last update, m = U - 1 - j, straight into its tape
          // row (the adjoint replays m < min(U, kHist): adj_ray)
          const int m = U - 1 - j;
          if (m < kHist && tape) ORT_ST(tape[(int64_t)(7 + m) * a.n_rays], t);
        }
        if constexpr (!kSl) {
          if constexpr (FAST)
            t = ort::fast::newton_step(r, t, f, nx, ny, nz, bad);
          else
            t = ort::newton_step(r, t, f, nx, ny, nz);
        } else if constexpr (FAST) {
          t = ort::fast::newton_step_slope(r, t, f, nx, ny, bad);  // (steep: bad)
        } else {
          t = ort::newton_step_any(r, t, f, nx, ny, nz);
        }
      } else if constexpr (!kSl) {
        nnx = nx;
        nny = ny;
        nnz = nz;
      } else if constexpr (FAST) {
        ort::fast::unit_normal_from_slope(nx, ny, nnx, nny, nnz, bad);
      } else if (nz == -1.0) {  // the slopes: their unit normal, as kNormal forms it
        ort::unit_normal3(nx, ny, ort::sqrt(nx * nx + ny * ny + 1.0), nnx, nny, nnz);
      } else {  // steep or NaN: the evaluation returned the unit normal itself
        nnx = nx;
        nny = ny;
        nnz = nz;
      }
    }
  }
  report_newton(a, si, active && !(FAST && bad), group, group_uniform, mask, last_bad, U);
  if constexpr ((FEAT & F_TAPE) != 0) {
    // the iterate rows no update fills (m >= U) get the root: every tape row is written
    // (the tape is the trace op's output; the adjoint reads only m < min(U, kHist))
    if (tape) {
#pragma unroll
      for (int m = 0; m < kHist; ++m)
        if (m >= U) ORT_ST(tape[(int64_t)(7 + m) * a.n_rays], t);
    }
  }
  hn = true;  // every active lane evaluated j == U (inactive lanes store nothing)
  return t;
}

// F_IA: the surface's interaction model after propagation / OPD / clipping
// (standard_surface.py:225 -> interactions/*.py). unnorm tracks the reference's
// rays.is_normalized flag, which only a thin lens clears (homogeneous.py:55-57).
template <uint32_t FEAT>
__device__ inline void interact(const KArgs& a, const ort_surface& s, ort::Ray& r,
                                const ort_surface_optics& o, int lam, double wl,
                                bool& unnorm) {
  const bool refl = (s.flags & ORT_SURF_REFLECTIVE) != 0;
  const PD p = cst(a.coef) + s.ia_off;
  if (s.interaction == ORT_IA_THIN_LENS) {
    ort::thin_lens(r, p[0], o.n_pre, refl ? -o.n_pre : o.n_post);
    unnorm = true;
    return;
  }
  double nx, ny, nz;
  ort::surface_normal<(FEAT & F_KM)>(s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed,
                                     r, nx, ny, nz);
  if (s.interaction == ORT_IA_REFRACT_REFLECT) {
    if (refl)
      ort::reflect(r, nx, ny, nz);
    else
      ort::refract(r, nx, ny, nz, o.u);
    return;
  }
  double w = wl;
  if constexpr ((FEAT & F_WRAY) == 0) w = a.n_lambda == 1 ? cst(a.lambdas)[0] : a.lambdas[lam];
  if (s.interaction == ORT_IA_PHASE)
    ort::phase_interact(r, p, nx, ny, nz, o.n_pre, refl ? o.n_pre : o.n_post, refl, w);
  else
    ort::diffract(r, p, nx, ny, nz, o.n_pre, o.n_post, refl, w);
}

// Occupancy of the Newton kernels: the Zernike kernels (without freeform kinds) need
// ~115 VGPRs (4 waves per SIMD); capped at 80 (6 waves, ~128 B scratch per lane) the TMA
// forward runs 9% faster on the MI355X (334 -> 305 us per 1M-ray launch, rocprofv3; 5
// waves: 313 us). The even-asphere kernels already fit 6 waves; the rest keep the
// compiler's choice. ORT_TRACE_WAVES overrides the target for A/B builds.
// The taping forward (F_TAPE: up to 11 rows of stores per surface) runs
// best at 4 waves: TMA 1M rays, taped trace 374 / 328 / 300 us at 6 / 5 / 4 waves per
// SIMD (rocprofv3 A/B); re-measured with the Cartesian Zernike form (131 VGPRs uncapped),
// config 5 step 0.750-0.761 / 0.732-0.733 / 0.774-0.775 ms at 3 / 4 / 5 waves.
// The Newton kernels' deferred-check pass (FAST = true in trace_ray) is compiled for the
// lenses whose Newton surfaces are even / odd aspheres (the kinds ort_fastpath.h has
// sequences for) without interactions, per-ray wavelengths or a tape; ORT_NO_NEWTON_FAST
// (A/B builds) keeps the single exact pass. Measured (config 3, RT-asph 60M rays, rocprofv3
// PMC + A/B on the MI355X, round 4): every ray stays inside the ranges
// (tools/fast_probe.py: 0 re-traced waves), the pass issues 2,598 fp64 VALU instructions
// per wave instead of 2,725 and 1,611 SALU instead of 2,363 -- but its range tests add as
// many non-fp64 VALU instructions as the div / sqrt sequences save (4,079 vs 4,060 VALU
// per wave in all), so the launch time is the exact pass's: 7.15-7.17 ms at 6 waves per
// SIMD (80 VGPRs) vs 7.16-7.20 ms exact-only (79 VGPRs); at the compiler's 99 VGPRs
// (5 waves) 7.29-7.31 ms. TraceWaves: 6 for the wave-uniform-row (F_MONO) kernels
// measured here, the compiler's choice for the others. The taped Zernike forward (config
// 5): 5 waves (96 VGPRs, 96 B of scratch) vs 4 (123 VGPRs) after the non-temporal tape
// stores, config 5 step 0.689 / 0.679 vs 0.692 / 0.694 ms (A/B, r04_ab_occupancy_c5.log;
// the adjoint at 4 waves instead of 3 measured 540 vs 417 us there). Round 5, with the
// degree-specialised Horner schemes: 4 waves (123 VGPRs, no scratch) 0.5259 / 0.5267 ms,
// 5 waves (96 VGPRs, 100 B of scratch) 0.5275 / 0.5227, 6 waves (80, 164 B) 0.567 / 0.593
// (profiles/r05_ab_fwd_occupancy.log): 4 waves, the same time without the spill traffic.
// The deferred-check even / odd kernels after the round-5 slope-form updates: 6 waves (80
// VGPRs, 56 B of scratch whose stores reach HBM: config 3 WRITE_SIZE 5.54 GB per launch for
// 3.84 GB of outputs) 6.89-6.91 ms, 5 waves (96 VGPRs, no scratch) 6.73-6.75 ms, 4 waves
// 7.01-7.02 ms (tools/gpu_r05p.sh, profiles/r05_ab_c3_occupancy.log): 5.
template <uint32_t FEAT>
constexpr bool kNewtonFast =
#ifdef ORT_NO_NEWTON_FAST
    false;
#else
    (FEAT & F_KM) != 0 && (FEAT & F_KM & ~(ort::KM_EVEN | ort::KM_ODD)) == 0 &&
    (FEAT & (F_IA | F_WRAY | F_TAPE)) == 0;
#endif

// The verify rounds' grid-stride form (F_STRIDE) usually returns at once and re-traces
// only after a schedule correction: 2 waves per SIMD, so it carries no scratch (its
// dispatch sets up no spill space).
template <uint32_t FEAT>
struct TraceWaves {
  static constexpr int value =
      (FEAT & F_STRIDE) != 0 ? 2
      : ((FEAT & ort::KM_ZERN) != 0 && (FEAT & (ort::KM_FREE | F_IA)) == 0)
          ? ((FEAT & F_TAPE) != 0 ? 4 : 6)
          : ((kNewtonFast<FEAT> && (FEAT & F_MONO) != 0) ? 5 : 1);
};
#ifdef ORT_TRACE_WAVES
#define ORT_TRACE_OCC __attribute__((amdgpu_waves_per_eu(ORT_TRACE_WAVES)))
#else
#define ORT_TRACE_OCC __attribute__((amdgpu_waves_per_eu(TraceWaves<FEAT>::value)))
#endif
// The device side of the host's DeviceLens.verify (raytrace.py) for one workgroup: per
// (group, Newton surface) the stop rule of newton_raphson.py:140-149 (grid_sag.py:108-140:
// index >= 1) read from the conv_mask window and last_bad of the launch that ran `sched`.
// Only the first wrong surface of a group is corrected (the later surfaces' statistics
// depend on it), in place in `sched` (memory this workgroup may write: global in
// ort_newton_fixup, LDS in a verify-and-re-trace launch). Returns the workgroup-wide
// code: 0 right, 1 corrected (re-run), 2 the window cannot decide (host). codes: LDS
// [kBlock / 64]. Every thread of the workgroup must call it.
__device__ inline int newton_decide(const ort_surface* surf, int32_t n_surf, int64_t n_groups,
                                    const ort_newton_stat* stats, int32_t conv_base,
                                    int32_t* sched, int32_t* codes) {
  constexpr int W = 128;  // stop indices per conv_mask window
  int code = 0;
  for (int64_t g = threadIdx.x; g < n_groups; g += kBlock) {
    for (int s = 0; s < n_surf; ++s) {
      const ort_surface sf = surf[s];
      if (!scheduled_geometry(sf.geometry)) continue;
      int32_t* U_p = sched + g * n_surf + s;
      const int U = *U_p;
      const int max_iter = sf.max_iter;
      const int k_min = sf.geometry == ORT_GEOM_GRID_SAG ? 1 : 0;
      if (U < k_min) {  // grid_sag.py:111-129 always makes the first update
        *U_p = k_min;
        code = max(code, 1);
        break;
      }
      const ort_newton_stat st = stats[g * n_surf + s];
      // first stop index k in [k_min, U) every ray passed, from the window
      int k = -1;
      bool undecided = false;
      for (int i = k_min; i < U; ++i) {
        const int b = i - conv_base;
        if (b < 0 || b >= W) {
          undecided = true;
          break;
        }
        const uint64_t word = b < 64 ? st.conv_mask[0] : st.conv_mask[1];
        if ((word >> (b & 63)) & 1ull) {
          k = i;
          break;
        }
      }
      if (undecided) {
        code = 2;
        break;
      }
      if (k >= 0) {  // every ray passed before update U: the reference stops there
        *U_p = k;
        code = max(code, 1);
        break;
      }
      if (U < max_iter && st.last_bad >= U) {  // not all passed at U: it goes on
        *U_p = U >= 8 ? max_iter : min(max_iter, max(2 * U + 2, 8));
        code = max(code, 1);
        break;
      }
    }
  }
  // workgroup max of the codes (fixed order, LDS)
  for (int o = 32; o > 0; o >>= 1) code = max(code, __shfl_xor(code, o, 64));
  if ((threadIdx.x & 63) == 0) codes[threadIdx.x >> 6] = code;
  __syncthreads();
  int c = 0;
  for (int w = 0; w < kBlock / 64; ++w) c = max(c, codes[w]);
  __syncthreads();  // codes free for reuse
  return c;
}


__device__ inline void store_ray(const KArgs& a, int64_t rid, const ort::Ray& r) {
  ORT_ST(a.out.x[rid], r.x);
  ORT_ST(a.out.y[rid], r.y);
  ORT_ST(a.out.z[rid], r.z);
  ORT_ST(a.out.L[rid], r.L);
  ORT_ST(a.out.M[rid], r.M);
  ORT_ST(a.out.N[rid], r.N);
  ORT_ST(a.out.i[rid], ort::intensity(r));
  ORT_ST(a.out.opd[rid], r.opd);
}

// One ray through every surface (and the image-space propagate) for trace_kernel.
// FAST: ort_fastpath.h's sequences with their range failures ORed into `bad` (see
// kNewtonFast); the lane's records, tape rows and Newton statistics are written only while
// it is active (the exact pass rewrites a bad lane's).
template <uint32_t FEAT, bool FAST>
__device__ inline __attribute__((always_inline)) ort::Ray trace_ray(const KArgs& a, int64_t rid, bool active, int64_t group,
                                     bool group_uniform, const int32_t* sched, int& range_bits,
                                     bool& bad) {
  // lanes past the end compute on ray 0 and store nothing; a lane of a valid ray that is
  // not active (the exact pass: its ray is stored already) traces its own ray, so a
  // wave-uniform row (F_MONO's readfirstlane) is the wave's own
  const int64_t r_ld = rid < a.n_rays ? rid : 0;
  // segment / wavelength of this ray
  const int64_t sidx = a.seg ? r_ld / a.seg_len : 0;
  int lam = 0;
  double wl = 0.0;  // F_WRAY: this ray's wavelength
  ort::Ray r;
  if constexpr (FEAT & F_GEN) {
    const ort_segment sg = a.seg[sidx];
    lam = sg.lambda_idx;
    const int64_t p = a.pupil_per_ray ? r_ld : (r_ld - sidx * a.seg_len);
    if constexpr (FAST)
      r = ort::fast::generate_ray(sg, a.px[p], a.py[p], a.apod, bad);
    else
      r = ort::generate_ray(sg, a.px[p], a.py[p], a.apod);
  } else {
    if (a.seg) lam = a.seg[sidx].lambda_idx;
    if constexpr ((FEAT & F_WRAY) != 0) wl = a.w[r_ld];
    r.x = a.in.x[r_ld];
    r.y = a.in.y[r_ld];
    r.z = a.in.z[r_ld];
    r.L = a.in.L[r_ld];
    r.M = a.in.M[r_ld];
    r.N = a.in.N[r_ld];
    r.i = a.in.i[r_ld];
    r.opd = a.in.opd[r_ld];
    r.att = 0.0;
    // the fast flat-surface refraction assumes finite directions (ort_fastpath.h)
    if constexpr (FAST) ORT_CHK(bad, !(::fabs(r.L) < __builtin_inf() && ::fabs(r.M) < __builtin_inf()));
  }
  bool unnorm = false;  // F_IA: rays.is_normalized == False after a thin lens
  if constexpr ((FEAT & F_GEN) != 0) {
    if (a.apod && (uint32_t)cst(a.apod)->kind > (uint32_t)ORT_APOD_TUKEY)
      range_bits |= ORT_STATUS_BAD_APODIZATION;
  }

#ifdef ORT_PREFETCH_SURF  // (A/B builds) surface si + 1's record loaded during surface si
  ort_surface s_next = cst(a.surf)[a.start_surface < a.n_surf ? a.start_surface : 0];
#endif
  for (int si = a.start_surface; si < a.n_surf; ++si) {
#ifdef ORT_PREFETCH_SURF
    const ort_surface s = s_next;
    s_next = cst(a.surf)[si + 1 < a.n_surf ? si + 1 : si];
#else
    const ort_surface s = cst(a.surf)[si];
#endif
    const ort_surface_optics o = surface_optics<FEAT>(a, s, lam, si, wl);
    double* tp = nullptr;  // F_TAPE: this surface's tape rows of this ray
    if constexpr ((FEAT & F_TAPE) != 0) {
      tp = a.tape + tape_row0(a.surf, si) * a.n_rays + rid;
      if (active) {
        ORT_ST(tp[0], r.x);
        ORT_ST(tp[a.n_rays], r.y);
        ORT_ST(tp[2 * a.n_rays], r.z);
        ORT_ST(tp[3 * a.n_rays], r.L);
        ORT_ST(tp[4 * a.n_rays], r.M);
        ORT_ST(tp[5 * a.n_rays], r.N);
      }
    }
    localize(a, s, r);
    double t;
    bool hn = false;  // (hnx, hny, hnz): the Newton geometry's normal at t
    double hnx = 0.0, hny = 0.0, hnz = 0.0;
    const bool radius_inf = (s.flags & ORT_SURF_RADIUS_INF) != 0;
    if (!known_geometry(s.geometry)) range_bits |= ORT_STATUS_BAD_GEOMETRY;
    if (s.geometry == ORT_GEOM_PLANE) {
      if constexpr (FAST)
        t = ort::fast::distance_plane(r, bad);
      else
        t = ort::distance_plane(r);
    } else if (s.geometry == ORT_GEOM_STANDARD) {
      if constexpr (FAST)
        t = ort::fast::distance_conic(r, s, radius_inf, bad);
      else
        t = ort::distance_conic(r, s.radius, s.conic, radius_inf);
    } else {
      if constexpr ((FEAT & F_KM) != 0) {
        t = newton_distance<FEAT, FAST>(a, s, si, r, active, group, group_uniform, range_bits,
                                        hn, hnx, hny, hnz, active ? tp : nullptr, sched, bad);
      } else {
        t = __builtin_nan("");  // unreachable: the host sets geometry_mask
      }
    }
    if constexpr ((FEAT & F_TAPE) != 0) {
      if (active) ORT_ST(tp[6 * a.n_rays], t);
    }
    const double n_pre = o.n_pre, u = o.u, alpha = o.alpha_pre;
    if constexpr ((FEAT & F_IA) != 0) {
      ort::propagate(r, t, alpha);
      if (unnorm) {  // homogeneous.py:55-57
        ort::normalize_dir(r);
        unnorm = false;
      }
      ort::add_opd(r, t, n_pre);
      if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
      if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
      interact<FEAT>(a, s, r, o, lam, wl, unnorm);
    } else if constexpr (FAST) {
      // the closed kernel's fast surface step (closed_surfaces), the Newton surfaces with
      // the normal of their last evaluation
      ort::propagate(r, t, alpha);
      ort::add_opd(r, t, n_pre);
      if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
      if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
      const bool refl = (s.flags & ORT_SURF_REFLECTIVE) != 0;
      const bool is_plane = s.geometry == ORT_GEOM_PLANE;
      if (!hn && !refl && (is_plane || (radius_inf && s.geometry == ORT_GEOM_STANDARD))) {
        ort::fast::refract_flat(r, u, o.u_sq, bad);  // normal (0, 0, +-1): reduced exactly
      } else {
        double nx, ny, nz;
        if (hn) {
          nx = hnx; ny = hny; nz = hnz;
        } else if (is_plane) {
          nx = 0.0; ny = 0.0; nz = 1.0;
        } else if (s.flags & ORT_SURF_INV_R2) {
          ort::fast::normal_conic_rcp(r.x, r.y, s, nx, ny, nz, bad);
        } else {
          ort::normal_conic(r.x, r.y, s.radius, s.conic, nx, ny, nz);
        }
        if (refl)
          ort::reflect(r, nx, ny, nz);
        else
          ort::fast::refract(r, nx, ny, nz, u, o.u_sq, bad);
      }
    } else if constexpr ((FEAT & F_KM) != 0) {
      if (hn) {  // finish_surface with the normal of the last Newton evaluation
        ort::propagate(r, t, alpha);
        ort::add_opd(r, t, n_pre);
        if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
        if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
        if (s.flags & ORT_SURF_REFLECTIVE)
          ort::reflect(r, hnx, hny, hnz);
        else
          ort::refract(r, hnx, hny, hnz, u);
      } else {
        ort::finish_surface<(FEAT & F_KM)>(r, s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed, t, n_pre, u,
                                           alpha);
      }
    } else {
      // closed-form geometries only: plane / conic normal inline
      ort::propagate(r, t, alpha);
      ort::add_opd(r, t, n_pre);
      if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
#ifndef ORT_NO_AP_PROG
      if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
#endif
      double nx, ny, nz;
      if (s.geometry == ORT_GEOM_PLANE) {
        nx = 0.0; ny = 0.0; nz = 1.0;
      } else if (s.flags & ORT_SURF_INV_R2) {
        ort::normal_conic_rcp(r.x, r.y, s.radius, s.conic, s.inv_r2, nx, ny, nz);
      } else {
        ort::normal_conic(r.x, r.y, s.radius, s.conic, nx, ny, nz);
      }
      if (s.flags & ORT_SURF_REFLECTIVE)
        ort::reflect(r, nx, ny, nz);
      else
        ort::refract(r, nx, ny, nz, u);
    }
    globalize(a, s, r);
    if constexpr ((FEAT & F_REC) != 0) {
      if ((s.flags & ORT_SURF_RECORD) && active) {
        double* base = a.rec + (int64_t)s.rec_slot * 8 * a.n_rays + rid;
        ORT_ST(base[0 * a.n_rays], r.x);
        ORT_ST(base[1 * a.n_rays], r.y);
        ORT_ST(base[2 * a.n_rays], r.z);
        ORT_ST(base[3 * a.n_rays], r.L);
        ORT_ST(base[4 * a.n_rays], r.M);
        ORT_ST(base[5 * a.n_rays], r.N);
        ORT_ST(base[6 * a.n_rays], ort::intensity(r));
        ORT_ST(base[7 * a.n_rays], r.opd);
      }
    }
  }
  // real_ray_tracer.py:84-89: image-space propagate by the last surface's thickness
  // (final_mat < 0: plain SurfaceGroup.trace, no propagate)
  if (a.final_mat >= 0) {
    ort::propagate(r, a.final_thickness, final_alpha<FEAT>(a, lam, wl));
    if constexpr ((FEAT & F_IA) != 0) {
      if (unnorm) ort::normalize_dir(r);
    }
  }
  return r;
}

// The rays of (virtual) block vb of nb: the body of trace_kernel's grid-stride loop
template <uint32_t FEAT>
__device__ __forceinline__ void trace_block(const KArgs& a, const int32_t* sched, int64_t vb,
                                            int64_t nb) {
  const int64_t rid =
      a.block_remap ? pair_major_ray(a, vb, nb) : vb * kBlock + threadIdx.x;
  const bool active = rid < a.n_rays;
  const int64_t r_ld = active ? rid : 0;  // inactive lanes compute on ray 0, store nothing
  // kNewtonFast: first the whole ray on ort_fastpath.h's deferred-check sequences; the
  // lanes that stayed inside their ranges store it (bit-identical to the exact path) and
  // leave, the rest fall through to the exact trace below on their own (divergent, rare),
  // reporting their Newton statistics per lane
  bool redo = false;
  if constexpr (kNewtonFast<FEAT>) {
    if (a.newton_mode == ORT_NEWTON_SCHEDULE && !a.exact_only) {
      bool bad = false;
      int fast_bits = 0;
      int64_t fgroup = 0;
      bool fgroup_uniform = true;
      fgroup = r_ld / a.group_len;
      const int64_t g0 = __shfl(fgroup, 0, 64);
      fgroup_uniform = __all(fgroup == g0);
      const ort::Ray rf = trace_ray<FEAT, true>(a, rid, active, fgroup, fgroup_uniform, sched,
                                                fast_bits, bad);
      bad = bad | !ort::fast::state_ok(rf);
#ifdef ORT_FAST_PROBE  // measurement builds only (tools/fast_probe.py): mark, do not redo
      if (bad) {
        ort::Ray rb = rf;
        rb.x = __builtin_nan("");
        if (active) store_ray(a, rid, rb);
        return;
      }
#endif
      if (!bad) {
        if (fast_bits && active && a.status) atomicOr(a.status, fast_bits);
        if (active) store_ray(a, rid, rf);
        return;
      }
      redo = true;
    }
  }

  // segment / wavelength / Newton group of this ray
  const int64_t sidx = a.seg ? r_ld / a.seg_len : 0;
  int lam = 0;
  double wl = 0.0;  // F_WRAY: this ray's wavelength
  ort::Ray r;
  if constexpr (FEAT & F_GEN) {
    const ort_segment sg = a.seg[sidx];
    lam = sg.lambda_idx;
    const int64_t p = a.pupil_per_ray ? r_ld : (r_ld - sidx * a.seg_len);
    r = ort::generate_ray(sg, a.px[p], a.py[p], a.apod);
  } else {
    if (a.seg) lam = a.seg[sidx].lambda_idx;
    if constexpr ((FEAT & F_WRAY) != 0) wl = a.w[r_ld];
    r.x = a.in.x[r_ld];
    r.y = a.in.y[r_ld];
    r.z = a.in.z[r_ld];
    r.L = a.in.L[r_ld];
    r.M = a.in.M[r_ld];
    r.N = a.in.N[r_ld];
    r.i = a.in.i[r_ld];
    r.opd = a.in.opd[r_ld];
    r.att = 0.0;
  }
  int64_t group = 0;
  bool group_uniform = true;
  if constexpr ((FEAT & F_KM) != 0) {
    group = r_ld / a.group_len;
    if (redo) {  // divergent (the fast pass's bad lanes only): no wave-wide reductions
      group_uniform = false;
    } else {
      const int64_t g0 = __shfl(group, 0, 64);
      group_uniform = __all(group == g0);
    }
  }
  int range_bits = 0;
  bool unnorm = false;  // F_IA: rays.is_normalized == False after a thin lens
  if constexpr ((FEAT & F_GEN) != 0) {
    if (a.apod && (uint32_t)cst(a.apod)->kind > (uint32_t)ORT_APOD_TUKEY)
      range_bits |= ORT_STATUS_BAD_APODIZATION;
  }

#ifdef ORT_PREFETCH_SURF  // (A/B builds) surface si + 1's record loaded during surface si
  ort_surface s_next = cst(a.surf)[a.start_surface < a.n_surf ? a.start_surface : 0];
#endif
  for (int si = a.start_surface; si < a.n_surf; ++si) {
#ifdef ORT_PREFETCH_SURF
    const ort_surface s = s_next;
    s_next = cst(a.surf)[si + 1 < a.n_surf ? si + 1 : si];
#else
    const ort_surface s = cst(a.surf)[si];
#endif
    const ort_surface_optics o = surface_optics<FEAT>(a, s, lam, si, wl);
    double* tp = nullptr;  // F_TAPE: this surface's tape rows of this ray
    if constexpr ((FEAT & F_TAPE) != 0) {
      tp = a.tape + tape_row0(a.surf, si) * a.n_rays + rid;
      if (active) {
        ORT_ST(tp[0], r.x);
        ORT_ST(tp[a.n_rays], r.y);
        ORT_ST(tp[2 * a.n_rays], r.z);
        ORT_ST(tp[3 * a.n_rays], r.L);
        ORT_ST(tp[4 * a.n_rays], r.M);
        ORT_ST(tp[5 * a.n_rays], r.N);
      }
    }
    localize(a, s, r);
    double t;
    bool hn = false;  // (hnx, hny, hnz): the Newton geometry's normal at t
    double hnx = 0.0, hny = 0.0, hnz = 0.0;
    if (!known_geometry(s.geometry)) range_bits |= ORT_STATUS_BAD_GEOMETRY;
    if (s.geometry == ORT_GEOM_PLANE) {
      t = ort::distance_plane(r);
    } else if (s.geometry == ORT_GEOM_STANDARD) {
      t = ort::distance_conic(r, s.radius, s.conic, (s.flags & ORT_SURF_RADIUS_INF) != 0);
    } else {
      if constexpr ((FEAT & F_KM) != 0) {
        bool unused = false;
        t = newton_distance<FEAT>(a, s, si, r, active, group, group_uniform, range_bits, hn,
                                  hnx, hny, hnz, active ? tp : nullptr, sched, unused);
      } else {
        t = __builtin_nan("");  // unreachable: the host sets geometry_mask
      }
    }
    if constexpr ((FEAT & F_TAPE) != 0) {
      if (active) ORT_ST(tp[6 * a.n_rays], t);
    }
    const double n_pre = o.n_pre, u = o.u, alpha = o.alpha_pre;
    if constexpr ((FEAT & F_IA) != 0) {
      ort::propagate(r, t, alpha);
      if (unnorm) {  // homogeneous.py:55-57
        ort::normalize_dir(r);
        unnorm = false;
      }
      ort::add_opd(r, t, n_pre);
      if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
      if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
      interact<FEAT>(a, s, r, o, lam, wl, unnorm);
    } else if constexpr ((FEAT & F_KM) != 0) {
      if (hn) {  // finish_surface with the normal of the last Newton evaluation
        ort::propagate(r, t, alpha);
        ort::add_opd(r, t, n_pre);
        if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
        if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
        if (s.flags & ORT_SURF_REFLECTIVE)
          ort::reflect(r, hnx, hny, hnz);
        else
          ort::refract(r, hnx, hny, hnz, u);
      } else {
        ort::finish_surface<(FEAT & F_KM)>(r, s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed, t, n_pre, u,
                                           alpha);
      }
    } else {
      // closed-form geometries only: plane / conic normal inline
      ort::propagate(r, t, alpha);
      ort::add_opd(r, t, n_pre);
      if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
#ifndef ORT_NO_AP_PROG
      if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
#endif
      double nx, ny, nz;
      if (s.geometry == ORT_GEOM_PLANE) {
        nx = 0.0; ny = 0.0; nz = 1.0;
      } else if (s.flags & ORT_SURF_INV_R2) {
        ort::normal_conic_rcp(r.x, r.y, s.radius, s.conic, s.inv_r2, nx, ny, nz);
      } else {
        ort::normal_conic(r.x, r.y, s.radius, s.conic, nx, ny, nz);
      }
      if (s.flags & ORT_SURF_REFLECTIVE)
        ort::reflect(r, nx, ny, nz);
      else
        ort::refract(r, nx, ny, nz, u);
    }
    globalize(a, s, r);
    if constexpr ((FEAT & F_REC) != 0) {
      if ((s.flags & ORT_SURF_RECORD) && active) {
        double* base = a.rec + (int64_t)s.rec_slot * 8 * a.n_rays + rid;
        ORT_ST(base[0 * a.n_rays], r.x);
        ORT_ST(base[1 * a.n_rays], r.y);
        ORT_ST(base[2 * a.n_rays], r.z);
        ORT_ST(base[3 * a.n_rays], r.L);
        ORT_ST(base[4 * a.n_rays], r.M);
        ORT_ST(base[5 * a.n_rays], r.N);
        ORT_ST(base[6 * a.n_rays], ort::intensity(r));
        ORT_ST(base[7 * a.n_rays], r.opd);
      }
    }
  }
  // real_ray_tracer.py:84-89: image-space propagate by the last surface's thickness
  // (final_mat < 0: plain SurfaceGroup.trace, no propagate)
  if (a.final_mat >= 0) {
    ort::propagate(r, a.final_thickness, final_alpha<FEAT>(a, lam, wl));
    if constexpr ((FEAT & F_IA) != 0) {
      if (unnorm) ort::normalize_dir(r);
    }
  }

  if (range_bits && active && a.status) atomicOr(a.status, range_bits);
  if constexpr ((FEAT & F_RMS) != 0) rms_epilogue(a, r, active, vb);
  if (!active) return;
  store_ray(a, rid, r);
}

template <uint32_t FEAT>
__global__ __launch_bounds__(kBlock) ORT_TRACE_OCC void trace_kernel(const KArgs a) {
  if (a.run_if && *cst(a.run_if) != 1) return;  // a device-side re-trace that is not needed
  // verify-and-re-trace (ort_options.verify_*): every workgroup derives the decision of
  // ort_newton_fixup from the previous launch's statistics into its own copy of the
  // schedule, workgroup 0 publishes it (verify_flag, sched_out), and the rays are traced
  // on that copy only when the schedule was corrected
  const int32_t* sched = a.sched;
  __shared__ int32_t vsched[ORT_VERIFY_MAX_SCHED];
  __shared__ int32_t vcodes[kBlock / 64];
  if constexpr ((FEAT & F_KM) != 0) {
    if (a.vstats) {
      const int64_t ng = (a.n_rays + a.group_len - 1) / a.group_len;
      const int nsch = (int)ng * a.n_surf;  // <= ORT_VERIFY_MAX_SCHED (host-checked)
      // the schedule's loads issued together with the flag's, so either path below waits
      // for one memory round trip, not two (the no-op rounds after a settled one are
      // mostly that wait)
      constexpr int kPre = ORT_VERIFY_MAX_SCHED / kBlock;
      int32_t pre[kPre];
#pragma unroll
      for (int q = 0; q < kPre; ++q) {
        const int k = threadIdx.x + q * kBlock;
        pre[q] = k < nsch ? a.sched[k] : 0;
      }
      const int prev = a.vprev ? *a.vprev : 1;
      if (prev != 1) {  // the previous launch did not run: nothing to verify
        if (blockIdx.x == 0) {
#pragma unroll
          for (int q = 0; q < kPre; ++q) {
            const int k = threadIdx.x + q * kBlock;
            if (k < nsch) a.sched_out[k] = pre[q];
          }
          if (threadIdx.x == 0) *a.vflag = prev;
        }
        return;
      }
#pragma unroll
      for (int q = 0; q < kPre; ++q) {
        const int k = threadIdx.x + q * kBlock;
        if (k < nsch) vsched[k] = pre[q];
      }
      __syncthreads();
      const int c = newton_decide(a.surf, a.n_surf, ng, a.vstats, a.conv_base, vsched, vcodes);
      if (blockIdx.x == 0) {
        for (int k = threadIdx.x; k < nsch; k += kBlock) a.sched_out[k] = vsched[k];
        if (threadIdx.x == 0) *a.vflag = c;
      }
      if (c != 1) return;
      sched = vsched;
    }
  }
  const int64_t nb = (a.n_rays + kBlock - 1) / kBlock;
  if constexpr ((FEAT & F_STRIDE) != 0) {
    // a verify-and-re-trace round: at most kVerifyGrid workgroups stride over the nb
    // blocks of rays (the usual outcome is "nothing to re-trace", so the round costs the
    // dispatch of a chip's worth of workgroups, not one per 256 rays). Its own
    // instantiation: the loop raises the register pressure of the body, and the first
    // launch of a call runs the loop-free kernel.
    for (int64_t vb = blockIdx.x; vb < nb; vb += gridDim.x) trace_block<FEAT>(a, sched, vb, nb);
  } else {
    trace_block<FEAT>(a, sched, blockIdx.x, nb);
  }
}

// Closed-form lenses (planes, spheres, conics: no Newton surface) -- the DoubleGauss /
// Cooke / ReverseTelephoto path. One ray per lane: at <= 64 VGPRs the kernel runs 8 waves
// per SIMD, which hides the fp64 div/sqrt latency better than 2 or 4 rays per lane
// (measured: 2 rays/lane 7% slower at 5 waves/SIMD, 4 rays/lane 28% slower).
// Per surface: one batch of scalar loads (surface record + optics of this wavelength).
//
// FAST = true: the surface math of ort_fastpath.h (range checks deferred into `bad`);
// FAST = false: ort_core.h's per-operation exact path. The kernel runs the fast trace and
// re-traces on the exact path only the lanes whose `bad` is set (operands outside the
// ranges where the short sequences are the IEEE results: NaN / missed rays, zeros, ...),
// so every output is the exact path's.
template <uint32_t FEAT, bool FAST>
__device__ inline ort::Ray closed_ray_in(const KArgs& a, int64_t r_ld, int& lam, double& wl,
                                         bool& bad) {
  ort::Ray r;
  if constexpr ((FEAT & F_GEN) != 0) {
    const int64_t sidx = a.n_seg == 1 ? 0 : r_ld / a.seg_len;
    const ort_segment sg = a.n_seg == 1 ? cst(a.seg)[0] : a.seg[sidx];
    lam = sg.lambda_idx;
    const int64_t p = a.pupil_per_ray ? r_ld : (r_ld - sidx * a.seg_len);
    // no apodization here: trace_closed_kernel applies it to the stored intensity
    // (non-temporal pupil loads measured no gain: 66.7 / 66.3 vs 66.3 / 65.9 us, config 4
    // mixed; the pupil is re-read from L2 when segments share it)
    if constexpr (FAST)
      r = ort::fast::generate_ray(sg, a.px[p], a.py[p], nullptr, bad);
    else
      r = ort::generate_ray(sg, a.px[p], a.py[p], nullptr);
  } else {
    if (a.seg) lam = a.seg[a.n_seg == 1 ? 0 : r_ld / a.seg_len].lambda_idx;
    if constexpr ((FEAT & F_WRAY) != 0) wl = a.w[r_ld];
    r.x = a.in.x[r_ld];
    r.y = a.in.y[r_ld];
    r.z = a.in.z[r_ld];
    r.L = a.in.L[r_ld];
    r.M = a.in.M[r_ld];
    r.N = a.in.N[r_ld];
    r.i = a.in.i[r_ld];
    r.opd = a.in.opd[r_ld];
    r.att = 0.0;
    // the fast flat-surface refraction assumes finite directions (ort_fastpath.h)
    if constexpr (FAST) bad = bad | !(::fabs(r.L) < __builtin_inf() && ::fabs(r.M) < __builtin_inf());
  }
  return r;
}

// apod: F_GEN | F_REC with an apodization, the pupil factor of this ray, multiplied into
// every recorded intensity (the generated ray would carry it from the start,
// ray_generator.py:91-95); 1 otherwise
template <uint32_t FEAT, bool FAST>
__device__ inline void closed_surfaces(const KArgs& a, ort::Ray& r, int lam, double wl,
                                       int64_t rid, bool active, bool& bad, bool& geom_bad,
                                       double apod = 1.0) {
#ifdef ORT_PREFETCH_SURF  // (A/B builds) surface si + 1's record loaded during surface si
  ort_surface s_next = cst(a.surf)[a.start_surface < a.n_surf ? a.start_surface : 0];
#endif
  for (int si = a.start_surface; si < a.n_surf; ++si) {
#ifdef ORT_PREFETCH_SURF
    const ort_surface s = s_next;
    s_next = cst(a.surf)[si + 1 < a.n_surf ? si + 1 : si];
#else
    const ort_surface s = cst(a.surf)[si];
#endif
    const ort_surface_optics o = surface_optics<FEAT>(a, s, lam, si, wl);
    if constexpr ((FEAT & F_AXIAL) != 0)
      r.z = r.z + -s.cs_t[2];  // x + -0 and y + -0 are identities
    else
      localize(a, s, r);
    const bool is_plane = s.geometry == ORT_GEOM_PLANE;
    const bool radius_inf = (s.flags & ORT_SURF_RADIUS_INF) != 0;
    double t;
    if constexpr (FAST) {
      t = is_plane ? ort::fast::distance_plane(r, bad)
                   : ort::fast::distance_conic(r, s, radius_inf, bad);
    } else {
      t = is_plane ? ort::distance_plane(r) : ort::distance_conic(r, s.radius, s.conic, radius_inf);
    }
    if constexpr (FAST) {
      // not a closed-form id: a uniform test, left to the exact pass (below)
      ORT_CHK(bad, s.geometry > ORT_GEOM_STANDARD || s.geometry < ORT_GEOM_PLANE);
    } else if (!is_plane && s.geometry != ORT_GEOM_STANDARD) {  // NaN rays + status
      t = __builtin_nan("");
      geom_bad = true;
    }
#ifndef ORT_NO_ALPHA_FLAGS
    if constexpr ((FEAT & F_WRAY) != 0)
      ort::propagate(r, t, o.alpha_pre);
    else
      ort::propagate_flagged(r, t, o.alpha_pre, s.flags);
#else
    ort::propagate(r, t, o.alpha_pre);
#endif
    ort::add_opd(r, t, o.n_pre);
    if (s.flags & ORT_SURF_APERTURE) ort::clip_radial(r, s.ap_rmax2, s.ap_rmin2);
#ifndef ORT_NO_AP_PROG
    if (s.flags & ORT_SURF_APERTURE_PROG) ort::clip_program(r, cst(a.coef) + s.ap_off, s.ap_len);
#endif
    const bool refl = (s.flags & ORT_SURF_REFLECTIVE) != 0;
#ifndef ORT_NO_FLAT_FAST
    constexpr bool kFlat = FAST;
#else
    constexpr bool kFlat = false;
#endif
    if (kFlat && !refl && (is_plane || radius_inf)) {
      ort::fast::refract_flat(r, o.u, o.u_sq, bad);  // normal (0, 0, +-1): reduced exactly
    } else {
      double nx, ny, nz;
      if (is_plane) {
        nx = 0.0; ny = 0.0; nz = 1.0;
      } else if (s.flags & ORT_SURF_INV_R2) {
        if constexpr (FAST)
          ort::fast::normal_conic_rcp(r.x, r.y, s, nx, ny, nz, bad);
        else
          ort::normal_conic_rcp(r.x, r.y, s.radius, s.conic, s.inv_r2, nx, ny, nz);
      } else {
        ort::normal_conic(r.x, r.y, s.radius, s.conic, nx, ny, nz);
      }
      if (refl) {
        ort::reflect(r, nx, ny, nz);
      } else {
        if constexpr (FAST)
          ort::fast::refract(r, nx, ny, nz, o.u, o.u_sq, bad);
        else
          ort::refract(r, nx, ny, nz, o.u);
      }
    }
    if constexpr ((FEAT & F_AXIAL) != 0) {
      r.x = r.x + 0.0;  // the reference's translate by +cs_t (= +0): -0 becomes +0
      r.y = r.y + 0.0;
      r.z = r.z + s.cs_t[2];
    } else {
      globalize(a, s, r);
    }
    if constexpr ((FEAT & F_REC) != 0) {
      if ((s.flags & ORT_SURF_RECORD) && active) {
        double* b = a.rec + (int64_t)s.rec_slot * 8 * a.n_rays + rid;
        ORT_ST(b[0 * a.n_rays], r.x);
        ORT_ST(b[1 * a.n_rays], r.y);
        ORT_ST(b[2 * a.n_rays], r.z);
        ORT_ST(b[3 * a.n_rays], r.L);
        ORT_ST(b[4 * a.n_rays], r.M);
        ORT_ST(b[5 * a.n_rays], r.N);
        if constexpr ((FEAT & F_GEN) != 0)
          ORT_ST(b[6 * a.n_rays], a.apod ? apod * ort::intensity(r) : ort::intensity(r));
        else
          ORT_ST(b[6 * a.n_rays], ort::intensity(r));
        ORT_ST(b[7 * a.n_rays], r.opd);
      }
    }
  }
}

template <uint32_t FEAT>
__global__ __launch_bounds__(kClosedBlock) __attribute__((amdgpu_waves_per_eu(8))) void trace_closed_kernel(const KArgs a) {
  int64_t rid;
  bool active;
  if constexpr ((FEAT & F_SPOT) != 0) {  // pair-aligned chunks (KArgs.spot_part1)
    const int64_t pair = blockIdx.x / a.spot_chunks;
    const int64_t j = (int64_t)(blockIdx.x - pair * a.spot_chunks) * kClosedBlock + threadIdx.x;
    rid = pair * a.seg_len + j;
    active = j < a.seg_len && rid < a.n_rays;
  } else {
    rid = (int64_t)blockIdx.x * kClosedBlock + threadIdx.x;
    active = rid < a.n_rays;
  }
  const int64_t r_ld = active ? rid : 0;
  int lam = 0;
  double wl = 0.0;  // F_WRAY: this ray's wavelength
  bool bad = false, geom_bad = false;
  // recorded intensities of apodized generated rays carry the pupil factor (the stored
  // image intensity gets it below); the record kernels alone pay for it up front
  double apod_f = 1.0;
  if constexpr ((FEAT & F_GEN) != 0 && (FEAT & F_REC) != 0) {
    if (a.apod) {
      const int64_t sidx = a.n_seg == 1 ? 0 : r_ld / a.seg_len;
      const int64_t p = a.pupil_per_ray ? r_ld : (r_ld - sidx * a.seg_len);
      apod_f = ort::apodize(*cst(a.apod), a.px[p], a.py[p]);
    }
  }
#ifndef ORT_NO_DEFERRED_CHECKS
  ort::Ray r = closed_ray_in<FEAT, true>(a, r_ld, lam, wl, bad);
  closed_surfaces<FEAT, true>(a, r, lam, wl, rid, active, bad, geom_bad, apod_f);
  bad = bad | !ort::fast::state_ok(r);  // the upper-range failures (ort_fastpath.h)
  if (__builtin_expect(bad, 0)) {  // this lane left the fast path's ranges: exact re-trace
    r = closed_ray_in<FEAT, false>(a, r_ld, lam, wl, bad);
    closed_surfaces<FEAT, false>(a, r, lam, wl, rid, active, bad, geom_bad, apod_f);
  }
#else
  ort::Ray r = closed_ray_in<FEAT, false>(a, r_ld, lam, wl, bad);
  closed_surfaces<FEAT, false>(a, r, lam, wl, rid, active, bad, geom_bad, apod_f);
#endif
  if (a.final_mat >= 0) ort::propagate(r, a.final_thickness, final_alpha<FEAT>(a, lam, wl));
  if (geom_bad && a.status && threadIdx.x == 0) atomicOr(a.status, (int)ORT_STATUS_BAD_GEOMETRY);
  if constexpr ((FEAT & F_GEN) != 0) {
    if (a.apod && a.status && threadIdx.x == 0 &&
        (uint32_t)cst(a.apod)->kind > (uint32_t)ORT_APOD_TUKEY)
      atomicOr(a.status, (int)ORT_STATUS_BAD_APODIZATION);
  }
  double inten = ort::intensity(r);
#ifndef ORT_NO_APOD
  if constexpr ((FEAT & F_GEN) != 0) {
    // Pupil apodization (ray_generator.py:91-95), applied to the stored intensity: the
    // trace only ever multiplies the intensity (absorption) or zeroes it (clipping), so
    // apod * (1 * e^att or 0) is the value the ray would carry from an apodized start,
    // with the apodization code outside the traced loop.
    if (a.apod) {
      const int64_t sidx = a.n_seg == 1 ? 0 : r_ld / a.seg_len;
      const int64_t p = a.pupil_per_ray ? r_ld : (r_ld - sidx * a.seg_len);
      inten = ort::apodize(*cst(a.apod), a.px[p], a.py[p]) * inten;
    }
  }
#endif
  if constexpr ((FEAT & F_SPOT) != 0) spot_epilogue<FEAT>(a, r, inten, active);
  if (!active) return;
  ORT_ST(a.out.x[rid], r.x);
  ORT_ST(a.out.y[rid], r.y);
  ORT_ST(a.out.z[rid], r.z);
  ORT_ST(a.out.L[rid], r.L);
  ORT_ST(a.out.M[rid], r.M);
  ORT_ST(a.out.N[rid], r.N);
  ORT_ST(a.out.i[rid], inten);
  ORT_ST(a.out.opd[rid], r.opd);
}

// Sum over the 64 lanes of a wave. With the whole wave active: DPP row operations
// (VALU moves, no LDS round trip per step): quad_perm xor 1 and xor 2, row_half_mirror,
// row_mirror (a row of 16 summed in every lane), row_bcast15 / row_bcast31 (rows
// accumulated into lane 63), then lane 63 read into a scalar. Otherwise the xor
// butterfly through ds_bpermute. Either way a fixed order: deterministic run to run.
template <int CTRL, int ROW_MASK>
__device__ inline double dpp_step(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROW_MASK, 0xf,
                                             false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ inline double wave_sum(double v) {
  if (__builtin_amdgcn_read_exec() == ~0ull) {
    v += dpp_step<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dpp_step<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dpp_step<0x141, 0xf>(v);  // row_half_mirror
    v += dpp_step<0x140, 0xf>(v);  // row_mirror
    v += dpp_step<0x142, 0xa>(v);  // row_bcast15 -> rows 1, 3
    v += dpp_step<0x143, 0xc>(v);  // row_bcast31 -> rows 2, 3
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------------
// Forward-mode VJP (ORT_VJP_UNROLLED): vjp_ray (ort_sweep.h) per lane; each block writes
// its P sums (wave sums, then the block's four waves in order) to partial[block][P] and
// vjp_reduce_kernel adds, per parameter, the blocks' sums in index order to grad: the
// same bits run to run (no atomics).
// ---------------------------------------------------------------------------------
template <int P, uint32_t KM>
__global__ __launch_bounds__(kBlock) void vjp_kernel(const KArgs a, const JArgs j) {
  const int64_t rid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = rid < a.n_rays;
  double acc[P];
  vjp_ray<P, KM>(a, j, rid, active, acc);
  __shared__ double part[kBlock / 64][P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const double v = wave_sum(acc[k]);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < P) {
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) v += part[w][threadIdx.x];
    j.partial[(int64_t)blockIdx.x * P + threadIdx.x] = v;
  }
}

// One block per parameter k < P of the chunk: grad[p0 + k] += the blocks' partials summed
// in a fixed order (strided per thread, wave sums, the four waves in order).
template <int P>
__global__ __launch_bounds__(kBlock) void vjp_reduce_kernel(const JArgs j, int64_t n_block) {
  const int k = blockIdx.x;
  if (j.p0 + k >= j.n_param) return;  // uniform
  double v = 0.0;
  for (int64_t b = threadIdx.x; b < n_block; b += kBlock) v += j.partial[b * P + k];
  v = wave_sum(v);
  __shared__ double ws[kBlock / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < kBlock / 64; ++w) s += ws[w];
    j.grad[j.p0 + k] += s;
  }
}

// ---------------------------------------------------------------------------------
// Geometry primitives of one surface in its local frame (geometries/*.py: sag(x, y),
// surface_normal(rays), distance(rays)) -- the reference's per-geometry API, used by
// its geometry tests and by analysis code that probes a surface.
// ---------------------------------------------------------------------------------
struct GArgs {
  int32_t surface;
  int32_t mode;  // 0: sag / normal at (x, y); 1: distance of the rays in a.in
  const double* x;
  const double* y;
  double* sag;
  double* nx;
  double* ny;
  double* nz;
  double* t;
};

template <uint32_t KM>
__global__ __launch_bounds__(kBlock) void geom_kernel(const KArgs a, const GArgs g) {
  const int64_t rid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool active = rid < a.n_rays;
  const int64_t r_ld = active ? rid : 0;
  const ort_surface s = cst(a.surf)[g.surface];
  bool range_error = false;
  int range_bits = 0;
  if (g.mode == 0) {
    const double x = g.x[r_ld], y = g.y[r_ld];
    double z, nx, ny, nz;
    if (s.geometry == ORT_GEOM_PLANE) {  // plane.py:45-59, :79-98
      z = 0.0;
      nx = 0.0; ny = 0.0; nz = 1.0;
    } else if (s.geometry == ORT_GEOM_STANDARD) {  // standard.py:73-87, :154-167
      z = ort::sag_conic(x * x + y * y, s.radius, s.conic);
      ort::normal_conic(x, y, s.radius, s.conic, nx, ny, nz);
    } else {
      if constexpr (KM != 0) {
        z = ort::newton_sagnorm<KM>(s, s.radius, s.conic, cst(a.coef), cst(a.zern), kNoSeed, x, y, true,
                                    range_error, nx, ny, nz);
      } else {
        z = nx = ny = nz = __builtin_nan("");
      }
    }
    if (active) {
      if (g.sag) g.sag[rid] = z;
      if (g.nx) g.nx[rid] = nx;
      if (g.ny) g.ny[rid] = ny;
      if (g.nz) g.nz[rid] = nz;
    }
  } else {
    ort::Ray r;
    r.x = a.in.x[r_ld];
    r.y = a.in.y[r_ld];
    r.z = a.in.z[r_ld];
    r.L = a.in.L[r_ld];
    r.M = a.in.M[r_ld];
    r.N = a.in.N[r_ld];
    r.i = 1.0;
    r.opd = 0.0;
    r.att = 0.0;
    double t;
    if (s.geometry == ORT_GEOM_PLANE) {
      t = ort::distance_plane(r);
    } else if (s.geometry == ORT_GEOM_STANDARD) {
      t = ort::distance_conic(r, s.radius, s.conic, (s.flags & ORT_SURF_RADIUS_INF) != 0);
    } else {
      if constexpr (KM != 0) {
        bool hn, bad = false;
        double hnx, hny, hnz;
        t = newton_distance<KM>(a, s, g.surface, r, active, 0, true, range_bits, hn, hnx, hny,
                                hnz, nullptr, a.sched, bad);
      } else {
        t = __builtin_nan("");
      }
    }
    if (active && g.t) g.t[rid] = t;
  }
  if (range_error) range_bits |= range_bit(s);
  if (range_bits && active && a.status) atomicOr(a.status, range_bits);
}

typedef void (*KernelFn)(const KArgs);
typedef void (*VjpFn)(const KArgs, const JArgs);
typedef void (*VjpReduceFn)(const JArgs, int64_t);
typedef void (*GeomFn)(const KArgs, const GArgs);

// kernel selection (defined in the ort_k_*.hip translation units)
KernelFn select_trace(uint32_t feat);      // Newton lenses, any F_GEN / F_REC  (ort_k_trace*.hip)
int closed_block();                        // its block size                   (ort_k_closed.hip)
KernelFn select_closed(uint32_t feat);     // closed-form lenses                (ort_k_closed.hip)
KernelFn select_generate();                // ray generation only               (ort_k_closed.hip)
KernelFn select_trace_w(uint32_t feat);    // Newton lenses, per-ray wavelengths (ort_k_trace_w.hip)
KernelFn select_trace_mono(uint32_t feat); // Newton lenses, F_GEN, wave-uniform wavelength row
                                           // (ort_k_trace_mono.hip)
KernelFn select_trace_ia(uint32_t feat);   // thin-lens / phase / grating lenses (ort_k_trace_ia.hip)
KernelFn select_trace_tape(uint32_t feat); // Newton lenses, F_GEN, writing the adjoint tape
                                           // (ort_k_trace_tape.hip)
// n(w), k(w) of one material (ort_material_nk)                            (ort_k_closed.hip)
void launch_material_nk(const ort_material* mats, const double* coef, int32_t mat,
                        const double* w, int64_t n, double* n_out, double* k_out,
                        hipStream_t stream);
VjpFn select_vjp(int tangents, uint32_t km);  // tangents 1, 2 or 4             (ort_k_vjp*.hip)
VjpReduceFn select_vjp_reduce(int tangents); // its fixed-order reduction      (ort_k_vjp.hip)
GeomFn select_geom(uint32_t km);           // per-geometry primitives           (ort_k_geom.hip)
int launch_pupil(const ort_pupil& d, double* px, double* py, hipStream_t stream);  // ort_k_pupil.hip

}  // namespace ortk
