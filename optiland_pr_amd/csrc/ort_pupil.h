// ort_pupil.h -- pupil sampling on the device (distribution.py:72-408).
//
// Point k of a distribution computed from its index alone, so a trace can be fed from
// HBM-resident pupil coordinates generated in one launch (ort_generate_pupil) instead
// of NumPy on the host plus a host-to-device copy:
//   uniform           linspace grid masked to r^2 <= 1 (row table from the host)
//   line_x / line_y   linspace(-1 or 0, 1, n) on one axis
//   cross             the y arm, then the x arm without a duplicated origin
//   ring, hexapolar   linspace angles, (r cos t, r sin t)
//   random            numpy.random.default_rng: PCG64 draws (the state before each
//                     chunk of 256 draws and the 128-bit affine jump to each lane come
//                     from the host), u = (next64 >> 11) * 2^-53, r = u1,
//                     t = 2 pi u2, (sqrt(r) cos t, sqrt(r) sin t)
// linspace follows numpy's arithmetic (i * step + start, the last point = stop), so the
// grid kinds are bit-identical to NumPy. cos / sin are correctly rounded (double-double
// evaluation around a 257-entry table); NumPy's (glibc's, <= 0.55 ulp) differ from the
// correctly rounded value in ~0.15% of arguments, by one ulp.
#pragma once

#include <math.h>
#include <stdint.h>

#include "../../include/optiland_rt.h"

#ifndef ORT_HD
#define ORT_HD __host__ __device__
#endif
#ifndef ORT_INLINE
#define ORT_INLINE ORT_HD inline __attribute__((always_inline))
#endif

#if defined(__HIPCC__)
#define ORT_TABLE __constant__
#else
#define ORT_TABLE
#endif
#include "ort_sincos_table.h"

namespace ort {

// ---- double-double arithmetic (exact error terms with fma; no contraction) ---------
struct DD {
  double hi, lo;
};
ORT_INLINE DD two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
ORT_INLINE DD fast_two_sum(double a, double b) {  // |a| >= |b|
  const double s = a + b;
  return {s, b - (s - a)};
}
ORT_INLINE DD two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
ORT_INLINE DD dd_add(DD a, DD b) {
  DD s = two_sum(a.hi, b.hi);
  const DD t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}
ORT_INLINE DD dd_mul(DD a, DD b) {
  DD p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return fast_two_sum(p.hi, p.lo);
}
ORT_INLINE DD dd_neg(DD a) { return {-a.hi, -a.lo}; }

// Correctly rounded sin and cos of x in [0, 2 pi] (relative error of the double-double
// result ~1e-30 before the final rounding). x = a_j + r, a_j = j pi / 128 the nearest
// table node (|r| <= pi / 256, r exact in double-double since a_j is held to 3 doubles),
// sin / cos of r by their Taylor series (leading terms in double-double), then the
// angle-addition formulas with the table's double-double sin a_j, cos a_j. The zeros of
// sin / cos sit on table nodes, so the result keeps full relative precision there.
ORT_INLINE void cr_sincos(double x, double& s_out, double& c_out) {
  int j = (int)(x * (128.0 / 3.141592653589793) + 0.5);
  j = j < 0 ? 0 : (j > 256 ? 256 : j);
  const double* T = ort_sincos_table[j];
  DD r = two_sum(x, -T[0]);
  r = dd_add(r, DD{-T[1], -T[2]});
  const DD r2 = dd_mul(r, r);
  const double t = r2.hi;
  // sin r = r (1 - t/3! + t^2/5! - t^3/7! + t^4/9! - t^5/11! + t^6/13!), t = r^2: the
  // t and t^2 terms in double-double, the rest (< 1e-15 relative) in double
  const DD s6 = dd_mul(r2, DD{-ORT_INVF3_HI, -ORT_INVF3_LO});
  const DD r4 = dd_mul(r2, r2);
  const DD s120 = dd_mul(r4, DD{ORT_INVF5_HI, ORT_INVF5_LO});
  const double st =
      t * t * t * (-ORT_INVF7_HI + t * (ORT_INVF9_HI + t * (-ORT_INVF11_HI + t * ORT_INVF13_HI)));
  const DD ps = dd_add(dd_add(DD{1.0, 0.0}, s6), dd_add(s120, DD{st, 0.0}));
  const DD sr = dd_mul(r, ps);
  // cos r = 1 - t/2! + t^2/4! - t^3/6! + t^4/8! - t^5/10! + t^6/12!
  const DD c2 = DD{-0.5 * r2.hi, -0.5 * r2.lo};
  const DD c24 = dd_mul(r4, DD{ORT_INVF4_HI, ORT_INVF4_LO});
  const double ct =
      t * t * t * (-ORT_INVF6_HI + t * (ORT_INVF8_HI + t * (-ORT_INVF10_HI + t * ORT_INVF12_HI)));
  const DD cr = dd_add(dd_add(DD{1.0, 0.0}, c2), dd_add(c24, DD{ct, 0.0}));
  const DD sa{T[3], T[4]}, ca{T[5], T[6]};
  const DD s = dd_add(dd_mul(sa, cr), dd_mul(ca, sr));
  const DD c = dd_add(dd_mul(ca, cr), dd_neg(dd_mul(sa, sr)));
  s_out = s.hi + s.lo;
  c_out = c.hi + c.lo;
}

// numpy.linspace(start, stop, num)[i]: i * step + start, the last point = stop
ORT_INLINE double linspace_at(double start, double stop, int64_t num, int64_t i) {
  if (num == 1) return start;
  if (i == num - 1) return stop;
  const double step = (stop - start) / (double)(num - 1);
  return (double)i * step + start;
}

// ---- PCG64 (numpy.random.PCG64: 128-bit LCG, XSL-RR output) ---------------------------
#if defined(__SIZEOF_INT128__)
typedef unsigned __int128 u128;
ORT_INLINE u128 mk128(uint64_t lo, uint64_t hi) { return ((u128)hi << 64) | lo; }
ORT_INLINE double pcg64_double(u128 s) {  // output of the state after a step
  const uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
  const uint64_t x = hi ^ lo;
  const unsigned rot = (unsigned)(hi >> 58);
  const uint64_t v = (x >> rot) | (x << ((64u - rot) & 63u));
  return (double)(v >> 11) * (1.0 / 9007199254740992.0);
}
#endif

// ---- point k of the distribution ------------------------------------------------------
ORT_INLINE void pupil_point(const ort_pupil& d, int64_t k, double& px, double& py) {
  switch (d.kind) {
    case ORT_PUPIL_UNIFORM: {  // distribution.py:161-186
      // rows[2 r] = grid row index, rows[2 r + 1] = first column; starts[r] = first point
      int lo = 0, hi = d.n_rows - 1;
      while (lo < hi) {  // last row with start <= k
        const int mid = (lo + hi + 1) >> 1;
        if (d.row_start[mid] <= k) lo = mid; else hi = mid - 1;
      }
      const int64_t col = d.row_col[2 * lo + 1] + (k - d.row_start[lo]);
      px = linspace_at(-1.0, 1.0, d.n, col);
      py = linspace_at(-1.0, 1.0, d.n, d.row_col[2 * lo]);
      return;
    }
    case ORT_PUPIL_LINE_X:  // distribution.py:72-99
      px = linspace_at(d.positive_only ? 0.0 : -1.0, 1.0, d.n, k);
      py = 0.0;
      return;
    case ORT_PUPIL_LINE_Y:  // distribution.py:102-129
      px = 0.0;
      py = linspace_at(d.positive_only ? 0.0 : -1.0, 1.0, d.n, k);
      return;
    case ORT_PUPIL_CROSS: {  // distribution.py:223-265
      if (k < d.n) {
        px = 0.0;
        py = linspace_at(-1.0, 1.0, d.n, k);
      } else {
        int64_t i = k - d.n;
        if ((d.n & 1) && i >= d.n / 2) ++i;
        px = linspace_at(-1.0, 1.0, d.n, i);
        py = 0.0;
      }
      return;
    }
    case ORT_PUPIL_RING: {  // distribution.py:358-375
      const double t = linspace_at(0.0, 2.0 * 3.141592653589793, d.n + 1, k);
      cr_sincos(t, py, px);
      return;
    }
    case ORT_PUPIL_HEXAPOLAR: {  // distribution.py:189-220
      if (k == 0) {
        px = 0.0;
        py = 0.0;
        return;
      }
      // ring i >= 1 holds points 1 + 3 i (i - 1) .. 3 i (i + 1)
      int64_t i = (int64_t)((3.0 + ::sqrt(9.0 + 12.0 * (double)(k - 1))) / 6.0);
      while (i > 1 && 1 + 3 * i * (i - 1) > k) --i;
      while (1 + 3 * (i + 1) * i <= k) ++i;
      const int64_t jj = k - (1 + 3 * i * (i - 1));
      const double r = linspace_at(0.0, 1.0, d.n + 1, i);
      const double t = linspace_at(0.0, 2.0 * 3.141592653589793, 6 * i + 1, jj);
      double s, c;
      cr_sincos(t, s, c);
      px = r * c;
      py = r * s;
      return;
    }
    default: {  // ORT_PUPIL_RANDOM, distribution.py:132-158
#if defined(__SIZEOF_INT128__)
      const int64_t chunk = k >> 8;
      const int lane = (int)(k & 255);
      const uint64_t* J = d.rng_lane + 4 * lane;  // affine map of lane + 1 steps
      const u128 A = mk128(J[0], J[1]), C = mk128(J[2], J[3]);
      const uint64_t* S = d.rng_chunk + 4 * chunk;  // states before the chunk's draws
      const u128 s1 = A * mk128(S[0], S[1]) + C;
      const u128 s2 = A * mk128(S[2], S[3]) + C;
      const double u1 = pcg64_double(s1);
      const double u2 = pcg64_double(s2);
      const double t = 0.0 + 6.283185307179586 * u2;  // uniform(0, 2 pi)
      const double rr = 0.0 + 1.0 * u1;              // uniform(0, 1)
      double s, c;
      cr_sincos(t, s, c);
      const double q = ::sqrt(rr);
      px = q * c;
      py = q * s;
#else
      px = py = NAN;
#endif
      return;
    }
  }
}

}  // namespace ort
