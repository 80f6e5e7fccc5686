// ort_fastpath.h -- the closed-form surface math (plane / conic, ray generation) with
// DEFERRED range checks, for trace_closed_kernel (ort_kernels.h).
//
// ort_core.h's sqrt / shared_div / sdiv run the correctly rounded gfx950 sequences
// without their range wrappers and fall back per operation (a divergent branch around
// every op) when an operand leaves the range where the wrappers are identities. Here the
// same instruction sequences run unconditionally and each operation only ORs "an operand
// was outside that range" into a per-lane flag; a lane that ends its ray with the flag
// set re-traces the whole ray on the per-operation path. Every value a lane keeps is
// therefore bit-identical to ort_core.h's (and so to the reference's IEEE operations):
// inside the ranges the fast sequences ARE the IEEE results, outside them the ray is
// recomputed. What goes away is the exec-mask bookkeeping and the taken branch per op.
//
// Ranges (the same as ort_core.h):
//   sqrt(x):   2^-767 <= x < inf
//   a / b:     2^-300 <= |b| <= 2^300 and 2^-300 <= |a| <= 2^300, or a == +0: the
//              quotient sequence q0 = a y, r = fma(-b, q0, a), q = fma(r, y, q0) then
//              yields +0 * sign(b) exactly (q0 carries the sign, r = +0); -0 and every
//              other value outside the range takes the exact path.
//
// Upper bounds (and the divisors' lower bound) are not tested per operation. Past them the short sequences do not return
// a wrong FINITE value, only a non-finite one: sqrt(+inf) gives NaN (rsq = 0, g = inf*0);
// a numerator large enough to matter overflows q0 = a y to inf and the quotient to inf or
// NaN. Non-finite values are sticky in the ray state -- a non-finite t makes the OPD
// (opd += |t n|, a sum of non-negative terms) non-finite for good, a non-finite direction
// or position makes the next t non-finite or is itself an output -- so the kernel tests
// the finished state once (state_ok) and re-traces such lanes exactly. Only the
// numerators' and sqrt's lower bounds (where the sequences would underflow into a finite,
// wrongly rounded result) and the divisors' upper bound (a reciprocal small enough to
// underflow a quotient) stay per operation.
//
// Formulas and their order follow ort_core.h (and through it the reference files cited
// there); only the check placement differs. Host compilation: plain IEEE operations.
#pragma once

#include "ort_core.h"

namespace ort {
namespace fast {

// Lens constants: from the host table (ort_surface.two_r / one_plus_k / r_sq,
// ort_surface_optics.u_sq) or recomputed per wave (ORT_NO_HOSTCONST; same values)
#ifdef ORT_NO_HOSTCONST
#define ORT_TWO_R(s) (2.0 * (s).radius)
#define ORT_ONE_PLUS_K(s) (1.0 + (s).conic)
#define ORT_R_SQ(s) ((s).radius * (s).radius)
#define ORT_U_SQ(u, u_sq) ((u) * (u))
#else
#define ORT_TWO_R(s) ((s).two_r)
#define ORT_ONE_PLUS_K(s) ((s).one_plus_k)
#define ORT_R_SQ(s) ((s).r_sq)
#define ORT_U_SQ(u, u_sq) (u_sq)
#endif

// ORT_FAST_NOCHECK (timing experiments only, never a shipped build): drop the range
// checks to measure what they cost
#ifdef ORT_FAST_NOCHECK
#define ORT_CHK(bad, cond) ((void)0)
#else
#define ORT_CHK(bad, cond) ((bad) = (bad) | (cond))
#endif

ORT_INLINE bool is_pos_zero(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_class(v, 1 << 6);  // v_cmp_class_f64: +0 only
#else
  return v == 0.0 && !signbit(v);
#endif
}

// sqrt(x) for 2^-767 <= x < inf (ort_core.h sqrt)
ORT_INLINE double sqrt(double x, bool& bad) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  ORT_CHK(bad, !(x >= 0x1p-767));  // +inf gives NaN: left to state_ok
  return g;
#else
  (void)bad;
  return ::sqrt(x);
#endif
}

// sqrt(x) where x >= 1 unless NaN (sums of squares plus 1): only the upper bound could
// fail, and +inf / NaN give NaN, which state_ok catches: no test
ORT_INLINE double sqrt_ge1(double x, bool& bad) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  (void)bad;
  return g;
#else
  (void)bad;
  return ::sqrt(x);
#endif
}

ORT_INLINE SharedDiv shared_div(double b, bool& bad) {
  SharedDiv d;
  d.b = b;
  d.ok = true;
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  d.y = y;
  // |b| <= 2^300 (false for NaN). Below 2^-1021 (zero and subnormal divisors included)
  // the reciprocal is infinite and every quotient non-finite -- NaN for a zero
  // numerator, +-inf or NaN otherwise -- which state_ok catches; in between the
  // refined reciprocal is accurate and, as every numerator is >= 2^-300 or an exact zero
  // (sdiv / sdiv0 / num_ok), q0 = a y cannot underflow (|q| >= 2^-600).
  ORT_CHK(bad, !(::fabs(b) <= 0x1p300));
#else
  (void)bad;
  d.y = 0.0;
#endif
  return d;
}

// the divisor is known to lie in [1, inf) unless NaN (a norm of (., ., 1))
// (no test: the divisor is a norm sqrt(s), s = a^2 + b^2 + 1 >= 1, so it is at most
// sqrt(DBL_MAX) < 2^512 -- its refined reciprocal >= 2^-512 is accurate and the quotients
// of the checked numerators (|a| >= 2^-300 or +-0, and -1) stay normal -- or, with s
// overflowed, +inf, whose zero reciprocal makes every quotient NaN for state_ok; NaN
// likewise. Round 6: the b <= 2^300 test this had was one of those that cannot fail on a
// finite result.)
ORT_INLINE SharedDiv shared_div_ge1(double b, bool& bad) {
  SharedDiv d;
  d.b = b;
  d.ok = true;
  (void)bad;
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  d.y = y;
#else
  (void)bad;
  d.y = 0.0;
#endif
  return d;
}

ORT_INLINE double quot(double a, const SharedDiv& d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double q0 = a * d.y;
  const double r = fma(-d.b, q0, a);
  return fma(r, d.y, q0);
#else
  return a / d.b;
#endif
}

// The same quotient for a divisor known to be > 0 with the residual formed negated:
// rn = fma(b, q0, -a) = -r exactly, and fma(-rn, y, q0) rounds q0 + r y exactly as
// fma(r, y, q0) does, but an exact-zero numerator keeps its sign (+-0 / b = +-0): for
// a = -0, rn = (-0) + (+0) = +0 and (-rn) y + q0 = (-0) + (-0) = -0, where the plain
// form's r = +0 turns -0 / b into +0. The negations are free operand modifiers. (For
// b < 0 the plain form is the one that is right for both zeros.)
ORT_INLINE double quot_pos(double a, const SharedDiv& d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double q0 = a * d.y;
  const double rn = fma(d.b, q0, -a);
  return fma(-rn, d.y, q0);
#else
  return a / d.b;
#endif
}

// |a| >= 2^-300 (false for 0 and NaN); a numerator past 2^300 overflows into a
// non-finite quotient (see the header)
ORT_INLINE bool num_ok(double a) { return ::fabs(a) >= 0x1p-300; }

// a / b, |a| >= 2^-300
ORT_INLINE double sdiv(double a, const SharedDiv& d, bool& bad) {
  ORT_CHK(bad, !num_ok(a));
  return quot(a, d);
}
// a / b, |a| >= 2^-300 or a == +0 (coordinates on a symmetry plane)
ORT_INLINE double sdiv0(double a, const SharedDiv& d, bool& bad) {
  ORT_CHK(bad, !(num_ok(a) || is_pos_zero(a)));
  return quot(a, d);
}

// a / b as one IEEE division
ORT_INLINE double div(double a, double b, bool& bad) {
  const SharedDiv d = shared_div(b, bad);
  return sdiv0(a, d, bad);
}

// rays/ray_generator.py:71-106 + fields/field_types.py:160-181 (ort_core.h generate_ray)
ORT_INLINE Ray generate_ray(const ort_segment& s, double px, double py,
                            const ort_apodization* apod, bool& bad) {
  Ray r;
  double x0, y0;
  if (s.mode == ORT_GEN_INFINITE) {
    x0 = px * s.epd / 2.0 * s.vx + s.x_off;
    y0 = py * s.epd / 2.0 * s.vy + s.y_off;
  } else {
    x0 = s.x_off;
    y0 = s.y_off;
  }
  const double z0 = s.z0;
  double x1, y1;
  if (s.mode == ORT_GEN_TELECENTRIC) {
    x1 = px * s.vx + x0;
    y1 = py * s.vy + y0;
  } else {
    x1 = px * s.epd * s.vx / 2.0;
    y1 = py * s.epd * s.vy / 2.0;
  }
  const double z1 = s.epl;
  const double dx = x1 - x0, dy = y1 - y0, dz = z1 - z0;
  const double mag = sqrt(dx * dx + dy * dy + dz * dz, bad);
  ORT_CHK(bad, (mag < 1e-9));  // the (0, 0, 1) branch of ray_generator.py:82-89
  const SharedDiv dm = shared_div(mag, bad);
  // mag > 0: quot_pos is exact for zero numerators of either sign
  ORT_CHK(bad, !((num_ok(dx) || dx == 0.0) && (num_ok(dy) || dy == 0.0) &&
                 (num_ok(dz) || dz == 0.0)));
  r.L = quot_pos(dx, dm);
  r.M = quot_pos(dy, dm);
  r.N = quot_pos(dz, dm);
  r.x = x0;
  r.y = y0;
  r.z = z0;
  r.i = apod ? apodize(*apod, px, py) : 1.0;  // no range-sensitive operations
  r.opd = 0.0;
  r.att = 0.0;
  return r;
}

// The end-of-trace test of the header: every output of the ray state finite and below
// 2^1000 (false for NaN / inf; the bound also covers a quotient that would overflow only
// in the short sequence, |q| ~ 2^1023). The intensity is not tested: only the clip tests
// write it, on positions that are themselves tested here.
ORT_INLINE bool state_ok(const Ray& r) {
  constexpr double kMax = 0x1p1000;
  return ::fabs(r.x) < kMax && ::fabs(r.y) < kMax && ::fabs(r.z) < kMax &&
         ::fabs(r.L) < kMax && ::fabs(r.M) < kMax && ::fabs(r.N) < kMax && ::fabs(r.opd) < kMax;
}

// plane.py:61-77 (-z / N) and the plane branch of standard.py:100-103
ORT_INLINE double distance_plane(const Ray& r, bool& bad) { return div(-r.z, r.N, bad); }

// standard.py:89-140 (ort_core.h distance_conic); s.two_r = 2 R formed on the host
ORT_INLINE double distance_conic(const Ray& r, const ort_surface& s, bool radius_inf,
                                 bool& bad) {
  if (radius_inf) {
    const double Ns = ::fabs(r.N) > 1e-14 ? r.N : 1e-14;
    return div(-r.z, Ns, bad);
  }
  const double R = s.radius, k = s.conic;
  const double N2 = r.N * r.N;
  const double z2 = r.z * r.z;
  double a, b, c;
  if (k == 0.0) {
    a = r.L * r.L + r.M * r.M + N2;
    b = 2.0 * (r.L * r.x + r.M * r.y - r.N * R + r.N * r.z);
    c = 0.0 - ORT_TWO_R(s) * r.z + r.x * r.x + r.y * r.y + z2;
  } else {
    a = k * N2 + r.L * r.L + r.M * r.M + N2;
    b = 2.0 * (k * r.N * r.z + r.L * r.x + r.M * r.y - r.N * R + r.N * r.z);
    c = k * z2 - ORT_TWO_R(s) * r.z + r.x * r.x + r.y * r.y + z2;
  }
  const double d = b * b - 4.0 * a * c;
  const double sd = sqrt(d, bad);
  const SharedDiv a2 = shared_div(2.0 * a, bad);
  // nonzero numerators (checked): quot_pos and quot agree for either sign of a
  const double n1 = -b + sd, n2 = -b - sd;
  ORT_CHK(bad, !(num_ok(n1) && num_ok(n2)));
  const double t1 = quot_pos(n1, a2);
  const double t2 = quot_pos(n2, a2);
  const double z1 = r.z + t1 * r.N;
  const double zz2 = r.z + t2 * r.N;
  // a == 0 (the -c / b branch, standard.py:138) fails shared_div's range test
  return ::fabs(z1) <= ::fabs(zz2) ? t1 : t2;
}

// standard.py:154-167 with the host's inv_r2 = RN(1 / (R * R)) (ort_core.h
// normal_conic_rcp: the Markstein-corrected quotient needs no range check of its own --
// r^2 = 0 / inf / NaN give the reference's 1 - q)
ORT_INLINE void normal_conic_rcp(double x, double y, const ort_surface& s, double& nx,
                                 double& ny, double& nz, bool& bad) {
  const double r2 = x * x + y * y;
  const double a = ORT_ONE_PLUS_K(s) * r2;
  const double q0 = a * s.inv_r2;
  const double q = fma(fma(-ORT_R_SQ(s), q0, a), s.inv_r2, q0);
  const double denom = s.radius * sqrt(1.0 - q, bad);
  const SharedDiv dd = shared_div(denom, bad);
  const double dfdx = sdiv0(x, dd, bad);
  const double dfdy = sdiv0(y, dd, bad);
  const double mag = sqrt_ge1(dfdx * dfdx + dfdy * dfdy + 1.0, bad);
  const SharedDiv dm = shared_div_ge1(mag, bad);
  // dfdx = x / denom with x checked (|x| in [2^-300, 2^300] or +0) and |denom| <= 2^300:
  // |dfdx| >= 2^-600 or +-0, and |dfdx| <= mag -- in range for the positive divisor
  // mag, zeros of either sign included (quot_pos): no check left to make
  nx = quot_pos(dfdx, dm);
  ny = quot_pos(dfdy, dm);
  nz = quot(-1.0, dm);  // constant numerator: always in range
}

// rays/real_rays.py:511-547 (ort_core.h align_normal) for dot != 0: sign(dot) is +-1 and
// n * sign(dot) is n with its sign bit flipped when dot < 0 -- the same bits as the
// product; dot == 0 (sign 0) and NaN take the exact path
ORT_INLINE double align_normal(const Ray& r, double& nx, double& ny, double& nz, bool& bad) {
#ifdef ORT_NO_SIGN_XOR
  return ::ort::align_normal(r, nx, ny, nz);
#endif
  const double dot = r.L * nx + r.M * ny + r.N * nz;
  ORT_CHK(bad, !(::fabs(dot) > 0.0));
  const uint64_t sb = (uint64_t)__double_as_longlong(dot) & 0x8000000000000000ull;
  nx = __longlong_as_double((long long)((uint64_t)__double_as_longlong(nx) ^ sb));
  ny = __longlong_as_double((long long)((uint64_t)__double_as_longlong(ny) ^ sb));
  nz = __longlong_as_double((long long)((uint64_t)__double_as_longlong(nz) ^ sb));
  return ::fabs(dot);
}

// rays/real_rays.py:141-163 (ort_core.h refract); u_sq = RN(u * u) from the host table
ORT_INLINE void refract(Ray& r, double nx, double ny, double nz, double u, double u_sq,
                        bool& bad) {
  const double dot = align_normal(r, nx, ny, nz, bad);
  const double root = sqrt(1.0 - ORT_U_SQ(u, u_sq) * (1.0 - dot * dot), bad);
  const double L0 = r.L, M0 = r.M, N0 = r.N;
  r.L = u * L0 + nx * root - u * nx * dot;
  r.M = u * M0 + ny * root - u * ny * dot;
  r.N = u * N0 + nz * root - u * nz * dot;
}

// Refraction at a flat surface: the plane normal (0, 0, 1) (plane.py:79-98) or the
// infinite-radius conic's (+-0, +-0, -1) (standard.py:154-167). For finite L, M and
// N != 0 the reference's expressions reduce exactly:
//   dot = L*0 + M*0 + N*1 = N, sign(dot) = sign(N), |dot| = |N|;
//   L' = u L + (+-0) root - u (+-0) |N| = u L + 0.0 (the zero terms only turn a -0
//   product into +0, as adding +0 does), M' likewise;
//   N' = (u N + sign(N) root) - (u sign(N)) |N| = (u N + sign(N) root) - u N.
// N == 0 / NaN takes the exact path; a non-finite L or M only reaches here on a ray that
// already failed a check (or came in non-finite, which closed_ray_in flags).
ORT_INLINE void refract_flat(Ray& r, double u, double u_sq, bool& bad) {
  ORT_CHK(bad, !(::fabs(r.N) > 0.0));
  const double root = sqrt(1.0 - ORT_U_SQ(u, u_sq) * (1.0 - r.N * r.N), bad);
  const double uN = u * r.N;
  const double sroot = ::copysign(root, r.N);
  r.L = u * r.L + 0.0;
  r.M = u * r.M + 0.0;
  r.N = (uN + sroot) - uN;
}

// ---- Newton geometries (trace_kernel's deferred-check pass) --------------------------
// The quotient for a divisor of either sign with a numerator that may be +-0: IEEE's
// signed zero is quot_pos's for b > 0 and the plain form's for b < 0 (see quot_pos)
ORT_INLINE double quot_signed(double a, const SharedDiv& d) {
  return d.b > 0.0 ? quot_pos(a, d) : quot(a, d);
}
// numerator in range or an exact zero of either sign (quot_signed / quot_pos keep its sign)
ORT_INLINE bool num_ok0(double a) { return num_ok(a) || a == 0.0; }

// The asphere formulas divide by R (1 + q) and R q with q = sqrt(...) >= 0: the sign of a
// nonzero divisor is the radius's, a lens constant. With sR = +-1 that sign and the
// divisor's magnitude |R| (1 + q), |R| q (the same products: IEEE multiplication is
// sign-symmetric), a / b = (sR a) / |b| is quot_pos's form on a positive divisor -- the
// same IEEE quotient, signed zeros included (sR a flips an exact zero's sign exactly when
// b < 0) -- without quot_signed's two quotients and select. A zero divisor (q = 0)
// gives an infinite reciprocal and non-finite quotients, as the signed form does.
// |R| <= 2^149 (so |R| (1 + q) <= 2^150, R^2 <= 2^298: inside shared_div's range) is
// tested once per evaluation (lens_range) instead of a test per divisor.
ORT_INLINE SharedDiv shared_div_pos(double b) {
  bool unused = false;
  return shared_div_ge1(b, unused);  // (the same refinement, no test of its own)
}
ORT_INLINE bool lens_range(double R) { return ::fabs(R) <= 0x1p149; }

// kSlope's direct slopes (ort_core.h): norm^2 < 1e28 checked (a steeper normal or NaN
// takes the exact path, which forms the reference's expression from the unit normal)
ORT_INLINE void slope_out(double dfdx, double dfdy, double& nx, double& ny, double& nz,
                          bool& bad) {
#ifdef ORT_SLOPE_MAXCHK  // (A/B builds) |dfdx|, |dfdy| < 7e13 implies the sum < 9.8e27 + 1
  // < 1e28: the same guarantee in two compares -- no measurable gain on the MI355X
  // (profiles/r06_ab_slopemax.log, r06_ab_c3_slope_opk.log)
  ORT_CHK(bad, !(::fabs(dfdx) < 7e13 && ::fabs(dfdy) < 7e13));
#else
  ORT_CHK(bad, !(dfdx * dfdx + dfdy * dfdy + 1.0 < 1e28));
#endif
  nx = dfdx;
  ny = dfdy;
  nz = -1.0;
}

// the unit normal (dz/dx, dz/dy, -1) / norm from kSlope's direct slopes (norm^2 < 1e28
// checked by slope_out): the tail of the kNormal evaluations, operation for operation
ORT_INLINE void unit_normal_from_slope(double dfdx, double dfdy, double& nx, double& ny,
                                       double& nz, bool& bad) {
  const double mag = sqrt_ge1(dfdx * dfdx + dfdy * dfdy + 1.0, bad);
  const SharedDiv dm = shared_div_ge1(mag, bad);
  ORT_CHK(bad, !(num_ok0(dfdx) && num_ok0(dfdy)));
  nx = quot_pos(dfdx, dm);
  ny = quot_pos(dfdy, dm);
  nz = quot(-1.0, dm);
}

// even_asphere.py:82-129 (ort_core.h sagnorm_even): the same operations in the same order,
// the divisions and square roots as the deferred-check sequences; mode: kNormal or kSlope
template <class PD>
ORT_INLINE double sagnorm_even(double x, double y, const ort_surface& s, PD C,
                               int nc, int mode, double& nx, double& ny, double& nz,
                               bool& bad) {
  const double R = s.radius;
  const double aR = ::fabs(R), sR = R > 0.0 ? 1.0 : -1.0;  // (lens constants)
  ORT_CHK(bad, !lens_range(R));
  const double r2 = x * x + y * y;
  const double a = ORT_ONE_PLUS_K(s) * r2;  // (1 + k) r2: +-0 at the vertex
  const SharedDiv rr = shared_div_pos(ORT_R_SQ(s));
  ORT_CHK(bad, !num_ok0(a));
  const double q = sqrt(1.0 - quot_pos(a, rr), bad);
  const SharedDiv dz = shared_div_pos(aR * (1.0 + q));
  ORT_CHK(bad, !num_ok0(r2));
  double P, D;  // the term sums by Horner in r2 (ort_core.h even_horner)
  ort::even_horner(r2, C, nc, P, D);
  const double z = quot_pos(sR * r2, dz) + r2 * P;
  const SharedDiv dd = shared_div_pos(aR * q);
  ORT_CHK(bad, !(num_ok0(x) && num_ok0(y)));
  double dfdx = quot_pos(sR * x, dd);
  double dfdy = quot_pos(sR * y, dd);
  dfdx = dfdx + x * D;
  dfdy = dfdy + y * D;
  if (mode == kSlope) {
    slope_out(dfdx, dfdy, nx, ny, nz, bad);
    return z;
  }
  const double mag = sqrt_ge1(dfdx * dfdx + dfdy * dfdy + 1.0, bad);
  const SharedDiv dm = shared_div_ge1(mag, bad);
  ORT_CHK(bad, !(num_ok0(dfdx) && num_ok0(dfdy)));
  nx = quot_pos(dfdx, dm);
  ny = quot_pos(dfdy, dm);
  nz = quot(-1.0, dm);
  return z;
}

// odd_asphere.py:73-130 (ort_core.h sagnorm_odd); non-finite per-term slopes zeroed
template <class PD>
ORT_INLINE double sagnorm_odd(double x, double y, const ort_surface& s, PD C,
                              int nc, int mode, double& nx, double& ny, double& nz,
                              bool& bad) {
  const double R = s.radius;
  const double aR = ::fabs(R), sR = R > 0.0 ? 1.0 : -1.0;  // (lens constants)
  ORT_CHK(bad, !lens_range(R));
  const double r2 = x * x + y * y;
  const double r = sqrt(r2, bad);  // the vertex itself (r2 = 0) takes the exact path
  const double a = ORT_ONE_PLUS_K(s) * r2;
  const SharedDiv rr = shared_div_pos(ORT_R_SQ(s));
  ORT_CHK(bad, !num_ok0(a));
  const double q = sqrt(1.0 - quot_pos(a, rr), bad);
  const SharedDiv dz = shared_div_pos(aR * (1.0 + q));
  ORT_CHK(bad, !num_ok0(r2));
  double z = quot_pos(sR * r2, dz);
  double rp = r;
  for (int i = 0; i < nc; ++i) {
    z = z + C[i] * rp;
    rp = rp * r;
  }
  const SharedDiv dd = shared_div_pos(aR * q);
  ORT_CHK(bad, !(num_ok0(x) && num_ok0(y)));
  double dfdx = quot_pos(sR * x, dd);
  double dfdy = quot_pos(sR * y, dd);
  const SharedDiv dr = shared_div(r, bad);
  double rq = quot_pos(1.0, dr);  // 1 / r
  for (int i = 0; i < nc; ++i) {
    const double f = (double)(i + 1);
    double xt = f * x * C[i] * rq;
    double yt = f * y * C[i] * rq;
    if (!isfinite(xt)) xt = 0.0;
    if (!isfinite(yt)) yt = 0.0;
    rq = (i == 0) ? 1.0 : (i == 1 ? r : rq * r);
    dfdx = dfdx + xt;
    dfdy = dfdy + yt;
  }
  if (mode == kSlope) {
    slope_out(dfdx, dfdy, nx, ny, nz, bad);
    return z;
  }
  const double mag = sqrt_ge1(dfdx * dfdx + dfdy * dfdy + 1.0, bad);
  const SharedDiv dm = shared_div_ge1(mag, bad);
  ORT_CHK(bad, !(num_ok0(dfdx) && num_ok0(dfdy)));
  nx = quot_pos(dfdx, dm);
  ny = quot_pos(dfdy, dm);
  nz = quot(-1.0, dm);
  return z;
}

// newton_raphson.py:154-166 from kSlope's slopes (ort_core.h newton_step_slope)
ORT_INLINE double newton_step_slope(const Ray& r, double t, double f, double fx, double fy,
                                    bool& bad) {
  const double df = fx * r.L + fy * r.M - r.N;
  const double dfs = ::fabs(df) > 1e-14 ? df : 1e-14;
  const SharedDiv dd = shared_div(dfs, bad);
  ORT_CHK(bad, !num_ok0(f));
  return t - quot_signed(f, dd);
}

// newton_raphson.py:154-166 (ort_core.h newton_step)
ORT_INLINE double newton_step(const Ray& r, double t, double f, double nx, double ny,
                              double nz, bool& bad) {
  const double nzs = ::fabs(nz) > 1e-14 ? nz : 1e-14;
  const SharedDiv dn = shared_div(nzs, bad);
  const double mnx = -nx, mny = -ny;
  ORT_CHK(bad, !(num_ok0(mnx) && num_ok0(mny)));
  const double fx = quot_signed(mnx, dn);
  const double fy = quot_signed(mny, dn);
  const double df = fx * r.L + fy * r.M - r.N;
  const double dfs = ::fabs(df) > 1e-14 ? df : 1e-14;
  const SharedDiv dd = shared_div(dfs, bad);
  ORT_CHK(bad, !num_ok0(f));
  return t - quot_signed(f, dd);
}

}  // namespace fast
}  // namespace ort
