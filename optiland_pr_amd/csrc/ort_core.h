// ort_core.h -- per-ray fp64 arithmetic of the sequential real-ray trace.
//
// Every function here is a scalar, per-ray restatement of one reference formula, in
// the reference's evaluation order (NumPy evaluates each expression left to right with
// one IEEE rounding per operation; this file is compiled with -ffp-contract=off so the
// compiler may not fuse a*b+c). The wave-level control (Newton convergence votes,
// segment lookup, record stores) lives in ort_trace.hip.
//
// The ray-dependent quantities are templated on a scalar type T: `double` for the
// trace itself, and `Dual<P>` (value + P forward-mode tangents) for the derivative
// kernels behind the autograd op (ort_trace_pupil_vjp). The value part of a Dual is
// computed by the same operations in the same order, so it is bit-identical to the
// double trace. Lens parameters (radius, conic, coefficients) stay `double`, except the
// Zernike coefficients, which the derivative kernels seed with tangents (ZSeed).
//
// Reference files are cited as path:line under optiland/.
#pragma once

#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/optiland_rt.h"

#ifndef ORT_HD
#define ORT_HD __host__ __device__
#endif
#define ORT_INLINE ORT_HD inline __attribute__((always_inline))

namespace ort {

// ---------------------------------------------------------------------------------
// forward-mode dual numbers (derivative kernels only)
// ---------------------------------------------------------------------------------
template <int P>
struct Dual {
  double v;
  double d[P];
  ORT_HD Dual() {}
  ORT_HD Dual(double x) : v(x) {
#pragma unroll
    for (int k = 0; k < P; ++k) d[k] = 0.0;
  }
};

// the double overloads stay visible next to the Dual ones below
using ::acos;
using ::cos;
using ::exp;
using ::fabs;
using ::sin;

// IEEE sqrt. gfx950 lowers a correctly rounded fp64 sqrt to v_rsq_f64 and two Goldschmidt
// / Newton refinements wrapped in an input scaling (x < 2^-767) and a zero / +inf class
// fix-up. For 2^-767 <= x < inf the wrappers are identities, so that range runs the
// refinement alone -- the same instructions on the same values, bit-identical to sqrt(x)
// -- and every other input (0, tiny, inf, NaN, negative) takes the full sequence.
ORT_INLINE double sqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(ORT_NO_FAST_SQRT)
  // the refinement runs unconditionally (no data-dependent branch around the common
  // case); the rare out-of-range lanes redo it with the full sequence
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
  if (__builtin_expect(!(x >= 0x1p-767 && x < __builtin_inf()), 0)) g = ::sqrt(x);
  return g;
#else
  return ::sqrt(x);
#endif
}

ORT_INLINE double vv(double x) { return x; }
ORT_INLINE bool tangent_free(double) { return true; }
template <int P>
ORT_INLINE double vv(const Dual<P>& x) { return x.v; }
template <int P>
ORT_INLINE bool tangent_free(const Dual<P>& x) {
  bool z = true;
#pragma unroll
  for (int k = 0; k < P; ++k) z = z && x.d[k] == 0.0;
  return z;
}

template <int P>
ORT_INLINE Dual<P> operator+(const Dual<P>& a, const Dual<P>& b) {
  Dual<P> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] + b.d[k];
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator+(const Dual<P>& a, double b) {
  Dual<P> r = a;
  r.v = a.v + b;
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator+(double a, const Dual<P>& b) {
  Dual<P> r = b;
  r.v = a + b.v;
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator-(const Dual<P>& a) {
  Dual<P> r;
  r.v = -a.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = -a.d[k];
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator-(const Dual<P>& a, const Dual<P>& b) {
  Dual<P> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] - b.d[k];
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator-(const Dual<P>& a, double b) {
  Dual<P> r = a;
  r.v = a.v - b;
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator-(double a, const Dual<P>& b) {
  Dual<P> r;
  r.v = a - b.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = -b.d[k];
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator*(const Dual<P>& a, const Dual<P>& b) {
  Dual<P> r;
  r.v = a.v * b.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * b.v + a.v * b.d[k];
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator*(const Dual<P>& a, double b) {
  Dual<P> r;
  r.v = a.v * b;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * b;
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator*(double a, const Dual<P>& b) {
  Dual<P> r;
  r.v = a * b.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a * b.d[k];
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator/(const Dual<P>& a, const Dual<P>& b) {
  Dual<P> r;
  r.v = a.v / b.v;
  const double inv = 1.0 / b.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = (a.d[k] - r.v * b.d[k]) * inv;
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator/(const Dual<P>& a, double b) {
  Dual<P> r;
  r.v = a.v / b;
  const double inv = 1.0 / b;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * inv;
  return r;
}
template <int P>
ORT_INLINE Dual<P> operator/(double a, const Dual<P>& b) {
  Dual<P> r;
  r.v = a / b.v;
  const double s = -r.v / b.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = s * b.d[k];
  return r;
}
template <int P>
ORT_INLINE Dual<P> sqrt(const Dual<P>& a) {
  Dual<P> r;
  r.v = sqrt(a.v);
  const double h = 0.5 / r.v;
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * h;
  return r;
}
template <int P>
ORT_INLINE Dual<P> fabs(const Dual<P>& a) {  // torch.abs backward: sign(a) * g
  return a.v < 0.0 ? -a : (a.v > 0.0 ? a : Dual<P>(::fabs(a.v)));
}
template <int P>
ORT_INLINE Dual<P> cos(const Dual<P>& a) {
  Dual<P> r;
  r.v = ::cos(a.v);
  const double s = -::sin(a.v);
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * s;
  return r;
}
template <int P>
ORT_INLINE Dual<P> sin(const Dual<P>& a) {
  Dual<P> r;
  r.v = ::sin(a.v);
  const double c = ::cos(a.v);
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * c;
  return r;
}
template <int P>
ORT_INLINE Dual<P> acos(const Dual<P>& a) {
  Dual<P> r;
  r.v = ::acos(a.v);
  const double s = -1.0 / ::sqrt(1.0 - a.v * a.v);
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * s;
  return r;
}
template <int P>
ORT_INLINE Dual<P> exp(const Dual<P>& a) {
  Dual<P> r;
  r.v = ::exp(a.v);
#pragma unroll
  for (int k = 0; k < P; ++k) r.d[k] = a.d[k] * r.v;
  return r;
}

// ---------------------------------------------------------------------------------
// ray state
// ---------------------------------------------------------------------------------
// att accumulates the absorption exponent sum(-alpha t 1e3) (homogeneous.py:54); the
// intensity is i * exp(att), evaluated once per ray instead of once per surface
// (exp(a)exp(b) vs exp(a+b): a few ulps relative, see DESIGN.md Parity).
template <class T>
struct RayT {
  T x, y, z, L, M, N, i, opd, att;
};
using Ray = RayT<double>;

template <class T>
ORT_INLINE T intensity(const RayT<T>& r) {
  return vv(r.att) == 0.0 ? r.i : r.i * exp(r.att);
}

// ---------------------------------------------------------------------------------
// Division by a shared divisor. gfx950 lowers an IEEE fp64 a / b to
//   v_div_scale(b), v_rcp_f64, 2 x (fma, fma) Newton steps on the reciprocal,
//   q0 = a * y, r = fma(-b, q0, a), v_div_fmas(r, y, q0), v_div_fixup
// where the scale/fixup steps only act on extreme exponents, zeros, infinities and
// NaNs. For several numerators over one divisor the reciprocal refinement is done once
// and, inside a guarded exponent range where scale/fixup are identities, each quotient
// is the same three operations -- bit-identical to a / b. Outside the range (and on
// the host) it falls back to the plain division. Dual numbers always divide plainly
// (their value is then the same IEEE quotient).
// ---------------------------------------------------------------------------------
struct SharedDiv {
  double b, y;
  bool ok;
};

ORT_INLINE bool div_range_ok(double v) {
  const double av = ::fabs(v);
  return av >= 0x1p-300 && av <= 0x1p300;  // false for 0, inf, NaN
}

ORT_INLINE SharedDiv shared_div(double b) {
  SharedDiv d;
  d.b = b;
#if defined(__HIP_DEVICE_COMPILE__)
  d.ok = div_range_ok(b);
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  d.y = y;
#else
  d.ok = false;
  d.y = 0.0;
#endif
  return d;
}

ORT_INLINE double sdiv(double a, const SharedDiv& d) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double q0 = a * d.y;
  const double r = fma(-d.b, q0, a);
  double q = fma(r, d.y, q0);
  if (__builtin_expect(!(d.ok && div_range_ok(a)), 0)) q = a / d.b;
  return q;
#else
  return a / d.b;
#endif
}

// Quotients that only enter derivatives (the adjoint's reverse sweep and its local jets,
// whose results are compared at rtol 1e-10, never bit for bit). IEEE by default; the
// ORT_FAST_RDIV A/B builds take the reciprocal refined twice and one residual step
// (within an ulp, no scale / fix-up steps) -- measured no faster on the config-5 adjoint
// (one box, alternating: 268.97 / 261.66 us IEEE vs 273.28 / 267.99 us fast, the fast
// build's scratch 76 -> 100 B; profiles/r06_ab_rdiv.log).
ORT_INLINE double rrcp(double b) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(ORT_FAST_RDIV)
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  return fma(y, e, y);
#else
  return 1.0 / b;
#endif
}
ORT_INLINE double rdiv(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(ORT_FAST_RDIV)
  const double y = rrcp(b);
  const double q0 = a * y;
  return fma(fma(-b, q0, a), y, q0);
#else
  return a / b;
#endif
}

template <int P>
struct PlainDiv {
  Dual<P> b;
};
template <int P>
ORT_INLINE PlainDiv<P> shared_div(const Dual<P>& b) {
  return PlainDiv<P>{b};
}
template <int P>
ORT_INLINE Dual<P> sdiv(const Dual<P>& a, const PlainDiv<P>& d) {
  return a / d.b;
}
template <int P>
ORT_INLINE Dual<P> sdiv(double a, const PlainDiv<P>& d) {
  return a / d.b;
}
template <int P>
ORT_INLINE Dual<P> sdiv(const Dual<P>& a, const SharedDiv& d) {
  return a / d.b;
}

// a / d and b / d: two IEEE divisions sharing one reciprocal refinement
template <class T, class D>
ORT_INLINE void div2(const T& a, const T& b, const D& d, T& qa, T& qb) {
  const auto sd = shared_div(d);
  qa = sdiv(a, sd);
  qb = sdiv(b, sd);
}

// the normalised normal (dzdx, dzdy, -1) / norm of every Newton geometry
// (nx = dzdx / norm, ny = dzdy / norm, nz = -1 / norm): one reciprocal refinement
template <class T>
ORT_INLINE void unit_normal3(const T& dzdx, const T& dzdy, const T& norm, T& nx, T& ny, T& nz) {
  const auto sd = shared_div(norm);
  nx = sdiv(dzdx, sd);
  ny = sdiv(dzdy, sd);
  nz = sdiv(-1.0, sd);
}

// What a Newton geometry's evaluation returns besides the sag (want_normal):
//   kNoNormal  the sag alone;
//   kNormal    the unit normal (nx, ny, nz) of the interaction (and of the reference's
//              update, newton_raphson.py:150-157);
//   kSlope     the update's slopes (fx, fy, -1): the reference forms fx = -nx / nz_safe,
//              fy = -ny / nz_safe from the unit normal (nz_safe = nz floored at 1e-14 in
//              magnitude). With n = (dz/dx, dz/dy, -1) / norm that is dz/dx, dz/dy up to
//              the rounding of the normalisation, so the update takes the slopes directly
//              -- no norm, no four quotients -- while norm < 1e14 (norm^2 < 1e28). A
//              steeper normal (where the floor matters) or NaN: the even / odd / Zernike
//              kinds return the unit normal itself (nz != -1 tells it apart: nz = -1 / norm),
//              the freeform kinds the reference's (fx, fy, -1) from it; newton_step_any
//              and normal_of take either. Newton surfaces are held to 1e-9 mm and the
//              reference's update counts, not to bit-exactness (the stop rule compares
//              |f| with tol, far from the rounding of one step).
enum : int { kNoNormal = 0, kNormal = 1, kSlope = 2 };

// The Cartesian Zernike slopes are Gx / Rn off the disc rho^2 < kZernChainRho2 (normalised
// coordinates), the reference's eps-guarded polar chain on it (sagnorm_zernike)
constexpr double kZernChainRho2 = 1e-4;

// (fx, fy, -1) of the reference's update from a unit normal
template <class T>
ORT_INLINE void slope_from_normal(T& nx, T& ny, T& nz) {
  const T nzs = ::fabs(vv(nz)) > 1e-14 ? nz : T(1e-14);
  T fx, fy;
  div2(T(-nx), T(-ny), nzs, fx, fy);
  nx = fx;
  ny = fy;
  nz = T(-1.0);
}

// kSlope's direct form applies (norm^2 = dz/dx^2 + dz/dy^2 + 1 < 1e28, not NaN)
template <class T>
ORT_INLINE bool slope_direct(const T& dzdx, const T& dzdy) {
  return vv(dzdx * dzdx + dzdy * dzdy + 1.0) < 1e28;
}

// Zernike coefficient tangent seeds for the derivative kernels: term j (global index in
// lens.zern) is parameter param[j] (< 0: not differentiated); tangent slot k of this
// launch is parameter p0 + k.
struct ZSeed {
  const int32_t* param;
  int p0;
};

ORT_INLINE double zcoef(double c, int, const ZSeed&, double*) { return c; }
template <int P>
ORT_INLINE Dual<P> zcoef(double c, int j, const ZSeed& zs, Dual<P>*) {
  Dual<P> r(c);
  if (zs.param) {
    const int p = zs.param[j] - zs.p0;
#pragma unroll
    for (int k = 0; k < P; ++k) r.d[k] = (p == k) ? 1.0 : 0.0;
  }
  return r;
}

// ---------------------------------------------------------------------------------
// pupil apodization: apodization/*.py get_intensity(Px, Py), called from
// rays/ray_generator.py:91-95. The same operations in the same order as the NumPy
// expressions (x**2 is x * x, x**0.5 is sqrt, NumPy's fast scalar powers); exp / cos /
// pow are the device's libm (within an ulp or so of NumPy's: intensity parity is
// relative). Constants p[] come from the host (include/optiland_rt.h).
// ---------------------------------------------------------------------------------
ORT_INLINE double apod_pow(double x, double e) {
  // numpy fast_scalar_power: x**0 = 1, x**0.5 = sqrt, x**1 = x, x**2 = square
  if (e == 1.0) return x;
  if (e == 2.0) return x * x;
  if (e == 0.5) return sqrt(x);
  if (e == 0.0) return 1.0;
  return ::pow(x, e);
}

ORT_INLINE double apodize(const ort_apodization& a, double px, double py) {
  constexpr double kPi = 3.141592653589793;  // be.pi
  const double r2 = px * px + py * py;
  switch (a.kind) {
    case ORT_APOD_GAUSSIAN:  // gaussian.py: exp(-(Px**2 + Py**2) / (2 * sigma**2))
      return ::exp(-r2 / a.p[0]);
    case ORT_APOD_COSINE_SQUARED: {  // cosine_squared.py
      const double r = sqrt(r2);
      const double c = ::cos((kPi * r) / a.p[1]);
      return r < a.p[0] ? c * c : 0.0;
    }
    case ORT_APOD_HANN: {  // hann.py: R = D / 2, 0.5 * (1 - cos((2 * pi * r) / D))
      const double r = sqrt(r2);
      const double v = 0.5 * (1.0 - ::cos((2.0 * kPi * r) / a.p[1]));
      return r < a.p[0] ? v : 0.0;
    }
    case ORT_APOD_POLYNOMIAL: {  // polynomial.py: (1 - (r / R)**2)**p
      const double r = sqrt(r2);
      const double q = r / a.p[0];
      const double v = apod_pow(1.0 - q * q, a.p[1]);
      return r < a.p[0] ? v : 0.0;
    }
    case ORT_APOD_SUPER_GAUSSIAN:  // super_gaussian.py: exp(-((r2**0.5 / w)**n))
      return ::exp(-apod_pow(sqrt(r2) / a.p[0], a.p[1]));
    case ORT_APOD_TUKEY: {  // tukey.py
      const double r = sqrt(r2);
      if (r <= a.p[1]) return 1.0;
      if (r < a.p[0]) return 0.5 * (1.0 + ::cos(kPi * (r - a.p[1]) / a.p[2]));
      return 0.0;
    }
    case ORT_APOD_UNIFORM:  // uniform.py: ones
      return 1.0;
    default:  // not a kind this library knows: NaN rather than a silent 1
      return __builtin_nan("");
  }
}

// ---------------------------------------------------------------------------------
// ray generation: rays/ray_generator.py:49-106 + fields/field_types.py:160-181
// ---------------------------------------------------------------------------------
ORT_INLINE Ray generate_ray(const ort_segment& s, double px, double py,
                            const ort_apodization* apod = nullptr) {
  Ray r;
  double x0, y0;
  if (s.mode == ORT_GEN_INFINITE) {
    x0 = px * s.epd / 2.0 * s.vx + s.x_off;  // field_types.py:166
    y0 = py * s.epd / 2.0 * s.vy + s.y_off;  // field_types.py:167
  } else {
    x0 = s.x_off;
    y0 = s.y_off;
  }
  const double z0 = s.z0;
  double x1, y1;
  if (s.mode == ORT_GEN_TELECENTRIC) {  // ray_generator.py:70-73
    x1 = px * s.vx + x0;
    y1 = py * s.vy + y0;
  } else {
    x1 = px * s.epd * s.vx / 2.0;  // ray_generator.py:76
    y1 = py * s.epd * s.vy / 2.0;  // ray_generator.py:77
  }
  const double z1 = s.epl;
  const double dx = x1 - x0, dy = y1 - y0, dz = z1 - z0;
  double mag = sqrt(dx * dx + dy * dy + dz * dz);  // :80
  const bool is_zero = mag < 1e-9;                    // :82
  mag = is_zero ? 1.0 : mag;
  const SharedDiv dm = shared_div(mag);
  r.L = is_zero ? 0.0 : sdiv(dx, dm);
  r.M = is_zero ? 0.0 : sdiv(dy, dm);
  r.N = is_zero ? 1.0 : sdiv(dz, dm);
  r.x = x0;
  r.y = y0;
  r.z = z0;
  r.i = apod ? apodize(*apod, px, py) : 1.0;  // ray_generator.py:91-95
  r.opd = 0.0;
  r.att = 0.0;
  return r;
}

template <class T>
ORT_INLINE RayT<T> promote(const Ray& r) {
  RayT<T> o;
  o.x = T(r.x); o.y = T(r.y); o.z = T(r.z);
  o.L = T(r.L); o.M = T(r.M); o.N = T(r.N);
  o.i = T(r.i); o.opd = T(r.opd); o.att = T(r.att);
  return o;
}

// ---------------------------------------------------------------------------------
// coordinate systems: coordinate_system.py:73-107, rays/base.py:28-42,
// rays/real_rays.py:90-130 (cos/sin precomputed on the host)
// ---------------------------------------------------------------------------------
template <class T>
ORT_INLINE void apply_cs_op(RayT<T>& r, const ort_cs_op& op) {
  const double a = op.p[0], b = op.p[1], c = op.p[2];
  switch (op.kind) {
    case ORT_CS_TRANSLATE:
      r.x = r.x + a;
      r.y = r.y + b;
      r.z = r.z + c;
      break;
    case ORT_CS_ROT_X: {
      const T y = r.y * a - r.z * b, z = r.y * b + r.z * a;
      const T M = r.M * a - r.N * b, N = r.M * b + r.N * a;
      r.y = y; r.z = z; r.M = M; r.N = N;
    } break;
    case ORT_CS_ROT_Y: {
      const T x = r.x * a + r.z * b, z = -r.x * b + r.z * a;
      const T L = r.L * a + r.N * b, N = -r.L * b + r.N * a;
      r.x = x; r.z = z; r.L = L; r.N = N;
    } break;
    default: {  // ORT_CS_ROT_Z
      const T x = r.x * a - r.y * b, y = r.x * b + r.y * a;
      const T L = r.L * a - r.M * b, M = r.L * b + r.M * a;
      r.x = x; r.y = y; r.L = L; r.M = M;
    } break;
  }
}

// ---------------------------------------------------------------------------------
// intersections
// ---------------------------------------------------------------------------------
// plane.py:61-77
template <class T>
ORT_INLINE T distance_plane(const RayT<T>& r) {
  return -r.z / r.N;
}

// standard.py:89-140
template <class T, class S>
ORT_INLINE T distance_conic(const RayT<T>& r, const S& R, const S& k, bool radius_inf) {
  if (radius_inf) {
    const T Ns = ::fabs(vv(r.N)) > 1e-14 ? r.N : T(1e-14);
    return -r.z / Ns;
  }
  const T N2 = r.N * r.N;
  const T z2 = r.z * r.z;
  T a, b, c;
  // 2*k*N*z + 2*L*x + 2*M*y - 2*N*R + 2*N*z: every "2*" is an exact scaling
  // b: every term of the reference's sum carries an exact factor 2 and 2 RN(v) == RN(2 v)
  // (outside the subnormal range), so the sum of the halves doubled once is the same
  // double as the reference's sum of doubled terms, with one multiply instead of five
  if (vv(k) == 0.0 && tangent_free(k)) {
    // sphere: k*N**2 = 0, 2*k*N*z = 0, k*z**2 = 0 and 0 + v == v, so the conic terms
    // drop out without changing a bit (for finite rays)
    a = r.L * r.L + r.M * r.M + N2;
    b = 2.0 * (r.L * r.x + r.M * r.y - r.N * R + r.N * r.z);
    c = 0.0 - 2.0 * R * r.z + r.x * r.x + r.y * r.y + z2;
  } else {
    a = k * N2 + r.L * r.L + r.M * r.M + N2;
    b = 2.0 * (k * r.N * r.z + r.L * r.x + r.M * r.y - r.N * R + r.N * r.z);
    c = k * z2 - 2.0 * R * r.z + r.x * r.x + r.y * r.y + z2;
  }
  const T d = b * b - 4.0 * a * c;
  const T sd = sqrt(d);
  const auto a2 = shared_div(2.0 * a);
  const T t1 = sdiv(-b + sd, a2);
  const T t2 = sdiv(-b - sd, a2);
  const T z1 = r.z + t1 * r.N;
  const T zz2 = r.z + t2 * r.N;
  T t = ::fabs(vv(z1)) <= ::fabs(vv(zz2)) ? t1 : t2;
  if (vv(a) == 0.0) t = -c / b;
  return t;
}

// standard.py:154-167
template <class T, class S>
ORT_INLINE void normal_conic(const T& x, const T& y, const S& R, const S& k, T& nx, T& ny,
                             T& nz) {
  const T r2 = x * x + y * y;
  const T denom = R * sqrt(1.0 - (1.0 + k) * r2 / (R * R));
  const auto dd = shared_div(denom);
  const T dfdx = sdiv(x, dd);
  const T dfdy = sdiv(y, dd);
  const T mag = sqrt(dfdx * dfdx + dfdy * dfdy + 1.0);  // dfdz**2 = (-1)**2 = 1
  const auto dm = shared_div(mag);
  nx = sdiv(dfdx, dm);
  ny = sdiv(dfdy, dm);
  nz = sdiv(-1.0, dm);
}

// normal_conic with the host's correctly rounded inv_r2 = RN(1 / (R * R)): the quotient
// (1 + k) r^2 / (R * R) is q0 = a inv_r2 corrected once by its exact residual, which is
// the correctly rounded quotient (Markstein's theorem; checked here on 4e8 random
// operands incl. all-ones and power-of-two divisors). Operands outside the normal range
// only occur for r^2 = 0 / inf / NaN, where 1 - q is the same as the reference's.
ORT_INLINE void normal_conic_rcp(double x, double y, double R, double k, double inv_r2,
                                 double& nx, double& ny, double& nz) {
  const double r2 = x * x + y * y;
  const double a = (1.0 + k) * r2;
  const double q0 = a * inv_r2;
  const double rr = R * R;
  const double q = fma(fma(-rr, q0, a), inv_r2, q0);
  const double denom = R * sqrt(1.0 - q);
  const auto dd = shared_div(denom);
  const double dfdx = sdiv(x, dd);
  const double dfdy = sdiv(y, dd);
  const double mag = sqrt(dfdx * dfdx + dfdy * dfdy + 1.0);
  const auto dm = shared_div(mag);
  nx = sdiv(dfdx, dm);
  ny = sdiv(dfdy, dm);
  nz = sdiv(-1.0, dm);
}

// base conic sag, standard.py:73-87 (shared by every Newton geometry)
template <class T, class S>
ORT_INLINE T sag_conic(const T& r2, const S& R, const S& k) {
  return r2 / (R * (1.0 + sqrt(1.0 - (1.0 + k) * r2 / (R * R))));
}

// x**p for the small integer exponents the asphere sums use. NumPy squares exactly
// for p == 2 and returns x for p == 1 and 1 for p == 0 (fast scalar power); other
// exponents go through libm pow in the reference and through repeated products here
// (1-ulp-level differences on a small correction term; see DESIGN.md Parity).
template <class T>
ORT_INLINE T ipow(const T& x, int p) {
  if (p == 0) return T(1.0);
  if (p < 0) return 1.0 / ipow(x, -p);
  T r = x;
#pragma unroll 1
  for (int q = 1; q < p; ++q) r = r * x;
  return r;
}

// The Newton step evaluates the sag AND the normal at the same point P(t)
// (newton_raphson.py:140-146 then :154-166), so the geometries below evaluate both in one
// pass: the conic square root sqrt(1 - (1 + k) r^2 / R^2) is the same IEEE expression in
// the sag (standard.py:73-87) and in the normal's denominator and is computed once;
// everything else keeps the reference's per-expression order. want_normal = false: the
// sag alone (the convergence check after the last update).

// even_asphere.py:82-98 (sag) + :100-129 (normal)
// The even asphere's term sums by Horner in r^2 (round 5):
//   P = C0 + r2 (C1 + r2 (C2 + ...)),  z = conic + r2 P
//   D = 2 C0 + r2 (4 C1 + r2 (6 C2 + ...)),  dz/dx = x / (R q) + x D  (dz/dy likewise)
// The reference adds C_i * r2 ** (i + 1) term by term through libm pow (even_asphere.py:
// 95-96, 119-121); this build already formed the powers as products (not the reference's
// bits), and Newton surfaces are held to 1e-9 mm with the reference's update counts, not to
// bit-exactness. Horner takes 2 operations per term for the sag and 3 for both slopes
// (was 3 and 9). The common term counts are unrolled at compile time (the coefficients'
// scalar loads issued together instead of one dependent load per loop trip).
template <int NC, class T, class PD>
ORT_INLINE void even_horner_n(const T& r2, PD C, T& P, T& D) {
  P = T(C[NC - 1]);
  D = T(2.0 * (double)NC * C[NC - 1]);
#pragma unroll
  for (int i = NC - 2; i >= 0; --i) {
    P = P * r2 + C[i];
    D = D * r2 + 2.0 * (double)(i + 1) * C[i];
  }
}

template <class T, class PD>
ORT_INLINE void even_horner(const T& r2, PD C, int nc, T& P, T& D) {
  switch (nc) {
    case 1: return even_horner_n<1>(r2, C, P, D);
    case 2: return even_horner_n<2>(r2, C, P, D);
    case 3: return even_horner_n<3>(r2, C, P, D);
    case 4: return even_horner_n<4>(r2, C, P, D);
    case 5: return even_horner_n<5>(r2, C, P, D);
    case 6: return even_horner_n<6>(r2, C, P, D);
    default: break;
  }
  if (nc <= 0) {
    P = T(0.0);
    D = T(0.0);
    return;
  }
  P = T(C[nc - 1]);
  D = T(2.0 * (double)nc * C[nc - 1]);
  for (int i = nc - 2; i >= 0; --i) {
    P = P * r2 + C[i];
    D = D * r2 + 2.0 * (double)(i + 1) * C[i];
  }
}

template <class T, class S, class PD>
ORT_INLINE T sagnorm_even(const T& x, const T& y, const S& R, const S& k, PD C, int nc,
                          int want_normal, T& nx, T& ny, T& nz) {
  const T r2 = x * x + y * y;
  const T q = sqrt(1.0 - (1.0 + k) * r2 / (R * R));
  T P, D;
  even_horner(r2, C, nc, P, D);
  const T z = r2 / (R * (1.0 + q)) + r2 * P;
  if (want_normal) {
    const T denom = R * q;
    T dfdx, dfdy;
    div2(x, y, denom, dfdx, dfdy);
    dfdx = dfdx + x * D;
    dfdy = dfdy + y * D;
    if (want_normal == kSlope && slope_direct(dfdx, dfdy)) {
      nx = dfdx;
      ny = dfdy;
      nz = T(-1.0);
      return z;
    }
    const T mag = sqrt(dfdx * dfdx + dfdy * dfdy + 1.0);
    unit_normal3(dfdx, dfdy, mag, nx, ny, nz);
  }
  return z;
}

// odd_asphere.py:73-89 (sag) + :91-130 (normal; non-finite per-term slopes are zeroed,
// :112-122)
template <class T, class S, class PD>
ORT_INLINE T sagnorm_odd(const T& x, const T& y, const S& R, const S& k, PD C, int nc,
                         int want_normal, T& nx, T& ny, T& nz) {
  const T r2 = x * x + y * y;
  const T r = sqrt(r2);
  const T q = sqrt(1.0 - (1.0 + k) * r2 / (R * R));
  T z = r2 / (R * (1.0 + q));
  T rp = r;  // r ** (i + 1)
  for (int i = 0; i < nc; ++i) {
    z = z + C[i] * rp;
    rp = rp * r;
  }
  if (want_normal) {
    const T denom = R * q;
    T dfdx, dfdy;
    div2(x, y, denom, dfdx, dfdy);
    T rq = 1.0 / r;  // r ** (i - 1): 1/r, 1, r, r*r, r*r*r, ...
    for (int i = 0; i < nc; ++i) {
      const double f = (double)(i + 1);
      T xt = f * x * C[i] * rq;
      T yt = f * y * C[i] * rq;
      if (!isfinite(vv(xt))) xt = T(0.0);
      if (!isfinite(vv(yt))) yt = T(0.0);
      rq = (i == 0) ? T(1.0) : (i == 1 ? r : rq * r);
      dfdx = dfdx + xt;
      dfdy = dfdy + yt;
    }
    if (want_normal == kSlope && slope_direct(dfdx, dfdy)) {
      nx = dfdx;
      ny = dfdy;
      nz = T(-1.0);
      return z;
    }
    const T mag = sqrt(dfdx * dfdx + dfdy * dfdy + 1.0);
    unit_normal3(dfdx, dfdy, mag, nx, ny, nz);
  }
  return z;
}

// ---- freeform Newton geometries (coefficient blocks: include/optiland_rt.h) ---------
// x ** p for the reference's integer powers, as successive products (p <= 2 exact as
// NumPy's fast paths; p >= 3 within an ulp of libm pow)
template <class T>
ORT_INLINE T np_sign(const T& v) {  // np.sign: 0 -> 0, NaN -> NaN
  const double d = vv(v);
  return T(d > 0.0 ? 1.0 : (d < 0.0 ? -1.0 : (d == d ? 0.0 : d)));
}

// polynomial.py:93-140: conic + sum_ij C_ij x^i y^j
template <class T, class S, class PD>
ORT_INLINE T sagnorm_poly(const T& x, const T& y, const S& R, const S& k, PD B,
                          bool want_normal,
                          T& nx, T& ny, T& nz) {
  const int ni = (int)B[0], nj = (int)B[1];
  const PD C = B + 2;
  const T r2 = x * x + y * y;
  const T q = sqrt(1.0 - (1.0 + k) * r2 / (R * R));
  T z = r2 / (R * (1.0 + q));
  T xi = T(1.0);  // x ** i
  for (int i = 0; i < ni; ++i) {
    T yj = T(1.0);  // y ** j
#pragma unroll 1
    for (int j = 0; j < nj; ++j) {
      z = z + C[i * nj + j] * xi * yj;
      yj = yj * y;
    }
    xi = xi * x;
  }
  if (want_normal) {
    const T denom = R * q;
    T dzdx, dzdy;
    div2(x, y, denom, dzdx, dzdy);
    T xm = T(1.0);  // x ** (i - 1)
    for (int i = 1; i < ni; ++i) {
      T yj = T(1.0);
#pragma unroll 1
      for (int j = 0; j < nj; ++j) {
        dzdx = dzdx + (double)i * C[i * nj + j] * xm * yj;
        yj = yj * y;
      }
      xm = xm * x;
    }
    T xi2 = T(1.0);
    for (int i = 0; i < ni; ++i) {
      T ym = T(1.0);  // y ** (j - 1)
#pragma unroll 1
      for (int j = 1; j < nj; ++j) {
        dzdy = dzdy + (double)j * C[i * nj + j] * xi2 * ym;
        ym = ym * y;
      }
      xi2 = xi2 * x;
    }
    const T norm = sqrt(dzdx * dzdx + dzdy * dzdy + 1.0);
    unit_normal3(dzdx, dzdy, norm, nx, ny, nz);
  }
  return z;
}

// chebyshev.py:104-202: T_n(u) = cos(n acos u), T_n'(u) = n sin(n acos u) / sqrt(1 - u^2)
// (the 1/norm chain factor is omitted by the reference's normal; kept as is); only
// non-zero coefficients contribute (chebyshev.py:126, 155). Range error on |u| > 1.
template <class T>
ORT_INLINE T cheb_t(int n, const T& u) {
  return cos((double)n * acos(u));
}
template <class T>
ORT_INLINE T cheb_dt(int n, const T& u) {
  return (double)n * sin((double)n * acos(u)) / sqrt(1.0 - u * u);
}

template <class T, class S, class PD>
ORT_INLINE T sagnorm_cheb(const T& x, const T& y, const S& R, const S& k, PD B,
                          bool want_normal,
                          bool& range_error, T& nx, T& ny, T& nz) {
  const int ni = (int)B[0], nj = (int)B[1];
  const double norm_x = B[2], norm_y = B[3];
  const PD C = B + 4;
  const T xn = x / norm_x;
  const T yn = y / norm_y;
  if (::fabs(vv(xn)) > 1.0 || ::fabs(vv(yn)) > 1.0) range_error = true;
  const T r2 = x * x + y * y;
  const T q = sqrt(1.0 - (1.0 + k) * r2 / (R * R));
  T z = r2 / (R * (1.0 + q));
  T dzdx, dzdy;
  if (want_normal) {
    const T denom = R * q;
    div2(x, y, denom, dzdx, dzdy);
  }
  for (int i = 0; i < ni; ++i) {
#pragma unroll 1
    for (int j = 0; j < nj; ++j) {
      const double c = C[i * nj + j];
      if (c == 0.0) continue;
      const T ti = cheb_t(i, xn), tj = cheb_t(j, yn);
      z = z + c * ti * tj;
      if (want_normal) {
        dzdx = dzdx + cheb_dt(i, xn) * c * tj;
        dzdy = dzdy + cheb_dt(j, yn) * c * ti;
      }
    }
  }
  if (want_normal) {
    const T norm = sqrt(dzdx * dzdx + dzdy * dzdy + 1.0);
    unit_normal3(dzdx, dzdy, norm, nx, ny, nz);
  }
  return z;
}

// biconic.py:69-158: z = cx x^2 / (1 + sqrt(1 - (1 + kx) cx^2 x^2)) + (same in y), with
// the reference's clamps
template <class T>
ORT_INLINE T biconic_profile(double c, double kk, const T& u) {
  const T v = 1.0 - (1.0 + kk) * (c * c) * (u * u);
  const T st = vv(v) < 1e-14 ? T(0.0) : v;
  const T den = 1.0 + sqrt(st);
  const T sden = ::fabs(vv(den)) < 1e-14 ? T(1e-14) : den;
  return (c * (u * u)) / sden;
}
template <class T>
ORT_INLINE T biconic_slope(double c, double kk, const T& u) {
  const T v = 1.0 - (1.0 + kk) * (c * c) * (u * u);
  const T st = vv(v) < 1e-14 ? T(1e-14) : v;
  const T ds = sqrt(st);
  const T sds = ::fabs(vv(ds)) < 1e-14 ? T(1e-14) : ds;
  return (c * u) / sds;
}

template <class T, class PD>
ORT_INLINE T sagnorm_biconic(const T& x, const T& y, PD B, bool want_normal, T& nx, T& ny,
                             T& nz) {
  const double cx = B[0], cy = B[1], kx = B[2], ky = B[3];
  const T zx = cx == 0.0 ? T(0.0) : biconic_profile(cx, kx, x);
  const T zy = cy == 0.0 ? T(0.0) : biconic_profile(cy, ky, y);
  if (want_normal) {
    const T dfdx = cx == 0.0 ? T(0.0) : biconic_slope(cx, kx, x);
    const T dfdy = cy == 0.0 ? T(0.0) : biconic_slope(cy, ky, y);
    const T mag = sqrt(dfdx * dfdx + dfdy * dfdy + 1.0);
    const T smag = vv(mag) < 1e-14 ? T(1.0) : mag;
    unit_normal3(dfdx, dfdy, smag, nx, ny, nz);
  }
  return zx + zy;
}

// toroidal.py:75-233: Y-Z profile z_y(y) (conic + even polynomial in y) swept around an
// axis at distance R_rot
template <class T, class PD>
ORT_INLINE T toroid_zy(PD B, const T& y, bool deriv) {
  const double c = B[1], kk = B[2];
  const bool has_yz = B[3] != 0.0;
  const int np = (int)B[4];
  const double eps = 1e-14;
  const T y2 = y * y;
  T z = T(0.0);
  if (has_yz) {
    const T v = 1.0 - (1.0 + kk) * (c * c) * y2;
    if (!deriv) {  // _calculate_zy, toroidal.py:75-107
      const T root = vv(v) < 0.0 ? T(0.0) : v;
      const T den = 1.0 + sqrt(root);
      const T sden = ::fabs(vv(den)) < eps ? T(eps) : den;
      z = (c * y2) / sden;
    } else {  // _calculate_zy_derivative, toroidal.py:109-141
      const T root = vv(v) < eps ? T(eps) : v;
      const T sq = sqrt(root);
      const T ssq = ::fabs(vv(sq)) < eps ? T(eps) : sq;
      z = (c * y) / ssq;
    }
  }
  if (np > 0) {
    T poly = T(0.0);
    T cur = deriv ? y : y2;
#pragma unroll 1
    for (int i = 0; i < np; ++i) {
      const double a = B[5 + i];
      if (!deriv) {
        poly = poly + a * cur;
      } else {
        const double pc = 2.0 * ((double)i + 1.0);
        poly = poly + a * pc * cur;
      }
      cur = cur * y2;
    }
    z = z + poly;
  }
  return z;
}

template <class T, class PD>
ORT_INLINE T sagnorm_toroidal(const T& x, const T& y, PD B, bool want_normal, T& nx, T& ny,
                              T& nz) {
  const double Rr = B[0];
  const double eps = 1e-14;
  const T zy = toroid_zy(B, y, false);
  const bool rinf = isinf(Rr);
  T z;
  T term = T(INFINITY);
  if (rinf) {
    z = zy;
  } else {
    const T d = Rr - zy;
    term = d * d - x * x;
    z = vv(term) < 0.0 ? T(NAN) : zy + (d - np_sign(d) * sqrt(term));
  }
  if (want_normal) {
    const T dzdy = toroid_zy(B, y, true);
    T fx, fy;
    if (rinf) {
      fx = T(0.0);
      fy = dzdy;
    } else {
      const bool valid = vv(term) >= 0.0;
      const T st = valid ? term : T(eps);
      const T sq = sqrt(st);
      const T ssq = ::fabs(vv(sq)) < eps ? T(eps) : sq;
      const double sR = Rr > 0.0 ? 1.0 : (Rr < 0.0 ? -1.0 : 0.0);
      fx = valid ? sR * x / ssq : T(0.0);
      fy = valid ? sR * (Rr - zy) * dzdy / ssq : T(0.0);
    }
    const T mag = sqrt(fx * fx + fy * fy + 1.0);
    const T smag = vv(mag) < eps ? T(1.0) : mag;
    const bool ok = vv(term) >= 0.0;
    nx = ok ? fx / smag : T(0.0);
    ny = ok ? fy / smag : T(0.0);
    nz = ok ? -1.0 / smag : T(-1.0);
  }
  return z;
}

// ---- Zernike: geometries/zernike.py:133-246 + zernike/base.py:42-299 ----------------
// Per term (n, m), with a = |m|, rho = r / R_norm, phi = atan2(yn, xn):
//   R_n^a(rho)   = sum_k a_k rho^(n-2k) = rho^a * P(rho^2)            (base.py:228-253)
//   dR/drho      = sum_k d_k rho^(n-2k-1), terms with n-2k-1 < 0 dropped (:259-299)
//                = rho^(a-1) * Q(rho^2)  (a >= 1),   rho * Q'(rho^2)  (a = 0)
// P, Q by Horner in rho^2 from the host's a_k, d_k (highest power first), rho^a and
// cos/sin(a phi) by one recurrence from cos phi = xn / rho, sin phi = yn / rho. The
// reference sums libm powers term by term and takes cos/sin of a*atan2: rounding-level
// differences (DESIGN.md Parity). A term whose coefficient is 0 adds exactly 0 to the
// sag and is skipped by the reference's normal (zernike.py:213-214), so it is skipped
// here -- unless the derivative kernels seed a tangent on it (the sag's derivative
// w.r.t. that coefficient is not zero).
ORT_INLINE bool zseeded(const ZSeed&, int, double*) { return false; }
template <int P>
ORT_INLINE bool zseeded(const ZSeed& zs, int j, Dual<P>*) {
  if (!zs.param) return false;
  const int p = zs.param[j] - zs.p0;
  return p >= 0 && p < P;
}

template <class T>
ORT_INLINE void polar_unit(const T& xn, const T& yn, const T& rho, T& c1, T& s1) {
  if (vv(rho) > 0.0) {
    div2(xn, yn, rho, c1, s1);
  } else {  // atan2(0, 0) = 0
    c1 = T(1.0);
    s1 = T(0.0);
  }
}

// ---- Zernike term sums in Cartesian form (ort_surface.zm_off / zm_deg, ABI v16) --------
// Up to radial order 6 the host also lowers sum_j c_j Z_j as a polynomial in the normalised
// coordinates, A[p][q] xn^p yn^q (p-major, q fastest; geometries.zernike_monomials: the
// exact integer expansion of R_n^|m|(rho) {cos|sin}(|m| phi) through Re / Im (xn + i yn)^a
// and rho^2 = xn^2 + yn^2), so a Newton evaluation is a two-level Horner scheme instead of
// a recurrence and a radial Horner per term. Nested Horner with derivatives (the inner
// level in yn, the outer in xn): value, gradient and Hessian w.r.t. (xn, yn).
template <class T>
struct IsPlain {
  static constexpr bool value = false;
};
template <>
struct IsPlain<double> {
  static constexpr bool value = true;
};

// The loops below take the degree N at run time; the block's entries A[o + q] are then
// scalar loads inside a loop with a run-time trip count, each waited for before its
// multiply (a dependent load chain per Newton evaluation). The degrees that occur (radial
// orders 2..6) are dispatched to copies with N a template parameter, fully unrolled: the
// same operations in the same order (bit-identical), with the block's loads issued up
// front. Other degrees (0, 1) keep the loop.
template <int N, class PD>
ORT_INLINE double zmono_value_n(PD A, double x, double y) {
  double F = 0.0;
#pragma unroll
  for (int p = N; p >= 0; --p) {
    const int o = p * (N + 1) - p * (p - 1) / 2, L = N - p;
    double B = A[o + L];
#pragma unroll
    for (int q = L - 1; q >= 0; --q) B = B * y + A[o + q];
    F = F * x + B;
  }
  return F;
}

template <int N, class PD>
ORT_INLINE void zmono_grad_n(PD A, double x, double y, double& F, double& Fx, double& Fy) {
  F = 0.0;
  Fx = 0.0;
  Fy = 0.0;
#pragma unroll
  for (int p = N; p >= 0; --p) {
    const int o = p * (N + 1) - p * (p - 1) / 2, L = N - p;
    double B = A[o + L], B1 = 0.0;
#pragma unroll
    for (int q = L - 1; q >= 0; --q) {
      B1 = B1 * y + B;
      B = B * y + A[o + q];
    }
    Fx = Fx * x + F;
    F = F * x + B;
    Fy = Fy * x + B1;
  }
}

template <int N, class PD>
ORT_INLINE void zmono_hess_n(PD A, double x, double y, double& F, double& Fx, double& Fy,
                             double& Fxx, double& Fxy, double& Fyy) {
  F = Fx = Fy = Fxx = Fxy = Fyy = 0.0;
#pragma unroll
  for (int p = N; p >= 0; --p) {
    const int o = p * (N + 1) - p * (p - 1) / 2, L = N - p;
    double B = A[o + L], B1 = 0.0, B2 = 0.0;
#pragma unroll
    for (int q = L - 1; q >= 0; --q) {
      B2 = B2 * y + 2.0 * B1;
      B1 = B1 * y + B;
      B = B * y + A[o + q];
    }
    Fxx = Fxx * x + 2.0 * Fx;
    Fx = Fx * x + F;
    F = F * x + B;
    Fxy = Fxy * x + Fy;
    Fy = Fy * x + B1;
    Fyy = Fyy * x + B2;
  }
}

template <class PD>
ORT_INLINE double zmono_value(PD A, int N, double x, double y) {
  switch (N) {
    case 2: return zmono_value_n<2>(A, x, y);
    case 3: return zmono_value_n<3>(A, x, y);
    case 4: return zmono_value_n<4>(A, x, y);
    case 5: return zmono_value_n<5>(A, x, y);
    case 6: return zmono_value_n<6>(A, x, y);
    default: break;
  }
  double F = 0.0;
  for (int p = N; p >= 0; --p) {
    const int o = p * (N + 1) - p * (p - 1) / 2, L = N - p;
    double B = A[o + L];
    for (int q = L - 1; q >= 0; --q) B = B * y + A[o + q];
    F = F * x + B;
  }
  return F;
}

template <class PD>
ORT_INLINE void zmono_grad(PD A, int N, double x, double y, double& F, double& Fx,
                           double& Fy) {
  switch (N) {
    case 2: return zmono_grad_n<2>(A, x, y, F, Fx, Fy);
    case 3: return zmono_grad_n<3>(A, x, y, F, Fx, Fy);
    case 4: return zmono_grad_n<4>(A, x, y, F, Fx, Fy);
    case 5: return zmono_grad_n<5>(A, x, y, F, Fx, Fy);
    case 6: return zmono_grad_n<6>(A, x, y, F, Fx, Fy);
    default: break;
  }
  F = 0.0;
  Fx = 0.0;
  Fy = 0.0;
  for (int p = N; p >= 0; --p) {
    const int o = p * (N + 1) - p * (p - 1) / 2, L = N - p;
    double B = A[o + L], B1 = 0.0;
    for (int q = L - 1; q >= 0; --q) {
      B1 = B1 * y + B;
      B = B * y + A[o + q];
    }
    Fx = Fx * x + F;
    F = F * x + B;
    Fy = Fy * x + B1;
  }
}

template <class PD>
ORT_INLINE void zmono_hess(PD A, int N, double x, double y, double& F, double& Fx, double& Fy,
                           double& Fxx, double& Fxy, double& Fyy) {
  switch (N) {
    case 2: return zmono_hess_n<2>(A, x, y, F, Fx, Fy, Fxx, Fxy, Fyy);
    case 3: return zmono_hess_n<3>(A, x, y, F, Fx, Fy, Fxx, Fxy, Fyy);
    case 4: return zmono_hess_n<4>(A, x, y, F, Fx, Fy, Fxx, Fxy, Fyy);
    case 5: return zmono_hess_n<5>(A, x, y, F, Fx, Fy, Fxx, Fxy, Fyy);
    case 6: return zmono_hess_n<6>(A, x, y, F, Fx, Fy, Fxx, Fxy, Fyy);
    default: break;
  }
  F = Fx = Fy = Fxx = Fxy = Fyy = 0.0;
  for (int p = N; p >= 0; --p) {
    const int o = p * (N + 1) - p * (p - 1) / 2, L = N - p;
    double B = A[o + L], B1 = 0.0, B2 = 0.0;
    for (int q = L - 1; q >= 0; --q) {
      B2 = B2 * y + 2.0 * B1;
      B1 = B1 * y + B;
      B = B * y + A[o + q];
    }
    Fxx = Fxx * x + 2.0 * Fx;
    Fx = Fx * x + F;
    F = F * x + B;
    Fxy = Fxy * x + Fy;
    Fy = Fy * x + B1;
    Fyy = Fyy * x + B2;
  }
}

// sag (zernike.py:133-161; sets range_error on |x/R_norm| > 1 or |y/R_norm| > 1,
// :234-246) and, with want_normal, the normal (zernike.py:163-231; the normal omits the
// normalisation constant: reference quirk)
template <class T, class S, class PD, class PZ>
ORT_INLINE T sagnorm_zernike(const T& x, const T& y, const S& R, const S& k, double Rn, PZ Tm,
                             int t0, int nt, PD coef, const ZSeed& zs, int want_normal,
                             bool& range_error, T& nx, T& ny, T& nz, int zm_off = 0,
                             int zm_deg = -1) {
  if constexpr (IsPlain<T>::value && IsPlain<S>::value) {
    if (zm_deg >= 0) {
      // Cartesian form: the sag from As, the normal's slopes from An's gradient mapped
      // through the reference's eps-guarded chain rule, d/dx = dF/drho drho/dx + dF/dphi
      // dphi/dx with dF/drho = (xn Fx + yn Fy) / rho and dF/dphi = xn Fy - yn Fx
      double xn, yn;
      div2(x, y, Rn, xn, yn);
      if (::fabs(xn) > 1.0 || ::fabs(yn) > 1.0) range_error = true;
      const double r2 = x * x + y * y;
      const double q = sqrt(1.0 - (1.0 + k) * r2 / (R * R));
      const double z = r2 / (R * (1.0 + q));
      const int K = (zm_deg + 1) * (zm_deg + 2) / 2;
      const PD As = coef + zm_off;
      const double F = zmono_value(As, zm_deg, xn, yn);
      if (want_normal) {
        double G, Gx, Gy;
        zmono_grad(As + K, zm_deg, xn, yn, G, Gx, Gy);
        double dzdx, dzdy;
        div2(x, y, R * q, dzdx, dzdy);
        const double eps = 1e-14;
        // The term sum's slopes. The reference forms them through (rho, phi) with eps guards
        // (zernike.py:190-214): dF/drho drho/dx + dF/dphi dphi/dx with drho/dx = (x / Rn^2) /
        // (rho + eps), dphi/dx = -yn / (rho^2 + eps) / Rn, dF/drho = (xn Gx + yn Gy) / rho,
        // dF/dphi = xn Gy - yn Gx (G: the block's Cartesian gradient). Without the guards
        // that is exactly Gx / Rn; with them it differs by ~eps / rho^2 relative, which
        // matters only near the axis (rho^2 < 1e-4: the guards bend the reference's normal
        // there, and its value on the axis is 0). So off that disc the slopes are Gx / Rn,
        // Gy / Rn (2 products instead of a square root and four divisions; < 1e-10
        // relative from the reference's), on it the reference's own chain. The adjoint's
        // pull-back (ort_sweep.h zern_adj) takes the same branch. (ORT_ZERN_POLAR_CHAIN,
        // A/B builds: the chain everywhere.)
        const double rho2n = xn * xn + yn * yn;
#ifndef ORT_ZERN_POLAR_CHAIN
        if (rho2n >= kZernChainRho2) {
          const double inv_rn = 1.0 / Rn;
          dzdx = dzdx + Gx * inv_rn;
          dzdy = dzdy + Gy * inv_rn;
        } else
#endif
        {
          const double rho = sqrt(rho2n);
          double xr, yr, drho_dx, drho_dy, qy, qx;
          div2(x, y, Rn * Rn, xr, yr);
          div2(xr, yr, rho + eps, drho_dx, drho_dy);
          div2(-(yn), xn, rho * rho + eps, qy, qx);
          const double inv_rn = 1.0 / Rn;
          const double G1 = xn * Gx + yn * Gy, G2 = xn * Gy - yn * Gx;
          const double Fr = rho > 0.0 ? G1 / rho : 0.0;
          dzdx = dzdx + (Fr * drho_dx + G2 * (qy * inv_rn));
          dzdy = dzdy + (Fr * drho_dy + G2 * (qx * inv_rn));
        }
        if (want_normal == kSlope && slope_direct(dzdx, dzdy)) {
          nx = dzdx;
          ny = dzdy;
          nz = -1.0;
          return z + F;
        }
        double norm = sqrt(dzdx * dzdx + dzdy * dzdy + 1.0);
        norm = norm < eps ? 1.0 : norm;
        unit_normal3(dzdx, dzdy, norm, nx, ny, nz);
      }
      return z + F;
    }
  }
  T xn, yn;
  div2(x, y, Rn, xn, yn);
  if (::fabs(vv(xn)) > 1.0 || ::fabs(vv(yn)) > 1.0) range_error = true;
  const T rho = sqrt(xn * xn + yn * yn);
  T c1, s1;
  polar_unit(xn, yn, rho, c1, s1);
  const T rho2 = rho * rho;
  const T r2 = x * x + y * y;
  const T q = sqrt(1.0 - (1.0 + k) * r2 / (R * R));
  const T z = r2 / (R * (1.0 + q));
  T total = T(0.0);  // python sum() starts at int 0; 0 + t == t exactly
  // normal: conic part + chain rule through (rho, phi) with the reference's eps guards
  const double eps = 1e-14;
  T dzdx, dzdy, drho_dx, drho_dy, dphi_dx, dphi_dy;
  if (want_normal) {
    const T denominator = R * q;
    div2(x, y, denominator, dzdx, dzdy);
    const double Rn2 = Rn * Rn;
    // (the reference returns zeros when EVERY rho is 0; per ray (x/Rn^2)/(0+eps) = 0 too)
    T xr, yr;
    div2(x, y, Rn2, xr, yr);
    div2(xr, yr, rho + eps, drho_dx, drho_dy);
    const T rho2e = rho2 + eps;
    const double inv_rn = 1.0 / Rn;
    T qy, qx;
    div2(T(-(yn)), xn, rho2e, qy, qx);
    dphi_dx = qy * inv_rn;
    dphi_dy = qx * inv_rn;  // "+(x_norm)": unary plus
  }
  for (int j = 0; j < nt; ++j) {
    const ort_zernike_term t = Tm[t0 + j];
    if (t.c == 0.0 && !zseeded(zs, t0 + j, (T*)nullptr)) continue;
    const int am = t.m >= 0 ? t.m : -t.m;
    // cos(am phi), sin(am phi), rho^am, rho^(am-1)
    T cm = T(1.0), sm = T(0.0), pm = T(1.0), pm1 = T(1.0);
#pragma unroll 1
    for (int qq = 0; qq < am; ++qq) {
      const T cn = cm * c1 - sm * s1;
      sm = sm * c1 + cm * s1;
      cm = cn;
      pm1 = pm;
      pm = pm * rho;
    }
    const PD a = coef + t.rad_off;
    T P = T(a[0]);
#pragma unroll 1
    for (int kk = 1; kk < t.n_rad; ++kk) P = P * rho2 + a[kk];
    const T rt = P * pm;  // R_n^am(rho)
    const T az = t.m >= 0 ? cm : sm;  // base.py:206-226
    const T c = zcoef(t.c, t0 + j, zs, (T*)nullptr);
    total = total + c * t.norm * rt * az;
    if (want_normal && t.c != 0.0) {
      const PD d = a + t.n_rad;
      T rd;
      if (am > 0) {
        T Q = T(d[0]);
#pragma unroll 1
        for (int kk = 1; kk < t.n_rad; ++kk) Q = Q * rho2 + d[kk];
        rd = Q * pm1;
      } else if (t.n_rad > 1) {
        T Q = T(d[0]);
#pragma unroll 1
        for (int kk = 1; kk < t.n_rad - 1; ++kk) Q = Q * rho2 + d[kk];
        rd = Q * rho;
      } else {
        rd = T(0.0);
      }
      T dr, dp;
      if (t.m == 0) {  // base.py:124-136
        dr = rd;
        dp = T(0.0);
      } else if (t.m > 0) {
        dr = rd * cm;
        dp = (double)(-t.m) * rt * sm;
      } else {
        dr = rd * sm;
        dp = (double)am * rt * cm;
      }
      dzdx = dzdx + c * (dr * drho_dx + dp * dphi_dx);
      dzdy = dzdy + c * (dr * drho_dy + dp * dphi_dy);
    }
  }
  if (want_normal) {
    if (want_normal == kSlope && slope_direct(dzdx, dzdy)) {
      nx = dzdx;
      ny = dzdy;
      nz = T(-1.0);
      return z + total;
    }
    T norm = sqrt(dzdx * dzdx + dzdy * dzdy + 1.0);
    norm = vv(norm) < eps ? T(1.0) : norm;
    unit_normal3(dzdx, dzdy, norm, nx, ny, nz);
  }
  return z + total;
}

// Reverse-mode companion of sagnorm_zernike for the coefficients (adjoint VJP): the sag
// and the normal's slopes are linear in c_j, so for every term j of the surface
//   g_j = w_sag * d sag / d c_j + w_dx * d dzdx / d c_j + w_dy * d dzdy / d c_j
// is handed to emit(j, g_j) -- one pass over the terms, whatever the number of
// coefficients. The slope part follows the reference's normal, which only sums terms
// with c_j != 0 (zernike.py:213-214) and omits the normalisation constant.
template <class PD, class PZ, class F>
ORT_INLINE void zernike_coef_adjoint(double x, double y, double Rn, PZ Tm, int t0, int nt,
                                     PD coef, double w_sag, double w_dx, double w_dy,
                                     F&& emit) {
  double xn, yn;
  div2(x, y, Rn, xn, yn);
  const double rho = sqrt(xn * xn + yn * yn);
  double c1, s1;
  if (rho > 0.0) {
    div2(xn, yn, rho, c1, s1);
  } else {
    c1 = 1.0;
    s1 = 0.0;
  }
  const double rho2 = rho * rho;
  const double eps = 1e-14;
  const double Rn2 = Rn * Rn;
  double xr, yr, drho_dx, drho_dy;
  div2(x, y, Rn2, xr, yr);
  div2(xr, yr, rho + eps, drho_dx, drho_dy);
  const double rho2e = rho2 + eps;
  const double inv_rn = 1.0 / Rn;
  double qy, qx;
  div2(-(yn), xn, rho2e, qy, qx);
  const double dphi_dx = qy * inv_rn;
  const double dphi_dy = qx * inv_rn;
  // cos / sin(am phi), rho^am, rho^(am - 1) of the previous term: the recurrence resumes
  // from there when |m| does not decrease (Z(n, +-m) pairs share it), else restarts --
  // the same products in the same order as a restart from am = 0 (the values are equal)
  int prev_am = 0;
  double cm = 1.0, sm = 0.0, pm = 1.0, pm1 = 1.0;
  for (int j = 0; j < nt; ++j) {
    const ort_zernike_term t = Tm[t0 + j];
    const int am = t.m >= 0 ? t.m : -t.m;
    if (am < prev_am) {
      cm = 1.0;
      sm = 0.0;
      pm = 1.0;
      pm1 = 1.0;
      prev_am = 0;
    }
#pragma unroll 1
    for (int qq = prev_am; qq < am; ++qq) {
      const double cn = cm * c1 - sm * s1;
      sm = sm * c1 + cm * s1;
      cm = cn;
      pm1 = pm;
      pm = pm * rho;
    }
    prev_am = am;
    const PD a = coef + t.rad_off;
    double P = a[0];
#pragma unroll 1
    for (int kk = 1; kk < t.n_rad; ++kk) P = P * rho2 + a[kk];
    const double rt = P * pm;
    const double az = t.m >= 0 ? cm : sm;
    double g = w_sag * (t.norm * rt * az);
    if (t.c != 0.0) {
      const PD d = a + t.n_rad;
      double rd = 0.0;
      if (am > 0) {
        double Q = d[0];
#pragma unroll 1
        for (int kk = 1; kk < t.n_rad; ++kk) Q = Q * rho2 + d[kk];
        rd = Q * pm1;
      } else if (t.n_rad > 1) {
        double Q = d[0];
#pragma unroll 1
        for (int kk = 1; kk < t.n_rad - 1; ++kk) Q = Q * rho2 + d[kk];
        rd = Q * rho;
      }
      double dr, dp;
      if (t.m == 0) {
        dr = rd;
        dp = 0.0;
      } else if (t.m > 0) {
        dr = rd * cm;
        dp = (double)(-t.m) * rt * sm;
      } else {
        dr = rd * sm;
        dp = (double)am * rt * cm;
      }
      g += w_dx * (dr * drho_dx + dp * dphi_dx) + w_dy * (dr * drho_dy + dp * dphi_dy);
    }
    emit(t0 + j, g);
  }
}

// Second-order local model of a Zernike surface at (x, y), in plain doubles, for the
// adjoint VJP: the sag and its gradient, the slopes (dzdx, dzdy) the reference's normal is
// built from (zernike.py:163-231: conic part x / (R q) plus the terms' chain rule through
// rho and phi, without the normalisation constant) and their Jacobian. The adjoint needs
// exactly these -- the Newton update's f, f_x, f_y and the normal's x / y derivatives --
// and the dual-number evaluation of sagnorm_zernike it replaces carries three values
// through every operation (with the adjoint state alive around it the kernel spilled).
// Per term c R(rho) A(phi), R = H(rho^2) rho^|m| from the radial table, the sums
//   Q_r = sum c R' A, Q_p = sum c R A', Q_rr = sum c R'' A, Q_rp = sum c R' A',
//   Q_pp = sum c R A''  (A'' = -m^2 A)
// are formed once over the terms and mapped to x, y by the derivatives of rho = r / R_n
// and phi = atan2(y, x) (1 / rho guarded by the reference's eps, as its normal does).
// Values agree with sagnorm_zernike's to rounding, not bit for bit: they enter only the
// derivative. Zero coefficients are skipped, as the reference's normal skips them.
struct SurfJet {
  double z, zx, zy;      // sag, d sag / dx, d sag / dy (the terms' normalisation included)
  double sx, sy;         // the normal's slopes
  double sxx, sxy, syy;  // d sx / dx, d sx / dy, d sy / dy
  double syx;            // d sy / dx (= sxy for a gradient field; the eps-guarded chain of
                         // the reference's normal near the Zernike axis is not one)
};

template <class PD, class PZ>
ORT_INLINE void zernike_jet(double x, double y, double R, double k, double Rn, PZ Tm, int t0,
                            int nt, PD coef, SurfJet& J, int zm_off = 0, int zm_deg = -1) {
  // base conic (standard.py:73-87, 154-167): z = r2 / (R (1 + q)), slope x / (R q)
  const double r2 = x * x + y * y;
  const double q = sqrt(1.0 - rdiv((1.0 + k) * r2, R * R));
  const double iRq = rrcp(R * q);
  const double h = (1.0 + k) * iRq * iRq * iRq;  // (1 + k) / (R q)^3
  J.z = rdiv(r2, R * (1.0 + q));
  J.sx = x * iRq;
  J.sy = y * iRq;
  J.sxx = iRq + h * x * x;
  J.sxy = h * x * y;
  J.syy = iRq + h * y * y;
  const double iRn = rrcp(Rn);
  const double xn = x * iRn, yn = y * iRn;
  if (zm_deg >= 0) {  // Cartesian form (zmono_*): exact derivatives of both polynomials
    const int K = (zm_deg + 1) * (zm_deg + 2) / 2;
    double F, Fx, Fy, G, Gx, Gy, Gxx, Gxy, Gyy;
    zmono_grad(coef + zm_off, zm_deg, xn, yn, F, Fx, Fy);
    zmono_hess(coef + zm_off + K, zm_deg, xn, yn, G, Gx, Gy, Gxx, Gxy, Gyy);
    J.z += F;
    J.zx = J.sx + Fx * iRn;
    J.zy = J.sy + Fy * iRn;
    const double rho2n = xn * xn + yn * yn;
#ifndef ORT_ZERN_POLAR_CHAIN
    // (ORT_JET_NO_DISC, A/B builds only: the unguarded derivatives on the disc too)
#ifdef ORT_JET_NO_DISC
    if (true) {
#else
    if (rho2n >= kZernChainRho2) {
#endif
      J.sx += Gx * iRn;
      J.sy += Gy * iRn;
      const double iRn2 = iRn * iRn;
      J.sxx += Gxx * iRn2;
      J.sxy += Gxy * iRn2;
      J.syx = J.sxy;
      J.syy += Gyy * iRn2;
      return;
    }
#endif
    // near the axis the forward's slopes are the reference's eps-guarded chain
    // (sagnorm_zernike): S = Rn sx = a G1 u - c G2 v, T = Rn sy = a G1 v + c G2 u with
    // u, v = xn, yn, a = 1 / (rho (rho + eps)), c = 1 / (rho^2 + eps), G1 = u Gx + v Gy,
    // G2 = u Gy - v Gx -- differentiated as the reference's autograd does, the block's
    // gradient carrying its Hessian (no symmetry: the guarded chain is no gradient field)
    const double eps = 1e-14;
    const double u = xn, v = yn;
    const double rho = sqrt(rho2n);
    if (rho > 0.0) {
      const double a = rrcp(rho * (rho + eps)), c = rrcp(rho2n + eps);
      const double ka = -a * a * rdiv(2.0 * rho + eps, rho), kc = -2.0 * c * c;  // a_u = ka u
      const double G1 = u * Gx + v * Gy, G2 = u * Gy - v * Gx;
      const double G1u = Gx + u * Gxx + v * Gxy, G1v = Gy + u * Gxy + v * Gyy;
      const double G2u = Gy + u * Gxy - v * Gxx, G2v = u * Gyy - Gx - v * Gxy;
      const double aG1 = a * G1, cG2 = c * G2;
      const double pa = ka * G1, pc = kc * G2;  // d(a G1) = pa (u, v) + a dG1, likewise c
      const double iRn2 = iRn * iRn;
      const double E = pa * u - pc * v, H = pa * v + pc * u;
      const double au = a * u, av = a * v, cu = c * u, cv = c * v;
      J.sx += (aG1 * u - cG2 * v) * iRn;
      J.sy += (aG1 * v + cG2 * u) * iRn;
      J.sxx += (u * E + au * G1u - cv * G2u + aG1) * iRn2;
      J.syx = J.sxy + (u * H + av * G1u + cu * G2u + cG2) * iRn2;
      J.sxy += (v * E + au * G1v - cv * G2v - cG2) * iRn2;
      J.syy += (v * H + av * G1v + cu * G2v + aG1) * iRn2;
    } else {  // on the axis: the forward's slopes are 0 + the conic's (Fr = 0, G2 = 0)
      const double iRn2 = iRn * iRn;
      J.sxx += Gxx * iRn2;
      J.sxy += Gxy * iRn2;
      J.syx = J.sxy;
      J.syy += Gyy * iRn2;
    }
    return;
  }
  const double rho = sqrt(xn * xn + yn * yn);
  double c1 = 1.0, s1 = 0.0;  // cos / sin phi (atan2(0, 0) = 0)
  if (rho > 0.0) {
    const double ir = rrcp(rho);
    c1 = xn * ir;
    s1 = yn * ir;
  }
  const double u = rho * rho;
  double Z = 0.0, Gr = 0.0, Gp = 0.0, Qr = 0.0, Qp = 0.0, Qrr = 0.0, Qrp = 0.0, Qpp = 0.0;
  for (int j = 0; j < nt; ++j) {
    const ort_zernike_term t = Tm[t0 + j];
    if (t.c == 0.0) continue;
    const int am = t.m >= 0 ? t.m : -t.m;
    double cm = 1.0, sm = 0.0, pw = 1.0;  // cos(am phi), sin(am phi), rho^am
#pragma unroll 1
    for (int qq = 0; qq < am; ++qq) {
      const double cn = cm * c1 - sm * s1;
      sm = sm * c1 + cm * s1;
      cm = cn;
      pw = pw * rho;
    }
    // H(u) and its first two derivatives (Horner), R = H rho^am
    const PD a = coef + t.rad_off;
    double H = a[0], H1 = 0.0, H2 = 0.0;
#pragma unroll 1
    for (int kk = 1; kk < t.n_rad; ++kk) {
      H2 = H2 * u + H1;
      H1 = H1 * u + H;
      H = H * u + a[kk];
    }
    H2 = 2.0 * H2;
    const double F = 2.0 * u * H1 + am * H;  // rho^(1 - am) R'
    double P, P1, P2;  // R, R', R''
    if (am == 0) {
      P = H;
      P1 = 2.0 * rho * H1;
      P2 = 2.0 * H1 + 4.0 * u * H2;
    } else if (am == 1) {
      P = H * rho;
      P1 = F;
      P2 = 2.0 * rho * (3.0 * H1 + 2.0 * u * H2);
    } else {
      const double pw2 = rdiv(pw, rho * rho);  // rho^(am - 2) (rho > 0 here, else pw = 0)
      P = H * pw;
      P1 = rho > 0.0 ? F * rdiv(pw, rho) : 0.0;
      P2 = rho > 0.0 ? pw2 * ((am - 1.0) * F + 2.0 * u * ((2.0 + am) * H1 + 2.0 * u * H2))
                     : (am == 2 ? 2.0 * H : 0.0);
    }
    double A, A1;  // A(phi), dA / dphi (base.py:206-226: cos m phi, sin |m| phi)
    if (t.m > 0) {
      A = cm;
      A1 = -(double)am * sm;
    } else if (t.m < 0) {
      A = sm;
      A1 = (double)am * cm;
    } else {
      A = 1.0;
      A1 = 0.0;
    }
    const double cz = t.c, cn = t.c * t.norm;
    Z += cn * P * A;
    Gr += cn * P1 * A;
    Gp += cn * P * A1;
    Qr += cz * P1 * A;
    Qp += cz * P * A1;
    Qrr += cz * P2 * A;
    Qrp += cz * P1 * A1;
    Qpp -= cz * (double)(am * am) * P * A;
  }
  const double eps = 1e-14;
  const double ir = rrcp((rho + eps) * Rn);  // 1 / (rho R_n), guarded
  const double rx = c1 * iRn, ry = s1 * iRn;  // d rho / dx, d rho / dy
  const double px = -s1 * ir, py = c1 * ir;    // d phi / dx, d phi / dy
  const double rxx = s1 * s1 * ir * iRn, rxy = -c1 * s1 * ir * iRn, ryy = c1 * c1 * ir * iRn;
  const double pxx = 2.0 * c1 * s1 * ir * ir, pxy = (s1 * s1 - c1 * c1) * ir * ir;
  J.z += Z;
  J.zx = J.sx + Gr * rx + Gp * px;
  J.zy = J.sy + Gr * ry + Gp * py;
  J.sx += Qr * rx + Qp * px;
  J.sy += Qr * ry + Qp * py;
  J.sxx += Qrr * rx * rx + 2.0 * Qrp * rx * px + Qpp * px * px + Qr * rxx + Qp * pxx;
  J.sxy += Qrr * rx * ry + Qrp * (rx * py + ry * px) + Qpp * px * py + Qr * rxy + Qp * pxy;
  J.syy += Qrr * ry * ry + 2.0 * Qrp * ry * py + Qpp * py * py + Qr * ryy - Qp * pxx;
  J.syx = J.sxy;
}

// the unit normal n = (sx, sy, -1) / |(sx, sy, -1)| of a jet and its x / y derivatives:
// dn = (dg - n (n . dg)) / |g| with dg = (sxx, sxy, 0) resp. (sxy, syy, 0)
template <int P>
ORT_INLINE void jet_normal(const SurfJet& J, Dual<P>& nx, Dual<P>& ny, Dual<P>& nz) {
  const double g = sqrt(J.sx * J.sx + J.sy * J.sy + 1.0);
  const double ig = rrcp(g);
  nx = Dual<P>(J.sx * ig);
  ny = Dual<P>(J.sy * ig);
  nz = Dual<P>(-ig);
  const double ex = nx.v * J.sxx + ny.v * J.syx, ey = nx.v * J.sxy + ny.v * J.syy;
  nx.d[0] = (J.sxx - nx.v * ex) * ig;
  ny.d[0] = (J.syx - ny.v * ex) * ig;
  nz.d[0] = -nz.v * ex * ig;
  nx.d[1] = (J.sxy - nx.v * ey) * ig;
  ny.d[1] = (J.syy - ny.v * ey) * ig;
  nz.d[1] = -nz.v * ey * ig;
}

// ---- Forbes Q-polynomials: forbes/geometry.py:83-640 + forbes/qpoly.py --------------
// The lens-only constants (orthonormal-basis coefficients, recurrence A/B/C, the Q-2D
// vertex slope) come precomputed in the coefficient block (optiland_pr_amd/forbes.py);
// the per-ray work is the Clenshaw recurrences below, in the reference's operation
// order. Integer powers u^3.. are products (the reference's libm pow: ulp-level).

// forbes/geometry.py:115-131 (_base_sag)
template <class T, class S>
ORT_INLINE T forbes_base_sag(const T& r2, const S& R, const S& k, bool rinf) {
  if (rinf) return T(0.0);
  const T a = 1.0 - (1.0 + k) * r2 / (R * R);
  const T sa = vv(a) < 0.0 ? T(0.0) : a;
  return r2 / (R * (1.0 + sqrt(sa)));
}

// forbes/geometry.py:133-150 (_base_sag_derivative: d z_base / d rho)
template <class T, class S>
ORT_INLINE T forbes_base_dsag(const T& rho, const T& r2, const S& R, const S& k, bool rinf) {
  if (rinf || vv(R) == 0.0) return T(0.0);
  const S c = 1.0 / R;
  const T a = 1.0 - (k + 1.0) * (c * c) * r2;
  const T sa = sqrt(vv(a) > 0.0 ? a : T(1e-12));
  return c * rho / sa;
}

// forbes/geometry.py:152-180 (_conic_correction_factor and its d/d rho)
template <class T, class S>
ORT_INLINE void forbes_conic_factor(const T& r2, const S& R, const S& k, bool rinf, T& f,
                                    T& df) {
  if (rinf) {
    f = T(1.0);
    df = T(0.0);
    return;
  }
  const S c = 1.0 / R;
  const S c2 = c * c;
  const T rho = sqrt(r2);
  const T na = 1.0 - k * c2 * r2;
  const T da = 1.0 - (k + 1.0) * c2 * r2;
  const T Nn = sqrt(vv(na) > 0.0 ? na : T(1e-12));
  const T Dd = sqrt(vv(da) > 0.0 ? da : T(1e-12));
  f = Nn / Dd;
  df = (c2 * rho) / (Nn * (Dd * Dd * Dd));
}

// Q-bfs Clenshaw over b_0..b_{L-1} at x = u^2 (qpoly.py:127-160): the sum
// S = 2 (alpha_0 + alpha_1); with want_d also dS/dx from the j = 1 recurrence
// (qpoly.py:163-192), both in one downward pass.
template <class T, class PD>
ORT_INLINE void qbfs_clenshaw(PD b, int L, const T& usq, bool want_d, T& s, T& ds) {
  if (L <= 0) {
    s = T(0.0);
    ds = T(0.0);
    return;
  }
  const int M = L - 1;
  const T p = 2.0 - 4.0 * usq;
  T a1 = T(0.0), a2 = T(0.0), d1 = T(0.0), d2 = T(0.0);  // alpha_{i+1}, alpha_{i+2}
#pragma unroll 1
  for (int i = M; i >= 0; --i) {
    T ai, di = T(0.0);
    if (i == M) {
      ai = T(b[i]);
    } else if (i == M - 1) {
      ai = b[i] + p * a1;
      if (want_d) di = -4.0 * a1;
    } else {
      ai = b[i] + p * a1 - a2;
      if (want_d) di = (i == M - 2) ? p * d1 - 4.0 * a1 : p * d1 - d2 - 4.0 * a1;
    }
    a2 = a1;
    a1 = ai;
    d2 = d1;
    d1 = di;
  }
  s = M > 0 ? 2.0 * (a1 + a2) : 2.0 * a1;
  ds = M > 0 ? 2.0 * (d1 + d2) : 2.0 * d1;
}

// One Q-2D azimuthal order (qpoly.py:389-430 sum, :443-466 d/d(u^2)): record
// L, d[L], A[L], B[L], C[L]; q2d_sum_from_alphas (qpoly.py:389-398) on both.
template <class T, class PD>
ORT_INLINE void q2d_clenshaw(PD rec, int m, const T& usq, bool want_d, T& s, T& ds) {
  const int L = (int)rec[0];
  if (L <= 0) {
    s = T(0.0);
    ds = T(0.0);
    return;
  }
  const PD D = rec + 1;
  const PD A = D + L;
  const PD Bc = A + L;
  const PD C = Bc + L;
  const int top = L - 1;
  T a1 = T(0.0), a2 = T(0.0), d1 = T(0.0), d2 = T(0.0), a3 = T(0.0), d3 = T(0.0);
#pragma unroll 1
  for (int n = top; n >= 0; --n) {
    T an, dn = T(0.0);
    if (n == top) {
      an = T(D[n]);
    } else {
      const T w = A[n] + Bc[n] * usq;
      if (n == top - 1) {
        an = D[n] + w * a1;
        if (want_d) dn = Bc[n] * a1;
      } else {
        an = D[n] + w * a1 - C[n + 1] * a2;
        if (want_d) dn = Bc[n] * a1 + w * d1 - C[n + 1] * d2;
      }
    }
    if (n == 3) {
      a3 = an;
      d3 = dn;
    }
    a2 = a1;
    a1 = an;
    d2 = d1;
    d1 = dn;
  }
  s = 0.5 * a1;
  ds = 0.5 * d1;
  if (m == 1 && top > 2) {
    s = s - 0.4 * a3;
    ds = ds - 0.4 * d3;
  }
}

template <class PD>
ORT_INLINE PD q2d_next(PD rec) {
  const int L = (int)rec[0];
  return rec + (L > 0 ? 1 + 4 * L : 1);
}

// forbes/geometry.py:243-266 (sag) and :296-327 (_surface_normal_analytical)
template <class T, class S, class PD>
ORT_INLINE T sagnorm_qbfs(const T& x, const T& y, const S& R, const S& k, bool rinf, PD B,
                          bool want_normal, T& nx, T& ny, T& nz) {
  const double nr = B[0];
  const int L = (int)B[1];
  const bool dep_normal = B[2] != 0.0;
  const PD b = B + 3;
  const T r2 = x * x + y * y;
  const T usq = r2 / (nr * nr);
  T ps, unused;
  qbfs_clenshaw(b, L, usq, false, ps, unused);
  T cf, dcf;
  forbes_conic_factor(r2, R, k, rinf, cf, dcf);
  const T dep = usq * (1.0 - usq) * cf * ps;
  const T z = forbes_base_sag(r2, R, k, rinf) + (vv(usq) > 1.0 ? T(0.0) : dep);
  if (want_normal) {
    const T rho = sqrt(r2 + 1e-12);
    T dfr = forbes_base_dsag(rho, r2, R, k, rinf);
    if (dep_normal) {
      const T u = rho / nr;
      T pv, pd;
      qbfs_clenshaw(b, L, u * u, true, pv, pd);
      const T dpdu = pd * 2.0 * u;
      const T dpre = (2.0 * u - 4.0 * (u * u * u)) / nr;
      const T dpoly = dpdu / nr;
      const T uu = u * u;
      const T q = uu - uu * uu;
      const T dd = dpre * cf * pv + q * dcf * pv + q * cf * dpoly;
      dfr = dfr + (vv(u) >= 1.0 ? T(0.0) : dd);
    }
    const T dfx = dfr * (x / rho);
    const T dfy = dfr * (y / rho);
    const T mag = sqrt(dfx * dfx + dfy * dfy + 1.0);
    const T sm = vv(mag) < 1e-12 ? T(1.0) : mag;
    nx = dfx / sm;
    ny = dfy / sm;
    nz = -1.0 / sm;
  }
  return z;
}

// qpoly.py:469-520 (compute_z_zprime_q2d): the m = 0 Q-bfs part and the m > 0 orders at
// (u, theta); c1 / s1 = cos / sin theta, cos / sin (m theta) by recurrence.
template <class T, class PD>
ORT_INLINE void q2d_sums(PD B, const T& u, const T& c1, const T& s1, bool want_d, T& p0,
                         T& dp0, T& pg, T& dr, T& dt) {
  const int L0 = (int)B[3];
  const T usq = u * u;
  T d0;
  qbfs_clenshaw(B + 4, L0, usq, want_d, p0, d0);
  dp0 = d0 * 2.0 * u;
  PD rec = B + 4 + L0;
  const int M = (int)rec[0];
  ++rec;
  pg = T(0.0);
  dr = T(0.0);
  dt = T(0.0);
  T cm = c1, sm = s1;  // cos / sin (m theta)
  T um = u;            // u ** m
  T um1 = T(1.0);      // u ** (m - 1)
#pragma unroll 1
  for (int m = 1; m <= M; ++m) {
    T sa, dsa, sb, dsb;
    q2d_clenshaw(rec, m, usq, want_d, sa, dsa);
    rec = q2d_next(rec);
    q2d_clenshaw(rec, m, usq, want_d, sb, dsb);
    rec = q2d_next(rec);
    const T term = um * (cm * sa + sm * sb);
    pg = m == 1 ? term : pg + term;
    if (want_d) {
      const T two_usq = 2.0 * usq;
      const T at = cm * (two_usq * dsa + (double)m * sa);
      const T bt = sm * (two_usq * dsb + (double)m * sb);
      const T rt = um1 * (at + bt);
      const T tt = (double)m * um * (-sa * sm + sb * cm);
      dr = m == 1 ? rt : dr + rt;
      dt = m == 1 ? tt : dt + tt;
    }
    const T cn = cm * c1 - sm * s1;
    sm = sm * c1 + cm * s1;
    cm = cn;
    um1 = um;
    um = um * u;
  }
}

// forbes/geometry.py:420-450 (sag) and :545-610 (_surface_normal_analytical)
template <class T, class S, class PD>
ORT_INLINE T sagnorm_q2d(const T& x, const T& y, const S& R, const S& k, bool rinf, PD B,
                         bool want_normal, T& nx, T& ny, T& nz) {
  const double nr = B[0];
  const T r2 = x * x + y * y;
  const T rho0 = sqrt(r2);
  T c1, s1;
  polar_unit(x, y, rho0, c1, s1);  // theta = atan2(y, x)
  T cf, dcf;
  forbes_conic_factor(r2, R, k, rinf, cf, dcf);
  T z;
  {
    const T u = sqrt(r2 + 1e-12) / nr;
    T p0, dp0, pg, dr, dt;
    q2d_sums(B, u, c1, s1, false, p0, dp0, pg, dr, dt);
    const T uu = u * u;
    const T total = uu * (1.0 - uu) * cf * p0 + cf * pg;
    z = forbes_base_sag(r2, R, k, rinf) + (vv(u) > 1.0 ? T(0.0) : total);
  }
  if (want_normal) {
    T dfx, dfy;
    if (vv(rho0) < 1e-12) {  // the vertex: analytical slope of the m = 1 order
      dfx = T(B[1]);
      dfy = T(B[2]);
    } else {
      const T u = rho0 / nr;
      T p0, dp0, pg, dr, dt;
      q2d_sums(B, u, c1, s1, true, p0, dp0, pg, dr, dt);
      const T dp0r = dp0 / nr;
      const T drr = dr / nr;
      const T uu = u * u;
      const T dpre = (2.0 * u - 4.0 * (u * u * u)) / nr;
      const T q = uu - uu * uu;
      const T ds0 = (dpre * p0 + q * dp0r) * cf + q * p0 * dcf;
      const T dsg = dcf * pg + cf * drr;
      const bool out = vv(u) > 1.0;
      const T dsr = out ? T(0.0) : ds0 + dsg;
      const T dst = out ? T(0.0) : cf * dt;
      const T ct = x / rho0, st = y / rho0;
      const T dsx = ct * dsr - (st / rho0) * dst;
      const T dsy = st * dsr + (ct / rho0) * dst;
      const T dbr = forbes_base_dsag(rho0, r2, R, k, rinf);
      dfx = dbr * ct + dsx;
      dfy = dbr * st + dsy;
    }
    const T mag = sqrt(dfx * dfx + dfy * dfy + 1.0);
    const T smg = vv(mag) < 1e-12 ? T(1.0) : mag;
    nx = dfx / smg;
    ny = dfy / smg;
    nz = -1.0 / smg;
  }
  return z;
}

// ---- grid sag: geometries/grid_sag.py:61-149 ------------------------------------------
// Block (lens.coef at coef_off): nx, ny, x grid, y grid, sag[ny][nx]. Per-lane table reads
// go through the generic address space (divergent indices).
struct GridView {
  const double* x;
  const double* y;
  const double* z;
  int nx, ny;
};

template <class PD>
ORT_INLINE GridView grid_view(PD C) {
  GridView g;
  g.nx = (int)C[0];
  g.ny = (int)C[1];
  g.x = (const double*)(C + 2);
  g.y = g.x + g.nx;
  g.z = g.y + g.ny;
  return g;
}

// numpy.searchsorted(v, x, side="right") - 1, NaN sorting last
ORT_INLINE int grid_cell(const double* v, int n, double x) {
  if (!(x == x)) return n - 1;
  int lo = 0, hi = n;  // first index with v[k] > x
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (v[mid] <= x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo - 1;
}

// grid_sag.py:61-101: bilinear sag (NaN off the grid) and its x / y derivatives
ORT_INLINE double grid_interp(const GridView& g, double x, double y, double& dsdx,
                              double& dsdy) {
  int i = grid_cell(g.x, g.nx, x);
  int j = grid_cell(g.y, g.ny, y);
  const bool off = (x < g.x[0]) || (x > g.x[g.nx - 1]) || (y < g.y[0]) || (y > g.y[g.ny - 1]);
  i = i < 0 ? 0 : i;
  j = j < 0 ? 0 : j;
  i = i >= g.nx - 1 ? g.nx - 2 : i;
  j = j >= g.ny - 1 ? g.ny - 2 : j;
  const double x1 = g.x[i], x2 = g.x[i + 1], y1 = g.y[j], y2 = g.y[j + 1];
  const double* r0 = g.z + (int64_t)j * g.nx + i;
  const double z11 = r0[0], z12 = r0[1], z21 = r0[g.nx], z22 = r0[g.nx + 1];
  const double tx = (x - x1) / (x2 - x1);
  const double ty = (y - y1) / (y2 - y1);
  const double z_y1 = z11 * (1.0 - tx) + z12 * tx;
  const double z_y2 = z21 * (1.0 - tx) + z22 * tx;
  const double sag = z_y1 * (1.0 - ty) + z_y2 * ty;
  dsdx = ((z12 - z11) * (1.0 - ty) + (z22 - z21) * ty) / (x2 - x1);
  dsdy = ((z21 - z11) * (1.0 - tx) + (z22 - z12) * tx) / (y2 - y1);
  return off ? __builtin_nan("") : sag;
}

// grid_sag.py:103-106, 142-149: normal (-ds/dx, -ds/dy, 1) normalised
ORT_INLINE double sagnorm_grid(const GridView& g, double x, double y, bool want_normal,
                               double& nx, double& ny, double& nz) {
  double dsdx, dsdy;
  const double sag = grid_interp(g, x, y, dsdx, dsdy);
  if (want_normal) {
    const double mag = sqrt(dsdx * dsdx + dsdy * dsdy + 1.0);
    const SharedDiv dm = shared_div(mag);
    nx = sdiv(-dsdx, dm);
    ny = sdiv(-dsdy, dm);
    nz = sdiv(1.0, dm);
  }
  return sag;
}

// grid_sag.py:111-126: one Newton update from t (returns dt = -f / f')
ORT_INLINE double grid_step(const GridView& g, const Ray& r, double t) {
  const double xi = r.x + t * r.L;
  const double yi = r.y + t * r.M;
  const double zi = r.z + t * r.N;
  double dsdx, dsdy;
  const double f = grid_interp(g, xi, yi, dsdx, dsdy) - zi;
  const double fp = dsdx * r.L + dsdy * r.M - r.N;
  return -f / fp;
}

// grid_sag.py:131-140: rays that end off the grid get NaN
ORT_INLINE double grid_final(const GridView& g, const Ray& r, double t) {
  const double xf = r.x + t * r.L;
  const double yf = r.y + t * r.M;
  const bool off =
      (xf < g.x[0]) || (xf > g.x[g.nx - 1]) || (yf < g.y[0]) || (yf > g.y[g.ny - 1]);
  return off ? __builtin_nan("") : t;
}

// ---- NURBS: geometries/nurbs/nurbs_geometry.py (ort_nurbs.h) ----------------------------
#include "ort_nurbs.h"

// Sag and normal of a Newton-iterated geometry (EvenAsphere / OddAsphere / Zernike).
// KM is a bitmask of the Newton kinds compiled in (KM_EVEN | KM_ODD | KM_ZERN): a lens
// only pays registers for the kinds it contains.
// KM_FREE covers the freeform kinds (XY polynomial, Chebyshev, biconic, toroidal, Forbes
// Q-bfs / Q-2D, grid sag) with a runtime switch; KM_NURBS the NURBS surfaces.
// KM_NURBS (bit 16, clear of the kernels' other specialisation bits, ort_sweep.h): NURBS
// surfaces, compiled only into the kernels of lenses that have one (ort_k_trace_ia.hip,
// ort_k_geom.hip)
enum : unsigned { KM_EVEN = 1u, KM_ODD = 2u, KM_ZERN = 4u, KM_FREE = 8u, KM_NURBS = 1u << 16 };

// R, K: the surface's radius and conic (double, or seeded duals in the derivative kernels)
template <unsigned KM, class T, class S, class PD, class PZ>
ORT_INLINE T newton_sagnorm(const ort_surface& s, const S& R, const S& K, PD coef, PZ zern,
                            const ZSeed& zs, const T& x, const T& y, int want_normal,
                            bool& range_error, T& nx, T& ny, T& nz) {
  const PD C = coef + s.coef_off;
  if constexpr ((KM & KM_EVEN) != 0) {
    if (KM == KM_EVEN || s.geometry == ORT_GEOM_EVEN_ASPHERE)
      return sagnorm_even(x, y, R, K, C, s.n_coef, want_normal, nx, ny, nz);
  }
  if constexpr ((KM & KM_ODD) != 0) {
    if ((KM & ~KM_ODD) == 0 || s.geometry == ORT_GEOM_ODD_ASPHERE)
      return sagnorm_odd(x, y, R, K, C, s.n_coef, want_normal, nx, ny, nz);
  }
  if constexpr ((KM & KM_ZERN) != 0) {
    if ((KM & ~KM_ZERN) == 0 || s.geometry == ORT_GEOM_ZERNIKE)
      return sagnorm_zernike(x, y, R, K, s.norm_radius, zern, s.coef_off, s.n_coef, coef, zs,
                             want_normal, range_error, nx, ny, nz, s.zm_off, s.zm_deg);
  }
  if constexpr ((KM & KM_NURBS) != 0) {  // primal kernels only (no derivative kernels)
    if (s.geometry == ORT_GEOM_NURBS) {
      if constexpr (std::is_same<T, double>::value) {
        const T z = sagnorm_nurbs(nurbs_view(C), s.tol, s.max_iter, x, y,
                                  want_normal != kNoNormal, nx, ny, nz);
        if (want_normal == kSlope) slope_from_normal(nx, ny, nz);
        return z;
      } else {
        nx = ny = nz = T(NAN);
        return T(NAN);
      }
    }
  }
  if constexpr ((KM & KM_FREE) != 0) {
    // the freeform kinds form the unit normal; kSlope's (fx, fy, -1) from it
    const bool wn = want_normal != kNoNormal;
    T z;
    switch (s.geometry) {
      case ORT_GEOM_POLYNOMIAL:
        z = sagnorm_poly(x, y, R, K, C, wn, nx, ny, nz);
        break;
      case ORT_GEOM_CHEBYSHEV: {
        bool cerr = false;
        z = sagnorm_cheb(x, y, R, K, C, wn, cerr, nx, ny, nz);
        if (cerr) range_error = true;
        break;
      }
      case ORT_GEOM_BICONIC:
        z = sagnorm_biconic(x, y, C, wn, nx, ny, nz);
        break;
      case ORT_GEOM_FORBES_QBFS:
        z = sagnorm_qbfs(x, y, R, K, (s.flags & ORT_SURF_RADIUS_INF) != 0, C, wn, nx, ny, nz);
        break;
      case ORT_GEOM_FORBES_Q2D:
        z = sagnorm_q2d(x, y, R, K, (s.flags & ORT_SURF_RADIUS_INF) != 0, C, wn, nx, ny, nz);
        break;
      case ORT_GEOM_GRID_SAG:  // primal kernels only (no derivative kernels for grids)
        if constexpr (std::is_same<T, double>::value) {
          z = sagnorm_grid(grid_view(C), x, y, wn, nx, ny, nz);
        } else {
          nx = ny = nz = z = T(NAN);
        }
        break;
      case ORT_GEOM_TOROIDAL:
        z = sagnorm_toroidal(x, y, C, wn, nx, ny, nz);
        break;
      default:  // an id this library does not know: NaN, never another kind's sag
        nx = ny = nz = T(NAN);
        return T(NAN);
    }
    if (want_normal == kSlope) slope_from_normal(nx, ny, nz);
    return z;
  }
  nx = ny = nz = T(NAN);
  return T(NAN);
}

template <unsigned KM, class T, class S, class PD, class PZ>
ORT_INLINE void newton_normal(const ort_surface& s, const S& R, const S& K, PD coef, PZ zern,
                              const ZSeed& zs, const T& x, const T& y, T& nx, T& ny, T& nz) {
  bool rerr = false;  // the normal never raises (zernike.py:163-231)
  (void)newton_sagnorm<KM>(s, R, K, coef, zern, zs, x, y, true, rerr, nx, ny, nz);
}

// One Newton evaluation at t (newton_raphson.py:140-146): returns f(t) = sag(P(t)) - z(t)
// and, with want_normal, the normal at P(t) for the update.
template <unsigned KM, class T, class S, class PD, class PZ>
ORT_INLINE T newton_eval(const ort_surface& s, const S& R, const S& K, PD coef, PZ zern,
                         const ZSeed& zs, const RayT<T>& r, const T& t, int want_normal,
                         bool& range_error, T& nx, T& ny, T& nz) {
  const T xi = r.x + t * r.L;
  const T yi = r.y + t * r.M;
  const T zi = r.z + t * r.N;
  return newton_sagnorm<KM>(s, R, K, coef, zern, zs, xi, yi, want_normal, range_error, nx, ny,
                            nz) - zi;
}

// newton_raphson.py:154-166: t_new = t - f / f'(t) from the update's slopes (fx, fy) at
// P(t) (an evaluation with want_normal = kSlope)
template <class T>
ORT_INLINE T newton_step_slope(const RayT<T>& r, const T& t, const T& f, const T& fx,
                               const T& fy) {
  const T df = fx * r.L + fy * r.M - r.N;
  const T dfs = ::fabs(vv(df)) > 1e-14 ? df : T(1e-14);
  return t - f / dfs;
}

// the same from a unit normal (the reference's own form)
template <class T>
ORT_INLINE T newton_step(const RayT<T>& r, const T& t, const T& f, T nx, T ny, T nz) {
  slope_from_normal(nx, ny, nz);
  return newton_step_slope(r, t, f, nx, ny);
}

// the update from a kSlope evaluation: its slopes (nz == -1) or its unit normal
template <class T>
ORT_INLINE T newton_step_any(const RayT<T>& r, const T& t, const T& f, const T& nx,
                             const T& ny, const T& nz) {
  if (vv(nz) == -1.0) return newton_step_slope(r, t, f, nx, ny);
  return newton_step(r, t, f, nx, ny, nz);
}

// ---------------------------------------------------------------------------------
// per-surface physics
// ---------------------------------------------------------------------------------
// propagation/homogeneous.py:30-57 (alpha = 4 pi k / w, applied only when k > 0)
template <class T>
ORT_INLINE void propagate(RayT<T>& r, const T& t, double alpha) {
  r.x = r.x + t * r.L;
  r.y = r.y + t * r.M;
  r.z = r.z + t * r.N;
  if (alpha > 0.0) r.att = r.att + -alpha * t * 1e3;
}

// propagate with the surface's absorption decided by its ORT_SURF_ALPHA_* flags when
// every wavelength row agrees (a scalar branch instead of a per-lane select); same values
template <class T>
ORT_INLINE void propagate_flagged(RayT<T>& r, const T& t, double alpha, int32_t flags) {
  r.x = r.x + t * r.L;
  r.y = r.y + t * r.M;
  r.z = r.z + t * r.N;
  if (flags & ORT_SURF_ALPHA_NONE) return;
  if ((flags & ORT_SURF_ALPHA_ALL) || alpha > 0.0) r.att = r.att + -alpha * t * 1e3;
}

// surfaces/standard_surface.py:218
template <class T>
ORT_INLINE void add_opd(RayT<T>& r, const T& t, double n_pre) {
  r.opd = r.opd + fabs(t * n_pre);
}

// physical_apertures/radial.py:50-63 + rays/real_rays.py:132-139
template <class T>
ORT_INLINE void clip_radial(RayT<T>& r, double rmax2, double rmin2) {
  const double radius2 = vv(r.x * r.x + r.y * r.y);
  const bool inside = (radius2 <= rmax2) && (radius2 >= rmin2);
  if (!inside) {
    r.i = T(0.0);
    r.att = T(0.0);
  }
}

// General physical apertures (physical_apertures/*.py): the postfix program described
// at ort_aperture_op, evaluated on the local (x, y); clips like clip_radial. The stack of
// booleans is a bit mask (at most 32 deep).
template <class PD>
ORT_INLINE bool aperture_contains(PD p, int len, double x, double y) {
  uint32_t st = 0;
  int sp = 0;
  for (int q = 0; q < len;) {
    const int op = (int)p[q];
    bool v = false;
    switch (op) {
      case ORT_AP_RADIAL: {  // radial.py:62, offset_radial.py:57-58
        const double dx = x - p[q + 3], dy = y - p[q + 4];
        const double r2 = dx * dx + dy * dy;
        v = (r2 <= p[q + 2]) && (r2 >= p[q + 1]);
        q += 5;
      } break;
      case ORT_AP_ELLIPSE: {  // elliptical.py:53-55
        const double dx = x - p[q + 1], dy = y - p[q + 2];
        v = (dx * dx / p[q + 3] + dy * dy / p[q + 4]) <= 1.0;
        q += 5;
      } break;
      case ORT_AP_RECT:  // rectangular.py:54-59
        v = (p[q + 1] <= x) && (x <= p[q + 2]) && (p[q + 3] <= y) && (y <= p[q + 4]);
        q += 5;
        break;
      case ORT_AP_POLYGON: {  // matplotlib point_in_path: even-odd crossings, closed
        const int n = (int)p[q + 1];
        const PD v0 = p + q + 2;
        if (isfinite(x) && isfinite(y) && n > 0) {
          double vx0 = v0[2 * (n - 1)], vy0 = v0[2 * (n - 1) + 1];
          // edges (v_{k-1} -> v_k) for k = 0..n-1 with v_{-1} = v_{n-1}: the same edge set
          // as matplotlib's v_0 -> v_1 -> ... -> v_{n-1} -> v_0, the same test per edge
          bool yflag0 = vy0 >= y;
          bool in = false;
          for (int k = 0; k < n; ++k) {
            const double vx1 = v0[2 * k], vy1 = v0[2 * k + 1];
            const bool yflag1 = vy1 >= y;
            if (yflag0 != yflag1 &&
                (((vy1 - y) * (vx0 - vx1) >= (vx1 - x) * (vy0 - vy1)) == yflag1))
              in = !in;
            yflag0 = yflag1;
            vx0 = vx1;
            vy0 = vy1;
          }
          v = in;
        }
        q += 2 + 2 * n;
      } break;
      default: {  // boolean ops (base.py:255-340)
        const bool b = (st >> (sp - 1)) & 1u, a = (st >> (sp - 2)) & 1u;
        sp -= 2;
        v = op == ORT_AP_UNION ? (a || b) : (op == ORT_AP_INTERSECT ? (a && b) : (a && !b));
        q += 1;
      } break;
    }
    st = (st & ~(1u << sp)) | ((uint32_t)v << sp);
    ++sp;
  }
  return sp > 0 && ((st >> (sp - 1)) & 1u);
}

template <class T, class PD>
ORT_INLINE void clip_program(RayT<T>& r, PD prog, int len) {
  if (!aperture_contains(prog, len, vv(r.x), vv(r.y))) {
    r.i = T(0.0);
    r.att = T(0.0);
  }
}

// rays/real_rays.py:511-547: sign(dot) flip (np.sign: 0 -> 0, NaN -> NaN), |dot|
template <class T>
ORT_INLINE T align_normal(const RayT<T>& r, T& nx, T& ny, T& nz) {
  const T dot = r.L * nx + r.M * ny + r.N * nz;
  const double dv = vv(dot);
  const double sgn = dv > 0.0 ? 1.0 : (dv < 0.0 ? -1.0 : (dv == dv ? 0.0 : dv));
  nx = nx * sgn;
  ny = ny * sgn;
  nz = nz * sgn;
  return fabs(dot);
}

// rays/real_rays.py:141-163; u = n1 / n2 comes from the host table (the same IEEE
// quotient the reference forms per ray)
template <class T>
ORT_INLINE void refract(RayT<T>& r, T nx, T ny, T nz, double u) {
  const T dot = align_normal(r, nx, ny, nz);
  const T root = sqrt(1.0 - u * u * (1.0 - dot * dot));
  const T L0 = r.L, M0 = r.M, N0 = r.N;
  r.L = u * L0 + nx * root - u * nx * dot;
  r.M = u * M0 + ny * root - u * ny * dot;
  r.N = u * N0 + nz * root - u * nz * dot;
}

// rays/real_rays.py:165-181
template <class T>
ORT_INLINE void reflect(RayT<T>& r, T nx, T ny, T nz) {
  const T dot = align_normal(r, nx, ny, nz);
  r.L = r.L - 2.0 * dot * nx;
  r.M = r.M - 2.0 * dot * ny;
  r.N = r.N - 2.0 * dot * nz;
}

// surface normal at the current (local) ray position
template <unsigned KM, class T, class S, class PD, class PZ>
ORT_INLINE void surface_normal(const ort_surface& s, const S& R, const S& K, PD coef, PZ zern,
                               const ZSeed& zs, const RayT<T>& r, T& nx, T& ny, T& nz) {
  switch (s.geometry) {
    case ORT_GEOM_PLANE:  // plane.py:79-98
      nx = T(0.0); ny = T(0.0); nz = T(1.0);
      break;
    case ORT_GEOM_STANDARD:
      if constexpr (std::is_same<T, double>::value && std::is_same<S, double>::value) {
        if (s.flags & ORT_SURF_INV_R2) {
          normal_conic_rcp(r.x, r.y, R, K, s.inv_r2, nx, ny, nz);
          break;
        }
      }
      normal_conic(r.x, r.y, R, K, nx, ny, nz);
      break;
    default:
      newton_normal<KM>(s, R, K, coef, zern, zs, r.x, r.y, nx, ny, nz);
  }
}

// everything in Surface.trace after the distance t is known
// (standard_surface.py:215-231 minus localize/globalize)
template <unsigned KM, class T, class S, class PD, class PZ>
ORT_INLINE void finish_surface(RayT<T>& r, const ort_surface& s, const S& R, const S& K,
                               PD coef, PZ zern, const ZSeed& zs, const T& t, double n_pre,
                               double u, double alpha_pre) {
  propagate(r, t, alpha_pre);
  add_opd(r, t, n_pre);
  if (s.flags & ORT_SURF_APERTURE) clip_radial(r, s.ap_rmax2, s.ap_rmin2);
  if (s.flags & ORT_SURF_APERTURE_PROG) clip_program(r, coef + s.ap_off, s.ap_len);
  T nx, ny, nz;
  surface_normal<KM>(s, R, K, coef, zern, zs, r, nx, ny, nz);
  if (s.flags & ORT_SURF_REFLECTIVE)
    reflect(r, nx, ny, nz);
  else
    refract(r, nx, ny, nz, u);
}

}  // namespace ort
