// ort_interact.h -- interaction models beyond refraction / reflection, per ray in fp64:
// thin lenses, phase profiles (generalised Snell's law) and diffraction gratings.
//
// Reference: optiland/interactions/{thin_lens_interaction_model,phase_interaction_model,
// diffractive_model}.py, optiland/phase/{constant,linear_grating,radial}.py,
// optiland/geometries/{plane_grating,standard_grating}.py (grating vectors) and
// optiland/rays/real_rays.py:183-509 (gratingdiffract, normalize). Every expression is
// evaluated in the reference's NumPy operation order (-ffp-contract=off), so the results
// are the reference's to the bit, except the radial phase's r**k for k >= 3 (NumPy calls
// libm pow; here a double-double product rounded once).
//
// Parameter blocks (lens.coef at ort_surface.ia_off) are described in
// include/optiland_rt.h at enum ort_interaction.
//
// T = double in the trace kernels; T = Dual<P> in the forward-mode VJP (vjp_ray), whose
// values are the same operations (a dual's value is its double expression, divisions
// plain IEEE) -- the derivatives follow every ray-dependent quantity, the parameter
// blocks, indices and wavelengths are constants.

#pragma once

#include "ort_core.h"

namespace ort {

// rays/real_rays.py:503-509: L, M, N divided by sqrt(L**2 + M**2 + N**2)
template <class T>
ORT_INLINE void normalize_dir(RayT<T>& r) {
  const T mag = sqrt(r.L * r.L + r.M * r.M + r.N * r.N);
  const auto d = shared_div(mag);
  r.L = sdiv(r.L, d);
  r.M = sdiv(r.M, d);
  r.N = sdiv(r.N, d);
}

// interactions/thin_lens_interaction_model.py:55-113: OPD of the paraxial phase
// transformation, slopes u' = (n1 u - x / f) / n2 (n2 = -n1 on a mirror), direction
// (u'x, u'y, 1) left unnormalised (the next propagation normalises it).
template <class T>
ORT_INLINE void thin_lens(RayT<T>& r, double f, double n1, double n2) {
  r.opd = r.opd - (r.x * r.x + r.y * r.y) / (2.0 * f);
  const auto dn = shared_div(r.N);
  const T ux1 = sdiv(r.L, dn);
  const T uy1 = sdiv(r.M, dn);
  const double inv_n2 = 1.0 / n2;
  const SharedDiv df = shared_div(f);
  r.L = inv_n2 * (n1 * ux1 - sdiv(r.x, df));
  r.M = inv_n2 * (n1 * uy1 - sdiv(r.y, df));
  r.N = T(1.0);
}

// x**k for an integer k >= 1, rounded once: NumPy squares exactly for k == 2 and passes
// x through for k == 1; for k >= 3 it calls libm pow, whose result is the correctly
// rounded power in all but astronomically rare cases -- a double-double product
// rounded at the end gives that same value.
ORT_INLINE double pow_k(double x, int k) {
  if (k == 1) return x;
  if (k == 2) return x * x;
  double hi = x, lo = 0.0;
#pragma unroll 1
  for (int q = 1; q < k; ++q) {
    const double p = hi * x;
    const double e = fma(hi, x, -p);
    lo = fma(lo, x, e);
    hi = p;
  }
  return hi + lo;
}
// the dual power: the same value, d(x^k) = k x^(k-1) dx
template <int P>
ORT_INLINE Dual<P> pow_k(const Dual<P>& x, int k) {
  Dual<P> r(pow_k(x.v, k));
  const double dk = k == 1 ? 1.0 : (double)k * pow_k(x.v, k - 1);
#pragma unroll
  for (int q = 0; q < P; ++q) r.d[q] = dk * x.d[q];
  return r;
}

// phase/*.py get_phase + get_gradient at (x, y); the z gradient is 0 for every profile
template <class PD, class T>
ORT_INLINE void phase_profile(PD p, const T& x, const T& y, T& phase, T& gx, T& gy) {
  const int kind = (int)p[0];
  if (kind == ORT_PHASE_CONSTANT) {  // constant.py: full_like(x, phase), zero gradient
    phase = T(p[2]);
    gx = T(0.0);
    gy = T(0.0);
  } else if (kind == ORT_PHASE_LINEAR) {  // linear_grating.py:60-92
    phase = p[2] * x + p[3] * y;
    gx = T(p[2]);
    gy = T(p[3]);
  } else {  // radial.py:26-75: phi = sum a_i r2**(i+1), d phi / dr = sum 2 (i+1) a_i r**(2i+1)
    const int n = (int)p[2];
    const T r2 = x * x + y * y;
    phase = T(0.0);
#pragma unroll 1
    for (int i = 0; i < n; ++i) phase = phase + p[3 + i] * pow_k(r2, i + 1);
    const T r = sqrt(r2);
    T dr = T(0.0);
#pragma unroll 1
    for (int i = 0; i < n; ++i)
      dr = dr + p[3 + i] * 2.0 * (double)(i + 1) * pow_k(r, 2 * (i + 1) - 1);
    const bool at0 = vv(r) == 0.0;
    const T q = dr / (at0 ? T(1.0) : r);
    gx = at0 ? T(0.0) : q * x;
    gy = at0 ? T(0.0) : q * y;
  }
}

// interactions/phase_interaction_model.py:45-132 (the normal is used as the geometry
// returns it, not aligned with the ray)
template <class PD, class T>
ORT_INLINE void phase_interact(RayT<T>& r, PD p, const T& nx, const T& ny, const T& nz,
                               double n1, double n2, bool reflective, double w) {
  const double k0 = 6.283185307179586 / w;  // 2 * be.pi / rays.w
  const T kix = n1 * k0 * r.L;
  const T kiy = n1 * k0 * r.M;
  const T kiz = n1 * k0 * r.N;
  T phase, gx, gy;
  phase_profile(p, r.x, r.y, phase, gx, gy);
  const double gz = 0.0;
  const T gdn = gx * nx + gy * ny + gz * nz;
  const T Gx = gx - gdn * nx, Gy = gy - gdn * ny, Gz = gz - gdn * nz;
  const T kdn = kix * nx + kiy * ny + kiz * nz;
  const T kx0 = kix - kdn * nx + Gx;
  const T ky0 = kiy - kdn * ny + Gy;
  const T kz0 = kiz - kdn * nz + Gz;
  const T par2 = kx0 * kx0 + ky0 * ky0 + kz0 * kz0;
  const double nk = n2 * k0;
  T rsq = nk * nk - par2;
  if (vv(rsq) < 0.0) {  // TIR / evanescent: rays.clip
    r.i = T(0.0);
    r.att = T(0.0);
  }
  rsq = (0.0 >= vv(rsq)) ? T(0.0) : rsq;  // np.maximum(0.0, R_sq): NaN propagates
  const T alpha = (reflective ? -1.0 : 1.0) * sqrt(rsq);
  const T kx = kx0 + alpha * nx;
  const T ky = ky0 + alpha * ny;
  const T kz = kz0 + alpha * nz;
  const T mag = sqrt(kx * kx + ky * ky + kz * kz);
  const auto dm = shared_div(mag);
  r.L = sdiv(kx, dm);
  r.M = sdiv(ky, dm);
  r.N = sdiv(kz, dm);
  r.opd = r.opd + -phase / k0;
  r.i = r.i * p[1];  // phase_profile.efficiency
}

// Grating vector at the local hit point: constant for PlaneGrating
// (plane_grating.py:105-124), from the groove tangent of the conic for
// StandardGratingGeometry (standard_grating.py:93-146, 224-247; n = the unaligned normal)
template <class PD, class T>
ORT_INLINE void grating_vector(PD p, const T& x, const T& y, const T& nx, const T& ny,
                               const T& nz, T& fx, T& fy, T& fz) {
  if (p[2] == 0.0) {
    fx = T(p[3]);
    fy = T(p[4]);
    fz = T(0.0);
    return;
  }
  const double ta = p[3], R2 = p[4], R3 = p[5], kp1 = p[6];
  const T r2 = x * x + y * y;
  const T s = sqrt((R2 - kp1 * r2) / R2);
  const T s1 = s + 1.0;
  const T dzdx = (x + y * ta) * (2.0 * R2 * s * s1 + kp1 * r2) / (R3 * s * (s1 * s1));
  const T nt = sqrt(1.0 + ta * ta + dzdx * dzdx);
  const auto dt = shared_div(nt);
  const T tx = sdiv(1.0, dt), ty = sdiv(T(ta), dt), tz = sdiv(dzdx, dt);
  const T gx = ny * tz - nz * ty;
  const T gy = -nx * tz + nz * tx;
  const T gz = nx * ty - ny * tx;
  const T mag = sqrt(gx * gx + gy * gy + gz * gz);
  const auto dm = shared_div(mag);
  fx = -sdiv(gx, dm);
  fy = -sdiv(gy, dm);
  fz = -sdiv(gz, dm);
}

// real_rays.py:183-498 (gratingdiffract) as called by diffractive_model.py:28-61:
// d = period / sqrt(fx**2 + fy**2), the normal aligned with the ray, the closed-form
// diffracted direction (every term in the reference's order), then normalize().
template <class PD, class T>
ORT_INLINE void diffract(RayT<T>& r, PD p, T nx, T ny, T nz, double n1, double n2,
                         bool reflective, double w) {
  T fx, fy, fz;
  grating_vector(p, r.x, r.y, nx, ny, nz, fx, fy, fz);
  const double m = p[0];
  const T d = p[1] / sqrt(fx * fx + fy * fy);
  const T L0 = r.L, M0 = r.M, N0 = r.N;
  align_normal(r, nx, ny, nz);
  const double n2c = reflective ? n2 * -1.0 : n2;
  const double n12 = n1 * n1, m2 = m * m, w2 = w * w;
  const T d2 = d * d;
  const T nx2 = nx * nx, ny2 = ny * ny, nz2 = nz * nz;
  // clang-format off
  const T D =
      -(L0 * L0) * d2 * n12 * ny2
      - L0 * L0 * d2 * n12 * nz2
      + 2.0 * L0 * M0 * d2 * n12 * nx * ny
      + 2.0 * L0 * N0 * d2 * n12 * nx * nz
      - 2.0 * L0 * d * fx * m * n1 * ny2 * w
      - 2.0 * L0 * d * fx * m * n1 * nz2 * w
      + 2.0 * L0 * d * fy * m * n1 * nx * ny * w
      + 2.0 * L0 * d * fz * m * n1 * nx * nz * w
      - M0 * M0 * d2 * n12 * nx2
      - M0 * M0 * d2 * n12 * nz2
      + 2.0 * M0 * N0 * d2 * n12 * ny * nz
      + 2.0 * M0 * d * fx * m * n1 * nx * ny * w
      - 2.0 * M0 * d * fy * m * n1 * nx2 * w
      - 2.0 * M0 * d * fy * m * n1 * nz2 * w
      + 2.0 * M0 * d * fz * m * n1 * ny * nz * w
      - N0 * N0 * d2 * n12 * nx2
      - N0 * N0 * d2 * n12 * ny2
      + 2.0 * N0 * d * fx * m * n1 * nx * nz * w
      + 2.0 * N0 * d * fy * m * n1 * ny * nz * w
      - 2.0 * N0 * d * fz * m * n1 * nx2 * w
      - 2.0 * N0 * d * fz * m * n1 * ny2 * w
      + d2 * (n2c * n2c) * nx2
      + d2 * (n2c * n2c) * ny2
      + d2 * (n2c * n2c) * nz2
      - fx * fx * m2 * ny2 * w2
      - fx * fx * m2 * nz2 * w2
      + 2.0 * fx * fy * m2 * nx * ny * w2
      + 2.0 * fx * fz * m2 * nx * nz * w2
      - fy * fy * m2 * nx2 * w2
      - fy * fy * m2 * nz2 * w2
      + 2.0 * fy * fz * m2 * ny * nz * w2
      - fz * fz * m2 * nx2 * w2
      - fz * fz * m2 * ny2 * w2;
  // clang-format on
  const T sD = sqrt(D);
  const T AL = L0 * d * n1 * ny2 + L0 * d * n1 * nz2 - M0 * d * n1 * nx * ny -
                    N0 * d * n1 * nx * nz + fx * m * ny2 * w + fx * m * nz2 * w -
                    fy * m * nx * ny * w - fz * m * nx * nz * w;
  const T AM = -L0 * d * n1 * nx * ny + M0 * d * n1 * nx2 + M0 * d * n1 * nz2 -
                    N0 * d * n1 * ny * nz - fx * m * nx * ny * w + fy * m * nx2 * w +
                    fy * m * nz2 * w - fz * m * ny * nz * w;
  const T PN = L0 * d * n1 * nx * nz + M0 * d * n1 * ny * nz - N0 * d * n1 * nx2 -
                    N0 * d * n1 * ny2 + fx * m * nx * nz * w + fy * m * ny * nz * w -
                    fz * m * nx2 * w - fz * m * ny2 * w;
  const auto dd = shared_div(d * n2c);
  if (reflective) {
    r.L = sdiv(AL - nx * sD, dd);
    r.M = sdiv(AM - ny * sD, dd);
    r.N = sdiv(-nz * sD, dd) - sdiv(PN, dd);
  } else {
    r.L = sdiv(AL + nx * sD, dd);
    r.M = sdiv(AM + ny * sD, dd);
    r.N = sdiv(nz * sD, dd) - sdiv(PN, dd);
  }
  normalize_dir(r);
}

}  // namespace ort
