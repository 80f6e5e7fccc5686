// ort_material.h -- per-ray dispersion: n(lambda), k(lambda) of one material
// (include/optiland_rt.h ort_material) for rays that each carry their own wavelength.
//
// The reference evaluates material.n(rays.w) / material.k(rays.w) for the whole
// wavelength array of a RealRays (materials/base.py:73-119) with the refractiveindex.info
// formulas of materials/material_file.py:250-428 and numpy.interp for tabulated data
// (:219-249, 422-428). Each formula here is that expression in the same operation order;
// lambda-independent subexpressions (1 + C0, C ** 2, C3 ** C4, ...) arrive precomputed
// by the host in NumPy. w ** 2 is the exact product (NumPy's square); other real powers
// use the device pow (NumPy's vectorised pow differs from it at the ulp level).
#pragma once

#include "ort_core.h"

namespace ort {

ORT_INLINE double wpow(double w, double e) {
  return e == 2.0 ? w * w : ::pow(w, e);
}

// numpy.interp(x, xp, fp) for increasing xp (numpy/_core/src/multiarray/compiled_base.c
// arr_interp): clamped ends, exact hits, slope * (x - xp[j]) + fp[j] with its NaN fallbacks
template <class PD>
ORT_INLINE double np_interp(double x, PD xp, PD fp, int n) {
  if (n == 1) return fp[0];  // one point: fp[0] everywhere (NaN included)
  if (x != x) return x;
  if (x <= xp[0]) return fp[0];
  if (x >= xp[n - 1]) return fp[n - 1];
  int lo = 0, hi = n - 1;  // xp[lo] <= x < xp[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (x >= xp[mid])
      lo = mid;
    else
      hi = mid;
  }
  if (xp[lo] == x) return fp[lo];
  const double slope = (fp[lo + 1] - fp[lo]) / (xp[lo + 1] - xp[lo]);
  double r = slope * (x - xp[lo]) + fp[lo];
  if (r != r) {
    r = slope * (x - xp[lo + 1]) + fp[lo + 1];
    if (r != r && fp[lo] == fp[lo + 1]) r = fp[lo];
  }
  return r;
}

// refractive index of material m at wavelength w (um)
template <class PD>
ORT_INLINE double material_n(const ort_material& m, PD coef, double w) {
  const PD c = coef + m.coef_off;
  const int nc = m.n_coef;
  switch (m.kind) {
    case ORT_MAT_IDEAL:
      return m.n_const;
    case 1: {  // Sellmeier: sqrt(1 + C0 + sum B w^2 / (w^2 - C^2))
      double n = c[0];
      for (int k = 1; k + 1 < nc; k += 2) n = n + c[k] * (w * w) / (w * w - c[k + 1]);
      return sqrt(n);
    }
    case 2: {  // Sellmeier-2: sqrt(1 + C0 + sum B w^2 / (w^2 - C))
      double n = c[0];
      for (int k = 1; k + 1 < nc; k += 2) n = n + c[k] * (w * w) / (w * w - c[k + 1]);
      return sqrt(n);
    }
    case 3:    // polynomial: sqrt(C0 + sum A w^e)
    case 5: {  // Cauchy: C0 + sum A w^e
      double n = c[0];
      for (int k = 1; k + 1 < nc; k += 2) n = n + c[k] * wpow(w, c[k + 1]);
      return m.kind == 3 ? sqrt(n) : n;
    }
    case 4: {  // RefractiveIndex.INFO
      double n = c[0] + c[1] * wpow(w, c[2]) / (w * w - c[3]) +
                 c[4] * wpow(w, c[5]) / (w * w - c[6]);
      for (int k = 7; k + 1 < nc; k += 2) n = n + c[k] * wpow(w, c[k + 1]);
      return sqrt(n);
    }
    case 6: {  // gases: 1 + C0 + sum B / (C - w^-2)
      double n = c[0];
      const double wm2 = ::pow(w, -2.0);
      for (int k = 1; k + 1 < nc; k += 2) n = n + c[k] / (c[k + 1] - wm2);
      return n;
    }
    case 7: {  // Herzberger
      const double d = w * w - 0.028;
      const double q = 1.0 / d;
      double n = c[0] + c[1] / d + c[2] * (q * q);
      for (int k = 3; k < nc; ++k) n = n + c[k] * wpow(w, (double)(2 * (k - 2)));
      return n;
    }
    case 8: {  // retro
      const double b = c[0] + c[1] * (w * w) / (w * w - c[2]) + c[3] * (w * w);
      return sqrt((1.0 + 2.0 * b) / (1.0 - b));
    }
    case 9: {  // exotic
      const double e = w - c[4];
      const double n = c[0] + c[1] / (w * w - c[2]) + c[3] * e / (e * e + c[5]);
      return sqrt(n);
    }
    case ORT_MAT_ABBE: {  // numpy.polyval: y = y * w + p_i from y = 0 (abbe.py:37-51)
      if (!(w >= 0.380 && w <= 0.750)) return __builtin_nan("");
      double y = 0.0;
      for (int k = 0; k < nc; ++k) y = y * w + c[k];
      return y;
    }
    default:  // ORT_MAT_TABULATED
      return np_interp(w, c, c + nc, nc);
  }
}

// extinction coefficient (material_file.py:219-249: 0 without k data)
template <class PD>
ORT_INLINE double material_k(const ort_material& m, PD coef, double w) {
  if (m.k_len <= 0) return m.k_const;
  return np_interp(w, coef + m.k_off, coef + m.k_off + m.k_len, m.k_len);
}

// homogeneous.py:49-54: alpha = 4 pi k / w, applied only when k > 0
ORT_INLINE double absorption_alpha(double k, double w) {
  return k > 0.0 ? 4.0 * M_PI * k / w : 0.0;
}

}  // namespace ort
