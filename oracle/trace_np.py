"""ORACLE -- NumPy CPU restatement of the reference's sequential real-ray trace.

TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker / CPU baseline.
The product path (optiland_pr_amd) never imports it and has no CPU fallback.

It restates, formula by formula and in the same evaluation order, the reference
(PriUVBio/optiland_Pr, Optiland 0.5.8 fork) NumPy-backend hot path:

  ray_generator.py:28-106, field_types.py:139-180      ray construction
  surface_group.py:232-244, standard_surface.py:186-233 surface loop
  coordinate_system.py:73-107, real_rays.py:90-130     localize / globalize
  plane.py:61-98, standard.py:73-167                   closed-form intersections
  newton_raphson.py:119-168                            Newton refinement (global stop)
  even_asphere.py:82-129, odd_asphere.py:73-130        asphere sag / normal
  zernike.py:133-246, zernike/base.py:42-299           Zernike sag / normal
  polynomial.py, chebyshev.py, biconic.py, toroidal.py  freeform sag / normal
  forbes/geometry.py:83-640, forbes/qpoly.py            Forbes Q-bfs / Q-2D sag / normal
  nurbs/nurbs_geometry.py:309-822 (oracle/nurbs_np.py)  NURBS sag / normal / distance
  homogeneous.py:30-57                                 propagate + absorption
  standard_surface.py:218                              OPD accumulation
  physical_apertures/radial.py:50-63, real_rays.py:132-139  radial clip
  real_rays.py:141-181, 511-547                        refract / reflect
  interactions/thin_lens_interaction_model.py:55-113   thin lens (+ normalize on the
                                                       next propagate, homogeneous.py:55-57)
  interactions/phase_interaction_model.py:45-132,      phase surfaces
    phase/{constant,linear_grating,radial}.py
  interactions/diffractive_model.py:28-61,             gratings
    real_rays.py:183-509, plane_grating.py:105-124,
    standard_grating.py:93-146, 224-247
  real_ray_tracer.py:84-89                             image-space propagate

Input is the lowered lens (optiland_pr_amd._abi structured arrays: the same bytes the
GPU reads). Pinned against the reference's own outputs by tests/test_oracle_golden.py
(fixtures made by tests/golden/gen_golden.py from /root/reference).
"""

from __future__ import annotations

import warnings

import numpy as np

# layout constants (data format shared with the product; no compute is imported)
from optiland_pr_amd import _abi

from . import nurbs_np


class ZernikeRangeError(ValueError):
    pass


# --------------------------------------------------------------------------------------
# rays
# --------------------------------------------------------------------------------------
class Rays:
    """SoA ray state (real_rays.py:46-88)."""

    __slots__ = ("x", "y", "z", "L", "M", "N", "i", "opd")

    def __init__(self, x, y, z, L, M, N, i, opd=None):
        self.x, self.y, self.z = (np.array(a, dtype=np.float64) for a in (x, y, z))
        self.L, self.M, self.N = (np.array(a, dtype=np.float64) for a in (L, M, N))
        self.i = np.array(i, dtype=np.float64)
        self.opd = np.zeros_like(self.x) if opd is None else np.array(opd, dtype=np.float64)

    def copy(self):
        return Rays(self.x, self.y, self.z, self.L, self.M, self.N, self.i, self.opd)

    def take(self, sl):
        return Rays(*(getattr(self, a)[sl] for a in _abi.RAY_FIELDS))

    def as_dict(self):
        return {a: getattr(self, a) for a in _abi.RAY_FIELDS}


def apodize(apod, px, py):
    """apodization/*.py get_intensity(Px, Py) (ray_generator.py:91-95) from the lowered
    record (_abi.APODIZATION: kind + the host-formed constants p, include/optiland_rt.h),
    the reference's NumPy expressions in the reference's order."""
    k, p = int(apod["kind"]), [float(v) for v in apod["p"]]
    with np.errstate(invalid="ignore", divide="ignore"):
        if k == _abi.APOD_UNIFORM:  # uniform.py
            return np.ones_like(px)
        if k == _abi.APOD_GAUSSIAN:  # gaussian.py:65-76
            return np.exp(-(px**2 + py**2) / p[0])
        r = (px**2 + py**2) ** 0.5
        if k == _abi.APOD_COSINE_SQUARED:  # cosine_squared.py:43-48
            return np.where(r < p[0], np.cos((np.pi * r) / p[1]) ** 2, 0.0)
        if k == _abi.APOD_HANN:  # hann.py
            return np.where(r < p[0], 0.5 * (1 - np.cos((2 * np.pi * r) / p[1])), 0.0)
        if k == _abi.APOD_POLYNOMIAL:  # polynomial.py
            return np.where(r < p[0], (1 - (r / p[0]) ** 2) ** p[1], 0.0)
        if k == _abi.APOD_SUPER_GAUSSIAN:  # super_gaussian.py
            return np.exp(-((r / p[0]) ** p[1]))
        if k == _abi.APOD_TUKEY:  # tukey.py
            taper = 0.5 * (1 + np.cos(np.pi * (r - p[1]) / p[2]))
            out = np.where(r <= p[1], 1.0, 0.0)
            return np.where((r > p[1]) & (r < p[0]), taper, out)
    raise ValueError(f"unknown apodization kind {k}")


def generate_rays(seg, px, py, apod=None):
    """ray_generator.py:49-106 with AngleField / ObjectHeightField get_ray_origins
    (field_types.py:139-181, 255-275), object-space telecentric aiming (:56-73) and the
    pupil apodization (:91-95).

    seg: one _abi.SEGMENT record (host scalars EPD, EPL, vx, vy, x_off, y_off, z0);
    apod: one _abi.APODIZATION record or None (intensity 1)."""
    epd, epl = float(seg["epd"]), float(seg["epl"])
    vx, vy = float(seg["vx"]), float(seg["vy"])
    mode = int(seg["mode"])
    if mode == _abi.GEN_INFINITE:
        x0 = px * epd / 2 * vx + float(seg["x_off"])  # field_types.py:166
        y0 = py * epd / 2 * vy + float(seg["y_off"])  # field_types.py:167
    else:
        x0 = np.full_like(px, float(seg["x_off"]))  # field_types.py:173-178
        y0 = np.full_like(px, float(seg["y_off"]))
    z0 = np.full_like(px, float(seg["z0"]))
    if mode == _abi.GEN_TELECENTRIC:  # ray_generator.py:70-73
        x1 = px * vx + x0
        y1 = py * vy + y0
    else:
        x1 = px * epd * vx / 2  # ray_generator.py:76
        y1 = py * epd * vy / 2  # ray_generator.py:77
    z1 = np.full_like(px, epl)
    mag = np.sqrt((x1 - x0) ** 2 + (y1 - y0) ** 2 + (z1 - z0) ** 2)  # :80
    is_zero = mag < 1e-9
    mag = np.where(is_zero, 1.0, mag)
    L = np.where(is_zero, 0.0, (x1 - x0) / mag)
    M = np.where(is_zero, 0.0, (y1 - y0) / mag)
    N = np.where(is_zero, 1.0, (z1 - z0) / mag)
    i = np.ones_like(px) if apod is None else apodize(apod, px, py)
    return Rays(x0, y0, z0, L, M, N, i)


# --------------------------------------------------------------------------------------
# coordinate systems
# --------------------------------------------------------------------------------------
def apply_cs(r: Rays, ops):
    """Apply lowered localize/globalize ops in order (coordinate_system.py:73-107)."""
    for op in ops:
        k = int(op["kind"])
        p = op["p"]
        if k == _abi.CS_TRANSLATE:  # rays/base.py:39-42
            r.x = r.x + p[0]
            r.y = r.y + p[1]
            r.z = r.z + p[2]
        elif k == _abi.CS_ROT_X:  # real_rays.py:96-102
            c, s = p[0], p[1]
            r.y, r.z, r.M, r.N = (r.y * c - r.z * s, r.y * s + r.z * c,
                                  r.M * c - r.N * s, r.M * s + r.N * c)
        elif k == _abi.CS_ROT_Y:  # real_rays.py:110-116
            c, s = p[0], p[1]
            r.x, r.z, r.L, r.N = (r.x * c + r.z * s, -r.x * s + r.z * c,
                                  r.L * c + r.N * s, -r.L * s + r.N * c)
        elif k == _abi.CS_ROT_Z:  # real_rays.py:124-130
            c, s = p[0], p[1]
            r.x, r.y, r.L, r.M = (r.x * c - r.y * s, r.x * s + r.y * c,
                                  r.L * c - r.M * s, r.L * s + r.M * c)
        else:
            raise ValueError(f"bad cs op {k}")


# --------------------------------------------------------------------------------------
# geometries
# --------------------------------------------------------------------------------------
def distance_plane(r: Rays):
    with warnings.catch_warnings():  # plane.py:73-75
        warnings.simplefilter("ignore")
        return -r.z / r.N


def distance_conic(r: Rays, R, k, radius_inf):
    """standard.py:89-140."""
    if radius_inf:
        N_safe = np.where(np.abs(r.N) > 1e-14, r.N, 1e-14)
        return -r.z / N_safe
    a = k * r.N**2 + r.L**2 + r.M**2 + r.N**2
    b = 2 * k * r.N * r.z + 2 * r.L * r.x + 2 * r.M * r.y - 2 * r.N * R + 2 * r.N * r.z
    c = k * r.z**2 - 2 * R * r.z + r.x**2 + r.y**2 + r.z**2
    d = b**2 - 4 * a * c
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        t1 = (-b + np.sqrt(d)) / (2 * a)
        t2 = (-b - np.sqrt(d)) / (2 * a)
        z1 = r.z + t1 * r.N
        z2 = r.z + t2 * r.N
        t = np.where(np.abs(z1) <= np.abs(z2), t1, t2)
        t = np.where(a == 0, -c / b, t)
    return t


def normal_conic(x, y, R, k):
    """standard.py:154-167."""
    r2 = x**2 + y**2
    denom = R * np.sqrt(1 - (1 + k) * r2 / R**2)
    dfdx = x / denom
    dfdy = y / denom
    dfdz = -1
    mag = np.sqrt(dfdx**2 + dfdy**2 + dfdz**2)
    return dfdx / mag, dfdy / mag, dfdz / mag


def sag_even(x, y, R, k, C):
    """even_asphere.py:82-98."""
    r2 = x**2 + y**2
    z = r2 / (R * (1 + np.sqrt(1 - (1 + k) * r2 / R**2)))
    for i, Ci in enumerate(C):
        z = z + Ci * r2 ** (i + 1)
    return z


def normal_even(x, y, R, k, C):
    """even_asphere.py:100-129."""
    r2 = x**2 + y**2
    denom = R * np.sqrt(1 - (1 + k) * r2 / R**2)
    dfdx = x / denom
    dfdy = y / denom
    for i, Ci in enumerate(C):
        dfdx = dfdx + 2 * (i + 1) * x * Ci * r2**i
        dfdy = dfdy + 2 * (i + 1) * y * Ci * r2**i
    mag = np.sqrt(dfdx**2 + dfdy**2 + 1)
    return dfdx / mag, dfdy / mag, -1 / mag


def sag_odd(x, y, R, k, C):
    """odd_asphere.py:73-89."""
    r2 = np.array(x**2 + y**2)
    r = np.sqrt(r2)
    z = r2 / (R * (1 + np.sqrt(1 - (1 + k) * r2 / R**2)))
    for i, Ci in enumerate(C):
        z = z + Ci * r ** (i + 1)
    return z


def normal_odd(x, y, R, k, C):
    """odd_asphere.py:91-130 (non-finite per-term slopes zeroed)."""
    r2 = x**2 + y**2
    r = np.sqrt(r2)
    denom = R * np.sqrt(1 - (1 + k) * r2 / R**2)
    dfdx = x / denom
    dfdy = y / denom
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        for i, Ci in enumerate(C):
            x_term = (i + 1) * x * Ci * r ** (i - 1)
            y_term = (i + 1) * y * Ci * r ** (i - 1)
            x_term[~np.isfinite(x_term)] = 0
            y_term[~np.isfinite(y_term)] = 0
            dfdx = dfdx + x_term
            dfdy = dfdy + y_term
    mag = np.sqrt(dfdx**2 + dfdy**2 + 1)
    return dfdx / mag, dfdy / mag, -1 / mag


def _radial(coef, term, r):
    """zernike/base.py:228-253: sum_k a_k r^(n-2k), a_k precomputed on the host."""
    n = int(term["n"])
    off, nr = int(term["rad_off"]), int(term["n_rad"])
    value = np.zeros_like(r)
    for kk in range(nr):
        value = value + coef[off + kk] * (r ** np.array(n - 2 * kk))
    return value


def _radial_derivative(coef, term, r):
    """zernike/base.py:272-299: sum_k d_k r^(n-2k-1) (d_k has (-1)^k (n-k)!/.. * (n-2k))."""
    n = int(term["n"])
    off, nr = int(term["rad_off"]), int(term["n_rad"])
    value = np.zeros_like(r)
    for kk in range(nr):
        if n - 2 * kk < 0:
            continue
        power_term = r ** np.array(n - 2 * kk - 1) if (n - 2 * kk - 1) >= 0 else 0
        value = value + coef[off + nr + kk] * power_term
    return value


def sag_zernike(x, y, R, k, terms, coef, norm_radius):
    """zernike.py:133-161 (standard/noll/fringe differ only in (n,m) order and norm)."""
    x_norm = x / norm_radius
    y_norm = y / norm_radius
    if np.any(np.abs(x_norm) > 1) or np.any(np.abs(y_norm) > 1):  # zernike.py:234-246
        raise ZernikeRangeError(
            "Zernike coordinates must be normalized to [-1, 1]. Consider updating the "
            "normalization radius to 1.1x the surface aperture."
        )
    rho = np.sqrt(x_norm**2 + y_norm**2)
    phi = np.arctan2(y_norm, x_norm)
    r2 = x**2 + y**2
    z = r2 / (R * (1 + np.sqrt(1 - (1 + k) * r2 / R**2)))
    # BaseZernike.poly: python sum() of terms, starting at int 0 (base.py:87-101)
    total = 0
    for t in terms:
        m = int(t["m"])
        az = np.cos(np.array(m) * phi) if m >= 0 else np.sin(np.abs(np.array(m)) * phi)
        total = total + float(t["c"]) * float(t["norm"]) * _radial(coef, t, rho) * az
    z += total
    return z


def normal_zernike(x, y, R, k, terms, coef, norm_radius):
    """zernike.py:163-231 (the normal omits the normalisation constant: reference quirk)."""
    r2 = x**2 + y**2
    denominator = R * np.sqrt(1 - (1 + k) * r2 / R**2)
    dzdx = x / denominator
    dzdy = y / denominator
    eps = 1e-14
    x_norm = x / norm_radius
    y_norm = y / norm_radius
    rho = np.sqrt(x_norm**2 + y_norm**2)
    phi = np.arctan2(y_norm, x_norm)
    if np.all(rho == 0):
        drho_dx = np.zeros_like(x)
        drho_dy = np.zeros_like(y)
    else:
        drho_dx = (x / (norm_radius**2)) / (rho + eps)
        drho_dy = (y / (norm_radius**2)) / (rho + eps)
    dphi_dx = -(y_norm) / (rho**2 + eps) * (1.0 / norm_radius)
    dphi_dy = +(x_norm) / (rho**2 + eps) * (1.0 / norm_radius)
    for t in terms:
        c = float(t["c"])
        if c == 0:
            continue
        m = int(t["m"])
        rt = _radial(coef, t, rho)
        rd = _radial_derivative(coef, t, rho)
        if m == 0:  # base.py:128-137
            dr, dphi = rd, 0.0
        elif m > 0:
            dr = rd * np.cos(m * phi)
            dphi = -m * rt * np.sin(m * phi)
        else:
            dr = rd * np.sin(abs(m) * phi)
            dphi = abs(m) * rt * np.cos(abs(m) * phi)
        dzdx += c * (dr * drho_dx + dphi * dphi_dx)
        dzdy += c * (dr * drho_dy + dphi * dphi_dy)
    nx = +dzdx
    ny = +dzdy
    norm = np.sqrt(nx**2 + ny**2 + 1)
    norm = np.where(norm < eps, 1.0, norm)
    return nx / norm, ny / norm, -np.ones_like(x) / norm


# ---- freeform Newton geometries ------------------------------------------------------
def sag_poly(x, y, R, k, C):
    """polynomial.py:93-108 (C: 2-D, be.atleast_2d)."""
    r2 = x**2 + y**2
    z = r2 / (R * (1 + np.sqrt(1 - (1 + k) * r2 / R**2)))
    for i in range(len(C)):
        for j in range(len(C[i])):
            z = z + C[i][j] * (x**i) * (y**j)
    return z


def normal_poly(x, y, R, k, C):
    """polynomial.py:111-140."""
    r2 = x**2 + y**2
    denom = R * np.sqrt(1 - (1 + k) * r2 / R**2)
    dzdx = x / denom
    dzdy = y / denom
    for i in range(1, len(C)):
        for j in range(len(C[i])):
            dzdx = dzdx + i * C[i][j] * (x ** (i - 1)) * (y**j)
    for i in range(len(C)):
        for j in range(1, len(C[i])):
            dzdy = dzdy + j * C[i][j] * (x**i) * (y ** (j - 1))
    norm = np.sqrt(dzdx**2 + dzdy**2 + 1)
    return dzdx / norm, dzdy / norm, -1 / norm


class ChebyshevRangeError(ValueError):
    pass


def _cheb_validate(xn, yn):
    """chebyshev.py:203-215."""
    if np.any(np.abs(xn) > 1) or np.any(np.abs(yn) > 1):
        raise ChebyshevRangeError("Chebyshev input coordinates must be normalized to [-1, 1]. "
                                  "Consider updating the normalization factors.")


def _cheb(n, x):
    return np.cos(n * np.arccos(x))  # chebyshev.py:176-188


def _cheb_d(n, x):
    return n * np.sin(n * np.arccos(x)) / np.sqrt(1 - x**2)  # chebyshev.py:190-201


def sag_cheb(x, y, R, k, C, norm_x, norm_y):
    """chebyshev.py:104-129."""
    xn = x / norm_x
    yn = y / norm_y
    _cheb_validate(xn, yn)
    r2 = x**2 + y**2
    z = r2 / (R * (1 + np.sqrt(1 - (1 + k) * r2 / R**2)))
    for i, j in np.argwhere(C != 0):
        z = z + C[i, j] * _cheb(i, xn) * _cheb(j, yn)
    return z


def normal_cheb(x, y, R, k, C, norm_x, norm_y):
    """chebyshev.py:131-174."""
    xn = x / norm_x
    yn = y / norm_y
    _cheb_validate(xn, yn)
    r2 = x**2 + y**2
    denom = R * np.sqrt(1 - (1 + k) * r2 / R**2)
    dzdx = x / denom
    dzdy = y / denom
    for i, j in np.argwhere(C != 0):
        dzdx = dzdx + (_cheb_d(i, xn) * C[i, j] * _cheb(j, yn))
        dzdy = dzdy + (_cheb_d(j, yn) * C[i, j] * _cheb(i, xn))
    norm = np.sqrt(dzdx**2 + dzdy**2 + 1)
    return dzdx / norm, dzdy / norm, -1 / norm


def sag_biconic(x, y, cx, cy, kx, ky):
    """biconic.py:69-103 (cx, cy, kx, ky as the reference's 0-d arrays)."""
    zx = np.zeros_like(x)
    zy = np.zeros_like(y)
    if not np.all(cx == 0):
        v = 1.0 - (1.0 + kx) * cx**2 * x**2
        st = np.where(v < 1e-14, 0.0, v)
        den = 1.0 + np.sqrt(st)
        zx = (cx * x**2) / np.where(np.abs(den) < 1e-14, 1e-14, den)
    if not np.all(cy == 0):
        v = 1.0 - (1.0 + ky) * cy**2 * y**2
        st = np.where(v < 1e-14, 0.0, v)
        den = 1.0 + np.sqrt(st)
        zy = (cy * y**2) / np.where(np.abs(den) < 1e-14, 1e-14, den)
    return zx + zy


def normal_biconic(x, y, cx, cy, kx, ky):
    """biconic.py:105-158."""
    if np.all(cx == 0):
        dfdx = np.zeros_like(x)
    else:
        v = 1.0 - (1.0 + kx) * cx**2 * x**2
        ds = np.sqrt(np.where(v < 1e-14, 1e-14, v))
        dfdx = (cx * x) / np.where(np.abs(ds) < 1e-14, 1e-14, ds)
    if np.all(cy == 0):
        dfdy = np.zeros_like(y)
    else:
        v = 1.0 - (1.0 + ky) * cy**2 * y**2
        ds = np.sqrt(np.where(v < 1e-14, 1e-14, v))
        dfdy = (cy * y) / np.where(np.abs(ds) < 1e-14, 1e-14, ds)
    mag = np.sqrt(dfdx**2 + dfdy**2 + 1.0)
    smag = np.where(mag < 1e-14, 1.0, mag)
    return dfdx / smag, dfdy / smag, -1.0 / smag


def _toroid_zy(y, R_yz, c, k, poly):
    """toroidal.py:75-107 (_calculate_zy)."""
    y2 = y**2
    z_y = np.zeros_like(y)
    if np.isfinite(R_yz) and R_yz != 0:
        v = 1.0 - (1.0 + k) * c**2 * y2
        root = np.where(v < 0, 0.0, v)
        den = 1.0 + np.sqrt(root)
        z_y = (c * y2) / np.where(np.abs(den) < 1e-14, 1e-14, den)
    if len(poly) > 0:
        p = np.zeros_like(y)
        cur = y2
        for a in poly:
            p = p + a * cur
            cur = cur * y2
        z_y = z_y + p
    return z_y


def _toroid_dzy(y, R_yz, c, k, poly):
    """toroidal.py:109-141 (_calculate_zy_derivative)."""
    y2 = y**2
    d = np.zeros_like(y)
    if np.isfinite(R_yz) and R_yz != 0:
        v = 1.0 - (1.0 + k) * c**2 * y2
        sq = np.sqrt(np.where(v < 1e-14, 1e-14, v))
        d = (c * y) / np.where(np.abs(sq) < 1e-14, 1e-14, sq)
    if len(poly) > 0:
        p = np.zeros_like(y)
        cur = y
        for i, a in enumerate(poly):
            p = p + a * (2.0 * (i + 1.0)) * cur
            cur = cur * y2
        d = d + p
    return d


def sag_toroidal(x, y, R_rot, R_yz, c, k, poly):
    """toroidal.py:143-167."""
    z_y = _toroid_zy(y, R_yz, c, k, poly)
    if np.isinf(R_rot):
        return z_y
    term = (R_rot - z_y) ** 2 - x**2
    with np.errstate(invalid="ignore"):
        return np.where(term < 0, np.nan,
                        z_y + ((R_rot - z_y) - np.sign(R_rot - z_y) * np.sqrt(term)))


def normal_toroidal(x, y, R_rot, R_yz, c, k, poly):
    """toroidal.py:169-233."""
    eps = 1e-14
    z_y = _toroid_zy(y, R_yz, c, k, poly)
    dz_dy = _toroid_dzy(y, R_yz, c, k, poly)
    if np.isinf(R_rot):
        fx = np.zeros_like(x)
        fy = dz_dy
        term = np.inf
    else:
        term = (R_rot - z_y) ** 2 - x**2
        valid = term >= 0
        sq = np.sqrt(np.where(valid, term, eps))
        ssq = np.where(np.abs(sq) < eps, eps, sq)
        fx = np.where(valid, np.sign(R_rot) * x / ssq, 0.0)
        fy = np.where(valid, np.sign(R_rot) * (R_rot - z_y) * dz_dy / ssq, 0.0)
    mag = np.sqrt(fx**2 + fy**2 + 1.0)
    smag = np.where(mag < eps, 1.0, mag)
    nx, ny, nz = fx / smag, fy / smag, -1.0 / smag
    return (np.where(term >= 0, nx, 0.0), np.where(term >= 0, ny, 0.0),
            np.where(term >= 0, nz, -1.0))


# ---- Forbes Q-bfs / Q-2D (forbes/geometry.py:83-640, forbes/qpoly.py) -----------------
# The lens-only tables (orthonormal-basis coefficients, recurrence A/B/C, vertex slope)
# are read from the lowered coefficient block (layout: include/optiland_rt.h); the
# per-ray recurrences below follow qpoly.py's NumPy path operation by operation.
_FEPS = 1e-12


def _forbes_base_sag(r2, R, k):
    """forbes/geometry.py:115-131."""
    if np.isinf(R):
        return np.zeros_like(r2)
    a = 1 - (1 + k) * r2 / R**2
    return r2 / (R * (1 + np.sqrt(np.where(a < 0, 0, a))))


def _forbes_base_dsag(rho, r2, R, k):
    """forbes/geometry.py:133-150."""
    if np.isinf(R) or R == 0:
        return np.zeros_like(rho)
    c = 1.0 / R
    a = 1 - (k + 1) * c**2 * r2
    return c * rho / np.sqrt(np.where(a > 0, a, 1e-12))


def _forbes_conic(r2, R, k):
    """forbes/geometry.py:152-180."""
    if np.isinf(R):
        return 1.0, 0.0
    c2 = (1.0 / R) ** 2
    rho = np.sqrt(r2)
    na = 1 - k * c2 * r2
    da = 1 - (k + 1) * c2 * r2
    Nn = np.sqrt(np.where(na > 0, na, 1e-12))
    Dd = np.sqrt(np.where(da > 0, da, 1e-12))
    return Nn / Dd, (c2 * rho) / (Nn * Dd**3)


def _qbfs_alphas(b, usq, j):
    """qpoly.py:127-192: alphas[0] (sum recurrence) and, for j = 1, alphas[1]."""
    m = len(b) - 1
    al = np.zeros((j + 1, m + 1) + np.shape(usq))
    p = 2 - 4 * usq
    al[0][m] = b[m]
    if m > 0:
        al[0][m - 1] = b[m - 1] + p * al[0][m]
    for i in range(m - 2, -1, -1):
        al[0][i] = b[i] + p * al[0][i + 1] - al[0][i + 2]
    if j and m - 1 >= 0:
        al[1][m - 1] = -4 * al[0][m]
        if m - 2 >= 0:
            al[1][m - 2] = p * al[1][m - 1] - 4 * al[0][m - 1]
        for n in range(m - 3, -1, -1):
            al[1][n] = p * al[1][n + 1] - al[1][n + 2] - 4 * al[0][n + 1]
    return al


def _qbfs_sum(b, usq, j=0):
    """(S, dS/d usq): 2 (alpha_0 + alpha_1), or 2 alpha_0 for one term."""
    if len(b) == 0:
        z = np.zeros_like(usq)
        return z, z
    al = _qbfs_alphas(b, usq, j)
    if len(b) > 1:
        return 2 * (al[0][0] + al[0][1]), (2 * (al[1][0] + al[1][1]) if j else None)
    return 2 * al[0][0], (2 * al[1][0] if j else None)


def _q2d_records(B):
    """Parse the Q-2D block: (norm, vdx, vdy, b0, [(m, rec_a, rec_b), ...])."""
    nr, vdx, vdy, L0 = B[0], B[1], B[2], int(B[3])
    b0 = list(B[4:4 + L0])
    pos = 4 + L0
    M = int(B[pos])
    pos += 1
    orders = []
    for m in range(1, M + 1):
        recs = []
        for _ in range(2):
            L = int(B[pos])
            if L == 0:
                recs.append(None)
                pos += 1
                continue
            body = np.asarray(B[pos + 1:pos + 1 + 4 * L]).reshape(4, L)
            recs.append(body)
            pos += 1 + 4 * L
        orders.append((m, recs[0], recs[1]))
    return nr, vdx, vdy, b0, orders


def _q2d_order(rec, m, usq):
    """qpoly.py:415-466 (clenshaw_q2d + its j = 1 derivative) and :389-398
    (q2d_sum_from_alphas) for one azimuthal order: (S, dS/d usq)."""
    D, A, Bc, C = rec
    top = len(D) - 1
    al = np.zeros((2, top + 1) + np.shape(usq))
    al[0][top] = D[top]
    if top > 0:
        al[0][top - 1] = D[top - 1] + (A[top - 1] + Bc[top - 1] * usq) * al[0][top]
    for n in range(top - 2, -1, -1):
        al[0][n] = D[n] + (A[n] + Bc[n] * usq) * al[0][n + 1] - C[n + 1] * al[0][n + 2]
    if top - 1 >= 0:
        al[1][top - 1] = Bc[top - 1] * al[0][top]
        for n in range(top - 2, -1, -1):
            al[1][n] = (Bc[n] * al[0][n + 1] + (A[n] + Bc[n] * usq) * al[1][n + 1]
                        - C[n + 1] * al[1][n + 2])
    out = []
    for a in al:
        s = 0.5 * a[0]
        if m == 1 and top > 2:
            s -= 2 / 5 * a[3]
        out.append(s)
    return out


def _q2d_sums(B, u, t):
    """qpoly.py:469-520 compute_z_zprime_q2d."""
    nr, vdx, vdy, b0, orders = _q2d_records(B)
    usq = u * u
    z = np.zeros_like(u)
    p0, dp0 = z, z
    if b0:
        p0, d = _qbfs_sum(b0, usq, 1)
        dp0 = d * 2 * u
    pg, dr, dt = [], [], []
    for m, ra, rb in orders:
        sa = sb = dsa = dsb = 0
        if ra is not None:
            sa, dsa = _q2d_order(ra, m, usq)
        if rb is not None:
            sb, dsb = _q2d_order(rb, m, usq)
        um = u**m
        ct, st = np.cos(m * t), np.sin(m * t)
        pg.append(um * (ct * sa + st * sb))
        umm1 = u ** (m - 1) if m > 0 else np.ones_like(u)
        two = 2 * usq
        dr.append(umm1 * (ct * (two * dsa + m * sa) + st * (two * dsb + m * sb)))
        dt.append(m * um * (-sa * st + sb * ct))
    sm = (lambda v: np.sum(np.stack(v), axis=0) if v else z)
    return p0, dp0, sm(pg), sm(dr), sm(dt)


def sag_qbfs(x, y, R, k, B):
    """forbes/geometry.py:243-266."""
    nr, L = np.array(B[0]), int(B[1])
    b = list(B[3:3 + L])
    r2 = x**2 + y**2
    usq = r2 / (nr**2)
    ps = _qbfs_sum(b, usq)[0] if L else np.zeros_like(usq)
    cf, _ = _forbes_conic(r2, R, k)
    dep = usq * (1 - usq) * cf * ps
    return _forbes_base_sag(r2, R, k) + np.where(usq > 1, 0.0, dep)


def normal_qbfs(x, y, R, k, B):
    """forbes/geometry.py:268-327 (NumPy: the analytical branch)."""
    nr, L, dep = np.array(B[0]), int(B[1]), B[2] != 0.0
    b = list(B[3:3 + L])
    r2 = x**2 + y**2
    rho = np.sqrt(r2 + _FEPS)
    dfr = _forbes_base_dsag(rho, r2, R, k)
    if dep:
        u = rho / nr
        pv, pd = _qbfs_sum(b, u**2, 1)
        dpdu = pd * 2 * u
        dpre = (2 * u - 4 * u**3) / nr
        cf, dcf = _forbes_conic(r2, R, k)
        usq = u**2
        dd = (dpre * cf * pv + (usq - usq**2) * dcf * pv + (usq - usq**2) * cf * (dpdu / nr))
        dfr = dfr + np.where(u >= 1, 0.0, dd)
    dfx, dfy = dfr * (x / rho), dfr * (y / rho)
    mag = np.sqrt(dfx**2 + dfy**2 + 1)
    sm = np.where(mag < _FEPS, 1.0, mag)
    return dfx / sm, dfy / sm, -1 / sm


def sag_q2d(x, y, R, k, B):
    """forbes/geometry.py:420-450."""
    nr = np.array(B[0])
    r2 = x**2 + y**2
    rho = np.sqrt(r2 + _FEPS)
    u = rho / nr
    t = np.arctan2(y, np.where(rho < _FEPS, x + 1e-12, x))
    p0, _, pg, _, _ = _q2d_sums(B, u, t)
    cf, _ = _forbes_conic(r2, R, k)
    usq = u**2
    total = usq * (1 - usq) * cf * p0 + cf * pg
    return _forbes_base_sag(r2, R, k) + np.where(u > 1, 0.0, total)


def normal_q2d(x, y, R, k, B):
    """forbes/geometry.py:545-610 (NumPy: the analytical branch)."""
    nr, vdx, vdy = np.array(B[0]), B[1], B[2]
    r2 = x**2 + y**2
    rho = np.sqrt(r2)
    isv = rho < _FEPS
    rs = np.where(isv, _FEPS, rho)
    u = rho / nr
    t = np.arctan2(y, x)
    p0, dp0, pg, dr, dt = _q2d_sums(B, u, t)
    cf, dcf = _forbes_conic(r2, R, k)
    usq = u**2
    dpre = (2 * u - 4 * u**3) / nr
    ds0 = (dpre * p0 + (usq - usq**2) * (dp0 / nr)) * cf + (usq - usq**2) * p0 * dcf
    dsg = (dcf * pg) + (cf * (dr / nr))
    dsr = np.where(u > 1, 0.0, ds0 + dsg)
    dst = np.where(u > 1, 0.0, cf * dt)
    ct, st = x / rs, y / rs
    dsx = ct * dsr - (st / rs) * dst
    dsy = st * dsr + (ct / rs) * dst
    dbr = _forbes_base_dsag(rho, r2, R, k)
    dfx = np.where(isv, vdx, dbr * ct + dsx)
    dfy = np.where(isv, vdy, dbr * st + dsy)
    mag = np.sqrt(dfx**2 + dfy**2 + 1)
    sm = np.where(mag < _FEPS, 1.0, mag)
    return dfx / sm, dfy / sm, -1.0 / sm


def _grid(B):
    n, m = int(B[0]), int(B[1])
    xg = np.asarray(B[2:2 + n], dtype=np.float64)
    yg = np.asarray(B[2 + n:2 + n + m], dtype=np.float64)
    zg = np.asarray(B[2 + n + m:2 + n + m + n * m], dtype=np.float64).reshape(m, n)
    return xg, yg, zg


def grid_interpolate(B, x, y):
    """grid_sag.py:61-101 (bilinear sag, its derivatives, NaN outside the grid)."""
    xg, yg, zg = _grid(B)
    i = np.searchsorted(xg, x, side="right") - 1
    j = np.searchsorted(yg, y, side="right") - 1
    nan_mask = (x < xg[0]) | (x > xg[-1]) | (y < yg[0]) | (y > yg[-1])
    i = np.where(i < 0, 0, i)
    j = np.where(j < 0, 0, j)
    i = np.where(i >= len(xg) - 1, len(xg) - 2, i)
    j = np.where(j >= len(yg) - 1, len(yg) - 2, j)
    x1, x2 = xg[i], xg[i + 1]
    y1, y2 = yg[j], yg[j + 1]
    z11, z12 = zg[j, i], zg[j, i + 1]
    z21, z22 = zg[j + 1, i], zg[j + 1, i + 1]
    tx = (x - x1) / (x2 - x1)
    ty = (y - y1) / (y2 - y1)
    z_y1 = z11 * (1 - tx) + z12 * tx
    z_y2 = z21 * (1 - tx) + z22 * tx
    sag = z_y1 * (1 - ty) + z_y2 * ty
    ds_dx = ((z12 - z11) * (1 - ty) + (z22 - z21) * ty) / (x2 - x1)
    ds_dy = ((z21 - z11) * (1 - tx) + (z22 - z12) * tx) / (y2 - y1)
    return np.where(nan_mask, np.nan, sag), ds_dx, ds_dy


def normal_grid(B, x, y):
    """grid_sag.py:142-149."""
    _, ds_dx, ds_dy = grid_interpolate(B, x, y)
    nx, ny, nz = -ds_dx, -ds_dy, np.ones_like(x)
    mag = np.sqrt(nx**2 + ny**2 + nz**2)
    return nx / mag, ny / mag, nz / mag


def distance_grid(r: Rays, B, tol, max_iter, sched=None):
    """grid_sag.py:108-140: Newton from t = 0, global stop max|dt| < tol checked after
    each update, rays off the grid -> NaN. Returns (t, updates)."""
    xg, yg, _ = _grid(B)
    t = np.zeros_like(r.x)
    updates = 0
    for _ in range(max_iter):
        if sched is not None and updates >= sched:
            break
        x_i = r.x + t * r.L
        y_i = r.y + t * r.M
        z_i = r.z + t * r.N
        sag, ds_dx, ds_dy = grid_interpolate(B, x_i, y_i)
        f = sag - z_i
        f_prime = ds_dx * r.L + ds_dy * r.M - r.N
        dt = -f / f_prime
        t = t + dt
        updates += 1
        if sched is None and np.max(np.abs(dt)) < tol:
            break
    x_f = r.x + t * r.L
    y_f = r.y + t * r.M
    oob = (x_f < xg[0]) | (x_f > xg[-1]) | (y_f < yg[0]) | (y_f > yg[-1])
    return np.where(oob, np.nan, t), updates


def _geometry_fns(table, s):
    g = int(s["geometry"])
    R, k = float(s["radius"]), float(s["conic"])
    off, nc = int(s["coef_off"]), int(s["n_coef"])
    if g == _abi.GEOM_EVEN_ASPHERE:
        C = [float(c) for c in table.coef[off:off + nc]]
        return (lambda x, y: sag_even(x, y, R, k, C)), (lambda x, y: normal_even(x, y, R, k, C))
    if g == _abi.GEOM_ODD_ASPHERE:
        C = [float(c) for c in table.coef[off:off + nc]]
        return (lambda x, y: sag_odd(x, y, R, k, C)), (lambda x, y: normal_odd(x, y, R, k, C))
    if g == _abi.GEOM_ZERNIKE:
        terms = table.zern[off:off + nc]
        nr = float(s["norm_radius"])
        return ((lambda x, y: sag_zernike(x, y, R, k, terms, table.coef, nr)),
                (lambda x, y: normal_zernike(x, y, R, k, terms, table.coef, nr)))
    B = [float(c) for c in table.coef[off:off + nc]]
    if g == _abi.GEOM_POLYNOMIAL:
        ni, nj = int(B[0]), int(B[1])
        C = np.array(B[2:2 + ni * nj]).reshape(ni, nj)
        return (lambda x, y: sag_poly(x, y, R, k, C)), (lambda x, y: normal_poly(x, y, R, k, C))
    if g == _abi.GEOM_CHEBYSHEV:
        ni, nj = int(B[0]), int(B[1])
        nx_, ny_ = np.array(B[2]), np.array(B[3])
        C = np.array(B[4:4 + ni * nj]).reshape(ni, nj)
        return ((lambda x, y: sag_cheb(x, y, R, k, C, nx_, ny_)),
                (lambda x, y: normal_cheb(x, y, R, k, C, nx_, ny_)))
    if g == _abi.GEOM_BICONIC:
        cx, cy, kx, ky = (np.array(v) for v in B[:4])
        return ((lambda x, y: sag_biconic(x, y, cx, cy, kx, ky)),
                (lambda x, y: normal_biconic(x, y, cx, cy, kx, ky)))
    if g == _abi.GEOM_TOROIDAL:
        R_rot, c_yz, k_yz, has_yz, n_poly = B[:5]
        poly = np.asarray(B[5:5 + int(n_poly)])
        R_rot = np.array(R_rot)
        # the reference keeps R_yz itself; only its finiteness / non-zero test matters here
        R_yz = np.array(1.0 if has_yz else np.inf)
        c = np.float64(c_yz)
        k_ = np.array(k_yz)
        return ((lambda x, y: sag_toroidal(x, y, R_rot, R_yz, c, k_, poly)),
                (lambda x, y: normal_toroidal(x, y, R_rot, R_yz, c, k_, poly)))
    if g == _abi.GEOM_GRID_SAG:
        return ((lambda x, y: grid_interpolate(B, x, y)[0]),
                (lambda x, y: normal_grid(B, x, y)))
    if g == _abi.GEOM_NURBS:  # nurbs_geometry.py:696-822 (oracle/nurbs_np.py)
        blk = nurbs_np.unpack(B)
        tol, max_iter = float(s["tol"]), int(s["max_iter"])
        return ((lambda x, y: nurbs_np.sag(blk, x, y, tol, max_iter)),
                (lambda x, y: nurbs_np.surface_normal(blk, x, y, tol, max_iter)))
    if g in (_abi.GEOM_FORBES_QBFS, _abi.GEOM_FORBES_Q2D):
        Rf, kf = np.array(R), np.array(k)
        sag_f, nrm_f = ((sag_qbfs, normal_qbfs) if g == _abi.GEOM_FORBES_QBFS
                        else (sag_q2d, normal_q2d))
        return (lambda x, y: sag_f(x, y, Rf, kf, B)), (lambda x, y: nrm_f(x, y, Rf, kf, B))
    raise ValueError(g)


def distance_newton(r: Rays, table, s, sched=None):
    """newton_raphson.py:119-168. Returns (t, updates). The stop test is GLOBAL over all
    rays of this trace call: max(|f|) < tol (NaN never passes). If sched is given,
    exactly that many updates are made instead."""
    if int(s["geometry"]) == _abi.GEOM_NURBS:  # its own (u, v) solve, no update count
        off, nc = int(s["coef_off"]), int(s["n_coef"])
        blk = nurbs_np.unpack(table.coef[off:off + nc])
        return nurbs_np.distance(blk, r.x, r.y, r.z, r.L, r.M, r.N, float(s["tol"]),
                                 int(s["max_iter"])), -1
    if int(s["geometry"]) == _abi.GEOM_GRID_SAG:
        off, nc = int(s["coef_off"]), int(s["n_coef"])
        with np.errstate(invalid="ignore", divide="ignore"):
            return distance_grid(r, table.coef[off:off + nc], float(s["tol"]),
                                 int(s["max_iter"]), sched)
    sag, normal = _geometry_fns(table, s)
    t = distance_conic(r, float(s["radius"]), float(s["conic"]),
                       bool(int(s["flags"]) & _abi.SURF_RADIUS_INF))
    tol, max_iter = float(s["tol"]), int(s["max_iter"])
    updates = 0
    for it in range(max_iter):
        if sched is not None and it >= sched:
            break
        x_int = r.x + t * r.L
        y_int = r.y + t * r.M
        z_int = r.z + t * r.N
        f_t = sag(x_int, y_int) - z_int
        if sched is None and np.max(np.abs(f_t)) < tol:
            break
        nx, ny, nz = normal(x_int, y_int)
        nz_safe = np.where(np.abs(nz) > 1e-14, nz, 1e-14)
        fx = -nx / nz_safe
        fy = -ny / nz_safe
        df_dt = fx * r.L + fy * r.M - r.N
        safe_df_dt = np.where(np.abs(df_dt) > 1e-14, df_dt, 1e-14)
        t = t - f_t / safe_df_dt
        updates += 1
    return t, updates


def sag_surface(x, y, table, s):
    """Geometry.sag(x, y): plane.py:45-59 (0), standard.py:73-87 (conic), Newton kinds
    through their own sag (even_asphere.py:82-98, odd_asphere.py:73-89, zernike.py:133-161)."""
    g = int(s["geometry"])
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if g == _abi.GEOM_PLANE:
        return np.zeros_like(y)
    if g == _abi.GEOM_STANDARD:
        R, k = float(s["radius"]), float(s["conic"])
        r2 = x**2 + y**2
        with np.errstate(invalid="ignore", divide="ignore"):
            return r2 / (R * (1 + np.sqrt(1 - (1 + k) * r2 / R**2)))
    with np.errstate(invalid="ignore", divide="ignore"):
        return _geometry_fns(table, s)[0](x, y)


def surface_normal(r: Rays, table, s):
    g = int(s["geometry"])
    if g == _abi.GEOM_PLANE:  # plane.py:79-98
        return np.zeros_like(r.x), np.zeros_like(r.x), np.ones_like(r.x)
    if g == _abi.GEOM_STANDARD:
        return normal_conic(r.x, r.y, float(s["radius"]), float(s["conic"]))
    return _geometry_fns(table, s)[1](r.x, r.y)


# --------------------------------------------------------------------------------------
# propagation / interaction
# --------------------------------------------------------------------------------------
def propagate(r: Rays, t, alpha):
    """homogeneous.py:30-57; alpha = 4*pi*k/w precomputed (k>0 <=> alpha>0)."""
    r.x = r.x + t * r.L
    r.y = r.y + t * r.M
    r.z = r.z + t * r.N
    if alpha > 0:
        r.i = r.i * np.exp(-alpha * t * 1e3)


def propagate_w(r: Rays, t, k, w):
    """homogeneous.py:30-57 with per-ray k(w) and w: absorption when any k > 0."""
    r.x = r.x + t * r.L
    r.y = r.y + t * r.M
    r.z = r.z + t * r.N
    if np.any(k > 0):
        alpha = 4 * np.pi * k / w
        r.i = r.i * np.exp(-alpha * t * 1e3)


# -- per-ray dispersion (materials/material_file.py:219-428 on the lowered ort_material
#    records: wavelength-independent subexpressions were formed by the host lowering) --
def material_n(table, mi, w):
    m = table.mat_table[mi]
    kind, nc, off = int(m["kind"]), int(m["n_coef"]), int(m["coef_off"])
    c = table.coef[off:off + (2 * nc if kind == _abi.MAT_TABULATED else nc)]
    if kind == _abi.MAT_IDEAL:  # ideal.py: constant n
        return np.full_like(w, float(m["n_const"]))
    if kind == _abi.MAT_TABULATED:  # :422-428
        return np.interp(w, c[:nc], c[nc:])
    if kind in (1, 2):  # Sellmeier (C ** 2 pre-formed) / Sellmeier-2
        n = c[0]
        for k in range(1, len(c), 2):
            n = n + c[k] * w**2 / (w**2 - c[k + 1])
        return np.sqrt(n)
    if kind in (3, 5):  # polynomial / Cauchy
        n = c[0]
        for k in range(1, len(c), 2):
            n = n + c[k] * w ** c[k + 1]
        return np.sqrt(n) if kind == 3 else n
    if kind == 4:
        n = c[0] + c[1] * w ** c[2] / (w**2 - c[3]) + c[4] * w ** c[5] / (w**2 - c[6])
        for k in range(7, len(c), 2):
            n = n + c[k] * w ** c[k + 1]
        return np.sqrt(n)
    if kind == 6:
        n = c[0]
        for k in range(1, len(c), 2):
            n = n + c[k] / (c[k + 1] - w**-2)
        return n
    if kind == 7:
        n = c[0] + c[1] / (w**2 - 0.028) + c[2] * (1 / (w**2 - 0.028)) ** 2
        for k in range(3, len(c)):
            n = n + c[k] * w ** (2 * (k - 2))
        return n
    if kind == 8:
        b = c[0] + c[1] * w**2 / (w**2 - c[2]) + c[3] * w**2
        return np.sqrt((1 + 2 * b) / (1 - b))
    if kind == 9:
        n = c[0] + c[1] / (w**2 - c[2]) + c[3] * (w - c[4]) / ((w - c[4]) ** 2 + c[5])
        return np.sqrt(n)
    if kind == _abi.MAT_ABBE:  # abbe.py:37-51
        if np.any(w < 0.380) or np.any(w > 0.750):
            raise ValueError("Wavelength out of range for this model.")
        return np.atleast_1d(np.polyval(c, w))
    raise ValueError(kind)


def material_k(table, mi, w):
    m = table.mat_table[mi]
    kl, ko = int(m["k_len"]), int(m["k_off"])
    if kl == 0:
        return np.full_like(w, float(m["k_const"]))
    return np.interp(w, table.coef[ko:ko + kl], table.coef[ko + kl:ko + 2 * kl])


def _align(r: Rays, nx, ny, nz):
    """real_rays.py:511-547."""
    dot = r.L * nx + r.M * ny + r.N * nz
    sgn = np.sign(dot)
    return nx * sgn, ny * sgn, nz * sgn, np.abs(dot)


def refract(r: Rays, nx, ny, nz, n1, n2):
    """real_rays.py:141-163."""
    u = n1 / n2
    nx, ny, nz, dot = _align(r, nx, ny, nz)
    with np.errstate(invalid="ignore"):
        root = np.sqrt(1 - u**2 * (1 - dot**2))
    L0, M0, N0 = r.L, r.M, r.N
    r.L = u * L0 + nx * root - u * nx * dot
    r.M = u * M0 + ny * root - u * ny * dot
    r.N = u * N0 + nz * root - u * nz * dot


def reflect(r: Rays, nx, ny, nz):
    """real_rays.py:165-181."""
    nx, ny, nz, dot = _align(r, nx, ny, nz)
    r.L = r.L - 2 * dot * nx
    r.M = r.M - 2 * dot * ny
    r.N = r.N - 2 * dot * nz


def normalize(r: Rays):
    """real_rays.py:503-509."""
    mag = np.sqrt(r.L**2 + r.M**2 + r.N**2)
    r.L, r.M, r.N = r.L / mag, r.M / mag, r.N / mag


def thin_lens(r: Rays, f, n1, n2):
    """thin_lens_interaction_model.py:69-111 (f: 0-d array as in the reference)."""
    f = np.asarray(f)
    r.opd = r.opd - (r.x**2 + r.y**2) / (2 * f)
    ux1 = r.L / r.N
    uy1 = r.M / r.N
    ux2 = 1 / n2 * (n1 * ux1 - r.x / f)
    uy2 = 1 / n2 * (n1 * uy1 - r.y / f)
    r.L, r.M, r.N = ux2, uy2, np.ones_like(ux2)


def _phase_profile(blk, x, y):
    """phase/constant.py, linear_grating.py:60-92, radial.py:26-75 -> phase, grad x, y."""
    kind = int(blk[0])
    if kind == _abi.PHASE_CONSTANT:
        return np.full_like(x, blk[2]), np.zeros_like(x), np.zeros_like(y)
    if kind == _abi.PHASE_LINEAR:
        kx, ky = float(blk[2]), float(blk[3])
        return kx * x + ky * y, np.full_like(x, kx), np.full_like(y, ky)
    coeffs = [float(c) for c in blk[3:3 + int(blk[2])]]
    r_squared = x**2 + y**2
    phase = np.zeros_like(x)
    for i, coeff in enumerate(coeffs):
        power = i + 1
        phase = phase + coeff * (r_squared**power)
    r = np.sqrt(r_squared)
    d_phi_dr = np.zeros_like(r)
    for i, coeff in enumerate(coeffs):
        power = i + 1
        d_phi_dr = d_phi_dr + coeff * 2 * power * (r ** (2 * power - 1))
    safe_r = np.where(r == 0, 1.0, r)
    dx = np.where(r == 0, 0.0, (d_phi_dr / safe_r) * x)
    dy = np.where(r == 0, 0.0, (d_phi_dr / safe_r) * y)
    return phase, dx, dy


def phase_interact(r: Rays, blk, nx, ny, nz, n1, n2, reflective, w):
    """phase_interaction_model.py:45-132."""
    if reflective:
        n2 = n1
    k0 = 2 * np.pi / w
    k_ix, k_iy, k_iz = n1 * k0 * r.L, n1 * k0 * r.M, n1 * k0 * r.N
    phase_val, gx, gy = _phase_profile(blk, r.x, r.y)
    gz = np.zeros_like(r.x)
    gdn = gx * nx + gy * ny + gz * nz
    Gx, Gy, Gz = gx - gdn * nx, gy - gdn * ny, gz - gdn * nz
    kdn = k_ix * nx + k_iy * ny + k_iz * nz
    kpx, kpy, kpz = k_ix - kdn * nx, k_iy - kdn * ny, k_iz - kdn * nz
    kox, koy, koz = kpx + Gx, kpy + Gy, kpz + Gz
    par2 = kox**2 + koy**2 + koz**2
    R_sq = (n2 * k0) ** 2 - par2
    r.i = np.where(R_sq < 0.0, np.zeros_like(r.i), r.i)
    R_sq = np.maximum(0.0, R_sq)
    alpha = (-1.0 if reflective else 1.0) * np.sqrt(R_sq)
    kx, ky, kz = kox + alpha * nx, koy + alpha * ny, koz + alpha * nz
    mag = np.sqrt(kx**2 + ky**2 + kz**2)
    r.L, r.M, r.N = kx / mag, ky / mag, kz / mag
    r.opd = r.opd + -phase_val / k0
    r.i = r.i * float(blk[1])


def grating_vector(blk, x, y, nx, ny, nz):
    """plane_grating.py:105-124 / standard_grating.py:93-146, 224-247 (the scalars tan,
    R**2, R**3, k + 1 formed by the lowering as the reference forms them)."""
    if float(blk[2]) == 0.0:
        ones = np.ones_like(x)
        return float(blk[3]) * ones, float(blk[4]) * ones, np.zeros_like(x)
    ta, R2, R3, kp1 = (float(v) for v in blk[3:7])
    s = np.sqrt((R2 - kp1 * (x**2 + y**2)) / R2)
    dzdx = (x + y * ta) * (2 * R2 * s * (s + 1) + kp1 * (x**2 + y**2)) / (R3 * s * (s + 1) ** 2)
    tx, ty, tz = np.ones_like(dzdx), np.ones_like(dzdx) * ta, dzdx
    nt = np.sqrt(tx**2 + ty**2 + tz**2)
    tx, ty, tz = tx / nt, ty / nt, tz / nt
    fx = ny * tz - nz * ty
    fy = -nx * tz + nz * tx
    fz = nx * ty - ny * tx
    mag = np.sqrt(fx**2 + fy**2 + fz**2)
    return -(fx / mag), -(fy / mag), -(fz / mag)


def diffract(r: Rays, blk, nx, ny, nz, n1, n2, reflective, w):
    """diffractive_model.py:37-56 + real_rays.py:183-498 (gratingdiffract)."""
    fx, fy, fz = grating_vector(blk, r.x, r.y, nx, ny, nz)
    m = float(blk[0])
    d = float(blk[1]) / np.sqrt(fx**2 + fy**2)
    L0, M0, N0 = r.L, r.M, r.N
    nx, ny, nz, _ = _align(r, nx, ny, nz)
    n2c = n2 * (-1 if reflective else 1)
    D = (-(L0**2) * d**2 * n1**2 * ny**2 - L0**2 * d**2 * n1**2 * nz**2
         + 2 * L0 * M0 * d**2 * n1**2 * nx * ny + 2 * L0 * N0 * d**2 * n1**2 * nx * nz
         - 2 * L0 * d * fx * m * n1 * ny**2 * w - 2 * L0 * d * fx * m * n1 * nz**2 * w
         + 2 * L0 * d * fy * m * n1 * nx * ny * w + 2 * L0 * d * fz * m * n1 * nx * nz * w
         - M0**2 * d**2 * n1**2 * nx**2 - M0**2 * d**2 * n1**2 * nz**2
         + 2 * M0 * N0 * d**2 * n1**2 * ny * nz + 2 * M0 * d * fx * m * n1 * nx * ny * w
         - 2 * M0 * d * fy * m * n1 * nx**2 * w - 2 * M0 * d * fy * m * n1 * nz**2 * w
         + 2 * M0 * d * fz * m * n1 * ny * nz * w
         - N0**2 * d**2 * n1**2 * nx**2 - N0**2 * d**2 * n1**2 * ny**2
         + 2 * N0 * d * fx * m * n1 * nx * nz * w + 2 * N0 * d * fy * m * n1 * ny * nz * w
         - 2 * N0 * d * fz * m * n1 * nx**2 * w - 2 * N0 * d * fz * m * n1 * ny**2 * w
         + d**2 * n2c**2 * nx**2 + d**2 * n2c**2 * ny**2 + d**2 * n2c**2 * nz**2
         - fx**2 * m**2 * ny**2 * w**2 - fx**2 * m**2 * nz**2 * w**2
         + 2 * fx * fy * m**2 * nx * ny * w**2 + 2 * fx * fz * m**2 * nx * nz * w**2
         - fy**2 * m**2 * nx**2 * w**2 - fy**2 * m**2 * nz**2 * w**2
         + 2 * fy * fz * m**2 * ny * nz * w**2
         - fz**2 * m**2 * nx**2 * w**2 - fz**2 * m**2 * ny**2 * w**2)
    with np.errstate(invalid="ignore"):
        sD = np.sqrt(D)
    AL = (L0 * d * n1 * ny**2 + L0 * d * n1 * nz**2 - M0 * d * n1 * nx * ny
          - N0 * d * n1 * nx * nz + fx * m * ny**2 * w + fx * m * nz**2 * w
          - fy * m * nx * ny * w - fz * m * nx * nz * w)
    AM = (-L0 * d * n1 * nx * ny + M0 * d * n1 * nx**2 + M0 * d * n1 * nz**2
          - N0 * d * n1 * ny * nz - fx * m * nx * ny * w + fy * m * nx**2 * w
          + fy * m * nz**2 * w - fz * m * ny * nz * w)
    PN = (L0 * d * n1 * nx * nz + M0 * d * n1 * ny * nz - N0 * d * n1 * nx**2
          - N0 * d * n1 * ny**2 + fx * m * nx * nz * w + fy * m * ny * nz * w
          - fz * m * nx**2 * w - fz * m * ny**2 * w)
    if reflective:
        r.L = (AL - nx * sD) / (d * n2c)
        r.M = (AM - ny * sD) / (d * n2c)
        r.N = -nz * sD / (d * n2c) - PN / (d * n2c)
    else:
        r.L = (AL + nx * sD) / (d * n2c)
        r.M = (AM + ny * sD) / (d * n2c)
        r.N = nz * sD / (d * n2c) - PN / (d * n2c)
    normalize(r)


def interact(r: Rays, table, s, n1, n2, w):
    """The surface's interaction model (standard_surface.py:225). Returns True when the
    rays are left unnormalised (thin lens)."""
    ia = int(s["interaction"])
    flags = int(s["flags"])
    refl = bool(flags & _abi.SURF_REFLECTIVE)
    blk = table.coef[int(s["ia_off"]):]
    if ia == _abi.IA_THIN_LENS:
        thin_lens(r, blk[0], n1, -n1 if refl else n2)
        return True
    nx, ny, nz = surface_normal(r, table, s)
    if ia == _abi.IA_REFRACT_REFLECT:
        if refl:
            reflect(r, nx, ny, nz)
        else:
            refract(r, nx, ny, nz, n1, n2)
    elif ia == _abi.IA_PHASE:
        phase_interact(r, blk, nx, ny, nz, n1, n2, refl, w)
    else:
        diffract(r, blk, nx, ny, nz, n1, n2, refl, w)
    return False


# --------------------------------------------------------------------------------------
# the trace
# --------------------------------------------------------------------------------------
class TraceResult:
    def __init__(self, rays, records, newton_updates):
        self.rays = rays
        self.records = records  # {surface index (traced, 0-based): Rays}
        self.newton_updates = newton_updates  # {surface index: updates}


def polygon_contains(vx, vy, x, y):
    """matplotlib Path.contains_points (the reference's numpy-backend
    path_contains_points, backend/numpy_backend.py:139-142): even-odd crossings of the
    implicitly closed polygon, per edge v0 -> v1 toggling when the edge straddles the
    horizontal through the point and
    ((vy1 - y) * (vx0 - vx1) >= (vx1 - x) * (vy0 - vy1)) == (vy1 >= y)."""
    inside = np.zeros(np.shape(x), dtype=bool)
    n = len(vx)
    for k in range(n):
        vx0, vy0 = vx[k - 1], vy[k - 1]
        vx1, vy1 = vx[k], vy[k]
        yf0, yf1 = vy0 >= y, vy1 >= y
        hit = (yf0 != yf1) & (((vy1 - y) * (vx0 - vx1) >= (vx1 - x) * (vy0 - vy1)) == yf1)
        inside ^= hit
    return inside & np.isfinite(x) & np.isfinite(y)


def aperture_contains(prog, x, y):
    """Evaluate a lowered aperture program (include/optiland_rt.h ort_aperture_op) with
    the reference's per-class contains() expressions: radial.py:54-63,
    offset_radial.py:46-58, elliptical.py:40-55, rectangular.py:40-60, polygon.py:50-66,
    base.py:255-340 (union / intersection / difference)."""
    stack = []
    q = 0
    while q < len(prog):
        op = int(prog[q])
        if op == _abi.AP_RADIAL:
            rmin2, rmax2, ox, oy = (float(v) for v in prog[q + 1:q + 5])
            radius2 = (x - ox) ** 2 + (y - oy) ** 2
            stack.append((radius2 <= rmax2) & (radius2 >= rmin2))
            q += 5
        elif op == _abi.AP_ELLIPSE:
            ox, oy, a2, b2 = (float(v) for v in prog[q + 1:q + 5])
            xx, yy = x - ox, y - oy
            stack.append((xx**2 / a2 + yy**2 / b2) <= 1)
            q += 5
        elif op == _abi.AP_RECT:
            x0, x1, y0, y1 = (float(v) for v in prog[q + 1:q + 5])
            stack.append((x0 <= x) & (x <= x1) & (y0 <= y) & (y <= y1))
            q += 5
        elif op == _abi.AP_POLYGON:
            n = int(prog[q + 1])
            v = np.asarray(prog[q + 2:q + 2 + 2 * n], dtype=np.float64).reshape(n, 2)
            stack.append(polygon_contains(v[:, 0], v[:, 1], x, y))
            q += 2 + 2 * n
        else:
            b = stack.pop()
            a = stack.pop()
            stack.append(a | b if op == _abi.AP_UNION else
                         (a & b if op == _abi.AP_INTERSECT else a & ~b))
            q += 1
    return stack[-1]


def trace_segment(table, rays: Rays, lam: int, record=False, sched=None, start=0, w=None):
    """One reference trace call: SurfaceGroup.trace (surface_group.py:232-244) over the
    traced surfaces, then the image-space propagate (real_ray_tracer.py:84-89).
    `rays` is modified in place (the reference mutates RealRays). w: per-ray
    wavelengths -- n and k then come from the material records per ray (as the reference
    evaluates material.n(rays.w)) instead of the lambda-th table row."""
    if w is not None:
        return _trace_segment_w(table, rays, w, record, sched, start)
    r = rays
    records = {}
    updates = {}
    unnorm = False
    n_tab = table.n_tab[lam]
    a_tab = table.alpha_tab[lam]
    w_lam = float(table.wavelengths[lam])
    for si in range(start, len(table.surfaces)):
        s = table.surfaces[si]
        g = int(s["geometry"])
        flags = int(s["flags"])
        # localize: translate(-t) of the root frame, then the remaining ops
        ct = s["cs_t"]
        r.x, r.y, r.z = r.x + -float(ct[0]), r.y + -float(ct[1]), r.z + -float(ct[2])
        apply_cs(r, table.cs_ops[int(s["cs_loc_off"]):int(s["cs_loc_off"]) + int(s["n_cs_loc"])])
        if g == _abi.GEOM_PLANE:
            t = distance_plane(r)
        elif g == _abi.GEOM_STANDARD:
            t = distance_conic(r, float(s["radius"]), float(s["conic"]),
                               bool(flags & _abi.SURF_RADIUS_INF))
        else:
            t, updates[si] = distance_newton(
                r, table, s, None if sched is None else sched.get(si))
        mp, mq = int(s["mat_pre"]), int(s["mat_post"])
        propagate(r, t, float(a_tab[mp]))
        if unnorm:  # homogeneous.py:55-57
            normalize(r)
        r.opd = r.opd + np.abs(t * n_tab[mp])  # standard_surface.py:218
        if flags & _abi.SURF_APERTURE:  # radial.py:50-63 + real_rays.py:132-139
            radius2 = r.x**2 + r.y**2
            inside = (radius2 <= float(s["ap_rmax2"])) & (radius2 >= float(s["ap_rmin2"]))
            r.i = np.where(~inside, np.zeros_like(r.i), r.i)
        if flags & _abi.SURF_APERTURE_PROG:  # physical_apertures/*.py contains + clip
            off, ln = int(s["ap_off"]), int(s["ap_len"])
            inside = aperture_contains(table.coef[off:off + ln], r.x, r.y)
            r.i = np.where(~inside, np.zeros_like(r.i), r.i)
        unnorm = interact(r, table, s, n_tab[mp], n_tab[mq], w_lam)
        apply_cs(r, table.cs_ops[int(s["cs_glob_off"]):int(s["cs_glob_off"]) + int(s["n_cs_glob"])])
        r.x, r.y, r.z = r.x + float(ct[0]), r.y + float(ct[1]), r.z + float(ct[2])
        if record:
            records[si] = r.copy()
    if table.final_mat >= 0:
        # real_ray_tracer.py:84-89 always propagates (by 0 for the samples), and applies
        # absorption only when k>0 of the image-space material.
        propagate(r, table.final_thickness, float(a_tab[table.final_mat]))
        if unnorm:
            normalize(r)
    return TraceResult(r, records, updates)


def _trace_segment_w(table, r: Rays, w, record, sched, start):
    records, updates = {}, {}
    unnorm = False
    w = np.asarray(w, dtype=np.float64)
    for si in range(start, len(table.surfaces)):
        s = table.surfaces[si]
        g = int(s["geometry"])
        flags = int(s["flags"])
        ct = s["cs_t"]
        r.x, r.y, r.z = r.x + -float(ct[0]), r.y + -float(ct[1]), r.z + -float(ct[2])
        apply_cs(r, table.cs_ops[int(s["cs_loc_off"]):int(s["cs_loc_off"]) + int(s["n_cs_loc"])])
        if g == _abi.GEOM_PLANE:
            t = distance_plane(r)
        elif g == _abi.GEOM_STANDARD:
            t = distance_conic(r, float(s["radius"]), float(s["conic"]),
                               bool(flags & _abi.SURF_RADIUS_INF))
        else:
            t, updates[si] = distance_newton(
                r, table, s, None if sched is None else sched.get(si))
        mp, mq = int(s["mat_pre"]), int(s["mat_post"])
        n_pre = material_n(table, mp, w)
        propagate_w(r, t, material_k(table, mp, w), w)
        if unnorm:
            normalize(r)
        r.opd = r.opd + np.abs(t * n_pre)  # standard_surface.py:218
        if flags & _abi.SURF_APERTURE:
            radius2 = r.x**2 + r.y**2
            inside = (radius2 <= float(s["ap_rmax2"])) & (radius2 >= float(s["ap_rmin2"]))
            r.i = np.where(~inside, np.zeros_like(r.i), r.i)
        if flags & _abi.SURF_APERTURE_PROG:
            off, ln = int(s["ap_off"]), int(s["ap_len"])
            inside = aperture_contains(table.coef[off:off + ln], r.x, r.y)
            r.i = np.where(~inside, np.zeros_like(r.i), r.i)
        unnorm = interact(r, table, s, n_pre, material_n(table, mq, w), w)
        apply_cs(r, table.cs_ops[int(s["cs_glob_off"]):int(s["cs_glob_off"]) + int(s["n_cs_glob"])])
        r.x, r.y, r.z = r.x + float(ct[0]), r.y + float(ct[1]), r.z + float(ct[2])
        if record:
            records[si] = r.copy()
    if table.final_mat >= 0:
        propagate_w(r, table.final_thickness, material_k(table, table.final_mat, w), w)
        if unnorm:
            normalize(r)
    return TraceResult(r, records, updates)


def trace_batch(table, rays: Rays, batch_lambda, seg_len, record=False):
    """Trace a batch of consecutive segments, each one reference trace call."""
    n = rays.x.size
    out = {a: np.empty(n) for a in _abi.RAY_FIELDS}
    ups = []
    recs = []
    nseg = max(1, len(batch_lambda))
    for sg in range(nseg):
        sl = slice(sg * seg_len, min(n, (sg + 1) * seg_len))
        sub = rays.take(sl)
        res = trace_segment(table, sub, int(batch_lambda[sg]) if len(batch_lambda) else 0,
                            record=record)
        for a in _abi.RAY_FIELDS:
            out[a][sl] = getattr(res.rays, a)
        ups.append(res.newton_updates)
        recs.append(res.records)
    return Rays(**{a: out[a] for a in ("x", "y", "z", "L", "M", "N", "i")}, opd=out["opd"]), ups, recs
