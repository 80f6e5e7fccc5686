"""Surface geometries (parameter holders lowered into the kernel's surface table).

Mirrors optiland/geometries/{plane,standard,newton_raphson,even_asphere,odd_asphere,
zernike}.py: same class names, constructor arguments and defaults. The arithmetic
(sag, intersection distance, normal) runs only in the HIP kernel
(optiland_pr_amd/csrc/ort_core.h); these classes just describe the surface.
"""

from __future__ import annotations

import dataclasses
import functools
import math

import numpy as np

from . import _abi
from .coordinate_system import CoordinateSystem


def scalar(v):
    """A plain float from a Python / NumPy number or a (possibly grad-requiring) torch
    scalar tensor -- geometry parameters may be autograd leaves (autodiff.py)."""
    if hasattr(v, "detach"):
        v = v.detach().cpu()
    return float(np.ravel(np.asarray(v, dtype=np.float64))[0])


class BaseGeometry:
    """geometries/base.py:14-110."""

    geometry_id: int = -1

    def __init__(self, coordinate_system: CoordinateSystem):
        self.cs = coordinate_system

    def flip(self):
        raise NotImplementedError

    # lowering hooks ------------------------------------------------------------------
    def lower_params(self):
        """-> (radius, conic, tol, max_iter, norm_radius, coefficients list)."""
        raise NotImplementedError

    def zernike_terms(self):
        return None

    # per-geometry API (geometries/base.py:61-110), evaluated on the MI355X in the
    # geometry's local frame; results are float64 device tensors
    def sag(self, x=0, y=0):
        """Sag z(x, y) (e.g. standard.py:73-87, even_asphere.py:82-98)."""
        from .raytrace import geometry_sag_normal

        return geometry_sag_normal(self, x, y)[0]

    def surface_normal(self, rays):
        """Unit normal (nx, ny, nz) at the rays' (x, y) (e.g. standard.py:154-167)."""
        from .raytrace import geometry_sag_normal

        return geometry_sag_normal(self, rays.x, rays.y)[1:]

    def distance(self, rays):
        """Distance along each ray to the surface (plane.py:61-77, standard.py:89-140,
        newton_raphson.py:119-168 with its global stop rule over `rays`)."""
        from .raytrace import geometry_distance

        return geometry_distance(self, rays)


class Plane(BaseGeometry):
    """geometries/plane.py:19-98 (t = -z/N, normal (0,0,1))."""

    geometry_id = _abi.GEOM_PLANE

    def __init__(self, coordinate_system):
        super().__init__(coordinate_system)
        self.radius = np.inf
        self.is_symmetric = True

    def flip(self):
        pass

    def lower_params(self):
        return np.inf, 0.0, 0.0, 0, 1.0, []


class StandardGeometry(BaseGeometry):
    """geometries/standard.py:19-167 (sphere / conic, closed form)."""

    geometry_id = _abi.GEOM_STANDARD

    def __init__(self, coordinate_system, radius, conic=0.0):
        super().__init__(coordinate_system)
        self.radius = float(radius)
        self.k = float(conic)
        self.is_symmetric = True

    def flip(self):
        self.radius = -self.radius

    def lower_params(self):
        return scalar(self.radius), scalar(self.k), 0.0, 0, 1.0, []


class PlaneGrating(Plane):
    """geometries/plane_grating.py:19-153: a plane carrying a grating (order, period,
    groove orientation angle) for the diffractive interaction."""

    def __init__(self, coordinate_system, grating_order, grating_period,
                 groove_orientation_angle):
        super().__init__(coordinate_system)
        self.grating_order = grating_order
        self.grating_period = grating_period
        self.groove_orientation_angle = groove_orientation_angle


class StandardGratingGeometry(StandardGeometry):
    """geometries/standard_grating.py:25-294: a sphere / conic carrying a grating (its
    distance and normal are the standard ones, standard_grating.py:148-222)."""

    def __init__(self, coordinate_system, radius, grating_order, grating_period,
                 groove_orientation_angle, conic=0.0):
        super().__init__(coordinate_system, radius, conic)
        self.grating_order = grating_order
        self.grating_period = grating_period
        self.groove_orientation_angle = groove_orientation_angle


class GridSagGeometry(BaseGeometry):
    """geometries/grid_sag.py:15-180: sag bilinearly interpolated on a rectangular grid
    (NaN outside it), intersected by its own Newton loop from t = 0 with the global stop
    rule max |dt| < tol."""

    geometry_id = _abi.GEOM_GRID_SAG

    def __init__(self, coordinate_system, x_coordinates, y_coordinates, sag_values,
                 tol=1e-6, max_iter=100):
        super().__init__(coordinate_system)
        self.x_grid = np.asarray(x_coordinates, dtype=np.float64)
        self.y_grid = np.asarray(y_coordinates, dtype=np.float64)
        self.sag_grid = np.asarray(sag_values, dtype=np.float64)
        self.tol = tol
        self.max_iter = max_iter
        self.is_symmetric = False
        self.radius = np.inf
        if self.sag_grid.shape != (len(self.y_grid), len(self.x_grid)):
            raise ValueError(
                f"Shape of sag_values {self.sag_grid.shape} must match "
                f"(len(y_coordinates), len(x_coordinates)) = "
                f"({len(self.y_grid)}, {len(self.x_grid)}).")
        if len(self.x_grid) < 2 or len(self.y_grid) < 2:
            raise ValueError("the sag grid needs at least 2 x 2 points")

    def flip(self):
        self.sag_grid = -self.sag_grid

    def lower_params(self):
        blk = [float(len(self.x_grid)), float(len(self.y_grid)), *self.x_grid.tolist(),
               *self.y_grid.tolist(), *self.sag_grid.ravel().tolist()]
        return np.inf, 0.0, float(self.tol), int(self.max_iter), 1.0, blk


class NewtonRaphsonGeometry(StandardGeometry):
    """geometries/newton_raphson.py:43-168 (conic initial guess + Newton refinement)."""

    def __init__(self, coordinate_system, radius, conic=0.0, tol=1e-10, max_iter=100):
        super().__init__(coordinate_system, radius, conic)
        self.tol = float(tol)
        self.max_iter = int(max_iter)


class EvenAsphere(NewtonRaphsonGeometry):
    """geometries/even_asphere.py:28-129: conic + sum_i C_i r^(2(i+1))."""

    geometry_id = _abi.GEOM_EVEN_ASPHERE

    def __init__(self, coordinate_system, radius, conic=0.0, tol=1e-10, max_iter=100,
                 coefficients=None):
        super().__init__(coordinate_system, radius, conic, tol, max_iter)
        self.coefficients = list(coefficients) if coefficients is not None else []
        self.is_symmetric = True

    def lower_params(self):
        return (scalar(self.radius), scalar(self.k), self.tol, self.max_iter, 1.0,
                [float(c) for c in self.coefficients])


class OddAsphere(EvenAsphere):
    """geometries/odd_asphere.py:20-130: conic + sum_i C_i r^(i+1)."""

    geometry_id = _abi.GEOM_ODD_ASPHERE


_ZERNIKE_TYPES = ("standard", "noll", "fringe")


def _index_to_number(kind, n, m):
    """zernike/standard.py:47-60, noll.py:59-78, fringe.py:53-68."""
    if kind == "standard":
        if (n - m) % 2 == 0:
            return (n * (n + 2) + m) // 2
        return None
    if kind == "noll":
        if (n - m) % 2 == 0:
            mod = n % 4
            if (m > 0 and mod <= 1) or (m < 0 and mod >= 2):
                c = 0
            elif (m >= 0 and mod >= 2) or (m <= 0 and mod <= 1):
                c = 1
            return int(n * (n + 1) / 2 + np.abs(m) + c)
        return None
    if kind == "fringe":
        if (n - m) % 2 == 0:
            return int((1 + (n + abs(m)) / 2) ** 2 - 2 * abs(m) + (1 - np.sign(m)) / 2)
        return None
    raise ValueError(kind)


def _norm_constant(kind, n, m):
    """standard.py:63-75 / noll.py:44-56: sqrt((2n+2)/(1+delta_m0)); fringe.py:38-50: 1."""
    if kind == "fringe":
        return np.array(1)
    denominator = 2 if m == 0 else 1
    return np.sqrt(np.array((2 * n + 2) / denominator))


@functools.lru_cache(maxsize=None)
def zernike_indices(kind, n_indices):
    """zernike/base.py:143-192 (_generate_indices): (n, m) sorted by the scheme's
    coefficient number."""
    numbers_present = np.full(n_indices + 1, False)
    numbers_present[0] = _index_to_number(kind, 0, 0) != 0
    number, indices = [], []
    n, m = 0, 0
    while not all(numbers_present):
        num = _index_to_number(kind, n, m)
        if num is not None:
            number.append(num)
            indices.append((n, m))
            if num <= n_indices:
                numbers_present[num] = True
        if m == n:
            n += 1
            m = -n
        else:
            m += 1
    srt = [e for _, e in sorted(zip(number, indices, strict=False))]
    return tuple(srt[:n_indices])


def _gamma(x):
    try:
        from scipy.special import gamma

        return gamma(x)
    except ImportError:  # pragma: no cover
        return np.float64(math.gamma(float(x)))


@functools.lru_cache(maxsize=None)
def radial_coefficients(n, m_abs):
    """Host precompute of the reference's per-term factorial weights.

    _radial_term (zernike/base.py:228-253): coeff_k = (-1)**k * num / denom,
    num = factorial(n-k), denom = k! * ((n+m)/2-k)! * ((n-m)/2-k)!, with
    be.factorial = scipy.special.gamma(n+1) (backend/numpy_backend.py:135-136).
    _radial_derivative (:272-299): d_k = (-1)**k * (num / denom) * (n - 2k).
    """
    s_max = (n - m_abs) // 2 + 1
    nn = np.array(n)
    ma = np.array(m_abs)
    a, d = [], []
    for k in range(s_max):
        num = _gamma(nn - k + 1)
        denom = _gamma(k + 1) * _gamma((nn + ma) // 2 - k + 1) * _gamma((nn - ma) // 2 - k + 1)
        a.append(float((-1) ** k * num / denom))
        factor = n - 2 * k
        d.append(float((-1) ** k * (num / denom) * factor))
    return tuple(a), tuple(d)


# Radial orders up to which a Zernike surface's term sum is also lowered in Cartesian
# (monomial) form and evaluated that way by the Newton kernels (ort_core.h zmono_*): the
# expansion's coefficients grow with the order (cancellation ~ eps x sum |coefficient|),
# so higher orders keep the polar recurrence.
ZM_MAX_DEG = 6


@functools.lru_cache(maxsize=None)
def zernike_monomials(n, m):
    """R_n^|m|(rho) * {cos m phi | sin |m| phi} (zernike/base.py:42-68, 228-253) as a
    polynomial in the normalised coordinates (xn, yn): {(p, q): coefficient of xn^p yn^q}.
    rho^a cos(a phi) = Re (xn + i yn)^a, rho^a sin(a phi) = Im (xn + i yn)^a and
    rho^2 = xn^2 + yn^2, with the reference's radial weights a_k (radial_coefficients):
    integers, so every coefficient here is an exact double."""
    a = abs(m)
    ak, _ = radial_coefficients(n, a)
    ang = {}
    for j in range(a + 1):  # binomial expansion of (xn + i yn)^a
        c = math.comb(a, j) * (-1) ** (j // 2)
        if (j % 2 == 0) == (m >= 0):
            ang[(a - j, j)] = c
    out = {}
    for k, w in enumerate(ak):
        e = (n - 2 * k - a) // 2  # rho^(n - 2k) = rho^a (rho^2)^e
        for i in range(e + 1):
            ce = math.comb(e, i)
            for (p, q), cz in ang.items():
                key = (p + 2 * i, q + 2 * (e - i))
                out[key] = out.get(key, 0.0) + w * ce * cz
    return out


def monomial_index(N):
    """(p, q) -> position in the p-major triangular block of degree N (ort_core.h)."""
    idx, k = {}, 0
    for p in range(N + 1):
        for q in range(N - p + 1):
            idx[(p, q)] = k
            k += 1
    return idx


def zernike_monomial_block(terms, on_device):
    """The Cartesian block of a Zernike surface (ort_surface.zm_off / zm_deg): degree N,
    then [As (K)] [An (K)] [Ms (nt x K)] [Mn (nt x K)] with K = (N+1)(N+2)/2:
    Mn[j] the monomials of term j, Ms[j] = norm_j * Mn[j]; As / An their sums weighted by
    the coefficients -- the sag's (normalised) and the normal's (the reference's normal
    omits the normalisation constant, zernike.py:163-231) -- formed in term order as
    acc = acc + c_j * M[j][k], the order ort_patch_zernike uses on the device (zeros when
    the coefficients live on the device and are patched there). None above ZM_MAX_DEG."""
    if not terms:
        return None
    N = max(int(t[2]) for t in terms)
    if N > ZM_MAX_DEG:
        return None
    idx = monomial_index(N)
    K = len(idx)
    Mn = np.zeros((len(terms), K))
    Ms = np.zeros((len(terms), K))
    for j, (c, norm, n, m, _a, _d) in enumerate(terms):
        for key, v in zernike_monomials(int(n), int(m)).items():
            Mn[j, idx[key]] = v
        Ms[j] = np.float64(norm) * Mn[j]
    As, An = [0.0] * K, [0.0] * K
    if not on_device:
        for j, t in enumerate(terms):
            c = float(t[0])
            for k in range(K):
                As[k] = As[k] + c * float(Ms[j, k])
                An[k] = An[k] + c * float(Mn[j, k])
    return N, As + An + [float(v) for v in Ms.ravel()] + [float(v) for v in Mn.ravel()]


@functools.lru_cache(maxsize=None)
def _zernike_structure(kind, n_c):
    """(norm, n, m, a_k, d_k) of the first n_c terms of a scheme: value-independent, so
    computed once (the lowering runs on every trace call)."""
    out = []
    for n, m in zernike_indices(kind, n_c):
        a, d = radial_coefficients(n, abs(m))
        out.append((float(_norm_constant(kind, n, m)), n, m, a, d))
    return tuple(out)


class ZernikePolynomialGeometry(NewtonRaphsonGeometry):
    """geometries/zernike.py:33-246: conic + sum_j c_j N_nm R_n^|m|(rho) {cos|sin}(m phi)."""

    geometry_id = _abi.GEOM_ZERNIKE

    def __init__(self, coordinate_system, radius, conic=0.0, tol=1e-10, max_iter=100,
                 coefficients=None, zernike_type="standard", norm_radius=1):
        super().__init__(coordinate_system, radius, conic, tol, max_iter)
        if zernike_type not in _ZERNIKE_TYPES:
            raise ValueError(
                "Zernike type must be one of 'standard', 'noll', or 'fringe', got "
                f"{zernike_type}")
        if norm_radius <= 0:
            raise ValueError(f"Normalization radius must be positive, got {norm_radius}")
        self.coefficients = np.atleast_1d(
            np.asarray(coefficients if coefficients is not None else [], dtype=np.float64))
        self.zernike_type = zernike_type
        self.norm_radius = float(norm_radius)
        self.is_symmetric = False

    def lower_params(self):
        return (scalar(self.radius), scalar(self.k), self.tol, self.max_iter,
                self.norm_radius, [])

    def zernike_terms(self, values=True):
        """-> list of (c, norm, n, m, a_k list, d_k list) in coefficient order; with
        values=False the coefficients are left as 0 placeholders (not read)."""
        coeffs = self.coefficients
        n_c = int(coeffs.numel()) if hasattr(coeffs, "numel") else len(coeffs)
        if not values:
            coeffs = np.zeros(n_c)
        elif hasattr(coeffs, "detach"):  # torch tensor (autograd leaf, autodiff.py)
            coeffs = coeffs.detach().cpu().numpy()
        return [(float(c), *st) for c, st in
                zip(coeffs, _zernike_structure(self.zernike_type, n_c), strict=True)]


class PolynomialGeometry(NewtonRaphsonGeometry):
    """geometries/polynomial.py:33-140: conic + sum_ij C_ij x^i y^j (C as be.atleast_2d)."""

    geometry_id = _abi.GEOM_POLYNOMIAL

    def __init__(self, coordinate_system, radius, conic=0.0, tol=1e-10, max_iter=100,
                 coefficients=None):
        super().__init__(coordinate_system, radius, conic, tol, max_iter)
        c = np.atleast_2d(np.asarray(coefficients if coefficients is not None else [],
                                     dtype=np.float64))
        if c.size == 0:
            c = np.zeros((1, 1))
        self.coefficients = c
        self.is_symmetric = False

    def lower_params(self):
        c = np.atleast_2d(np.asarray(self.coefficients, dtype=np.float64))
        block = [float(c.shape[0]), float(c.shape[1])] + [float(v) for v in c.ravel()]
        return scalar(self.radius), scalar(self.k), self.tol, self.max_iter, 1.0, block


class ChebyshevPolynomialGeometry(NewtonRaphsonGeometry):
    """geometries/chebyshev.py:33-215: conic + sum_ij C_ij T_i(x/norm_x) T_j(y/norm_y)."""

    geometry_id = _abi.GEOM_CHEBYSHEV

    def __init__(self, coordinate_system, radius, conic=0.0, tol=1e-10, max_iter=100,
                 coefficients=None, norm_x=1, norm_y=1):
        super().__init__(coordinate_system, radius, conic, tol, max_iter)
        self.coefficients = np.atleast_2d(np.asarray(
            coefficients if coefficients is not None else [], dtype=np.float64))
        self.norm_x = float(norm_x)
        self.norm_y = float(norm_y)
        self.is_symmetric = False

    def lower_params(self):
        c = np.atleast_2d(np.asarray(self.coefficients, dtype=np.float64))
        if c.size == 0:
            c = np.zeros((1, 0))
        block = [float(c.shape[0]), float(c.shape[1]), float(self.norm_x),
                 float(self.norm_y)] + [float(v) for v in c.ravel()]
        return scalar(self.radius), scalar(self.k), self.tol, self.max_iter, 1.0, block


class BiconicGeometry(NewtonRaphsonGeometry):
    """geometries/biconic.py:29-158: separate conic profiles in x and y; the Newton start
    guess is the (R_x, k_x) conic (newton_raphson.py:134)."""

    geometry_id = _abi.GEOM_BICONIC

    def __init__(self, coordinate_system, radius_x, radius_y, conic_x=0.0, conic_y=0.0,
                 tol=1e-10, max_iter=100):
        super().__init__(coordinate_system, radius_x, conic_x, tol, max_iter)
        self.Rx = float(radius_x)
        self.Ry = float(radius_y)
        self.kx = float(conic_x)
        self.ky = float(conic_y)
        self.is_symmetric = False

    @staticmethod
    def _curv(r):
        return 0.0 if (np.isinf(r) or r == 0) else 1.0 / r

    def lower_params(self):
        block = [self._curv(self.Rx), self._curv(self.Ry), self.kx, self.ky]
        return scalar(self.radius), scalar(self.k), self.tol, self.max_iter, 1.0, block


class ToroidalGeometry(NewtonRaphsonGeometry):
    """geometries/toroidal.py:26-233: a Y-Z conic + even polynomial profile swept about an
    axis at R_rot; the Newton start guess is the (R_yz, k = 0) sphere."""

    geometry_id = _abi.GEOM_TOROIDAL

    def __init__(self, coordinate_system, radius_x, radius_y, conic=0.0, coeffs_poly_y=None,
                 tol=1e-10, max_iter=100):
        super().__init__(coordinate_system, radius_y, 0.0, tol, max_iter)
        self.R_rot = float(radius_x)
        self.R_yz = float(radius_y)
        self.k_yz = float(conic)
        self.coeffs_poly_y = [float(c) for c in (coeffs_poly_y or [])]
        self.is_symmetric = False

    def lower_params(self):
        has_yz = bool(np.isfinite(self.R_yz) and self.R_yz != 0)
        c_yz = 1.0 / self.R_yz if has_yz else 0.0
        block = [self.R_rot, c_yz, self.k_yz, 1.0 if has_yz else 0.0,
                 float(len(self.coeffs_poly_y))] + self.coeffs_poly_y
        return scalar(self.radius), scalar(self.k), self.tol, self.max_iter, 1.0, block


@dataclasses.dataclass
class ForbesSolverConfig:
    """geometries/forbes/geometry.py:50-60."""

    tol: float = 1e-10
    max_iter: int = 100


@dataclasses.dataclass
class ForbesSurfaceConfig:
    """geometries/forbes/geometry.py:63-80 (terms: {n: c} for Q-bfs,
    {('a'|'b', m, n): c} for Q-2D)."""

    radius: float
    conic: float = 0.0
    norm_radius: float = 1.0
    terms: dict | None = None


class _ForbesBase(NewtonRaphsonGeometry):
    """geometries/forbes/geometry.py:83-180: base conic + Q-polynomial departure scaled by
    the conic correction factor; Newton-iterated like every NewtonRaphsonGeometry."""

    def __init__(self, coordinate_system, surface_config, solver_config=None):
        solver_config = solver_config or ForbesSolverConfig()
        super().__init__(coordinate_system, surface_config.radius, surface_config.conic,
                         solver_config.tol, solver_config.max_iter)
        self.surface_config = surface_config
        self.solver_config = solver_config
        self.norm_radius = float(surface_config.norm_radius)
        self.terms = dict(surface_config.terms or {})


class ForbesQbfsGeometry(_ForbesBase):
    """geometries/forbes/geometry.py:183-330: rotationally symmetric Q-bfs surface.

    Coefficient block: norm_radius, L, dep_normal, b_0 .. b_{L-1} (the orthonormal P_n
    coefficients, forbes.qbfs_to_pn); dep_normal = 0 when every coefficient is zero (the
    reference's normal then skips the departure, :300)."""

    geometry_id = _abi.GEOM_FORBES_QBFS

    def __init__(self, coordinate_system, surface_config, solver_config=None):
        super().__init__(coordinate_system, surface_config, solver_config)
        self.radial_terms = self.terms
        self.is_symmetric = True

    def lower_params(self):
        from .forbes import qbfs_to_pn

        t = {int(k): scalar(v) for k, v in self.radial_terms.items()}
        cs = [t.get(n, 0.0) for n in range(max(t) + 1)] if t and max(t) >= 0 else []
        b = qbfs_to_pn(cs)
        dep = 1.0 if any(c != 0.0 for c in cs) else 0.0
        block = [self.norm_radius, float(len(b)), dep] + b
        return scalar(self.radius), scalar(self.k), self.tol, self.max_iter, 1.0, block


class ForbesQ2dGeometry(_ForbesBase):
    """geometries/forbes/geometry.py:333-640: Q-2D freeform surface.

    Coefficient block: norm_radius, d/dx and d/dy of the sag at the vertex, the m = 0
    Q-bfs record (L, b_0 .. b_{L-1}), the highest azimuthal order M, then per order
    m = 1..M its cosine and sine Clenshaw records (forbes.q2d_order_block)."""

    geometry_id = _abi.GEOM_FORBES_Q2D

    def __init__(self, coordinate_system, surface_config, solver_config=None):
        super().__init__(coordinate_system, surface_config, solver_config)
        self.freeform_coeffs = self.terms
        self.is_symmetric = False

    def split(self):
        from .forbes import q2d_split

        cm0, ams, bms = q2d_split({k: scalar(v) for k, v in self.freeform_coeffs.items()})
        return [float(c) for c in cm0], ams, bms

    def lower_params(self):
        from .forbes import q2d_order_block, q2d_sum_at_zero, qbfs_to_pn

        cm0, ams, bms = self.split()
        # vertex slope (forbes/geometry.py:530-543): only the m = 1 order contributes
        vdx = q2d_sum_at_zero(ams[0], 1) / np.float64(self.norm_radius) if ams and ams[0] else 0.0
        vdy = q2d_sum_at_zero(bms[0], 1) / np.float64(self.norm_radius) if bms and bms[0] else 0.0
        b0 = qbfs_to_pn(cm0)
        block = [self.norm_radius, float(vdx), float(vdy), float(len(b0))] + b0
        block.append(float(len(ams)))
        for m in range(1, len(ams) + 1):
            block += q2d_order_block(ams[m - 1], m)
            block += q2d_order_block(bms[m - 1], m)
        return scalar(self.radius), scalar(self.k), self.tol, self.max_iter, 1.0, block


class NurbsGeometry(BaseGeometry):
    """geometries/nurbs/nurbs_geometry.py:29-932: a NURBS surface -- an explicit control
    net (control_points (3, n+1, m+1), weights, degrees, knots) or, with no control points,
    a bicubic least-squares fit of the conic (radius, conic) or of a plane over the window
    [x_center +- nurbs_norm_x] x [y_center +- nurbs_norm_y] once fit_surface() is called
    (the reference fits only then, nurbs_geometry.py:828-838). sag / surface_normal /
    distance solve for (u, v) on the MI355X (ort_nurbs.h); get_value / get_derivative /
    get_normals evaluate at given (u, v) on the host (nurbs.py)."""

    geometry_id = _abi.GEOM_NURBS

    def __init__(self, coordinate_system, radius=np.inf, conic=0.0, nurbs_norm_x=None,
                 nurbs_norm_y=None, x_center=0.0, y_center=0.0, control_points=None,
                 weights=None, u_degree=None, v_degree=None, u_knots=None, v_knots=None,
                 n_points_u=4, n_points_v=4, tol=1e-10, max_iter=100):
        from . import nurbs

        super().__init__(coordinate_system)
        self.radius = radius
        self.k = conic
        self.nurbs_norm_x = nurbs_norm_x
        self.nurbs_norm_y = nurbs_norm_y
        self.x_center = x_center
        self.y_center = y_center
        self.tol = tol
        self.max_iter = max_iter
        self.is_symmetric = False
        self.P = None if control_points is None else np.asarray(control_points, np.float64)
        self.W = None if weights is None else np.asarray(weights, np.float64)
        self.p, self.q = u_degree, v_degree
        self.U = None if u_knots is None else np.asarray(u_knots, np.float64)
        self.V = None if v_knots is None else np.asarray(v_knots, np.float64)
        if self.P is None:  # fitted on fit_surface()
            self.is_fitted = True
            self.ndim = 3
            self.P_size_u = n_points_u + 1
            self.P_size_v = n_points_v + 1
            return
        # nurbs_geometry.py:132-269: the missing parts of an explicit net take the
        # reference's defaults (unit weights; degree = points - 1, i.e. Bezier; clamped
        # uniform knots)
        self.is_fitted = False
        self.ndim = self.P.shape[0]
        nu, nv = self.P.shape[1], self.P.shape[2]
        self.P_size_u, self.P_size_v = nu, nv
        if self.W is None:
            self.W = np.ones((nu, nv))
        if self.p is None and self.U is None:
            self.p = nu - 1
        if self.q is None and self.V is None:
            self.q = nv - 1
        if self.U is None:
            self.U = nurbs.clamped_knots(nu, self.p)
        if self.V is None:
            self.V = nurbs.clamped_knots(nv, self.q)
        if self.p is None:
            self.p = len(self.U) - nu - 1
        if self.q is None:
            self.q = len(self.V) - nv - 1
        self.surface_type = ("NURBS" if weights is not None else
                             "Bezier" if u_knots is None and u_degree is None else "B-Spline")

    def __str__(self):
        return "NURBS"

    def flip(self):
        """nurbs_geometry.py:271-278."""
        self.radius = -self.radius
        self.P = self.P.copy()
        self.P[2] = -self.P[2]

    def fit_surface(self):
        """nurbs_geometry.py:828-932: fit the conic (or, with an infinite radius, a plane)."""
        from . import nurbs

        nx, ny = float(self.nurbs_norm_x), float(self.nurbs_norm_y)
        xc, yc = float(self.x_center), float(self.y_center)
        if np.isinf(scalar(self.radius)):
            P, W, p, q, U, V = nurbs.fit_plane(nx, ny, xc, yc, self.P_size_u, self.P_size_v)
        else:
            P, W, p, q, U, V = nurbs.fit_standard(scalar(self.radius), scalar(self.k), nx, ny,
                                                  xc, yc, self.P_size_u, self.P_size_v)
            self.P_size_u, self.P_size_v = P.shape[1], P.shape[2]
        self.surface_type = "NURBS"
        self.P, self.W, self.p, self.q, self.U, self.V = P, W, p, q, U, V

    def _net(self):
        if self.P is None:
            raise ValueError("the NURBS surface has no control net yet: call fit_surface()")
        return self.P, self.W, int(self.p), int(self.q), self.U, self.V

    def get_value(self, u, v):
        """nurbs_geometry.py:280-307: S(u, v), shape (3, ...) like u."""
        from . import nurbs

        u, v = np.asarray(u, np.float64), np.asarray(v, np.float64)
        if u.size != v.size:
            raise Exception("u and v must have the same size")
        S = nurbs.surface_point(*self._net(), u.ravel(), v.ravel())
        return S.reshape((S.shape[0],) + u.shape) if u.ndim > 1 else S

    def get_derivative(self, u, v, order_u, order_v):
        """nurbs_geometry.py:428-453: d^(order_u + order_v) S / du^order_u dv^order_v."""
        from . import nurbs

        u, v = np.asarray(u, np.float64), np.asarray(v, np.float64)
        dS = nurbs.surface_derivatives(*self._net(), u.ravel(), v.ravel(), order_u,
                                       order_v)[order_u][order_v]
        return dS.reshape((dS.shape[0],) + u.shape) if u.ndim > 1 else dS

    def get_normals(self, u, v):
        """nurbs_geometry.py:585-604."""
        from . import nurbs

        return nurbs.surface_normals(*self._net(), np.asarray(u, np.float64),
                                     np.asarray(v, np.float64))

    def lower_params(self):
        from . import nurbs

        blk = nurbs.lowered_block(*self._net())
        return scalar(self.radius), scalar(self.k), float(self.tol), int(self.max_iter), 1.0, blk
