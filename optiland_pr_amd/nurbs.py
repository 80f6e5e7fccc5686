"""NURBS surfaces: the host side of the reference's NurbsGeometry
(optiland/geometries/nurbs/nurbs_geometry.py, nurbs_fitting.py, nurbs_basis_functions.py).

Host work only -- forming the lowered control net. The least-squares fit of a standard
(conic) or plane surface to a control net (fit_surface), and the parameter-space
evaluations the reference's class exposes (get_value / get_derivative / get_normals at
given (u, v)). The ray-space work -- sag(x, y), surface_normal, distance(rays), each an
iterative (u, v) solve -- runs on the MI355X (ort_nurbs.h) through the geometry API of
geometries.BaseGeometry and inside the trace kernels.

Lowered block (GEOM_NURBS, include/optiland_rt.h):
    p, q, nu, nv, U[nu + p + 1], V[nv + q + 1], Pw[4][nu][nv] = (x w, y w, z w, w)
"""

from __future__ import annotations

from math import comb

import numpy as np

# degrees the kernels evaluate (ort_nurbs.h kNurbsMaxDeg): the reference's fitted surfaces
# are bicubic; an explicit net of higher degree is refused at lowering
MAX_DEGREE = 5


# ---- fitting: nurbs_fitting.py:19-244 (NURBS Book A9.7 / eqs. 9.4-9.5, 9.68-9.69) ------
def _basis_one(p, U, i, u):
    """nurbs_basis_functions.py:170-219 (A2.4): N_{i,p}(u)."""
    m = len(U) - 1
    if (i == 0 and u == U[0]) or (i == m - p - 1 and u == U[m]):
        return 1.0
    if u < U[i] or u >= U[i + p + 1]:
        return 0.0
    N = [0.0] * (p + i + 1)
    for j in range(p + 1):
        if U[i + j] <= u < U[i + j + 1]:
            N[j] = 1.0
    for k in range(1, p + 1):
        saved = 0.0
        if N[0] != 0.0:
            saved = ((u - U[i]) * N[0]) / (U[i + k] - U[i])
        for j in range(p - k + 1):
            ul, ur = U[i + j + 1], U[i + j + k + 1]
            if N[j + 1] == 0.0:
                N[j] = saved
                saved = 0.0
            else:
                t = N[j + 1] / (ur - ul)
                N[j] = saved + (ur - u) * t
                saved = (u - ul) * t
    return N[0]


def _chord_params(pts):
    """nurbs_fitting.py:167-198: chord-length parameters of one row of points."""
    n = len(pts)
    cds = [0.0] * (n + 1)
    cds[-1] = 1.0
    for i in range(1, n):
        cds[i] = np.linalg.norm(np.asarray(pts[i]) - np.asarray(pts[i - 1]))
    d = sum(cds[1:-1])
    return [sum(cds[0:i + 1]) / d for i in range(n)]


def _surface_params(points, su, sv):
    """nurbs_fitting.py:201-244: the averaged u and v parameters of the point grid."""
    ut = []
    for v in range(sv):
        ut += _chord_params([points[v + sv * u] for u in range(su)])
    uk = [sum(ut[u + su * v] for v in range(sv)) / sv for u in range(su)]
    vt = []
    for u in range(su):
        vt += _chord_params([points[v + sv * u] for v in range(sv)])
    vl = [sum(vt[v + sv * u] for u in range(su)) / su for v in range(sv)]
    return uk, vl


def _knots(p, n_data, n_ctrl, params):
    """nurbs_fitting.py:137-164 (eqs. 9.68-9.69)."""
    kv = [0.0] * (p + 1)
    d = float(n_data) / float(n_ctrl - p)
    for j in range(1, n_ctrl - p):
        i = int(j * d)
        a = (j * d) - i
        kv.append(((1.0 - a) * params[i - 1]) + (a * params[i]))
    return kv + [1.0] * (p + 1)


def _lu_solve(A, B):
    """A X = B column by column through one LU factorisation (scipy.linalg.lu_factor /
    lu_solve, as nurbs_fitting.py:57, 87 solves each coordinate), NumPy's solve without
    SciPy."""
    try:
        from scipy.linalg import lu_factor, lu_solve
    except ImportError:  # pragma: no cover
        return np.linalg.solve(A, B)
    lu = lu_factor(A)
    return np.stack([lu_solve(lu, B[:, d]) for d in range(B.shape[1])], axis=1)


def _fit_rows(rows, params, p, kv, n_ctrl):
    """One direction of A9.7: the end points interpolated, the interior control points the
    least-squares solution of (N^T N) P = N^T R (nurbs_fitting.py:48-89 / 91-132)."""
    n_data = len(params)
    Nm = np.array([[_basis_one(p, kv, j, params[i]) for j in range(1, n_ctrl - 1)]
                   for i in range(1, n_data - 1)])
    NtN = Nm.T @ Nm
    out = []
    for row in rows:  # row: n_data points (lists of dim floats)
        p0, pm = row[0], row[-1]
        rk = []
        for i in range(1, n_data - 1):
            n0 = _basis_one(p, kv, 0, params[i])
            nn = _basis_one(p, kv, n_ctrl - 1, params[i])
            rk.append([a - b * n0 - c * nn for a, b, c in zip(row[i], p0, pm, strict=True)])
        dim = len(p0)
        R = [[0.0] * dim for _ in range(n_ctrl - 2)]
        for i in range(1, n_ctrl - 1):
            for d in range(dim):
                for k, pt in enumerate(rk):
                    R[i - 1][d] += pt[d] * _basis_one(p, kv, i, params[k + 1])
        X = _lu_solve(NtN, np.asarray(R, dtype=np.float64))
        out.append([list(p0)] + [list(x) for x in X] + [list(pm)])
    return out


def approximate_surface(points, su, sv, pu, pv):
    """nurbs_fitting.py:19-134: control net (nu = su - 1, nv = sv - 1) approximating the
    su x sv data points (row-major in v) with degrees pu, pv. Returns (P[3][nu][nv], U, V)."""
    nu, nv = su - 1, sv - 1
    uk, vl = _surface_params(points, su, sv)
    ku = _knots(pu, su, nu, uk)
    kv = _knots(pv, sv, nv, vl)
    # u direction, one fit per data column j: (nu) x (sv) intermediate points
    cols = [[points[j + sv * i] for i in range(su)] for j in range(sv)]
    tmp = _fit_rows(cols, uk, pu, ku, nu)  # tmp[j][i]
    # v direction, one fit per intermediate row i
    rows = [[tmp[j][i] for j in range(sv)] for i in range(nu)]
    net = _fit_rows(rows, vl, pv, kv, nv)  # net[i][j]
    P = np.transpose(np.asarray(net, dtype=np.float64), (2, 0, 1))
    return P, np.asarray(ku), np.asarray(kv)


def clamped_knots(n_ctrl, p):
    """The uniform clamped knot vector the reference forms when none is given
    (nurbs_geometry.py:153-166)."""
    return np.concatenate((np.zeros(p), np.linspace(0, 1, n_ctrl - p + 1), np.ones(p)))


def fit_standard(radius, conic, nx, ny, xc, yc, su, sv):
    """nurbs_geometry.py:840-885: a bicubic fit of the conic sag on the su x sv grid over
    [xc - nx, xc + nx] x [yc - ny, yc + ny]."""
    x = np.linspace(xc - nx, xc + nx, su)
    y = np.linspace(yc - ny, yc + ny, sv)
    X, Y = np.meshgrid(x, y)
    r2 = X**2 + Y**2
    Z = r2 / (radius * (1 + np.sqrt(1 - (1 + conic) * r2 / radius**2)))
    pts = np.stack((X.T, Y.T, Z.T), axis=0).reshape(3, -1).T.tolist()
    P, U, V = approximate_surface(pts, su, sv, 3, 3)
    return P, np.ones(P.shape[1:]), 3, 3, U, V


def fit_plane(nx, ny, xc, yc, su, sv):
    """nurbs_geometry.py:887-932: a flat bicubic net on the su x sv grid."""
    x = np.linspace(xc - nx, xc + nx, su)
    y = np.linspace(yc - ny, yc + ny, sv)
    X, Y = np.meshgrid(x, y)
    P = np.stack((X.T, Y.T, np.zeros_like(X).T), axis=0)
    return P, np.ones((su, sv)), 3, 3, clamped_knots(su, 3), clamped_knots(sv, 3)


# ---- parameter-space evaluation (host API): nurbs_basis_functions.py, nurbs_geometry.py
def basis(n, p, U, u):
    """nurbs_basis_functions.py:20-71 (eq. 2.5 over the whole table)."""
    u = np.atleast_1d(np.asarray(u, dtype=np.float64))
    m = n + p + 1
    N = np.zeros((p + 1, m, u.size))
    for i in range(m):
        N[0, i] = 1.0 * ((u >= U[i]) & (u < U[i + 1])) + 1.0 * ((u == U[-1]) & (i == n))
    for k in range(1, p + 1):
        m -= 1
        for i in range(m):
            d1, d2 = U[i + k] - U[i], U[i + k + 1] - U[i + 1]
            a = (u - U[i]) / d1 * N[k - 1, i] if d1 != 0 else 0.0
            b = (U[i + k + 1] - u) / d2 * N[k - 1, i + 1] if d2 != 0 else 0.0
            N[k, i] = a + b
    return N[p, :n + 1]


def basis_derivative(n, p, U, u, order):
    """nurbs_basis_functions.py:74-134 (eqs. 2.7 / 2.9)."""
    if order == 0:
        return basis(n, p, U, u)
    Nl = basis_derivative(n, p - 1, U, u, order - 1)
    Nl = np.concatenate((Nl, np.zeros((1, Nl.shape[1]))), axis=0)
    out = np.zeros((n + 1, Nl.shape[1]))
    for i in range(n + 1):
        d1, d2 = U[i + p] - U[i], U[i + p + 1] - U[i + 1]
        a = p * Nl[i] / d1 if d1 != 0 else 0.0
        b = p * Nl[i + 1] / d2 if d2 != 0 else 0.0
        out[i] = a - b
    return out


def _homogeneous(P, W):
    return np.concatenate((P * W[None], W[None]), axis=0)


def surface_derivatives(P, W, p, q, U, V, u, v, ku, kv):
    """nurbs_geometry.py:455-583: S^(k, l)(u, v) for k <= ku, l <= kv (eq. 4.20);
    [k][l] -> (ndim, N)."""
    Pw = _homogeneous(P, W)
    nu, nv = Pw.shape[1], Pw.shape[2]
    Aw = [[(np.sum(np.matmul(Pw, basis_derivative(nv - 1, q, V, v, l))
                   * basis_derivative(nu - 1, p, U, u, k)[None], axis=1)
            if k <= p and l <= q else np.zeros((Pw.shape[0], np.size(u))))
           for l in range(kv + 1)] for k in range(ku + 1)]
    rows = []
    for k in range(ku + 1):
        cols = []
        for L in range(kv + 1):
            t = Aw[k][L][:-1]
            for i in range(1, k + 1):
                t = t - comb(k, i) * Aw[i][0][-1] * rows[k - i][L]
            for j in range(1, L + 1):
                t = t - comb(L, j) * Aw[0][j][-1] * cols[L - j]
            for i in range(1, k + 1):
                for j in range(1, L + 1):
                    t = t - comb(k, i) * comb(L, j) * Aw[i][j][-1] * rows[k - i][L - j]
            cols.append(t / Aw[0][0][-1])
        rows.append(cols)
    return rows


def surface_point(P, W, p, q, U, V, u, v):
    """nurbs_geometry.py:309-374: the point S(u, v) (perspective map of eq. 4.15)."""
    Pw = _homogeneous(P, W)
    nu, nv = Pw.shape[1], Pw.shape[2]
    Sw = np.sum(np.matmul(Pw, basis(nv - 1, q, V, v)) * basis(nu - 1, p, U, u)[None], axis=1)
    return Sw[:-1] / Sw[-1]


def surface_normals(P, W, p, q, U, V, u, v):
    """nurbs_geometry.py:585-604: cross(S_u, S_v) / |cross(S_u, S_v)|."""
    D = surface_derivatives(P, W, p, q, U, V, u, v, 1, 1)
    n = np.cross(D[1][0], D[0][1], axisa=0, axisb=0, axisc=0)
    return n / np.sum(n**2, axis=0) ** 0.5


def lowered_block(P, W, p, q, U, V):
    """The coefficient block of the lowered surface (layout in the module docstring)."""
    P = np.asarray(P, dtype=np.float64)
    W = np.asarray(W, dtype=np.float64)
    if P.ndim != 3 or P.shape[0] != 3:
        raise ValueError("NURBS control points must have shape (3, n+1, m+1)")
    nu, nv = P.shape[1], P.shape[2]
    if W.shape != (nu, nv):
        raise ValueError(f"NURBS weights must have shape {(nu, nv)}")
    p, q = int(p), int(q)
    U = np.asarray(U, dtype=np.float64).ravel()
    V = np.asarray(V, dtype=np.float64).ravel()
    if U.size != nu + p + 1 or V.size != nv + q + 1:
        raise ValueError("NURBS knot vectors must have n + p + 2 and m + q + 2 entries")
    if not (1 <= p <= MAX_DEGREE and 1 <= q <= MAX_DEGREE):
        raise ValueError(f"NURBS degrees 1..{MAX_DEGREE} are lowered (got {p}, {q})")
    for K, d in ((U, p), (V, q)):  # the kernels evaluate the span's window (ort_nurbs.h)
        if np.any(np.diff(K) < 0) or np.any(K[:d + 1] != K[0]) or np.any(K[-d - 1:] != K[-1]):
            raise ValueError("NURBS knot vectors must be non-decreasing and clamped "
                             "(first and last degree + 1 knots equal)")
    Pw = _homogeneous(P, W)
    return [float(p), float(q), float(nu), float(nv), *U.tolist(), *V.tolist(),
            *Pw.ravel().tolist()]
