"""Forbes Q-polynomial tables (host side of ForbesQbfsGeometry / ForbesQ2dGeometry).

The reference (geometries/forbes/qpoly.py, after prysm) evaluates Q-bfs and Q-2D sums by
Clenshaw recurrences whose coefficients -- the orthonormalisation constants f, g, h
(Q-bfs) and F, G, gamma (Q-2D), the three-term recurrence A, B, C, and the change of
basis from the user's Q coefficients to the orthonormal P coefficients -- depend only on
the lens, not on the ray. They are formed here once per lowering, with the reference's
arithmetic (same Python / NumPy scalar operations in the same order, so the same
doubles), and handed to the kernel in the surface's coefficient block; the kernel only
runs the per-ray recurrences (csrc/ort_core.h sagnorm_qbfs / sagnorm_q2d).
"""

from __future__ import annotations

import functools
from collections import defaultdict

import numpy as np
from scipy import special


# ---- Q-bfs: qpoly.py:60-90 -------------------------------------------------------------
@functools.lru_cache(maxsize=None)
def qbfs_f(n: int):
    if n == 0:
        return 2.0
    if n == 1:
        return np.sqrt(19) / 2
    return np.sqrt(float(n * (n + 1) + 3) - qbfs_g(n - 1) ** 2 - qbfs_h(n - 2) ** 2)


@functools.lru_cache(maxsize=None)
def qbfs_g(k: int):
    """g_{k} (the reference's g_qbfs(n_minus_1 = k))."""
    if k == 0:
        return -1 / 2
    return -(1 + qbfs_g(k - 1) * qbfs_h(k - 1)) / qbfs_f(k)


@functools.lru_cache(maxsize=None)
def qbfs_h(k: int):
    """h_{k} (the reference's h_qbfs(n_minus_2 = k)); n = k + 2."""
    n = k + 2
    return -n * (n - 1) / (2 * qbfs_f(k))


def qbfs_to_pn(cs) -> list:
    """Q-bfs coefficients -> orthonormal P_n coefficients (qpoly.py:93-124): a backward
    solve of the bidiagonal-plus-one system f, g, h."""
    cs = [np.float64(c) for c in cs]
    m = len(cs) - 1
    if m < 0:
        return []
    b = [0.0] * (m + 1)
    b[m] = cs[m] / qbfs_f(m)
    if m == 0:
        return [float(v) for v in b]
    b[m - 1] = (cs[m - 1] - qbfs_g(m - 1) * b[m]) / qbfs_f(m - 1)
    for i in range(m - 2, -1, -1):
        b[i] = (cs[i] - qbfs_g(i) * b[i + 1] - qbfs_h(i) * b[i + 2]) / qbfs_f(i)
    return [float(v) for v in b]


# ---- Q-2D: qpoly.py:263-380 ------------------------------------------------------------
@functools.lru_cache(maxsize=None)
def q2d_gamma(n: int, m: int):
    if n == 1 and m == 2:
        return 3 / 8
    if n == 1 and m > 2:
        k = m - 1
        return ((2 * k + 1) / (2 * (k - 1))) * q2d_gamma(1, k)
    k = n - 1
    return (((k + 1) * (2 * m + 2 * k - 1)) / ((m + k - 2) * (2 * k + 1))) * q2d_gamma(k, m)


def _delta(i, j):
    return 1 if i == j else 0


@functools.lru_cache(maxsize=None)
def q2d_G(n: int, m: int):
    if n == 0:
        return special.factorial2(2 * m - 1) / (2 ** (m + 1) * special.factorial(m - 1))
    if m == 1:
        return (-((2 * n**2 - 1) * (n**2 - 1)) / (8 * (4 * n**2 - 1))
                - 1 / 24 * _delta(n, 1))
    num = (2 * n * (m + n - 1) - m) * ((n + 1) * (2 * m + 2 * n - 1))
    den = ((m + 2 * n - 2) * (m + 2 * n - 1)) * ((m + 2 * n) * (2 * n + 1))
    return (-num / den) * q2d_gamma(n, m)


@functools.lru_cache(maxsize=None)
def q2d_F(n: int, m: int):
    if n == 0 and m == 1:
        return 0.25
    if n == 0:
        return m**2 * special.factorial2(2 * m - 3) / (2 ** (m + 1) * special.factorial(m - 1))
    if m == 1:
        return ((4 * (n - 1) ** 2 * n**2 + 1) / (8 * (2 * n - 1) ** 2)
                + 11 / 32 * _delta(n, 1))
    chi = m + n - 2
    num = 2 * n * chi * (3 - 5 * m + 4 * n * chi) + m**2 * (3 - m + 4 * n * chi)
    den = ((m + 2 * n - 3) * (m + 2 * n - 2)) * ((m + 2 * n - 1) * (2 * n - 1))
    return (num / den) * q2d_gamma(n, m)


@functools.lru_cache(maxsize=None)
def q2d_f(n: int, m: int):
    if n == 0:
        return np.sqrt(q2d_F(0, m))
    return np.sqrt(q2d_F(n, m) - q2d_g(n - 1, m) ** 2)


@functools.lru_cache(maxsize=None)
def q2d_g(n: int, m: int):
    return q2d_G(n, m) / q2d_f(n, m)


def q2d_to_pnm(cns, m: int) -> list:
    """Q-2D coefficients of one azimuthal order -> orthonormal P_n^m coefficients
    (qpoly.py:337-355): a backward bidiagonal solve."""
    m = abs(m)
    top = len(cns) - 1
    if top < 0:
        return []
    d = [0.0] * (top + 1)
    d[top] = cns[top] / q2d_f(top, m)
    for n in range(top - 1, -1, -1):
        d[n] = (cns[n] - q2d_g(n, m) * d[n + 1]) / q2d_f(n, m)
    return [float(v) for v in d]


_ABC_SPECIAL = {  # (m, n) -> (A, B, C), qpoly.py:358-364
    (1, 0): (2, -1, 0),
    (1, 1): (-4 / 3, -8 / 3, -11 / 3),
    (1, 2): (9 / 5, -24 / 5, 0),
    (2, 0): (3, -2, 0),
    (3, 0): (5, -4, 0),
}


def q2d_abc(n: int, m: int):
    """Three-term recurrence coefficients (qpoly.py:367-386), special cases first."""
    if (m, n) in _ABC_SPECIAL:
        return tuple(float(v) for v in _ABC_SPECIAL[(m, n)])
    d = (4 * n**2 - 1) * (m + n - 2) * (m + 2 * n - 3)
    if d == 0:
        d = 1e-99
    a = ((2 * n - 1) * (m + 2 * n - 2) * (4 * n * (m + n - 2) + (m - 3) * (2 * m - 1))) / d
    b = (-2 * (2 * n - 1) * (m + 2 * n - 3) * (m + 2 * n - 2) * (m + 2 * n - 1)) / d
    c = (n * (2 * n - 3) * (m + 2 * n - 1) * (2 * m + 2 * n - 3)) / d
    return float(a), float(b), float(c)


def q2d_split(freeform_coeffs: dict):
    """Zemax-style {('a'|'b', m, n): c} -> (cm0, ams, bms) (forbes/geometry.py:382-418 +
    qpoly.py:585-613): m = 0 terms, then per azimuthal order 1..M the cosine and sine
    radial lists, zero-padded; an order with no terms has an empty list."""
    internal = {}
    for key, value in (freeform_coeffs or {}).items():
        kind, i1, i2 = key
        kind = str(kind).lower()
        if kind == "a":
            internal[(int(i2), int(i1))] = value
        elif kind == "b":
            internal[(int(i2), int(i1), "sin")] = value
    order = sorted(internal, key=lambda k: (k[0], abs(k[1]), 0 if len(k) == 2 else 1))
    cms, ac, bc = [], defaultdict(list), defaultdict(list)
    for key in order:
        n, m = key[0], (-key[1] if len(key) == 3 else key[1])
        c = internal[key]
        if m == 0:
            cms.extend([0.0] * (n + 1 - len(cms)))
            cms[n] = c
            continue
        lst = ac[abs(m)] if m > 0 else bc[abs(m)]
        lst.extend([0.0] * (n + 1 - len(lst)))
        lst[n] = c
    top = max([0] + list(ac) + list(bc))
    return cms, [ac.get(i, []) for i in range(1, top + 1)], [bc.get(i, []) for i in range(1, top + 1)]


def q2d_sum_at_zero(cns, m: int):
    """Clenshaw sum of one azimuthal order at u^2 = 0 (the vertex-slope constant,
    forbes/geometry.py:530-543): 0.5 alpha_0 (- 2/5 alpha_3 for m = 1 with > 3 terms)."""
    d = q2d_to_pnm(cns, m)
    top = len(d) - 1
    al = np.zeros(len(d))
    if top < 0:
        return 0.5 * al[0] if len(al) else 0.0
    al[top] = d[top]
    if top > 0:
        a, b, _ = q2d_abc(top - 1, m)
        al[top - 1] = d[top - 1] + (a + b * 0.0) * al[top]
    for n in range(top - 2, -1, -1):
        a, b, _ = q2d_abc(n, m)
        c = q2d_abc(n + 1, m)[2]
        al[n] = d[n] + (a + b * 0.0) * al[n + 1] - c * al[n + 2]
    s = 0.5 * al[0]
    if m == 1 and len(cns) - 1 > 2:
        s -= 2 / 5 * al[3]
    return s


def q2d_order_block(cns, m: int) -> list:
    """One azimuthal order's Clenshaw record: L, then d_0..d_{L-1} (P^m basis),
    A_0..A_{L-1}, B_0..B_{L-1}, C_0..C_{L-1} (A/B/C at index n for recurrence step n)."""
    L = len(cns)
    if L == 0:
        return [0.0]
    d = q2d_to_pnm(cns, m)
    abc = [q2d_abc(n, m) for n in range(L)]
    return ([float(L)] + d + [v[0] for v in abc] + [v[1] for v in abc]
            + [v[2] for v in abc])
