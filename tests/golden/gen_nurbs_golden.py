"""NURBS golden vectors: the REFERENCE's NurbsGeometry (optiland/geometries/nurbs/*.py)
fitted and evaluated on the inputs of its own tests (tests/test_nurbs_geometry.py: radius
100, conic -1, 20 x 20 fit window, 10 x 10 points) plus seeded random points and rays on
four more surfaces (an off-centre conic fit, a plane fit, an explicit rational B-spline
with non-uniform knots and weights).

Test infrastructure only, run in the build container (never on the GPU box):

    PYTHONPATH=tests/golden/shims:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_nurbs_golden.py

(tests/golden/shims/numba.py stands in for numba's @jit, which nurbs_basis_functions.py:3
imports: the functions then run as the plain NumPy code they are, as they do under the
reference's own torch backend, nurbs_basis_functions.py:8-14.)

Writes tests/golden/nurbs.npz (arrays "<case>/<name>") and nurbs.json (the specs). Per
case: the fitted / given control net (P, W, p, q, U, V), get_value and get_derivative on a
(u, v) grid, sag(x, y) and surface_normal at seeded points, and distance(rays) for seeded
rays (one reference call over all rays of the case). The reference restarts a diverging
(u, v) iteration from numpy.random values (nurbs_geometry.py:711-714); the generator seeds
numpy's generator; the points and rays that restarted are marked (`*_restarted`): they
converge to the same root from any restart, so they are compared like the rest.
"""

from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

import optiland.backend as be  # noqa: E402
from optiland.coordinate_system import CoordinateSystem  # noqa: E402
from optiland.geometries.nurbs.nurbs_geometry import NurbsGeometry  # noqa: E402

be.set_backend("numpy")


def _explicit_net():
    """A 6 x 5 rational control net over [-6, 6] x [-5, 5]: a weak bowl with an xy twist,
    non-uniform weights, u degree 3 / v degree 2 on clamped non-uniform knots."""
    xs = np.linspace(-6.0, 6.0, 6)
    ys = np.linspace(-5.0, 5.0, 5)
    X, Y = np.meshgrid(xs, ys, indexing="ij")
    Z = (X**2 + Y**2) / 90.0 + 0.004 * X * Y - 0.01 * Y
    W = 1.0 + 0.15 * np.cos(0.7 * X) * np.sin(0.5 * Y + 0.3)
    U = [0.0, 0.0, 0.0, 0.0, 0.35, 0.6, 1.0, 1.0, 1.0, 1.0]
    V = [0.0, 0.0, 0.0, 0.45, 0.7, 1.0, 1.0, 1.0]
    return np.stack([X, Y, Z]), W, 3, 2, U, V


SPECS = {
    # tests/test_nurbs_geometry.py:18-93
    "fit_conic": dict(kind="fit", radius=100.0, conic=-1.0, nurbs_norm_x=20.0,
                      nurbs_norm_y=20.0, n_points_u=10, n_points_v=10, window=17.0),
    "fit_offcentre": dict(kind="fit", radius=-50.0, conic=0.3, nurbs_norm_x=12.0,
                          nurbs_norm_y=9.0, x_center=1.5, y_center=-2.0, n_points_u=6,
                          n_points_v=8, window=7.0),
    "fit_sphere": dict(kind="fit", radius=40.0, conic=0.0, nurbs_norm_x=8.0,
                       nurbs_norm_y=8.0, n_points_u=8, n_points_v=8, window=7.0),
    "fit_plane": dict(kind="fit", radius=float("inf"), conic=0.0, nurbs_norm_x=5.0,
                      nurbs_norm_y=5.0, n_points_u=4, n_points_v=4, window=4.5),
    "explicit": dict(kind="explicit", window=4.5),
}


def build(spec):
    cs = CoordinateSystem()
    if spec["kind"] == "fit":
        g = NurbsGeometry(cs, radius=spec["radius"], conic=spec["conic"],
                          nurbs_norm_x=spec["nurbs_norm_x"], nurbs_norm_y=spec["nurbs_norm_y"],
                          x_center=spec.get("x_center", 0.0), y_center=spec.get("y_center", 0.0),
                          n_points_u=spec["n_points_u"], n_points_v=spec["n_points_v"])
        g.fit_surface()
        return g
    P, W, p, q, U, V = _explicit_net()
    return NurbsGeometry(cs, control_points=P, weights=W, u_degree=p, v_degree=q,
                         u_knots=np.asarray(U), v_knots=np.asarray(V), tol=1e-10)


class _Rays:
    def __init__(self, x, y, z=None, L=None, M=None, N=None):
        self.x, self.y, self.z, self.L, self.M, self.N = x, y, z, L, M, N


def _restarted(call):
    """Run `call` twice: with numpy.random.rand answering NaN (the reference draws one value
    per iteration whether or not any (u, v) left the unit square, nurbs_geometry.py:711-714,
    so the points that restarted come out NaN) and then with the seeded generator (the
    recorded result). Returns (result, mask of the points that needed a restart)."""
    orig = be.rand
    be.rand = lambda *a, **k: float("nan")
    try:
        probe = call()
    finally:
        be.rand = orig
    out = call()
    first = probe[0] if isinstance(probe, tuple) else probe
    return out, ~np.isfinite(np.asarray(first, dtype=np.float64))


def case(name, spec, rng):
    g = build(spec)
    out = {"P": np.asarray(g.P, dtype=np.float64), "W": np.asarray(g.W, dtype=np.float64),
           "U": np.asarray(g.U, dtype=np.float64), "V": np.asarray(g.V, dtype=np.float64),
           "pq": np.array([g.p, g.q], dtype=np.int64)}
    uv = np.array([0.0, 0.13, 0.5, 0.77, 1.0])
    uu, vv = [a.ravel() for a in np.meshgrid(uv, uv, indexing="ij")]
    uu = np.concatenate([uu, rng.uniform(0, 1, 16)])
    vv = np.concatenate([vv, rng.uniform(0, 1, 16)])
    out["u"], out["v"] = uu, vv
    out["value"] = np.asarray(g.get_value(uu, vv), dtype=np.float64)
    for ou, ov in ((1, 0), (0, 1), (1, 1), (2, 0), (0, 2)):
        out[f"d{ou}{ov}"] = np.asarray(g.get_derivative(uu, vv, ou, ov), dtype=np.float64)
    out["normals_uv"] = np.asarray(g.get_normals(uu, vv), dtype=np.float64)
    w = spec["window"]
    xc, yc = spec.get("x_center", 0.0), spec.get("y_center", 0.0)
    base = [(0.0, 0.0), (10.0, 0.0)] if name == "fit_conic" else []
    pts = rng.uniform(-w, w, size=(2, 48))
    x = np.concatenate([[b[0] for b in base], xc + pts[0]])
    y = np.concatenate([[b[1] for b in base], yc + pts[1]])
    out["x"], out["y"] = x, y
    sag, r1 = _restarted(lambda: g.sag(x, y))
    nrm, r2 = _restarted(lambda: g.surface_normal(_Rays(x, y)))
    out["sag"] = np.asarray(sag, dtype=np.float64)
    out["normal"] = np.stack([np.asarray(c, dtype=np.float64) for c in nrm])
    # rays from z0 below the surface, small tilts, landing inside the window
    nr = 48
    p0 = rng.uniform(-0.8 * w, 0.8 * w, size=(2, nr))
    z0 = np.full(nr, -5.0) + rng.uniform(-1, 1, nr)
    L = rng.uniform(-0.06, 0.06, nr)
    M = rng.uniform(-0.06, 0.06, nr)
    N = np.sqrt(1.0 - L * L - M * M)
    rays = _Rays(xc + p0[0], yc + p0[1], z0, L, M, N)
    dist, r3 = _restarted(lambda: g.distance(rays))
    out["rx"], out["ry"], out["rz"] = rays.x, rays.y, rays.z
    out["rL"], out["rM"], out["rN"] = L, M, N
    out["distance"] = np.asarray(dist, dtype=np.float64)
    if name == "fit_conic":  # tests/test_nurbs_geometry.py:78-93: one axial ray from z = -10
        one = _Rays(np.zeros(1), np.zeros(1), np.full(1, -10.0), np.zeros(1), np.zeros(1),
                    np.ones(1))
        out["distance_axial"] = np.asarray(g.distance(one), dtype=np.float64)
    out["sag_restarted"], out["distance_restarted"] = r1 | r2, r3
    assert np.all(np.isfinite(out["sag"])) and np.all(np.isfinite(out["distance"])), name
    print(name, "restarted points:", int(np.sum(r1 | r2)), "rays:", int(np.sum(r3)))
    return out


def main():
    np.random.seed(20251018)
    rng = np.random.default_rng(7)
    arrays = {}
    for name, spec in SPECS.items():
        for k, v in case(name, spec, rng).items():
            arrays[f"{name}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "nurbs.npz"), **arrays)
    with open(os.path.join(HERE, "nurbs.json"), "w") as f:
        json.dump({k: {kk: (None if isinstance(vv, float) and np.isinf(vv) else vv)
                       for kk, vv in v.items()} for k, v in SPECS.items()}, f, indent=1)
    print("wrote nurbs.npz:", len(arrays), "arrays")


if __name__ == "__main__":
    main()
