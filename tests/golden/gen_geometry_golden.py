"""Per-geometry golden vectors: the REFERENCE's geometries (optiland/geometries/*.py)
evaluated on the inputs of its own geometry tests (tests/test_geometries.py:23-1230:
same constructor arguments, points and rays) plus seeded random points and rays.

Test infrastructure only, run in the build container (never on the GPU box):

    PYTHONPATH=tests/golden/shims:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_geometry_golden.py

Writes tests/golden/geometry.npz (arrays "<case>/<name>") and geometry.json (the
geometry specs). Every case records sag(x, y) and the normal at (x, y) for its points,
and distance(rays) for its rays (one reference call over all rays of the case, so the
Newton global stop rule spans them).
"""

from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

import optiland.backend as be  # noqa: E402
from optiland import geometries  # noqa: E402
from optiland.coordinate_system import CoordinateSystem  # noqa: E402
from optiland.rays import RealRays  # noqa: E402

be.set_backend("numpy")


def _coeffs(d, kind):
    start = 0 if kind == "standard" else 1
    return [d.get(i, 0.0) for i in range(start, max(d) + 1 + start)]


# name: (spec, extra literal points from the reference tests)
SPECS = {
    "plane": dict(kind="plane"),
    "sphere": dict(kind="standard", radius=10.0, conic=0.0),
    "parabola": dict(kind="standard", radius=-20.0, conic=-1.0),
    "conic": dict(kind="standard", radius=27.0, conic=0.5),
    "even_sag": dict(kind="even_asphere", radius=27.0, conic=0.0, coefficients=[1e-3, -1e-5]),
    "even_dist": dict(kind="even_asphere", radius=-41.1, conic=0.0,
                      coefficients=[1e-3, -1e-5, 1e-7]),
    "even_norm": dict(kind="even_asphere", radius=10.0, conic=0.5, coefficients=[1e-2]),
    "odd_sag": dict(kind="odd_asphere", radius=27.0, conic=0.0, coefficients=[1e-3, -1e-5]),
    "odd_dist": dict(kind="odd_asphere", radius=-41.1, conic=0.0,
                     coefficients=[1e-3, -1e-5, 1e-7]),
    "odd_norm": dict(kind="odd_asphere", radius=10.0, conic=0.5, coefficients=[1e-2, -1e-5]),
    "zern_standard": dict(kind="zernike", radius=22.0, conic=0.0, norm_radius=10.0,
                          zernike_type="standard",
                          coefficients=_coeffs({4: 0.5, 3: 0.2, 5: 0.3, 10: 0.1, 12: 0.2},
                                               "standard")),
    "zern_noll": dict(kind="zernike", radius=22.0, conic=0.0, norm_radius=10.0,
                      zernike_type="noll",
                      coefficients=_coeffs({4: 0.5, 5: 0.2, 6: 0.3, 11: 0.2, 15: 0.1}, "noll")),
    "zern_fringe": dict(kind="zernike", radius=22.0, conic=0.0, norm_radius=10.0,
                        zernike_type="fringe",
                        coefficients=_coeffs({4: 0.5, 6: 0.2, 11: 0.3, 13: 0.2, 27: 0.1},
                                             "fringe")),
    "zern_fringe_conic": dict(kind="zernike", radius=-50.0, conic=-0.8, norm_radius=12.0,
                              zernike_type="fringe",
                              coefficients=[0.0, 1e-3, -2e-3, 5e-3, 1e-3, 0.0, 2e-4, -1e-4]),
    "poly_sag": dict(kind="polynomial", radius=22.0, conic=0.0,
                     coefficients=[[0.0, 1e-2, -2e-3], [0.1, 1e-2, -1e-3], [0.2, 1e-2, 0.0]]),
    "poly_dist": dict(kind="polynomial", radius=-26.0, conic=0.1,
                      coefficients=[[0.0, 1e-2, 2e-3], [0.1, -1e-2, 1e-3], [0.2, 1e-2, 2e-4]]),
    "poly_1d": dict(kind="polynomial", radius=40.0, conic=-0.3,
                    coefficients=[0.0, 2e-3, 1e-4, -3e-6]),
    "cheb_sag": dict(kind="chebyshev", radius=22.0, conic=0.0, norm_x=10.0, norm_y=10.0,
                     coefficients=[[0.0, 1e-2, -2e-3], [0.1, 1e-2, -1e-3], [0.2, 1e-2, 0.0]]),
    "cheb_dist": dict(kind="chebyshev", radius=-26.0, conic=0.1, norm_x=10.0, norm_y=10.0,
                      coefficients=[[0.0, 1e-2, -2e-3], [0.1, 1e-2, -1e-3], [0.2, 1e-2, 0.0]]),
    "biconic": dict(kind="biconic", radius_x=10.0, radius_y=20.0, conic_x=0.5, conic_y=-0.5),
    "biconic_conics": dict(kind="biconic", radius_x=10.0, radius_y=20.0, conic_x=-1.0,
                           conic_y=0.5),
    "biconic_rx_inf": dict(kind="biconic", radius_x=float("inf"), radius_y=20.0,
                           conic_x=0.0, conic_y=0.0),
    "biconic_ry_inf": dict(kind="biconic", radius_x=-15.0, radius_y=float("inf"),
                           conic_x=0.2, conic_y=0.0),
    "toroid": dict(kind="toroidal", radius_x=100.0, radius_y=50.0, conic=-0.5,
                   coeffs_poly_y=[1e-5]),
    "toroid_cyl_x": dict(kind="toroidal", radius_x=float("inf"), radius_y=-50.0, conic=0.0,
                         coeffs_poly_y=[]),
    "toroid_cyl_y": dict(kind="toroidal", radius_x=100.0, radius_y=float("inf"), conic=0.0,
                         coeffs_poly_y=[]),
    "toroid_no_x": dict(kind="toroidal", radius_x=float("inf"), radius_y=50.0, conic=-1.1,
                        coeffs_poly_y=[1e-5, -2e-6]),
    "toroid_no_y": dict(kind="toroidal", radius_x=100.0, radius_y=float("inf"), conic=-0.9,
                        coeffs_poly_y=[1e-5, -2e-6]),
    "toroid_neg": dict(kind="toroidal", radius_x=-30.0, radius_y=-20.0, conic=0.3,
                       coeffs_poly_y=[2e-5, 1e-7]),
    # Forbes (tests/test_geometries.py:2103-2720): radial_terms as [n, c] pairs,
    # freeform_coeffs as [kind, m, n, c] (JSON has no tuple keys)
    "qbfs_zemax": dict(kind="forbes_qbfs", radius=21.723, conic=-4.428, norm_radius=6.336,
                       radial_terms=[[0, 1.614], [1, 0.348], [2, 0.150], [3, 0.033],
                                     [4, 0.030]]),
    "qbfs_plane_base": dict(kind="forbes_qbfs", radius=float("inf"), conic=0.0,
                            norm_radius=10.0, radial_terms=[[1, 1e-3]]),
    "qbfs_small": dict(kind="forbes_qbfs", radius=22.0, conic=-4.428, norm_radius=6.336,
                       radial_terms=[[0, 1.6e-4], [1, 0.3e-4], [2, 0.15e-4]]),
    "qbfs_sparse": dict(kind="forbes_qbfs", radius=50.0, conic=-1.0, norm_radius=10.0,
                        radial_terms=[[2, 1e-4]]),
    "qbfs_zero": dict(kind="forbes_qbfs", radius=-35.0, conic=0.3, norm_radius=8.0,
                      radial_terms=[[0, 0.0], [1, 0.0]]),
    "q2d_mixed": dict(kind="forbes_q2d", radius=50.0, conic=0.0, norm_radius=10.0,
                      freeform_coeffs=[["a", 0, 0, 1e-3], ["a", 0, 1, -2e-4],
                                       ["a", 1, 1, 2e-4], ["b", 1, 1, 3e-4],
                                       ["a", 2, 0, 1e-4], ["b", 3, 2, -5e-5],
                                       ["a", 1, 4, 1e-5], ["a", 1, 0, 4e-4]]),
    "q2d_dict": dict(kind="forbes_q2d", radius=123.4, conic=-0.9, norm_radius=45.6,
                     freeform_coeffs=[["a", 2, 2, 1e-4], ["b", 1, 1, -5e-5]]),
    "q2d_conic": dict(kind="forbes_q2d", radius=-40.0, conic=0.5, norm_radius=8.0,
                      freeform_coeffs=[["a", 1, 1, 3e-4], ["a", 1, 3, -1e-4],
                                       ["b", 1, 0, 2e-4], ["b", 2, 1, 1e-4],
                                       ["a", 4, 0, 5e-5], ["a", 0, 2, 2e-4]]),
    "q2d_sine_only": dict(kind="forbes_q2d", radius=100.0, conic=0.0, norm_radius=10.0,
                          freeform_coeffs=[["b", 1, 1, 1e-3]]),
}


SPECS["grid_tilt"] = dict(kind="grid_sag", x=[-1.0, 1.0], y=[-1.0, 1.0],  # test_grid_sag_geometry.py:49-76
                          sag=[[-0.1, 0.1], [-0.1, 0.1]])
SPECS["grid_bowl"] = dict(kind="grid_sag", x=[-9.0, -7.875, -6.75, -5.625, -4.5, -3.375, -2.25, -1.125, 0.0, 1.125, 2.25, 3.375, 4.5, 5.625, 6.75, 7.875, 9.0], y=[-7.0, -5.833333333333333, -4.666666666666666, -3.5, -2.333333333333333, -1.166666666666666, 0.0, 1.1666666666666679, 2.333333333333334, 3.5, 4.666666666666668, 5.833333333333334, 7.0], sag=[[2.796, 2.4005625, 2.05575, 1.7615625000000001, 1.518, 1.3250625, 1.1827500000000002, 1.0910625, 1.05, 1.0595625, 1.11975, 1.2305625, 1.3920000000000001, 1.6040625, 1.8667500000000001, 2.1800624999999996, 2.544], [2.4638888888888886, 2.071076388888889, 1.728888888888889, 1.4373263888888888, 1.1963888888888887, 1.0060763888888888, 0.8663888888888888, 0.7773263888888888, 0.7388888888888888, 0.7510763888888887, 0.8138888888888888, 0.9273263888888887, 1.0913888888888887, 1.3060763888888887, 1.5713888888888887, 1.887326388888889, 2.2538888888888886], [2.1862222222222223, 1.796034722222222, 1.456472222222222, 1.167534722222222, 0.9292222222222221, 0.741534722222222, 0.6044722222222221, 0.5180347222222221, 0.4822222222222221, 0.4970347222222221, 0.562472222222222, 0.6785347222222221, 0.845222222222222, 1.0625347222222221, 1.330472222222222, 1.6490347222222221, 2.018222222222222], [1.9629999999999999, 1.5754375, 1.2385, 0.9521875000000001, 0.7165, 0.5314375, 0.397, 0.31318750000000006, 0.28, 0.2974375, 0.36550000000000005, 0.4841875, 0.6535000000000001, 0.8734375, 1.144, 1.4651874999999999, 1.837], [1.7942222222222224, 1.4092847222222225, 1.0749722222222224, 0.7912847222222221, 0.5582222222222222, 0.37578472222222215, 0.2439722222222222, 0.16278472222222218, 0.13222222222222219, 0.15228472222222217, 0.22297222222222218, 0.3442847222222222, 0.5162222222222221, 0.7387847222222221, 1.0119722222222223, 1.3357847222222223, 1.7102222222222223], [1.679888888888889, 1.297576388888889, 0.9658888888888889, 0.6848263888888888, 0.4543888888888889, 0.2745763888888889, 0.14538888888888887, 0.06682638888888885, 0.038888888888888855, 0.06157638888888886, 0.13488888888888886, 0.2588263888888889, 0.4333888888888889, 0.6585763888888889, 0.9343888888888888, 1.2608263888888889, 1.6378888888888892], [1.62, 1.2403125, 0.91125, 0.6328125, 0.405, 0.2278125, 0.10125, 0.0253125, 0.0, 0.0253125, 0.10125, 0.2278125, 0.405, 0.6328125, 0.91125, 1.2403125, 1.62], [1.6145555555555555, 1.2374930555555554, 0.9110555555555555, 0.6352430555555555, 0.4100555555555556, 0.23549305555555558, 0.1115555555555556, 0.03824305555555559, 0.015555555555555597, 0.0434930555555556, 0.12205555555555561, 0.25124305555555565, 0.43105555555555564, 0.6614930555555556, 0.9425555555555556, 1.2742430555555555, 1.6565555555555558], [1.6635555555555555, 1.2891180555555555, 0.9653055555555556, 0.6921180555555557, 0.4695555555555556, 0.29761805555555565, 0.17630555555555558, 0.10561805555555559, 0.0855555555555556, 0.1161180555555556, 0.1973055555555556, 0.3291180555555556, 0.5115555555555557, 0.7446180555555557, 1.0283055555555556, 1.3626180555555556, 1.7475555555555555], [1.7670000000000001, 1.3951875, 1.074, 0.8034374999999999, 0.5835, 0.41418750000000004, 0.2955, 0.2274375, 0.21, 0.24318750000000003, 0.32699999999999996, 0.46143750000000006, 0.6465, 0.8821875, 1.1685, 1.5054375000000002, 1.893], [1.924888888888889, 1.5557013888888889, 1.2371388888888892, 0.9692013888888891, 0.751888888888889, 0.5852013888888891, 0.46913888888888905, 0.40370138888888907, 0.3888888888888891, 0.4247013888888891, 0.5111388888888891, 0.648201388888889, 0.8358888888888891, 1.074201388888889, 1.3631388888888891, 1.7027013888888891, 2.092888888888889], [2.137222222222223, 1.7706597222222225, 1.4547222222222222, 1.1894097222222224, 0.9747222222222223, 0.8106597222222223, 0.6972222222222224, 0.6344097222222224, 0.6222222222222223, 0.6606597222222225, 0.7497222222222224, 0.8894097222222224, 1.0797222222222222, 1.3206597222222225, 1.6122222222222224, 1.9544097222222223, 2.3472222222222228], [2.4040000000000004, 2.0400625, 1.72675, 1.4640624999999998, 1.252, 1.0905624999999999, 0.9797499999999999, 0.9195625000000001, 0.9099999999999999, 0.9510624999999999, 1.04275, 1.1850625, 1.378, 1.6215625, 1.91575, 2.2605625000000003, 2.656]])


def _forbes(spec):
    cfg = dict(radius=spec["radius"], conic=spec["conic"], norm_radius=spec["norm_radius"])
    if spec["kind"] == "forbes_qbfs":
        cfg["terms"] = {int(n): c for n, c in spec["radial_terms"]}
    else:
        cfg["terms"] = {(k, int(m), int(n)): c for k, m, n, c in spec["freeform_coeffs"]}
    return cfg


def build(spec):
    cs = CoordinateSystem()
    k = spec["kind"]
    if k == "plane":
        return geometries.Plane(cs)
    if k == "standard":
        return geometries.StandardGeometry(cs, radius=spec["radius"], conic=spec["conic"])
    if k == "even_asphere":
        return geometries.EvenAsphere(cs, radius=spec["radius"], conic=spec["conic"],
                                      coefficients=spec["coefficients"])
    if k == "odd_asphere":
        return geometries.OddAsphere(cs, radius=spec["radius"], conic=spec["conic"],
                                     coefficients=spec["coefficients"])
    if k == "zernike":
        return geometries.ZernikePolynomialGeometry(
            cs, radius=spec["radius"], conic=spec["conic"], coefficients=spec["coefficients"],
            norm_radius=spec["norm_radius"], zernike_type=spec["zernike_type"])
    if k == "polynomial":
        return geometries.PolynomialGeometry(cs, radius=spec["radius"], conic=spec["conic"],
                                             coefficients=np.array(spec["coefficients"]))
    if k == "chebyshev":
        return geometries.ChebyshevPolynomialGeometry(
            cs, radius=spec["radius"], conic=spec["conic"],
            coefficients=np.array(spec["coefficients"]), norm_x=spec["norm_x"],
            norm_y=spec["norm_y"])
    if k == "biconic":
        return geometries.BiconicGeometry(cs, radius_x=spec["radius_x"],
                                          radius_y=spec["radius_y"], conic_x=spec["conic_x"],
                                          conic_y=spec["conic_y"])
    if k == "toroidal":
        return geometries.ToroidalGeometry(cs, radius_x=spec["radius_x"],
                                           radius_y=spec["radius_y"], conic=spec["conic"],
                                           coeffs_poly_y=spec["coeffs_poly_y"])
    if k in ("forbes_qbfs", "forbes_q2d"):
        cls = (geometries.ForbesQbfsGeometry if k == "forbes_qbfs"
               else geometries.ForbesQ2dGeometry)
        return cls(cs, geometries.ForbesSurfaceConfig(**_forbes(spec)))
    if k == "grid_sag":
        return geometries.GridSagGeometry(cs, spec["x"], spec["y"], spec["sag"])
    raise ValueError(k)


def points(name, spec, rng):
    """Sag/normal evaluation points: the reference tests' points + seeded random ones
    inside the surface's valid region."""
    if spec["kind"] == "zernike":
        g = np.linspace(-10, 10, 10) * spec["norm_radius"] / 10.0
        X, Y = np.meshgrid(g, g)  # test_geometries.py:888-905
        r = rng.uniform(-1, 1, size=(2, 64)) * spec["norm_radius"] / np.sqrt(2)
        return np.concatenate([X.ravel(), r[0]]), np.concatenate([Y.ravel(), r[1]])
    if spec["kind"] == "chebyshev":  # |x / norm| <= 1 (chebyshev.py:203-215)
        base_x = [0.0, 1.0, -2.0, 0.0, 3.0, 8.0, 1.0, -2.0]
        base_y = [0.0, 1.0, -7.0, 0.0, -7.0, 2.1, 2.0, 3.0]
        r = rng.uniform(-9.5, 9.5, size=(2, 64))
        return np.concatenate([base_x, r[0]]), np.concatenate([base_y, r[1]])
    base_x = [0.0, 1.0, -2.0, 0.0, 3.0, 8.0, 1.0, -2.0, 10.0, -5.0]
    base_y = [0.0, 1.0, 3.0, 0.0, -7.0, 2.1, 2.0, -7.0, 1.0, 1.0]
    rad = min([abs(spec[k]) for k in ("radius", "radius_x", "radius_y") if k in spec] + [100.0])
    lim = 4.0 if rad < 15 else 8.0
    r = rng.uniform(-lim, lim, size=(2, 64))
    return np.concatenate([base_x, r[0]]), np.concatenate([base_y, r[1]])


def rays(name, spec, rng):
    """Distance rays: the reference tests' rays (test_geometries.py:173-205, 275-310,
    695-720) + seeded random rays starting in front of the vertex."""
    x = [1.0, 1.0, 2.0, 1.0]
    y = [2.0, 2.0, 3.0, 2.0]
    z = [-3.0, -3.0, -4.0, -10.2]
    L0, M0 = 0.222, -0.229
    L = [0.0, 0.0, 0.0, L0]
    M = [0.0, 0.0, 0.0, M0]
    N = [1.0, 1.0, 1.0, float(np.sqrt(1 - L0**2 - M0**2))]
    n = 48
    lim = 2.5 if spec["kind"] in ("zernike", "biconic") else 3.0
    rx = rng.uniform(-lim, lim, n)
    ry = rng.uniform(-lim, lim, n)
    rz = rng.uniform(-6.0, -1.0, n)
    a = rng.uniform(-0.15, 0.15, (2, n))
    rn = np.sqrt(1 - a[0] ** 2 - a[1] ** 2)
    return (np.concatenate([x, rx]), np.concatenate([y, ry]), np.concatenate([z, rz]),
            np.concatenate([L, a[0]]), np.concatenate([M, a[1]]), np.concatenate([N, rn]))


def main():
    rng = np.random.default_rng(2024)
    arrays = {}
    for name, spec in SPECS.items():
        g = build(spec)
        px, py = points(name, spec, rng)
        arrays[f"{name}/x"] = px
        arrays[f"{name}/y"] = py
        arrays[f"{name}/sag"] = np.asarray(g.sag(px, py), dtype=np.float64) * np.ones_like(px)
        rr = RealRays(px, py, np.zeros_like(px), np.zeros_like(px), np.zeros_like(px),
                      np.ones_like(px), np.ones_like(px), np.ones_like(px))
        nx, ny, nz = g.surface_normal(rr)
        for k, v in (("nx", nx), ("ny", ny), ("nz", nz)):
            arrays[f"{name}/{k}"] = np.asarray(v, dtype=np.float64) * np.ones_like(px)
        rx, ry, rz, rL, rM, rN = rays(name, spec, rng)
        for k, v in (("rx", rx), ("ry", ry), ("rz", rz), ("rL", rL), ("rM", rM), ("rN", rN)):
            arrays[f"{name}/{k}"] = v
        rr = RealRays(rx, ry, rz, rL, rM, rN, np.ones_like(rx), np.ones_like(rx))
        arrays[f"{name}/t"] = np.asarray(g.distance(rr), dtype=np.float64) * np.ones_like(rx)
    np.savez_compressed(os.path.join(HERE, "geometry.npz"), **arrays)
    with open(os.path.join(HERE, "geometry.json"), "w") as f:
        json.dump(SPECS, f, indent=1)
    print(f"{len(SPECS)} geometry cases")


if __name__ == "__main__":
    main()
