"""Shared helpers: the per-geometry golden cases (tests/golden/geometry.{json,npz}, made
by gen_geometry_golden.py from the reference) rebuilt with the NATIVE host API."""

import json
import os

import numpy as np

from optiland_pr_amd.coordinate_system import CoordinateSystem
from optiland_pr_amd.geometries import (
    EvenAsphere,
    OddAsphere,
    Plane,
    StandardGeometry,
    ZernikePolynomialGeometry,
)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def specs():
    with open(os.path.join(GOLDEN, "geometry.json")) as f:
        return json.load(f)


def arrays(name):
    d = np.load(os.path.join(GOLDEN, "geometry.npz"), allow_pickle=False)
    return {k.split("/", 1)[1]: d[k] for k in d.files if k.startswith(name + "/")}


def build(spec):
    cs = CoordinateSystem()
    k = spec["kind"]
    if k == "plane":
        return Plane(cs)
    if k == "standard":
        return StandardGeometry(cs, radius=spec["radius"], conic=spec["conic"])
    if k == "even_asphere":
        return EvenAsphere(cs, radius=spec["radius"], conic=spec["conic"],
                           coefficients=spec["coefficients"])
    if k == "odd_asphere":
        return OddAsphere(cs, radius=spec["radius"], conic=spec["conic"],
                          coefficients=spec["coefficients"])
    if k == "zernike":
        return ZernikePolynomialGeometry(cs, radius=spec["radius"], conic=spec["conic"],
                                         coefficients=spec["coefficients"],
                                         norm_radius=spec["norm_radius"],
                                         zernike_type=spec["zernike_type"])
    raise ValueError(k)


CASES = sorted(specs())
NEWTON_KINDS = ("even_asphere", "odd_asphere", "zernike")
