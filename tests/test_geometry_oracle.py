"""Pin the oracle's per-geometry functions (oracle/trace_np.py) against the reference's
geometry outputs on the inputs of its own geometry tests (tests/golden/geometry.npz,
gen_geometry_golden.py): sag, surface normal and distance (Newton global stop rule over
all rays of a call) for plane, conic, even/odd asphere and the three Zernike schemes.
Bit-exact: the oracle evaluates the reference's expressions in the reference's order.
Also the reference test suite's literal numbers (tests/test_geometries.py).
"""

import numpy as np
import pytest

from oracle import trace_np
from optiland_pr_amd.lowering import lower_geometry
from tests._geometry_cases import CASES, arrays, build, specs


def _oracle(name):
    spec = specs()[name]
    table = lower_geometry(build(spec))
    s = table.surfaces[0]
    a = arrays(name)
    sag = trace_np.sag_surface(a["x"], a["y"], table, s)
    r0 = trace_np.Rays(a["x"], a["y"], np.zeros_like(a["x"]), 0 * a["x"], 0 * a["x"],
                       np.ones_like(a["x"]), np.ones_like(a["x"]))
    with np.errstate(all="ignore"):
        nx, ny, nz = trace_np.surface_normal(r0, table, s)
    rays = trace_np.Rays(a["rx"], a["ry"], a["rz"], a["rL"], a["rM"], a["rN"],
                         np.ones_like(a["rx"]))
    g = int(s["geometry"])
    with np.errstate(all="ignore"):
        if g == 0:
            t = trace_np.distance_plane(rays)
        elif g == 1:
            t = trace_np.distance_conic(rays, float(s["radius"]), float(s["conic"]),
                                        bool(int(s["flags"]) & 2))
        else:
            t, _ = trace_np.distance_newton(rays, table, s)
    return a, sag, (nx, ny, nz), t


@pytest.mark.parametrize("name", CASES)
def test_oracle_geometry_bit_exact(name):
    a, sag, (nx, ny, nz), t = _oracle(name)
    np.testing.assert_array_equal(sag * np.ones_like(a["x"]), a["sag"])
    np.testing.assert_array_equal(nx * np.ones_like(a["x"]), a["nx"])
    np.testing.assert_array_equal(ny * np.ones_like(a["x"]), a["ny"])
    np.testing.assert_array_equal(nz * np.ones_like(a["x"]), a["nz"])
    np.testing.assert_array_equal(t, a["t"])


def test_reference_test_literals():
    """Numbers hard-coded in the reference's tests/test_geometries.py."""
    g = arrays("even_sag")
    np.testing.assert_allclose(g["sag"][1:3], [0.039022474574473776, 0.25313367948069593])
    np.testing.assert_allclose(arrays("even_dist")["t"][:4],
                               [2.9438901710409624, 2.9438901710409624, 3.8530733934173256,
                                10.625463223037386])
    np.testing.assert_allclose(arrays("odd_sag")["sag"][1:3],
                               [0.03845668813684687, 0.24529923075615997])
    np.testing.assert_allclose(arrays("odd_dist")["t"][:3], [2.94131486, 2.94131486, 3.84502393],
                               rtol=1e-8)
    z = arrays("zern_fringe")["sag"][:10]
    np.testing.assert_allclose(z[:3], [8.84770045, 6.57121389, 4.91876121], rtol=1e-8)
