"""NURBS surfaces on the CPU: the oracle (oracle/nurbs_np.py) and the host side of the
product (optiland_pr_amd/nurbs.py: the control-net fit and the parameter-space API) against
the reference's own outputs (tests/golden/nurbs.npz, tests/golden/gen_nurbs_golden.py: the
inputs of the reference's tests/test_nurbs_geometry.py plus seeded points and rays), and
the lowering of a NURBS surface. The per-ray kernel code (ort_nurbs.h) is exercised here
through the host build of the trace core (test_host_lens.py's nurbs_lens case) and on the
MI355X by test_gpu_nurbs.py."""

import os

import numpy as np
import pytest

from optiland_pr_amd import _abi, nurbs
from optiland_pr_amd.coordinate_system import CoordinateSystem
from optiland_pr_amd.geometries import NurbsGeometry

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "nurbs.npz"))
CASES = ("fit_conic", "fit_offcentre", "fit_sphere", "fit_plane", "explicit")
FITS = {  # gen_nurbs_golden.py SPECS (the fitted ones)
    "fit_conic": dict(radius=100.0, conic=-1.0, nurbs_norm_x=20.0, nurbs_norm_y=20.0,
                      n_points_u=10, n_points_v=10),
    "fit_offcentre": dict(radius=-50.0, conic=0.3, nurbs_norm_x=12.0, nurbs_norm_y=9.0,
                          x_center=1.5, y_center=-2.0, n_points_u=6, n_points_v=8),
    "fit_sphere": dict(radius=40.0, conic=0.0, nurbs_norm_x=8.0, nurbs_norm_y=8.0,
                       n_points_u=8, n_points_v=8),
    "fit_plane": dict(radius=np.inf, conic=0.0, nurbs_norm_x=5.0, nurbs_norm_y=5.0,
                      n_points_u=4, n_points_v=4),
}
# the geometry's own tolerance (NurbsGeometry default 1e-10) bounds the solves' residuals
TOL = 1e-10


def g(case, key):
    return GOLD[f"{case}/{key}"]


def geometry(case):
    """The native geometry of a golden case: fitted by optiland_pr_amd.nurbs, or the
    explicit net as the reference held it."""
    cs = CoordinateSystem()
    if case in FITS:
        geo = NurbsGeometry(cs, **FITS[case])
        geo.fit_surface()
        return geo
    return NurbsGeometry(cs, control_points=g(case, "P"), weights=g(case, "W"),
                         u_degree=int(g(case, "pq")[0]), v_degree=int(g(case, "pq")[1]),
                         u_knots=g(case, "U"), v_knots=g(case, "V"), tol=TOL)


def block(case):
    from oracle import nurbs_np

    P, W = g(case, "P"), g(case, "W")
    p, q = (int(v) for v in g(case, "pq"))
    return nurbs_np.unpack(nurbs.lowered_block(P, W, p, q, g(case, "U"), g(case, "V")))


@pytest.mark.parametrize("case", [c for c in CASES if c in FITS])
def test_fit_matches_reference(case):
    """nurbs_fitting.py:19-164 (A9.7 least squares) and nurbs_geometry.py:840-932."""
    geo = geometry(case)
    np.testing.assert_array_equal(geo.P, g(case, "P"))  # the same LU solves, bit for bit
    np.testing.assert_array_equal(geo.W, g(case, "W"))
    np.testing.assert_array_equal(geo.U, g(case, "U"))
    np.testing.assert_array_equal(geo.V, g(case, "V"))
    assert (geo.p, geo.q) == tuple(int(v) for v in g(case, "pq"))


@pytest.mark.parametrize("case", CASES)
def test_parameter_space_api_matches_reference(case):
    """get_value / get_derivative / get_normals (nurbs_geometry.py:280-604) on the host."""
    geo = geometry(case)
    u, v = g(case, "u"), g(case, "v")
    np.testing.assert_allclose(geo.get_value(u, v), g(case, "value"), rtol=1e-12, atol=1e-12)
    for k in ("d10", "d01", "d11", "d20", "d02"):
        # (components that vanish analytically come out as rounding noise of the
        # control net x basis-derivative scale, up to ~1e-8 on the 20 mm fits)
        ref = g(case, k)
        np.testing.assert_allclose(geo.get_derivative(u, v, int(k[1]), int(k[2])), ref,
                                   rtol=1e-10, atol=1e-8,
                                   err_msg=k)
    np.testing.assert_allclose(geo.get_normals(u, v), g(case, "normals_uv"), rtol=0,
                               atol=1e-12)


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case):
    """The oracle's sag / surface_normal / distance (global stop, fixed restart sequence)
    against the reference's (numpy.random restarts: the restarted points converge to the
    same root)."""
    from oracle import nurbs_np

    blk = block(case)
    x, y = g(case, "x"), g(case, "y")
    np.testing.assert_allclose(nurbs_np.value(blk, g(case, "u"), g(case, "v")),
                               g(case, "value"), rtol=0, atol=1e-12)
    np.testing.assert_allclose(nurbs_np.sag(blk, x, y, TOL, 100), g(case, "sag"), rtol=0,
                               atol=1e-11)
    np.testing.assert_allclose(np.stack(nurbs_np.surface_normal(blk, x, y, TOL, 100)),
                               g(case, "normal"), rtol=0, atol=1e-12)
    d = nurbs_np.distance(blk, g(case, "rx"), g(case, "ry"), g(case, "rz"), g(case, "rL"),
                          g(case, "rM"), g(case, "rN"), TOL, 100)
    np.testing.assert_allclose(d, g(case, "distance"), rtol=0, atol=1e-11)


def test_reference_test_values():
    """tests/test_nurbs_geometry.py:18-93's own expectations on the fitted paraboloid."""
    from oracle import nurbs_np

    blk = block("fit_conic")
    sag = nurbs_np.sag(blk, np.array([0.0, 10.0]), np.array([0.0, 0.0]), TOL, 100)
    np.testing.assert_allclose(sag, [0.0, 0.5], atol=1e-4)
    n = nurbs_np.surface_normal(blk, np.zeros(1), np.zeros(1), TOL, 100)
    np.testing.assert_allclose(np.ravel(n), [0.0, 0.0, 1.0], atol=1e-4)
    one = [np.zeros(1), np.zeros(1), np.full(1, -10.0), np.zeros(1), np.zeros(1), np.ones(1)]
    np.testing.assert_allclose(nurbs_np.distance(blk, *one, TOL, 100), [10.0], atol=1e-4)
    np.testing.assert_allclose(g("fit_conic", "distance_axial"), [10.0], atol=1e-4)


def test_lowered_block_layout_and_refusals():
    geo = geometry("explicit")
    R, k, tol, max_iter, _, blk = geo.lower_params()
    p, q = int(geo.p), int(geo.q)
    nu, nv = geo.W.shape
    assert blk[:4] == [float(p), float(q), float(nu), float(nv)]
    o = 4 + nu + p + 1 + nv + q + 1
    Pw = np.asarray(blk[o:]).reshape(4, nu, nv)
    np.testing.assert_array_equal(Pw[:3], geo.P * geo.W[None])
    np.testing.assert_array_equal(Pw[3], geo.W)
    assert tol == TOL and max_iter == 100
    with pytest.raises(ValueError, match="clamped"):
        nurbs.lowered_block(geo.P, geo.W, p, q, np.linspace(0, 1, nu + p + 1), geo.V)
    with pytest.raises(ValueError, match="degrees"):
        nurbs.lowered_block(np.zeros((3, 8, 8)), np.ones((8, 8)), 6, 3,
                            nurbs.clamped_knots(8, 6), nurbs.clamped_knots(8, 3))
    unfitted = NurbsGeometry(CoordinateSystem(), radius=50.0, nurbs_norm_x=5.0,
                             nurbs_norm_y=5.0)
    with pytest.raises(ValueError, match="fit_surface"):
        unfitted.lower_params()


def test_lens_lowering_classifies_nurbs_as_own_solver():
    """A NURBS surface lowers with GEOM_NURBS and is not a Newton surface of the schedule
    (its per-ray (u, v) solve has no update count); autograd refuses it."""
    from optiland_pr_amd.lowering import lower_surface_group
    from optiland_pr_amd.ops import _check_differentiable
    from tests._cases import build_lens

    lens = build_lens("nurbs_lens")
    table = lower_surface_group(lens.surface_group, [0.55])
    geo = table.surfaces["geometry"]
    assert list(geo) == [_abi.GEOM_NURBS, _abi.GEOM_NURBS, _abi.GEOM_PLANE]  # (traced surfaces)
    assert table.newton_surfaces == []
    with pytest.raises(NotImplementedError, match="NURBS"):
        _check_differentiable(table)


def test_reference_geometry_converts_through_the_adapter():
    """adapter._geometry turns the reference's NurbsGeometry (its P / W / p / q / U / V as
    the reference holds them) into the native one: the same lowered block."""
    from optiland_pr_amd import adapter

    class RefCS:
        x = y = z = rx = ry = rz = 0.0
        reference_cs = None

    class RefNurbs:  # the attribute set of nurbs_geometry.py:86-269 after fit_surface
        pass

    ref = RefNurbs()
    ref.__class__.__name__ = "NurbsGeometry"
    ref.cs = RefCS()
    ref.radius, ref.k, ref.tol, ref.max_iter = 40.0, 0.0, 1e-10, 100
    ref.nurbs_norm_x = ref.nurbs_norm_y = 8.0
    ref.x_center = ref.y_center = 0.0
    ref.P, ref.W = g("fit_sphere", "P"), g("fit_sphere", "W")
    ref.p, ref.q = (int(v) for v in g("fit_sphere", "pq"))
    ref.U, ref.V = g("fit_sphere", "U"), g("fit_sphere", "V")
    ref.is_fitted = True
    nat = adapter._geometry(ref)
    assert isinstance(nat, NurbsGeometry)
    assert nat.lower_params()[5] == nurbs.lowered_block(ref.P, ref.W, ref.p, ref.q, ref.U,
                                                        ref.V)


@pytest.fixture(scope="module")
def nurbs_exe(tmp_path_factory):
    import shutil
    import subprocess

    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    src = os.path.join(HERE, "native", "nurbs_main.cpp")
    out = tmp_path_factory.mktemp("nurbs") / "nurbs_main"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-o", str(out), src],
                   check=True)
    return str(out)


def _net(p, q, seed):
    rng = np.random.default_rng(seed)
    nu, nv = p + 3, q + 4
    X, Y = np.meshgrid(np.linspace(-6, 6, nu), np.linspace(-5, 5, nv), indexing="ij")
    Z = (X**2 + Y**2) / 100.0 + 0.003 * X * Y + rng.uniform(-0.02, 0.02, X.shape)
    W = rng.uniform(0.8, 1.2, X.shape)

    def knots(n, d):
        inner = np.sort(rng.uniform(0.1, 0.9, n - d - 1))
        return np.concatenate([np.zeros(d + 1), inner, np.ones(d + 1)])

    return np.stack([X, Y, Z]), W, knots(nu, p), knots(nv, q), rng


@pytest.mark.parametrize("pq", [(1, 1), (1, 2), (2, 2), (3, 2), (4, 3), (5, 5), (5, 1)])
def test_kernel_solves_match_oracle_every_degree(nurbs_exe, pq):
    """ort_nurbs.h compiled for the host (the code the kernels inline): sag, normal and
    distance on nets of degrees 1-5 against the oracle (global stop rule; the kernel code
    stops per ray), plus the golden nets."""
    import subprocess

    from oracle import nurbs_np

    p, q = pq
    P, W, U, V, rng = _net(p, q, 10 * p + q)
    B = np.asarray(nurbs.lowered_block(P, W, p, q, U, V))
    n = 256
    x, y = rng.uniform(-4.5, 4.5, size=(2, n))
    L, M = rng.uniform(-0.05, 0.05, size=(2, n))
    N = np.sqrt(1 - L * L - M * M)
    px, py = rng.uniform(-4, 4, size=(2, n))
    pz = rng.uniform(-6, -2, n)
    inp = b"".join([np.int32(B.size).tobytes(), B.tobytes(), np.float64(TOL).tobytes(),
                    np.int32(100).tobytes(), np.int32(n).tobytes(), x.tobytes(), y.tobytes(),
                    np.concatenate([px, py, pz, L, M, N]).tobytes()])
    r = subprocess.run([nurbs_exe], input=inp, capture_output=True, check=True)
    out = np.frombuffer(r.stdout, dtype=np.float64).reshape(5, n)
    blk = nurbs_np.unpack(B)
    np.testing.assert_allclose(out[0], nurbs_np.sag(blk, x, y, TOL, 100), rtol=0, atol=1e-11)
    np.testing.assert_allclose(out[1:4], np.stack(nurbs_np.surface_normal(blk, x, y, TOL, 100)),
                               rtol=0, atol=1e-12)
    np.testing.assert_allclose(out[4], nurbs_np.distance(blk, px, py, pz, L, M, N, TOL, 100),
                               rtol=0, atol=1e-11)


def test_kernel_solves_refuse_out_of_range_blocks(nurbs_exe):
    """A hand-made block outside the lowered range (degree 6, or fewer control points than
    degree + 1) evaluates to NaN instead of reading past its window (ort_nurbs.h)."""
    import subprocess

    P, W, U, V, _ = _net(3, 2, 1)
    good = np.asarray(nurbs.lowered_block(P, W, 3, 2, U, V))
    for bad in (6.0, 0.0):
        B = good.copy()
        B[0] = bad  # the u degree
        n = 4
        z = np.zeros(n)
        inp = b"".join([np.int32(B.size).tobytes(), B.tobytes(), np.float64(TOL).tobytes(),
                        np.int32(20).tobytes(), np.int32(n).tobytes(), z.tobytes(), z.tobytes(),
                        np.concatenate([z, z, z - 3, z, z, z + 1]).tobytes()])
        r = subprocess.run([nurbs_exe], input=inp, capture_output=True, check=True)
        out = np.frombuffer(r.stdout, dtype=np.float64)
        assert np.isnan(out).all(), bad


def test_unfitted_surface_json_round_trip_keeps_the_fit_grid():
    """lensio: a NURBS surface not fitted yet keeps its fit window and grid, so
    fit_surface after from_dict gives the same net."""
    import json

    from optiland_pr_amd.lensio import geometry_from_dict, geometry_to_dict

    geo = NurbsGeometry(CoordinateSystem(), radius=-50.0, conic=0.3, nurbs_norm_x=12.0,
                        nurbs_norm_y=9.0, x_center=1.5, y_center=-2.0, n_points_u=6,
                        n_points_v=8)
    back = geometry_from_dict(json.loads(json.dumps(geometry_to_dict(geo))))
    geo.fit_surface()
    back.fit_surface()
    np.testing.assert_array_equal(back.P, geo.P)
    np.testing.assert_array_equal(back.P, g("fit_offcentre", "P"))
