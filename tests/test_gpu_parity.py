"""GPU parity: the HIP trace (through the C ABI) against the reference's golden vectors and
the oracle, on the MI355X.

Stated parity tolerances:
  * closed-form lenses (plane / conic): x, y, z, L, M, N, opd BIT-EXACT; intensity
    relative 1e-12 (absorption exp is accumulated once per ray: exp(a)exp(b) vs exp(a+b)).
  * Newton lenses (even / odd asphere, Zernike): |dx|,|dy|,|dz|,|dopd| <= 1e-9 mm,
    |dL|,|dM|,|dN| <= 1e-11, intensity relative 1e-12 -- device products replace libm pow
    (r**k, k >= 3) and the cos/sin(m*atan2) of the Zernike azimuth is evaluated by the
    angle-addition recurrence.
  * NaN masks identical; Newton update counts identical to the reference's global rule.
"""

import numpy as np
import pytest

from tests._cases import ALL_CASES, CLOSED_FORM, FIELDS, native_case
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu

TOL = {"x": 1e-9, "y": 1e-9, "z": 1e-9, "opd": 1e-9, "L": 1e-11, "M": 1e-11, "N": 1e-11}


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need the MI355X (torch.cuda.is_available() is False)")
    from optiland_pr_amd import _native

    _native.load()
    return torch


def assert_parity(name, got, ref, closed_form, what=""):
    for a in FIELDS:
        g, r = np.asarray(got[a]), np.asarray(ref[a])
        assert g.shape == r.shape, (name, a)
        np.testing.assert_array_equal(np.isnan(g), np.isnan(r), err_msg=f"{name}{what}.{a} NaN")
        if a == "i":
            np.testing.assert_allclose(g, r, rtol=1e-12, atol=0, err_msg=f"{name}{what}.i")
        elif closed_form:
            np.testing.assert_array_equal(g, r, err_msg=f"{name}{what}.{a}")
        else:
            np.testing.assert_allclose(g, r, rtol=0, atol=TOL[a], err_msg=f"{name}{what}.{a}")


def gpu_trace_case(torch, name, meta, newton_mode="reference", record=False):
    from optiland_pr_amd.raytrace import DeviceLens, RealRays, trace_pupil

    lens, table, segs = native_case(name, meta, record=record)
    g = load_golden(name)
    n_p = meta["n_pupil"]
    n = n_p * len(segs)
    dl = DeviceLens(table)
    out = RealRays.empty(n, 0.0)
    px = torch.as_tensor(g["Px"], device="cuda")
    py = torch.as_tensor(g["Py"], device="cuda")
    rec = None
    if record:
        rec = torch.empty(table.n_rec * 8 * n, dtype=torch.float64, device="cuda")
    keys = [("pair", k) for k in range(len(segs))]
    trace_pupil(dl, segs, px, py, out, n, n_p, n_p, keys=keys, rec=rec,
                newton_mode=newton_mode)
    torch.cuda.synchronize()
    return dl, g, out.numpy(), rec, keys


@pytest.mark.parametrize("name", ALL_CASES)
def test_trace_pupil_vs_reference(torch, name, golden_index):
    """Fused generate + trace, every (field, wavelength) pair of the case in ONE launch,
    each pair its own Newton group (= one reference Optic.trace call)."""
    _, g, got, _, _ = gpu_trace_case(torch, name, golden_index[name])
    assert_parity(name, got, g, name in CLOSED_FORM)


@pytest.mark.parametrize("name", ["cooke", "dg", "rt_asph", "tma_fringe", "decentered"])
def test_trace_resident_rays_vs_reference(torch, name, golden_index):
    """ort_trace_sequential on resident rays = the reference's generated rays."""
    from optiland_pr_amd import _abi
    from optiland_pr_amd.raytrace import DeviceLens, RealRays, trace_rays

    meta = golden_index[name]
    _, table, segs = native_case(name, meta)
    g = load_golden(name)
    n_p = meta["n_pupil"]
    rin = RealRays(g["x0"], g["y0"], g["z0"], g["L0"], g["M0"], g["N0"], 1.0, 0.0)
    rout = RealRays.empty(len(rin), 0.0)
    dl = DeviceLens(table)
    trace_rays(dl, rin, rout, group_len=n_p, keys=[("p", k) for k in range(len(segs))],
               segments=segs, seg_len=n_p)
    torch.cuda.synchronize()
    assert_parity(name, rout.numpy(), g, name in CLOSED_FORM, " (resident)")
    # in-place (the reference mutates RealRays)
    trace_rays(dl, rin, rin, group_len=n_p, segments=segs, seg_len=n_p)
    torch.cuda.synchronize()
    assert_parity(name, rin.numpy(), g, name in CLOSED_FORM, " (in place)")
    assert _abi.RAY_FIELDS


@pytest.mark.parametrize("name", ["rt_asph", "rt_odd", "tma_fringe", "tma_standard",
                                  "grid_lens"])
def test_newton_schedule_matches_reference_global_rule(torch, name, golden_index):
    dl, g, _, _, keys = gpu_trace_case(torch, name, golden_index[name])
    ref = g["newton_updates"]
    for p, k in enumerate(keys):
        sched = dl.sched_cache[k]
        for s in dl.newton:
            assert int(sched[s]) == int(ref[p][s + 1]), (name, p, s)


@pytest.mark.parametrize("name", ["rt_asph", "tma_fringe"])
def test_newton_wave_mode_within_newton_tol(torch, name, golden_index):
    """ORT_NEWTON_WAVE stops a wavefront as soon as its own 64 rays have |f| < tol, one
    update earlier than the reference's global rule for some waves: the intersection is
    then only as exact as the Newton tolerance itself (tol = 1e-6 mm for add_surface
    aspheres, geometry_configs.py:48). Stated bound: 1e-6 mm / 1e-6 direction."""
    _, g, got, _, _ = gpu_trace_case(torch, name, golden_index[name], newton_mode="wave")
    for a in FIELDS:
        np.testing.assert_array_equal(np.isnan(got[a]), np.isnan(g[a]))
        np.testing.assert_allclose(got[a], g[a], rtol=1e-6 if a == "i" else 0,
                                   atol=0 if a == "i" else 1e-6, err_msg=f"{name} wave {a}")


def test_doublegauss_records(torch, golden_index):
    """Per-surface snapshots (standard_surface.py:266-286), bit-exact."""
    meta = golden_index["dg"]
    dl, g, got, rec, _ = gpu_trace_case(torch, "dg", meta, record=True)
    n_p = meta["n_pupil"]
    n_pairs = len(meta["fields"]) * len(meta["wavelengths"])
    recs = rec.view(dl.table.n_rec, 8, n_pairs, n_p).cpu().numpy()
    ref = g["records"]  # [pair][surface][8][n_p]
    for slot, si in enumerate(dl.table.rec_surfaces):
        for f, a in enumerate(FIELDS):
            r = ref[:, si + 1, f, :]
            if a == "i":
                np.testing.assert_allclose(recs[slot, f], r, rtol=1e-12)
            else:
                np.testing.assert_array_equal(recs[slot, f], r, err_msg=f"surf {si + 1} {a}")


def test_optic_trace_api(torch, golden_index):
    """Optic.trace (optic.py:584-609 -> RealRayTracer.trace) on the MI355X."""
    from optiland_pr_amd.samples import DoubleGauss

    meta = golden_index["dg"]
    g = load_golden("dg")
    n_p = meta["n_pupil"]
    lens = DoubleGauss()
    rays = lens.trace(0.0, 1.0, 0.5876, num_rays=32, distribution="uniform")
    got = rays.numpy()
    pair = meta["fields"].index([0.0, 1.0]) * len(meta["wavelengths"]) + 1
    sl = slice(pair * n_p, (pair + 1) * n_p)
    assert_parity("dg.Optic.trace", got, {a: g[a][sl] for a in FIELDS}, True)
    # SurfaceGroup image record is what SpotDiagram reads
    img_x = lens.surface_group.x[-1].cpu().numpy()
    np.testing.assert_array_equal(img_x, g["x"][sl])


def test_surface_group_trace_seam(torch, golden_index):
    """SurfaceGroup.trace(rays) in place (surface_group.py:232-244): with the image
    thickness 0 of the samples, equal to the golden image-plane rays."""
    from optiland_pr_amd.raytrace import RealRays
    from optiland_pr_amd.samples import CookeTriplet

    meta = golden_index["cooke"]
    g = load_golden("cooke")
    n_p = meta["n_pupil"]
    pair = 1 * len(meta["wavelengths"]) + 1  # field (0, 0.7), 0.55 um
    sl = slice(pair * n_p, (pair + 1) * n_p)
    lens = CookeTriplet()
    rays = RealRays(g["x0"][sl], g["y0"][sl], g["z0"][sl], g["L0"][sl], g["M0"][sl],
                    g["N0"][sl], 1.0, 0.55)
    lens.surface_group.trace(rays)
    torch.cuda.synchronize()
    assert_parity("cooke.SurfaceGroup.trace", rays.numpy(), {a: g[a][sl] for a in FIELDS}, True)


def test_zernike_range_error(torch):
    """zernike.py:234-246: ValueError when |x / R_norm| > 1 at a Newton iterate."""
    from optiland_pr_amd.raytrace import ZernikeRangeError
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    lens = ThreeMirrorAnastigmat()
    for s in lens.surface_group.surfaces[1:4]:
        s.geometry.norm_radius = 0.5
    lens.invalidate()
    with pytest.raises(ValueError, match="Zernike coordinates must be normalized"):
        lens.trace(0.0, 1.0, 0.587, num_rays=8, distribution="uniform")
    assert issubclass(ZernikeRangeError, ValueError)


@pytest.mark.parametrize("n", [0, 1, 255, 257, 1000])
def test_ragged_and_empty_batches(torch, n):
    """Sizes that are not multiples of the 256-ray block, and the empty batch."""
    from oracle import trace_np
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    rng = np.random.default_rng(n)
    r = np.sqrt(rng.uniform(size=n))
    th = rng.uniform(0, 2 * np.pi, size=n)
    px, py = r * np.cos(th), r * np.sin(th)
    dl = lens_for(lens, [0.55])
    seg = np.stack([segment_params(lens, 0.0, 1.0, 0)])
    out = RealRays.empty(n, 0.55)
    trace_pupil(dl, seg, torch.as_tensor(px, device="cuda"), torch.as_tensor(py, device="cuda"),
                out, n, max(n, 1), max(n, 1))
    torch.cuda.synchronize()
    if n == 0:
        assert len(out) == 0
        return
    ref = trace_np.trace_segment(dl.table, trace_np.generate_rays(seg[0], px, py), 0).rays
    assert_parity(f"cooke[n={n}]", out.numpy(), ref.as_dict(), True)


def test_nan_rays_propagate_like_reference(torch):
    """Rays that miss a surface become NaN (sqrt of a negative discriminant,
    standard.py:121-127) exactly where the oracle says so; the rest stay bit-exact."""
    from oracle import trace_np
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    n = 4096
    g = np.linspace(-8.0, 8.0, 64)  # pupil far outside the lens: rays miss the spheres
    px, py = (a.ravel() for a in np.meshgrid(g, g))
    dl = lens_for(lens, [0.55])
    seg = np.stack([segment_params(lens, 0.0, 1.0, 0)])
    out = RealRays.empty(n, 0.55)
    trace_pupil(dl, seg, torch.as_tensor(px, device="cuda"), torch.as_tensor(py, device="cuda"),
                out, n, n, n)
    torch.cuda.synchronize()
    with np.errstate(all="ignore"):
        ref = trace_np.trace_segment(dl.table, trace_np.generate_rays(seg[0], px, py), 0).rays
    got = out.numpy()
    assert np.isnan(ref.x).any()
    assert_parity("cooke[miss]", got, ref.as_dict(), True)


def test_doublegauss_1m_full_size_properties(torch, golden_index):
    """BASELINE config 2 size (1,000,000 random pupil rays, seed 0, Hy = 1, 0.5876 um):
    size-independent checks against the reference's full-size summary."""
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.samples import DoubleGauss

    ref = golden_index["_full"]["dg_1m"]
    d = RandomDistribution(seed=0)
    d.generate_points(1_000_000)
    rays = DoubleGauss().trace(0.0, 1.0, 0.5876, num_rays=1_000_000, distribution=d)
    x, y, opd = (getattr(rays, a).cpu().numpy() for a in ("x", "y", "opd"))
    assert x.size == ref["n"] and int(np.isnan(x).sum()) == ref["nan"]
    # bit-exact trace => identical NumPy reductions
    assert float(np.sum(x)) == ref["sum_x"]
    assert float(np.sum(y)) == ref["sum_y"]
    assert float(np.sum(opd)) == ref["sum_opd"]
    assert float(np.sum(x * x)) == ref["sum_x2"]
    assert [float(x[0]), float(y[0]), float(opd[0])] == ref["first"]
    assert [float(x[-1]), float(y[-1]), float(opd[-1])] == ref["last"]


@pytest.mark.parametrize("key", ["rt_asph_1m", "tma_1m"])
def test_newton_lenses_1m_full_size_properties(torch, golden_index, key):
    """Config 3's RT-asph and config 5's fringe-Zernike TMA at the BASELINE ray count
    (1,000,000 random pupil rays, seed 0, Hy = 1): the reference's own NumPy sums of the
    image x, y, opd (gen_golden.py --full-newton), the first / last ray, no NaNs and the
    Newton update count of every Newton surface under the global stop rule. Per-ray
    tolerance of the Newton kernels is 1e-9 mm; the stated bound on the 1M-ray sums is
    relative 1e-12 (x: absolute 1e-9 per ray summed in quadrature, 1e-6)."""
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.raytrace import lens_for
    from optiland_pr_amd.samples import ReverseTelephotoAsphere, ThreeMirrorAnastigmat

    ref = golden_index["_full"][key]
    lens, wl = ((ReverseTelephotoAsphere(), 0.5876) if key == "rt_asph_1m"
                else (ThreeMirrorAnastigmat(), 0.587))
    d = RandomDistribution(seed=0)
    d.generate_points(1_000_000)
    rays = lens.trace(0.0, 1.0, wl, num_rays=1_000_000, distribution=d)
    x, y, opd = (getattr(rays, a).cpu().numpy() for a in ("x", "y", "opd"))
    assert x.size == ref["n"] and int(np.isnan(x).sum()) == ref["nan"]
    np.testing.assert_allclose(float(np.sum(x)), ref["sum_x"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(float(np.sum(y)), ref["sum_y"], rtol=1e-12)
    np.testing.assert_allclose(float(np.sum(opd)), ref["sum_opd"], rtol=1e-12)
    np.testing.assert_allclose(float(np.sum(x * x)), ref["sum_x2"], rtol=1e-12)
    np.testing.assert_allclose([float(x[0]), float(y[0]), float(opd[0])], ref["first"],
                               rtol=0, atol=1e-9)
    np.testing.assert_allclose([float(x[-1]), float(y[-1]), float(opd[-1])], ref["last"],
                               rtol=0, atol=1e-9)
    dl = lens_for(lens, [wl])
    scheds = list(dl.sched_cache.values())
    assert scheds, "no verified Newton schedule was cached"
    for s_idx, u in ref["newton_updates"].items():
        assert int(scheds[-1][int(s_idx) - 1]) == u, (key, s_idx)


def test_unknown_geometry_id_fails_loudly(torch):
    """A geometry id outside enum ort_geometry is never traced as another kind: refused
    at the boundary when the lens's geometry_mask names it (ORT_ERR_ARG), NaN rays plus
    ORT_STATUS_BAD_GEOMETRY (-> ValueError) when only the surface record holds it."""
    from optiland_pr_amd import _native
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import DeviceLens, RealRays, lens_for, trace_pupil
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    table = lens_for(lens, [0.55]).table
    table.surfaces = table.surfaces.copy()
    table.surfaces[2]["geometry"] = 13  # (12 is NURBS since ABI v20)
    seg = np.stack([segment_params(lens, 0.0, 1.0, 0)])
    n = 256
    px = torch.linspace(-0.5, 0.5, n, dtype=torch.float64, device="cuda")
    py = torch.zeros(n, dtype=torch.float64, device="cuda")
    out = RealRays.empty(n, 0.55)
    dl = DeviceLens(table)
    with pytest.raises(RuntimeError, match="ORT_ERR_ARG"):
        trace_pupil(dl, seg, px, py, out, n, n, n)
    dl.c.geometry_mask = dl.geometry_mask & ~(1 << 13)  # a stale / inconsistent mask
    trace_pupil(dl, seg, px, py, out, n, n, n)
    torch.cuda.synchronize()
    assert np.isnan(out.numpy()["x"]).all()  # the closed-form kernel: NaN rays
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    import ctypes as C

    from optiland_pr_amd import _abi
    from optiland_pr_amd.raytrace import _ptr, _stream_handle, upload_segments

    seg_dev = upload_segments(seg, "cuda")
    batch = _native.ort_batch(n, n, n, 1, 0, seg_dev.data_ptr())
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, 0, None)
    out_c = out.c_struct()
    rc = _native.load().ort_trace_pupil(C.byref(dl.c), _ptr(px), _ptr(py), C.byref(out_c),
                                        C.byref(batch), C.byref(opt), None, None, _ptr(st),
                                        _stream_handle())
    assert rc == 0
    torch.cuda.synchronize()
    assert int(st.item()) & _abi.STATUS_BAD_GEOMETRY  # ... and the status bit when asked


@pytest.mark.parametrize("lens_name", ["cooke", "dg"])
def test_signed_zeros_bit_exact(torch, lens_name):
    """Rays on the symmetry planes (px = +-0, py = +-0, the on-axis chief ray) through
    convex and concave surfaces: every output equal to the oracle's INCLUDING the sign of
    zero results (the closed-form fast path's quotients keep signed zeros; a -0 input
    takes the exact path)."""
    from oracle import trace_np
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil
    from optiland_pr_amd.samples import CookeTriplet, DoubleGauss

    lens = CookeTriplet() if lens_name == "cooke" else DoubleGauss()
    v = np.linspace(-1.0, 1.0, 41)
    px = np.concatenate([np.zeros(41), v, -np.zeros(41), v, [0.0, -0.0, 0.0, -0.0]])
    py = np.concatenate([v, np.zeros(41), v, -np.zeros(41), [0.0, 0.0, -0.0, -0.0]])
    n = px.size
    wl = 0.55 if lens_name == "cooke" else 0.5876
    dl = lens_for(lens, [wl])
    for hx, hy in ((0.0, 0.0), (0.0, 1.0), (0.5, 0.0)):
        seg = np.stack([segment_params(lens, hx, hy, 0)])
        out = RealRays.empty(n, wl)
        trace_pupil(dl, seg, torch.as_tensor(px, device="cuda"),
                    torch.as_tensor(py, device="cuda"), out, n, n, n)
        torch.cuda.synchronize()
        ref = trace_np.trace_segment(dl.table, trace_np.generate_rays(seg[0], px, py), 0).rays
        got = out.numpy()
        for a in FIELDS:
            g, r = got[a], getattr(ref, a)
            if a == "i":
                np.testing.assert_allclose(g, r, rtol=1e-12, atol=0)
                continue
            np.testing.assert_array_equal(g, r, err_msg=f"{lens_name} ({hx},{hy}) {a}")
            np.testing.assert_array_equal(np.signbit(g), np.signbit(r),
                                          err_msg=f"{lens_name} ({hx},{hy}) sign of {a}")


@pytest.mark.parametrize("lens_name", ["cooke", "dg"])
def test_extreme_operands_bit_exact(torch, lens_name):
    """Resident rays whose operands sit at and beyond the edges of the closed-form fast
    path's ranges (ort_fastpath.h): denormal, tiny (2^-301 / 2^-299), huge (1e150 ..
    1.7e308), infinite and NaN positions, rays starting on the vertex (zero numerators),
    grazing / tiny / unnormalised / infinite directions. Lower-bound failures take the
    exact path per lane, upper-bound failures surface as a non-finite (or > 2^1000) ray
    state at the end of the fast trace; either way every output must equal the oracle's,
    bit for bit including the sign of zeros, and the NaN masks must agree."""
    import itertools

    from oracle import trace_np
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_rays
    from optiland_pr_amd.samples import CookeTriplet, DoubleGauss

    lens = CookeTriplet() if lens_name == "cooke" else DoubleGauss()
    wl = 0.55 if lens_name == "cooke" else 0.5876
    dl = lens_for(lens, [wl])
    inf, nan = np.inf, np.nan
    pos = [0.0, -0.0, 1e-310, -1e-310, 2.0**-301, -(2.0**-299), 1e-200, 1.5, -3.25, 1e150,
           -1e200, 1e300, 1.7e308, inf, nan]
    zs = [0.0, -10.0, -1e-300, 1e300]
    dirs = [(0.0, 0.0, 1.0), (0.6, 0.0, 0.8), (0.0, -0.28, 0.96), (1.0, 0.0, 1e-200),
            (1e-200, 1e-200, 1.0), (0.0, 0.0, -1.0), (2.0, 0.0, 2.0), (1e-200, 0.0, 1e-200),
            (inf, 0.0, 1.0), (0.0, 0.0, nan), (0.1, 0.2, 1e-310)]
    rows = [(x, y, z, *d) for x, y, z, d in itertools.product(pos, pos, zs, dirs)]
    x, y, z, L, M, N = (np.array(c, dtype=np.float64) for c in zip(*rows))
    n = x.size
    rin = RealRays(x, y, z, L, M, N, 1.0, wl)
    rout = RealRays.empty(n, wl)
    trace_rays(dl, rin, rout)
    torch.cuda.synchronize()
    with np.errstate(all="ignore"):
        ref = trace_np.trace_segment(
            dl.table, trace_np.Rays(x.copy(), y.copy(), z.copy(), L.copy(), M.copy(), N.copy(),
                                    np.ones(n)), 0).rays
    got = rout.numpy()
    for a in FIELDS:
        g, r = np.asarray(got[a]), np.asarray(getattr(ref, a))
        np.testing.assert_array_equal(np.isnan(g), np.isnan(r), err_msg=f"{lens_name} {a} NaN")
        ok = ~np.isnan(r)
        if a == "i":
            with np.errstate(all="ignore"):
                np.testing.assert_allclose(g[ok], r[ok], rtol=1e-12, atol=0)
            continue
        np.testing.assert_array_equal(g[ok], r[ok], err_msg=f"{lens_name} {a}")
        np.testing.assert_array_equal(np.signbit(g[ok]), np.signbit(r[ok]),
                                      err_msg=f"{lens_name} sign of {a}")
    assert np.isfinite(got["x"]).sum() > n // 20  # the set is not all NaN


def _extreme_rays(wl):
    import itertools

    from optiland_pr_amd.raytrace import RealRays

    inf, nan = np.inf, np.nan
    pos = [0.0, -0.0, 1e-310, -1e-310, 2.0**-301, -(2.0**-299), 1e-200, 1.5, -3.25, 1e150,
           -1e200, 1e300, 1.7e308, inf, nan]
    zs = [0.0, -10.0, -1e-300, 1e300]
    dirs = [(0.0, 0.0, 1.0), (0.6, 0.0, 0.8), (0.0, -0.28, 0.96), (1.0, 0.0, 1e-200),
            (1e-200, 1e-200, 1.0), (0.0, 0.0, -1.0), (2.0, 0.0, 2.0), (1e-200, 0.0, 1e-200),
            (inf, 0.0, 1.0), (0.0, 0.0, nan), (0.1, 0.2, 1e-310)]
    rows = [(x, y, z, *d) for x, y, z, d in itertools.product(pos, pos, zs, dirs)]
    cols = [np.array(c, dtype=np.float64) for c in zip(*rows)]
    return cols, RealRays(*cols, 1.0, wl)


def _assert_same_bits(got, exp, what):
    for a in FIELDS:
        g, e = np.asarray(got[a]), np.asarray(exp[a])
        np.testing.assert_array_equal(g.view(np.uint64), e.view(np.uint64),
                                      err_msg=f"{what} {a}")


@pytest.mark.parametrize("lens_name", ["rt_asph", "rt_odd"])
def test_newton_fast_pass_equals_exact_pass(torch, lens_name, golden_index):
    """The deferred-range-check pass for even / odd asphere Newton lenses (trace_ray<FEAT,
    true>: fast div / sqrt sequences, range failures flagged and re-traced on the exact
    sequences) against ORT_OPT_EXACT (every ray on the per-operation exact sequences): every
    output the SAME BITS (NaN payloads and signed zeros included) and the same Newton update
    counts, on the reference's golden pupils and on the extreme-operand set (denormal, tiny,
    huge, infinite and NaN positions, grazing / unnormalised directions), whose NaN masks
    must also equal the oracle's and whose moderate-magnitude rays its values to the Newton
    tolerances."""
    from oracle import trace_np
    from optiland_pr_amd.raytrace import DeviceLens, RealRays, lens_for, trace_pupil, \
        trace_rays
    from optiland_pr_amd.samples import ReverseTelephotoAsphere

    meta = golden_index[lens_name]
    _, table, segs = native_case(lens_name, meta)
    g = load_golden(lens_name)
    n_p = meta["n_pupil"]
    n = n_p * len(segs)
    px = torch.as_tensor(g["Px"], device="cuda")
    py = torch.as_tensor(g["Py"], device="cuda")
    res = {}
    for exact in (False, True):
        dl = DeviceLens(table)
        out = RealRays.empty(n, 0.0)
        keys = [("pair", k) for k in range(len(segs))]
        trace_pupil(dl, segs, px, py, out, n, n_p, n_p, keys=keys, exact_only=exact)
        torch.cuda.synchronize()
        res[exact] = (out.numpy(), [dl.sched_cache[k].copy() for k in keys])
    _assert_same_bits(res[False][0], res[True][0], f"{lens_name} golden pupil")
    for a, b in zip(res[False][1], res[True][1]):
        np.testing.assert_array_equal(a, b)
    assert_parity(lens_name, res[False][0], g, False)

    if lens_name != "rt_asph":
        return
    wl = 0.5876
    (x, y, z, L, M, N), rin = _extreme_rays(wl)
    n = x.size
    outs = {}
    for exact in (False, True):
        dl = lens_for(ReverseTelephotoAsphere(), [wl])
        rout = RealRays.empty(n, wl)
        trace_rays(dl, rin, rout, exact_only=exact)
        torch.cuda.synchronize()
        outs[exact] = rout.numpy()
    _assert_same_bits(outs[False], outs[True], "rt_asph extreme operands")
    with np.errstate(all="ignore"):
        ref = trace_np.trace_segment(
            dl.table, trace_np.Rays(x.copy(), y.copy(), z.copy(), L.copy(), M.copy(),
                                    N.copy(), np.ones(n)), 0).rays
    got = outs[False]
    moderate = np.ones(n, bool)
    for a in FIELDS:
        r = np.asarray(getattr(ref, a))
        np.testing.assert_array_equal(np.isnan(got[a]), np.isnan(r),
                                      err_msg=f"rt_asph extreme {a} NaN")
        moderate &= np.isfinite(r) & (np.abs(r) < 1e6)
    assert moderate.sum() > 50
    for a in FIELDS:
        r = np.asarray(getattr(ref, a))[moderate]
        gm = np.asarray(got[a])[moderate]
        if a == "i":
            np.testing.assert_allclose(gm, r, rtol=1e-12, atol=0)
        else:
            np.testing.assert_allclose(gm, r, rtol=0, atol=TOL[a], err_msg=f"extreme {a}")


@pytest.mark.parametrize("lens_name", ["cooke", "rt_asph"])
def test_wave_uniform_rows_and_chunk_major_blocks(torch, lens_name):
    """3 fields x 3 wavelengths of one shared 1024-point pupil: the segments sit on 64- and
    256-ray boundaries, so the launch takes the scalar wavelength-row kernels (F_MONO with
    n_lambda > 1) and, for the Newton lens, the XCD-aware chunk-major block order
    (pair_major_ray). Every pair must equal the oracle's trace of that pair alone:
    bit-exact for the closed-form lens, the Newton tolerances for RT-asph (incl. the
    reference's per-pair Newton update counts)."""
    from oracle import trace_np
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil
    from optiland_pr_amd.samples import CookeTriplet, ReverseTelephotoAsphere

    lens = CookeTriplet() if lens_name == "cooke" else ReverseTelephotoAsphere()
    wls = [0.4861, 0.5876, 0.6563]
    fields = [(0.0, 0.0), (0.0, 0.7), (0.3, 1.0)]
    n_p = 1024
    rng = np.random.default_rng(7)
    rr = np.sqrt(rng.uniform(size=n_p))
    th = rng.uniform(0.0, 2.0 * np.pi, size=n_p)
    px, py = rr * np.cos(th), rr * np.sin(th)
    dl = lens_for(lens, wls)
    seg = np.stack([segment_params(lens, hx, hy, wi) for hx, hy in fields
                    for wi in range(len(wls))])
    n = n_p * len(seg)
    out = RealRays.empty(n, 0.0)
    keys = [("wave_uniform", k) for k in range(len(seg))]
    trace_pupil(dl, seg, torch.as_tensor(px, device="cuda"), torch.as_tensor(py, device="cuda"),
                out, n, n_p, n_p, keys=keys)
    torch.cuda.synchronize()
    got = out.numpy()
    closed = lens_name == "cooke"
    for k, sg in enumerate(seg):
        with np.errstate(all="ignore"):
            res = trace_np.trace_segment(dl.table, trace_np.generate_rays(sg, px, py),
                                         int(sg["lambda_idx"]))
        sl = slice(k * n_p, (k + 1) * n_p)
        assert_parity(f"{lens_name}[pair {k}]", {a: got[a][sl] for a in FIELDS},
                      res.rays.as_dict(), closed)
        if not closed:
            for s in dl.newton:
                assert int(dl.sched_cache[keys[k]][s]) == int(res.newton_updates[s]), (k, s)


def test_resident_rays_wave_uniform_rows(torch):
    """ort_trace_sequential on resident rays of 3 (field, wavelength) segments of 256 rays
    each (segment boundaries on waves: the scalar wavelength-row closed-form kernel):
    every segment bit-exact against the oracle's trace of its rays at its wavelength."""
    from oracle import trace_np
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_rays
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    wls = [0.48, 0.55, 0.65]
    dl = lens_for(lens, wls)
    n_p = 256
    rng = np.random.default_rng(3)
    rr = np.sqrt(rng.uniform(size=n_p))
    th = rng.uniform(0.0, 2.0 * np.pi, size=n_p)
    px, py = rr * np.cos(th), rr * np.sin(th)
    seg = np.stack([segment_params(lens, 0.0, hy, wi) for wi, hy in enumerate((0.0, 0.5, 1.0))])
    gen = [trace_np.generate_rays(sg, px, py) for sg in seg]
    cat = {a: np.concatenate([getattr(g, a) for g in gen]) for a in ("x", "y", "z", "L", "M", "N")}
    rin = RealRays(cat["x"], cat["y"], cat["z"], cat["L"], cat["M"], cat["N"], 1.0, 0.0)
    rout = RealRays.empty(len(rin), 0.0)
    trace_rays(dl, rin, rout, group_len=n_p, keys=[("res_wu", k) for k in range(len(seg))],
               segments=seg, seg_len=n_p)
    torch.cuda.synchronize()
    got = rout.numpy()
    for k, sg in enumerate(seg):
        ref = trace_np.trace_segment(dl.table, trace_np.generate_rays(sg, px, py),
                                     int(sg["lambda_idx"])).rays
        sl = slice(k * n_p, (k + 1) * n_p)
        assert_parity(f"cooke resident[seg {k}]", {a: got[a][sl] for a in FIELDS},
                      ref.as_dict(), True)


def test_unknown_apodization_kind_raises(torch):
    """an apodization record with a kind the core does not know sets
    ORT_STATUS_BAD_APODIZATION (NaN intensities are never returned silently)."""
    from optiland_pr_amd.raytrace import lens_for
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    lens = ThreeMirrorAnastigmat()
    lens.set_apodization("GaussianApodization", sigma=0.6)
    lens.trace(0.0, 1.0, 0.587, num_rays=8, distribution="uniform")
    dl = lens_for(lens, [0.587])
    dl.apod.view(torch.int32)[0] = 99  # the uploaded record's kind
    with pytest.raises(ValueError, match="apodization"):
        lens.trace(0.0, 1.0, 0.587, num_rays=8, distribution="uniform")


@pytest.mark.parametrize("name", ["apod_gaussian", "apod_tukey"])
def test_apodized_records_carry_the_pupil_factor(torch, name, golden_index):
    """with records on, the closed-form kernel's per-surface intensity
    rows of an apodized lens carry the pupil factor (ray_generator.py:91-95 starts the
    rays apodized). The image surface's record equals the reference's image-plane rays
    (x, y bit-exact, i rel 1e-12), and it is the stored output intensity exactly."""
    meta = golden_index[name]
    dl, g, got, rec, _ = gpu_trace_case(torch, name, meta, record=True)
    n_p = meta["n_pupil"]
    n_pairs = len(meta["fields"]) * len(meta["wavelengths"])
    recs = rec.view(dl.table.n_rec, 8, n_pairs * n_p).cpu().numpy()
    last = list(dl.table.rec_surfaces).index(max(dl.table.rec_surfaces))
    np.testing.assert_array_equal(recs[last, 0], g["x"])
    np.testing.assert_array_equal(recs[last, 1], g["y"])
    np.testing.assert_allclose(recs[last, 6], g["i"], rtol=1e-12)
    np.testing.assert_array_equal(recs[last, 6], np.asarray(got["i"]))
    assert np.any(recs[last, 6] < 1.0)  # the pupil factor is really there


@pytest.mark.parametrize("name", ["tma_fringe", "tma_standard", "tma_noll"])
def test_zernike_cartesian_form_matches_polar(torch, name, golden_index, monkeypatch):
    """The Cartesian form of the Zernike term sums (ABI v16, ort_core.h zmono_*) against the
    polar evaluation of the same lens (ZM_MAX_DEG forced below every order: no block) on
    the golden pupils: equal Newton update counts, outputs within a few ulps of the ray
    scale (1e-12 mm, 1e-13 in the direction cosines) -- far inside the reference tolerances
    both paths are held to."""
    from optiland_pr_amd import geometries
    from optiland_pr_amd.raytrace import DeviceLens, RealRays, trace_pupil

    meta = golden_index[name]
    g = load_golden(name)
    n_p = meta["n_pupil"]
    px = torch.as_tensor(g["Px"], device="cuda")
    py = torch.as_tensor(g["Py"], device="cuda")
    res = {}
    for polar in (False, True):
        if polar:
            monkeypatch.setattr(geometries, "ZM_MAX_DEG", -1)
        _, table, segs = native_case(name, meta)
        assert (table.surfaces["zm_deg"] >= 0).any() != polar
        n = n_p * len(segs)
        dl = DeviceLens(table)
        out = RealRays.empty(n, 0.0)
        keys = [("pair", k) for k in range(len(segs))]
        trace_pupil(dl, segs, px, py, out, n, n_p, n_p, keys=keys)
        torch.cuda.synchronize()
        res[polar] = (out.numpy(), [dl.sched_cache[k].copy() for k in keys])
    for a, b in zip(res[False][1], res[True][1]):
        np.testing.assert_array_equal(a, b)
    for a in FIELDS:
        c, p = res[False][0][a], res[True][0][a]
        np.testing.assert_array_equal(np.isnan(c), np.isnan(p))
        tol = 1e-13 if a in ("L", "M", "N") else 1e-12
        np.testing.assert_allclose(c, p, rtol=1e-12 if a == "i" else 0,
                                   atol=0 if a == "i" else tol, err_msg=f"{name}.{a}")
