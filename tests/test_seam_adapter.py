"""The drop-in seam as the reference would call it -- adapter._trace_on_mi355x (the body
install() puts behind optiland's SurfaceGroup.trace, surface_group.py:232-244) -- on BOTH
dispatch keys of the custom op torch.ops.ort.trace_sequential: "cpu" (the host build of the
trace core, liboptiland_host.so: runs here in the CPU suite) and "cuda" (the HIP kernels,
-m gpu on the MI355X). Driven with the native classes, which carry the reference's class
names and attributes (the reference itself is not on the GPU box; tests/
test_reference_install.py drives the real reference objects through install()). Under
autograd everything goes through the op's VJP (ort_trace_sequential_vjp /
ort_host_trace_sequential_vjp).

Checks: in-place rays and every surface record bit-exact to the dg / cooke goldens; a
mixed-wavelength batch against mixed_w; gradients through the seam against the reference's
torch autograd (autograd_tma: Zernike coefficients, autograd_cooke: radius / conic /
thickness) at rtol 1e-8 / 1e-9; input-ray and record cotangents by gradcheck; skip, caching
and the fall-back rules.
"""

import numpy as np
import pytest

from tests.conftest import load_golden

FIELDS = ("x", "y", "z", "L", "M", "N", "i", "opd")
NAMES = ("x", "y", "z", "L", "M", "N", "intensity", "opd")


@pytest.fixture(scope="module", params=["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def dev(request):
    import torch

    from optiland_pr_amd import _native

    if request.param == "cuda":
        if not torch.cuda.is_available():
            pytest.fail("needs the MI355X")
        _native.load()
    else:
        _native.load_host()
    return request.param


@pytest.fixture(scope="module")
def torch():
    import torch

    return torch


def _rays(torch, g, sl, w, dev, requires_grad=False):
    from optiland_pr_amd.raytrace import RealRays

    r = RealRays(*(torch.as_tensor(g[f"{a}0"][sl], device=dev) for a in ("x", "y", "z", "L", "M", "N")),
                 1.0, w, device=dev)
    if requires_grad:
        for a in ("x", "y", "L", "M"):
            setattr(r, a, getattr(r, a).clone().requires_grad_(True))
    return r


def _generated(torch, lens, hx, hy, wl, num, dev, dist="uniform"):
    """Rays as RealRayTracer builds them (ray_generator.py:28-106): the oracle's generation
    (pinned bit-exact to the reference, tests/test_oracle_golden.py), moved to `dev`."""
    from oracle import trace_np
    from optiland_pr_amd.distribution import create_distribution
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays

    d = create_distribution(dist)
    d.generate_points(num)
    px = np.asarray(d.x, dtype=np.float64)
    py = np.asarray(d.y, dtype=np.float64)
    seg = segment_params(lens, hx, hy, 0)
    q = trace_np.generate_rays(seg, px, py)
    return RealRays(*(torch.as_tensor(np.ascontiguousarray(getattr(q, a)), device=dev)
                      for a in ("x", "y", "z", "L", "M", "N")), 1.0, wl, device=dev)


@pytest.mark.parametrize("case,pair", [("dg", 1), ("dg", 4), ("cooke", 4)])
def test_seam_rays_and_records_bit_exact(torch, dev, golden_index, case, pair):
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.samples import CookeTriplet, DoubleGauss

    meta = golden_index[case]
    g = load_golden(case)
    n_p = meta["n_pupil"]
    wl = meta["wavelengths"][pair % len(meta["wavelengths"])]
    sl = slice(pair * n_p, (pair + 1) * n_p)
    lens = DoubleGauss() if case == "dg" else CookeTriplet()
    sg = lens.surface_group
    rays = _rays(torch, g, sl, wl, dev)
    x_in = rays.x
    out = _trace_on_mi355x(sg, rays, 0)
    assert out is rays  # the reference returns the same RealRays, updated in place
    assert rays.x.device.type == dev
    for a in FIELDS:
        got = getattr(rays, a).cpu().numpy()
        if a == "i":
            np.testing.assert_allclose(got, g[a][sl], rtol=1e-12)
        else:
            np.testing.assert_array_equal(got, g[a][sl], err_msg=a)
    assert torch.equal(sg.surfaces[0].x, x_in)  # the object surface records the input
    if "records" in g:
        ref = g["records"][pair]
        for si in range(1, len(sg.surfaces)):
            for f, nm in enumerate(NAMES):
                got = getattr(sg.surfaces[si], nm).cpu().numpy()
                if nm == "intensity":
                    np.testing.assert_allclose(got, ref[si, f], rtol=1e-12)
                else:
                    np.testing.assert_array_equal(got, ref[si, f], err_msg=f"surf {si} {nm}")
    else:  # the image record equals the traced rays
        np.testing.assert_array_equal(sg.surfaces[-1].x.cpu().numpy(), g["x"][sl])


@pytest.mark.parametrize("name", ["dg", "cooke", "freeform"])
def test_seam_mixed_wavelengths(torch, dev, name):
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.raytrace import RealRays
    from tests._cases import build_lens

    g = load_golden("mixed_w")
    lens = build_lens(name)
    rays = RealRays(*(torch.as_tensor(g[f"{name}/in_{a}"], device=dev)
                      for a in ("x", "y", "z", "L", "M", "N", "i")),
                    torch.as_tensor(g[f"{name}/w"], device=dev), device=dev)
    _trace_on_mi355x(lens.surface_group, rays, 0)
    for a in FIELDS:
        got = getattr(rays, a).cpu().numpy()
        ref = g[f"{name}/{a}"]
        if a == "i":
            np.testing.assert_allclose(got, ref, rtol=1e-12)
        elif name == "dg":
            np.testing.assert_array_equal(got, ref, err_msg=a)
        else:
            tol = 1e-11 if a in ("L", "M", "N") else 1e-9
            np.testing.assert_allclose(got, ref, rtol=0, atol=tol, err_msg=a)


def _rms(torch, s):
    x, y = s.x, s.y
    r2 = (x - torch.mean(x)) ** 2 + (y - torch.mean(y)) ** 2
    return torch.sqrt(torch.mean(r2))


@pytest.mark.parametrize("scheme", ["fringe", "standard", "noll"])
def test_seam_gradient_zernike_matches_reference(torch, dev, scheme):
    """autograd_tma*: d rms / d (30 Zernike coefficients) of the TMA at field (0, 1),
    uniform 32, 0.587 um, through SurfaceGroup.trace (the reference's operand reads the
    image record, rms_spot_size operand/ray.py:300-340); fringe, standard and noll (whose
    Newton slope omits the normalisation constant: the adjoint VJP, every update taped)."""
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    g = load_golden("autograd_tma" if scheme == "fringe" else f"autograd_tma_{scheme}")
    lens = ThreeMirrorAnastigmat(scheme)
    rays = _generated(torch, lens, 0.0, 1.0, 0.587, 32, dev)
    leaves = []
    for si in (1, 2, 3):
        geo = lens.surface_group.surfaces[si].geometry
        t = torch.tensor(np.asarray(geo.coefficients, dtype=np.float64), device=dev,
                         requires_grad=True)
        geo.coefficients = t
        leaves.append(t)
    _trace_on_mi355x(lens.surface_group, rays, 0)
    loss = _rms(torch, lens.surface_group.surfaces[-1])
    np.testing.assert_allclose(float(loss.detach()), float(g["rms_value"]), rtol=1e-12)
    loss.backward()
    got = np.stack([t.grad.cpu().numpy() for t in leaves])
    scale = np.max(np.abs(g["rms_grad"]))
    np.testing.assert_allclose(got, g["rms_grad"], rtol=1e-8, atol=1e-9 * scale)


@pytest.mark.parametrize("th", [2, 6])
def test_seam_gradient_radius_conic_thickness_matches_reference(torch, dev, th):
    """autograd_cooke: d rms / d (radius 1, 3, 6, conic 5, thickness th) of the Cooke
    triplet, the thickness entering as the vertex z of every later surface (what the
    reference's set_thickness writes, optic_updater.py:64-85)."""
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.samples import CookeTriplet

    g = load_golden("autograd_cooke")
    lens = CookeTriplet()
    rays = _generated(torch, lens, 0.0, 1.0, 0.55, 24, dev)
    sg = lens.surface_group
    leaves = []
    for si in (1, 3, 6):
        t = torch.tensor(float(sg.surfaces[si].geometry.radius), dtype=torch.float64,
                         device=dev, requires_grad=True)
        sg.surfaces[si].geometry.radius = t
        leaves.append(t)
    t = torch.tensor(0.0, dtype=torch.float64, device=dev, requires_grad=True)
    sg.surfaces[5].geometry.k = t
    leaves.append(t)
    t0 = float(sg.surfaces[th].thickness)
    t = torch.tensor(t0, dtype=torch.float64, device=dev, requires_grad=True)
    for s in sg.surfaces[th + 1:]:
        s.geometry.cs.z = float(s.geometry.cs.z) + (t - t0)
    leaves.append(t)
    _trace_on_mi355x(sg, rays, 0)
    loss = _rms(torch, sg.surfaces[-1])
    np.testing.assert_allclose(float(loss.detach()), float(g[f"t{th}_value"]), rtol=1e-13)
    loss.backward()
    got = np.array([float(v.grad) for v in leaves])
    np.testing.assert_allclose(got, g[f"t{th}_grad"], rtol=1e-9, atol=1e-12)


def test_seam_gradcheck_rays_and_records(torch, dev):
    """Input-ray cotangents and record cotangents (central differences of the HIP
    forward): image and intermediate-surface records of the Cooke triplet w.r.t. the input
    x, y, L, M and a radius, all in one backward."""
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.raytrace import RealRays
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    base = _generated(torch, lens, 0.0, 0.7, 0.55, 2, dev, "hexapolar")  # 7 rays
    sg = lens.surface_group
    R0 = float(sg.surfaces[3].geometry.radius)

    def f(x, y, L, M, R):
        sg.surfaces[3].geometry.radius = R
        r = RealRays.__new__(RealRays)
        r.x, r.y, r.z = x, y, base.z
        r.L, r.M, r.N = L, M, torch.sqrt(1 - L * L - M * M)
        r.i, r.opd, r.w = base.i, base.opd, base.w
        _trace_on_mi355x(sg, r, 0)
        s2, s4 = sg.surfaces[2], sg.surfaces[4]
        return r.x, r.y, r.opd, s2.x, s2.L, s4.y, s4.opd

    inputs = tuple(getattr(base, a).clone().requires_grad_(True) for a in ("x", "y", "L", "M"))
    R = torch.tensor(R0, dtype=torch.float64, device=dev, requires_grad=True)
    assert torch.autograd.gradcheck(f, (*inputs, R), eps=1e-7, atol=1e-6, rtol=1e-5,
                                    nondet_tol=1e-12)


def test_seam_intensity_cotangents(torch, dev):
    """d i / d i_in through clipping and absorption (record and output intensity rows)."""
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.samples import GOLDEN_LENSES

    lens = GOLDEN_LENSES["cooke_aperture"]()
    rays = _generated(torch, lens, 0.0, 1.0, 0.55, 8, dev)
    i_in = (0.5 + torch.arange(rays.i.numel(), dtype=torch.float64, device=dev) / 100)
    rays.i = i_in.clone().requires_grad_(True)
    leaf = rays.i
    _trace_on_mi355x(lens.surface_group, rays, 0)
    loss = torch.sum(rays.i) + 2.0 * torch.sum(lens.surface_group.surfaces[2].intensity)
    loss.backward()
    ratio_img = (rays.i / i_in).detach()
    ratio_2 = (lens.surface_group.surfaces[2].intensity / i_in).detach()
    np.testing.assert_allclose(leaf.grad.cpu().numpy(), (ratio_img + 2.0 * ratio_2).cpu().numpy(),
                               rtol=1e-14)


def test_seam_skip_and_cache(torch, dev, golden_index):
    """skip = 3: surfaces before it keep empty records (SurfaceGroup.reset); a second call
    with an unchanged lens reuses the uploaded tables, an edited one re-uploads."""
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.samples import DoubleGauss

    meta = golden_index["dg"]
    g = load_golden("dg")
    n_p = meta["n_pupil"]
    pair = 1
    sl = slice(pair * n_p, (pair + 1) * n_p)
    wl = meta["wavelengths"][pair % len(meta["wavelengths"])]
    lens = DoubleGauss()
    sg = lens.surface_group
    # rays as they leave surface 2 (the golden record): trace surfaces 3.. only
    from optiland_pr_amd.raytrace import RealRays

    rec = g["records"][pair]
    rays = RealRays(*(torch.as_tensor(rec[2, f], device=dev) for f in range(7)), wl, device=dev)
    rays.opd = torch.as_tensor(rec[2, 7], device=dev)
    _trace_on_mi355x(sg, rays, 3)
    for a in ("x", "y", "z", "L", "M", "N", "opd"):
        np.testing.assert_array_equal(getattr(rays, a).cpu().numpy(), g[a][sl], err_msg=a)
    for si in (0, 1, 2):
        assert np.size(sg.surfaces[si].x) == 0
    np.testing.assert_array_equal(sg.surfaces[5].y.cpu().numpy(), rec[5, 1])
    (dl1,) = sg._ort_lenses.values()
    _trace_on_mi355x(sg, _rays(torch, g, sl, wl, dev), 0)
    assert list(sg._ort_lenses.values())[0] is dl1
    sg.surfaces[1].geometry.radius = float(sg.surfaces[1].geometry.radius) * 1.01
    _trace_on_mi355x(sg, _rays(torch, g, sl, wl, dev), 0)
    assert list(sg._ort_lenses.values())[0] is not dl1


def test_seam_refuses_undifferentiated_values(torch, dev):
    """A lens value the derivative kernels do not carry (a decenter, a normalisation
    radius) that requires grad makes the seam hand the call back to the reference loop
    (Unsupported) instead of detaching it; values that need no grad pass."""
    from optiland_pr_amd.adapter import Unsupported, _trace_on_mi355x
    from optiland_pr_amd.samples import CookeTriplet, ThreeMirrorAnastigmat

    lens = CookeTriplet()
    rays = _generated(torch, lens, 0.0, 1.0, 0.55, 4, dev)
    lens.surface_group.surfaces[2].geometry.cs.x = torch.tensor(0.0, dtype=torch.float64,
                                                                requires_grad=True)
    with pytest.raises(Unsupported, match="cs.x"):
        _trace_on_mi355x(lens.surface_group, rays, 0)
    with torch.no_grad():  # no autograd: nothing to differentiate, the trace runs
        _trace_on_mi355x(lens.surface_group, rays, 0)

    tma = ThreeMirrorAnastigmat()
    rays = _generated(torch, tma, 0.0, 1.0, 0.587, 4, dev)
    geo = tma.surface_group.surfaces[2].geometry
    geo.norm_radius = torch.tensor(float(geo.norm_radius), dtype=torch.float64,
                                   requires_grad=True)
    with pytest.raises(Unsupported, match="norm_radius"):
        _trace_on_mi355x(tma.surface_group, rays, 0)


def test_op_is_registered_and_custom(torch, dev):
    """The seam's one autograd node is the registered custom op."""
    from optiland_pr_amd.adapter import _trace_on_mi355x
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    rays = _generated(torch, lens, 0.0, 1.0, 0.55, 4, dev)
    R = torch.tensor(float(lens.surface_group.surfaces[1].geometry.radius),
                     dtype=torch.float64, device=dev, requires_grad=True)
    lens.surface_group.surfaces[1].geometry.radius = R
    _trace_on_mi355x(lens.surface_group, rays, 0)
    assert "trace_sequential" in type(rays.x.grad_fn).__name__ or \
        "ort" in str(rays.x.grad_fn.name())
