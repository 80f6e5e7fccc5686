"""GPU: autograd through the HIP trace (config 5) against the reference's torch-CPU
autograd (tests/golden/autograd_tma.npz, gen_autograd_golden.py; pinned against the
oracle by finite differences in test_autograd_oracle.py).

Tolerances: the forward values agree with the reference to a few ulps (the Zernike
azimuth is a recurrence here, atan2/cos/sin there); gradients computed in forward mode
(dual numbers) vs reverse mode differ by rounding only: rtol 1e-8, atol 1e-9 x max|g|.
"""

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WSUM_FIELDS = ("x", "y", "z", "L", "M", "N", "opd")


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("needs the MI355X")
    from optiland_pr_amd import _native

    _native.load()
    return torch


def _tma_with_leaves(torch, coeffs=None, device="cpu", scheme="fringe"):
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    lens = ThreeMirrorAnastigmat(scheme)
    leaves = []
    for k, si in enumerate((1, 2, 3)):
        g = lens.surface_group.surfaces[si].geometry
        c = np.asarray(g.coefficients if coeffs is None else coeffs[k], dtype=np.float64)
        t = torch.tensor(c, dtype=torch.float64, device=device, requires_grad=True)
        g.coefficients = t
        leaves.append(t)
    return lens, leaves


def _close(got, ref):
    scale = np.max(np.abs(ref))
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-9 * scale)


SCHEMES = ["fringe", "standard", "noll"]


def _golden(scheme):
    from tests.conftest import load_golden

    return load_golden("autograd_tma" if scheme == "fringe" else f"autograd_tma_{scheme}")


@pytest.mark.parametrize("scheme", SCHEMES)
def test_rms_spot_size_gradient_matches_reference(torch, scheme):
    """d rms / d c of the three Zernike mirrors against the reference's torch autograd
    (autograd_tma*.npz): fringe, and the standard / noll schemes whose Newton slope omits
    the normalisation constant (the adjoint serves them with every update taped)."""
    from optiland_pr_amd.operands import RayOperand

    g = _golden(scheme)
    lens, leaves = _tma_with_leaves(torch, scheme=scheme)
    loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 32, 0.587, "uniform")
    assert loss.requires_grad
    np.testing.assert_allclose(float(loss.detach()), float(g["rms_value"]), rtol=1e-12)
    loss.backward()
    got = np.stack([t.grad.numpy() for t in leaves])
    _close(got, g["rms_grad"])


@pytest.mark.parametrize("scheme", SCHEMES)
def test_weighted_output_gradient_matches_reference(torch, scheme):
    g = _golden(scheme)
    lens, leaves = _tma_with_leaves(torch, scheme=scheme)
    rays = lens.trace(0.0, -1.0, 0.587, num_rays=32, distribution="uniform")
    loss = 0.0
    for f in WSUM_FIELDS:
        w = torch.as_tensor(g[f"wsum_w_{f}"], device=rays.x.device)
        loss = loss + torch.sum(w * getattr(rays, f))
    np.testing.assert_allclose(float(loss.detach()), float(g["wsum_value"]), rtol=1e-11)
    loss.backward()
    got = np.stack([t.grad.numpy() for t in leaves])
    _close(got, g["wsum_grad"])


def test_tangent_chunking_agrees(torch):
    """1, 2 or 4 tangents per launch: the same derivatives (atomics order aside)."""
    from optiland_pr_amd.operands import RayOperand

    res = []
    old = os.environ.get("ORT_VJP_TANGENTS")
    try:
        for p in ("1", "2", "4"):
            os.environ["ORT_VJP_TANGENTS"] = p
            lens, leaves = _tma_with_leaves(torch)
            RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 16, 0.587, "hexapolar").backward()
            res.append(np.stack([t.grad.numpy() for t in leaves]))
    finally:
        if old is None:
            os.environ.pop("ORT_VJP_TANGENTS", None)
        else:
            os.environ["ORT_VJP_TANGENTS"] = old
    np.testing.assert_allclose(res[0], res[1], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(res[0], res[2], rtol=1e-13, atol=1e-15)


def test_gradcheck_nonzero_coefficients(torch):
    """torch.autograd.gradcheck (central differences) on the image x, y of a small batch.
    All coefficients non-zero: the reference (and this op) drop zero terms from the
    normal, which finite differences at c = 0 cannot see."""
    base = np.array([2e-5, -1e-5, 3e-5, 1e-4, 2e-4, -1e-4, 5e-5, 1e-5, -2e-5, 3e-5])
    lens, _ = _tma_with_leaves(torch, [base, base, base])
    geo = lens.surface_group.surfaces[2].geometry
    c0 = geo.coefficients.detach().clone().requires_grad_(True)

    def f(c):
        geo.coefficients = c
        r = lens.trace(0.0, 1.0, 0.587, num_rays=3, distribution="hexapolar")
        return r.x, r.y, r.opd

    assert torch.autograd.gradcheck(f, (c0,), eps=1e-7, atol=1e-6, rtol=1e-4,
                                    nondet_tol=1e-12)


def test_no_grad_mode_uses_plain_trace(torch):
    lens, leaves = _tma_with_leaves(torch)
    with torch.no_grad():
        rays = lens.trace(0.0, 1.0, 0.587, num_rays=8, distribution="uniform")
    assert not rays.x.requires_grad


def test_full_size_directional_derivative(torch):
    """Config 5 at its BASELINE size: 1M random pupil rays (seed 0), field Hy = 1.
    Size-independent checks: the VJP is linear in the cotangent, and grad . d matches a
    central difference of the HIP forward along a random direction d."""
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.operands import RayOperand

    d = RandomDistribution(seed=0)
    d.generate_points(1_000_000)
    lens, leaves = _tma_with_leaves(torch)
    loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 1_000_000, 0.587, d)
    loss.backward()
    grad = np.concatenate([t.grad.numpy() for t in leaves])
    assert np.all(np.isfinite(grad))

    rng = np.random.default_rng(7)
    direc = rng.standard_normal(grad.size)
    direc /= np.linalg.norm(direc)
    c0 = np.concatenate([t.detach().numpy() for t in leaves])
    h = 1e-7

    def value(c):
        lens2, _ = _tma_with_leaves(torch, c.reshape(3, 10))
        with torch.no_grad():
            return float(RayOperand.rms_spot_size(lens2, -1, 0.0, 1.0, 1_000_000, 0.587, d))

    fd = (value(c0 + h * direc) - value(c0 - h * direc)) / (2 * h)
    # zero coefficients: the normal skips them (reference quirk), so compare only the
    # non-zero ones along the direction
    nz = c0 != 0
    direc_nz = np.where(nz, direc, 0.0)
    fd_nz = (value(c0 + h * direc_nz) - value(c0 - h * direc_nz)) / (2 * h)
    assert np.dot(grad, direc_nz) == pytest.approx(fd_nz, rel=1e-5, abs=1e-9)
    assert np.isfinite(fd)


def test_vjp_linear_in_cotangent(torch):
    from optiland_pr_amd import autodiff
    from optiland_pr_amd.raytrace import RealRayTracer

    lens, leaves = _tma_with_leaves(torch)
    rays = RealRayTracer(lens).trace(0.0, 0.0, 0.587, 64, "hexapolar")
    n = rays.x.numel()
    gen = torch.Generator(device=rays.x.device).manual_seed(3)
    a = torch.randn(n, dtype=torch.float64, device=rays.x.device, generator=gen)
    b = torch.randn(n, dtype=torch.float64, device=rays.x.device, generator=gen)

    def g(cx, cy):
        return torch.autograd.grad((rays.x, rays.y), leaves, (cx, cy), retain_graph=True)

    ga, gb, gab = g(a, b * 0), g(a * 0, b), g(a, b)
    for u, v, w in zip(ga, gb, gab, strict=True):
        np.testing.assert_allclose((u + v).numpy(), w.numpy(), rtol=1e-10,
                                   atol=1e-12 * float(w.abs().max()))
    assert autodiff.wants_grad(lens)


@pytest.mark.parametrize("th", [2, 6])
def test_shape_parameter_gradients_match_reference(torch, th):
    """d rms / d (radius 1, 3, 6; conic 5; thickness after surface `th`) of the Cooke
    triplet vs the reference's torch autograd (autograd_cooke.npz; pinned against the
    oracle by finite differences in test_autograd_oracle.py)."""
    from optiland_pr_amd.operands import RayOperand
    from optiland_pr_amd.samples import CookeTriplet
    from tests.conftest import load_golden

    g = load_golden("autograd_cooke")
    lens = CookeTriplet()
    leaves = []
    for si in (1, 3, 6):
        t = torch.tensor(float(lens.surface_group.surfaces[si].geometry.radius),
                         dtype=torch.float64, requires_grad=True)
        lens.set_radius(t, si)
        leaves.append(t)
    t = torch.tensor(0.0, dtype=torch.float64, requires_grad=True)
    lens.set_conic(t, 5)
    leaves.append(t)
    t = torch.tensor(float(lens.surface_group.surfaces[th].thickness), dtype=torch.float64,
                     requires_grad=True)
    lens.set_thickness(t, th)
    leaves.append(t)
    loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 24, 0.55, "uniform")
    np.testing.assert_allclose(float(loss.detach()), float(g[f"t{th}_value"]), rtol=1e-13)
    loss.backward()
    got = np.array([float(v.grad) for v in leaves])
    np.testing.assert_allclose(got, g[f"t{th}_grad"], rtol=1e-9, atol=1e-12)


def test_gradcheck_radius_conic_zernike_mixed(torch):
    """gradcheck over a mixed parameter set on the TMA: a mirror radius, a conic and
    non-zero Zernike coefficients (all entering the Newton iteration)."""
    base = np.array([2e-5, -1e-5, 3e-5, 1e-4, 2e-4, -1e-4, 5e-5, 1e-5, -2e-5, 3e-5])
    lens, _ = _tma_with_leaves(torch, [base, base, base])
    g1 = lens.surface_group.surfaces[1].geometry
    g2 = lens.surface_group.surfaces[2].geometry
    for g in (lens.surface_group.surfaces[si].geometry for si in (1, 2, 3)):
        g.coefficients = g.coefficients.detach()
    R = torch.tensor(-100.0, dtype=torch.float64, requires_grad=True)
    k = torch.tensor(0.05, dtype=torch.float64, requires_grad=True)
    c = torch.tensor(base, dtype=torch.float64, requires_grad=True)

    def f(R_, k_, c_):
        g1.radius = R_
        g2.k = k_
        lens.surface_group.surfaces[3].geometry.coefficients = c_
        r = lens.trace(0.0, 1.0, 0.587, num_rays=3, distribution="hexapolar")
        return r.x, r.y, r.L

    assert torch.autograd.gradcheck(f, (R, k, c), eps=1e-7, atol=1e-6, rtol=1e-4,
                                    nondet_tol=1e-12)


def test_device_resident_coefficients(torch):
    """Coefficient leaves in HBM (the uploaded Zernike table patched on the device, no
    host round trip) give the same loss and gradients as host leaves, bit for bit; the
    Adam trajectory agrees to rounding (torch's CPU and CUDA Adam kernels themselves
    may round the update differently, which then feeds the next step)."""
    from optiland_pr_amd.operands import RayOperand

    res = {}
    for dev in ("cpu", "cuda"):
        lens, leaves = _tma_with_leaves(torch, device=dev)
        opt = torch.optim.Adam(leaves, lr=1e-6)
        losses, grads = [], []
        for _ in range(3):
            opt.zero_grad()
            loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 24, 0.587, "uniform")
            loss.backward()
            grads.append(np.stack([t.grad.cpu().numpy() for t in leaves]))
            opt.step()
            losses.append(float(loss.detach()))
        res[dev] = (losses, np.stack([t.detach().cpu().numpy() for t in leaves]), grads)
    assert res["cpu"][0][0] == res["cuda"][0][0]
    assert np.array_equal(res["cpu"][2][0], res["cuda"][2][0])  # first step: same inputs
    np.testing.assert_allclose(res["cpu"][0], res["cuda"][0], rtol=1e-12)
    for gc, gg in zip(res["cpu"][2], res["cuda"][2]):
        np.testing.assert_allclose(gc, gg, rtol=1e-9, atol=1e-12 * np.max(np.abs(gc)))
    np.testing.assert_allclose(res["cpu"][1], res["cuda"][1], rtol=0, atol=1e-15)


@pytest.mark.parametrize("name", ["tma_fringe", "rt_asph"])
def test_taped_forward_gradients_bit_identical(torch, name, monkeypatch):
    """The forward writes the adjoint tape (F_TAPE) and the backward runs only the reverse
    sweep: the same tape values as the adjoint's own re-trace, so the same gradients to
    the last bit (and the same loss). Both runs take the two-pass ort::rms_spot (the
    untaped trace cannot fuse the rms; test_fused_rms_matches_unfused compares the two
    reductions)."""
    from optiland_pr_amd import autodiff, operands

    monkeypatch.setattr(operands, "FUSED_RMS", False)
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.operands import RayOperand
    from tests._cases import build_lens

    d = RandomDistribution(seed=1)
    d.generate_points(20000)
    wl = 0.587 if name.startswith("tma") else 0.5876
    res = []
    old = autodiff.TAPED_FORWARD
    try:
        for taped in (False, True):
            autodiff.TAPED_FORWARD = taped
            lens = build_lens(name)
            leaves = []
            for s in lens.surface_group.surfaces[1:]:
                g = s.geometry
                if hasattr(g, "coefficients") and type(g).__name__ == "ZernikePolynomialGeometry":
                    t = torch.tensor(np.asarray(g.coefficients), dtype=torch.float64,
                                     device="cuda", requires_grad=True)
                    g.coefficients = t
                    leaves.append(t)
                elif type(g).__name__ == "EvenAsphere":
                    t = torch.tensor(float(g.radius), dtype=torch.float64, device="cuda",
                                     requires_grad=True)
                    g.radius = t
                    leaves.append(t)
            loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 20000, wl, d)
            loss.backward()
            res.append((float(loss.detach()), np.concatenate([t.grad.reshape(-1).cpu().numpy()
                                                     for t in leaves])))
    finally:
        autodiff.TAPED_FORWARD = old
    assert res[0][0] == res[1][0]
    np.testing.assert_array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("device", ["cpu", "cuda"])
def test_fused_rms_matches_unfused(torch, device, monkeypatch):
    """Config 5's loss with the rms in the taped forward's epilogue (F_RMS rows +
    ort_rms_finish, the gradient folded into the adjoint's cotangent load) against the trace
    followed by ort::rms_spot / ort::rms_spot_vjp (ORT_FUSED_RMS=0): same value to rounding
    (Chan's combination of per-workgroup moments vs the two-pass centroid), same
    coefficient gradients (rtol 1e-10), on 1M random rays; run twice, bit-identical."""
    from optiland_pr_amd import operands
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.operands import RayOperand

    d = RandomDistribution(seed=0)
    d.generate_points(1_000_000)
    res = {}
    for fused in (True, False, True):
        monkeypatch.setattr(operands, "FUSED_RMS", fused)
        lens, leaves = _tma_with_leaves(torch, device=device)
        loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 1_000_000, 0.587, d)
        loss.backward()
        g = np.concatenate([t.grad.cpu().numpy() for t in leaves])
        v = float(loss.detach())
        if fused in res:
            assert v == res[fused][0]
            np.testing.assert_array_equal(g, res[fused][1])
        res[fused] = (v, g)
    assert res[True][0] == pytest.approx(res[False][0], rel=1e-13)
    scale = np.max(np.abs(res[False][1]))
    np.testing.assert_allclose(res[True][1], res[False][1], rtol=1e-10, atol=1e-12 * scale)


# gen_autograd_golden.py IA_CASES: radius leaves (surfaces) and the wavelength per lens
IA_CASES = {"paraxial_lens": ((2, 3), 0.55), "phase_plate": ((2, 3), 0.55),
            "grating_curved": ((), 0.587)}


@pytest.mark.parametrize("name", sorted(IA_CASES))
def test_gradients_through_interaction_models(torch, name):
    """d rms / d (radii, thickness after surface 1) through thin-lens, phase and grating
    surfaces vs the reference's torch autograd (autograd_ia.npz, gen_autograd_golden.py
    --ia): the forward-mode VJP carries the interaction models in duals (vjp_ray; the
    adjoint has no reverse for them, autodiff.vjp_mode)."""
    from optiland_pr_amd import _abi, autodiff
    from optiland_pr_amd.operands import RayOperand
    from tests._cases import build_lens
    from tests.conftest import load_golden

    rsurf, wl = IA_CASES[name]
    g = load_golden("autograd_ia")
    lens = build_lens(name)
    leaves = []
    for si in rsurf:
        t = torch.tensor(float(lens.surface_group.surfaces[si].geometry.radius),
                         dtype=torch.float64, requires_grad=True)
        lens.set_radius(t, si)
        leaves.append(t)
    t = torch.tensor(float(lens.surface_group.surfaces[1].thickness), dtype=torch.float64,
                     requires_grad=True)
    lens.set_thickness(t, 1)
    leaves.append(t)
    loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 16, wl, "uniform")
    np.testing.assert_allclose(float(loss.detach()), float(g[f"{name}_value"]), rtol=1e-12)
    loss.backward()
    got = np.array([float(v.grad) for v in leaves])
    np.testing.assert_allclose(got, g[f"{name}_grad"], rtol=1e-9, atol=1e-13)
    from optiland_pr_amd.lowering import lower_surface_group

    table = lower_surface_group(lens.surface_group, [wl])
    assert autodiff.vjp_mode(table) == _abi.VJP_UNROLLED
