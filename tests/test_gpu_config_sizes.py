"""GPU parity at the BASELINE configs' own sizes, against summaries the
reference produced here (tests/golden/config_sizes.json, gen_config_sizes.py; and
index.json _full, gen_golden.py):

  config 1  the exact spot-diagram workload: Cooke triplet, Hy = 0 / 0.7 / 1, 0.55 um,
            uniform 128 (37,932 rays): image-plane sums per field equal the reference's
            (bit-exact trace => identical NumPy reductions), SpotDiagram centroids / radii
            (device reduction, another summation order) rtol 1e-12;
  config 3  3 of the 15 RT-asph (field, lambda) pairs at the full 4M random rays
            (seed = pair index): sums within the Newton tolerances of the reference's;
  config 4  3 of the 49 ReverseTelephoto (field, lambda) pairs at the full 2M random
            rays (seed = pair index) through the bench's per-ray-pupil launch: NumPy sums of
            x, y, opd, x^2, first / last ray identical to the reference's.
"""

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("needs the MI355X")
    from optiland_pr_amd import _native

    _native.load()
    return torch


@pytest.fixture(scope="module")
def sizes():
    with open(os.path.join(HERE, "golden", "config_sizes.json")) as f:
        return json.load(f)


def test_config1_spot_diagram_workload(torch, sizes, golden_index):
    from optiland_pr_amd.analysis import SpotDiagram
    from optiland_pr_amd.samples import CookeTriplet

    ref = sizes["config1"]
    lens = CookeTriplet()
    spot = SpotDiagram(lens, wavelengths=[0.55], num_rings=128, distribution="uniform")
    assert spot.rays.x.numel() == 3 * 12644
    geo = [[float(v) for v in row] for row in spot.geometric_spot_radius()]
    rms = [[float(v) for v in row] for row in spot.rms_spot_radius()]
    cen = [[float(a), float(b)] for a, b in spot.centroid()]
    np.testing.assert_allclose(geo, ref["geo"], rtol=1e-12)
    np.testing.assert_allclose(rms, ref["rms"], rtol=1e-12)
    np.testing.assert_allclose(cen, ref["centroid"], rtol=1e-12, atol=1e-15)
    # the image-plane rays of each field: the reference's own NumPy sums, bit for bit
    full = golden_index["_full"]["cooke_uniform128"]
    x = spot.rays.x.cpu().numpy().reshape(3, -1)
    y = spot.rays.y.cpu().numpy().reshape(3, -1)
    for f in range(3):
        assert x[f].size == full[f]["n"]
        assert float(np.sum(x[f])) == full[f]["sum_x"]
        assert float(np.sum(y[f])) == full[f]["sum_y"]
        assert float(np.mean(y[f])) == full[f]["mean_y"]
        assert float(np.std(y[f])) == full[f]["std_y"]


@pytest.mark.parametrize("pair", [0, 24, 48])
def test_config4_pairs_at_2m_rays(torch, sizes, pair):
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil
    from optiland_pr_amd.samples import ReverseTelephoto

    ref = sizes["config4"][str(pair)]
    lens = ReverseTelephoto()
    wls = [float(w) for w in np.linspace(0.4861, 0.6563, 7)]
    dl = lens_for(lens, wls)
    seg = np.stack([segment_params(lens, 0.0, ref["hy"], pair % 7)])
    assert wls[pair % 7] == ref["wavelength"]
    d = RandomDistribution(seed=pair)
    d.generate_points(2_000_000)
    px = torch.as_tensor(np.asarray(d.x), device="cuda")
    py = torch.as_tensor(np.asarray(d.y), device="cuda")
    n = px.numel()
    out = RealRays.empty(n, 0.0)
    trace_pupil(dl, seg, px, py, out, n, n, n, pupil_per_ray=True)
    x, y, opd = (getattr(out, a).cpu().numpy() for a in ("x", "y", "opd"))
    assert x.size == ref["n"] and int(np.isnan(x).sum()) == ref["nan"]
    assert float(np.sum(x)) == ref["sum_x"]
    assert float(np.sum(y)) == ref["sum_y"]
    assert float(np.sum(opd)) == ref["sum_opd"]
    assert float(np.sum(x * x)) == ref["sum_x2"]
    assert [float(x[0]), float(y[0]), float(opd[0])] == ref["first"]
    assert [float(x[-1]), float(y[-1]), float(opd[-1])] == ref["last"]


@pytest.mark.parametrize("pair", [0, 7, 14])
def test_config3_pairs_at_4m_rays(torch, sizes, pair):
    """Config 3's Newton lens at its own size: 3 of the 15 RT-asph (field, lambda) pairs at
    the full 4M random pupil rays (seed = pair index), one launch per pair with the Newton
    schedule verified against the reference's global stop rule. Newton tolerances: each ray
    within 1e-9 mm of the reference, so sums over 4M rays within 4M x 1e-12 relative
    scale; the first / last rays 1e-9 mm."""
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil
    from optiland_pr_amd.samples import ReverseTelephotoAsphere

    ref = sizes["config3"][str(pair)]
    lens = ReverseTelephotoAsphere()
    wls = [0.4861, 0.5876, 0.6563]
    assert wls[pair % 3] == ref["wavelength"]
    dl = lens_for(lens, wls)
    seg = np.stack([segment_params(lens, 0.0, ref["hy"], pair % 3)])
    d = RandomDistribution(seed=pair)
    d.generate_points(4_000_000)
    px = torch.as_tensor(np.asarray(d.x), device="cuda")
    py = torch.as_tensor(np.asarray(d.y), device="cuda")
    n = px.numel()
    out = RealRays.empty(n, 0.0)
    trace_pupil(dl, seg, px, py, out, n, n, n, keys=[("c3", pair)])
    x, y, opd = (getattr(out, a).cpu().numpy() for a in ("x", "y", "opd"))
    assert x.size == ref["n"] and int(np.isnan(x).sum()) == ref["nan"]
    np.testing.assert_allclose(float(np.sum(x)), ref["sum_x"], rtol=1e-12, atol=1e-5)
    np.testing.assert_allclose(float(np.sum(y)), ref["sum_y"], rtol=1e-12, atol=1e-5)
    np.testing.assert_allclose(float(np.sum(opd)), ref["sum_opd"], rtol=1e-12)
    np.testing.assert_allclose(float(np.sum(x * x)), ref["sum_x2"], rtol=1e-10)
    np.testing.assert_allclose([x[0], y[0], opd[0]], ref["first"], rtol=0, atol=1e-9)
    np.testing.assert_allclose([x[-1], y[-1], opd[-1]], ref["last"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("scheme", ["fringe", "standard", "noll"])
def test_config5_loss_and_gradient_at_1m_rays(torch, scheme):
    """Config 5 at its own size: the TMA loss rms_spot_size over 1M random pupil rays
    (seed 0, Hy = 1, 0.587 um) and d rms / d c for the 30 Zernike coefficients, as the
    reference's torch backend computes them (tests/golden/autograd_tma_1m.json and
    autograd_tma_{standard,noll}_1m.json, gen_autograd_golden.py --full): fringe, and
    SURVEY 8d.5's "standard" variant (whose Newton slope omits the normalisation
    constant; the adjoint serves it, every update taped). The pupil sample is NumPy's
    stream (sums bit-exact); the loss within rtol 1e-12 (reduction order), the gradient
    within rtol 1e-8 as the smaller autograd goldens (adjoint vs torch's unrolled
    graph)."""
    import json

    from optiland_pr_amd import autodiff
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.operands import RayOperand
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    name = "autograd_tma_1m" if scheme == "fringe" else f"autograd_tma_{scheme}_1m"
    path = os.path.join(HERE, "golden", name + ".json")
    with open(path) as f:
        ref = json.load(f)
    d = RandomDistribution(seed=0)
    d.generate_points(1_000_000)
    assert float(np.sum(np.asarray(d.x))) == ref["px_sum"]
    assert float(np.sum(np.asarray(d.y))) == ref["py_sum"]
    lens = ThreeMirrorAnastigmat(scheme)
    leaves = []
    for si in (1, 2, 3):
        g = lens.surface_group.surfaces[si].geometry
        t = torch.tensor(np.asarray(g.coefficients), dtype=torch.float64, device="cuda",
                         requires_grad=True)
        g.coefficients = t
        leaves.append(t)
    calls = []
    real_vjp = autodiff.vjp

    def spy(*a, **k):
        calls.append(k.get("mode"))
        return real_vjp(*a, **k)

    autodiff.vjp = spy
    try:
        rms = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 1_000_000, 0.587, d)
        rms.backward()
    finally:
        autodiff.vjp = real_vjp
    from optiland_pr_amd import _abi

    assert calls == [_abi.VJP_ADJOINT]  # one reverse sweep, for every scheme
    np.testing.assert_allclose(float(rms.detach()), ref["rms"], rtol=1e-12)
    got = np.stack([t.grad.cpu().numpy() for t in leaves])
    np.testing.assert_allclose(got, np.asarray(ref["grad"]), rtol=1e-8, atol=1e-12)
