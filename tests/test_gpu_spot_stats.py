"""GPU: the spot-diagram statistics kernel (ort_spot_stats) against the reference's
NumPy statistics (analysis/spot_diagram.py:317-357) evaluated on the same traced image
points (the SpotDiagram.data arrays, masked i > 0 and localized as :425-437 do).

Stated tolerance: count exact, max radius exact up to the centroid's rounding (rtol
1e-12), centroid and rms rtol 1e-12 (device tree sums vs NumPy pairwise sums); NaN
where NumPy gives NaN.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("needs the MI355X")
    from optiland_pr_amd import _native

    _native.load()
    return torch


def numpy_stats(spot):
    """spot_diagram.py:317-357 in NumPy on the masked, localized points."""
    data = [[(sd.x.cpu().numpy(), sd.y.cpu().numpy()) for sd in row] for row in spot.data]
    ref = spot._analysis_ref_wavelength_index
    out = []
    for row in data:
        cx, cy = np.mean(row[ref][0]), np.mean(row[ref][1])
        for x, y in row:
            xc, yc = x - cx, y - cy
            with np.errstate(all="ignore"):
                rms = np.sqrt(np.mean(xc**2 + yc**2))
                geo = np.max(np.sqrt(xc**2 + yc**2)) if x.size else np.nan
                mx, my = np.mean(x), np.mean(y)
            out.append((x.size, mx, my, rms, geo))
    return np.array(out, dtype=np.float64)


def check(spot):
    got = spot._stats.cpu().numpy()
    ref = numpy_stats(spot)
    np.testing.assert_array_equal(got[:, 0], ref[:, 0])
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_allclose(got[:, 1:], ref[:, 1:], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("coords", ["local", "global"])
def test_cooke_hexapolar(gpu, coords):
    from optiland_pr_amd.analysis import SpotDiagram
    from optiland_pr_amd.samples import CookeTriplet

    check(SpotDiagram(CookeTriplet(), coordinates=coords))


def test_decentered_local_frame(gpu):
    """Tilted / decentred elements: the localize ops of the image surface applied to
    points on the device."""
    from optiland_pr_amd.analysis import SpotDiagram
    from optiland_pr_amd.samples import DecenteredTriplet

    lens = DecenteredTriplet()
    check(SpotDiagram(lens, num_rings=12))
    lens.surface_group.surfaces[-1].geometry.cs.rx = 0.05  # tilt the image plane
    lens.surface_group.surfaces[-1].geometry.cs.y = 0.3
    lens.invalidate()
    check(SpotDiagram(lens, num_rings=12))


def test_many_chunks_uniform(gpu):
    """~1M points per pair: several 2048-ray chunks per pair, three pairs."""
    from optiland_pr_amd.analysis import SpotDiagram
    from optiland_pr_amd.samples import DoubleGauss

    spot = SpotDiagram(DoubleGauss(), fields=[(0, 0), (0, 1)], wavelengths="all",
                       num_rings=1129, distribution="uniform")
    check(spot)


def test_clipped_and_missing_rays(gpu):
    """An aperture that clips part of the pupil (i = 0 points leave the statistics) and
    a field where some rays miss a surface (NaN points propagate as in NumPy)."""
    from optiland_pr_amd.analysis import SpotDiagram
    from optiland_pr_amd.samples import CookeTripletApertures

    check(SpotDiagram(CookeTripletApertures(), num_rings=10))


def test_empty_spot(gpu):
    """Every ray clipped: count 0, NaN centroid / rms; geometric radius raises as
    NumPy's max of an empty array does."""
    from optiland_pr_amd.analysis import SpotDiagram
    from optiland_pr_amd.samples import CookeTriplet
    from optiland_pr_amd.surfaces import RadialAperture

    lens = CookeTriplet()
    lens.surface_group.surfaces[2].aperture = RadialAperture(r_max=1e-9, r_min=1e-10)
    lens.invalidate()
    spot = SpotDiagram(lens, fields=[(0, 0)], wavelengths=[0.55], num_rings=4)
    st = spot._stats.cpu().numpy()
    assert st[0, 0] == 0 and np.all(np.isnan(st[0, 1:4]))
    with pytest.raises(ValueError):
        spot.geometric_spot_radius()
