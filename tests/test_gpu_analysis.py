"""GPU: the trace's consumers against the reference's own goldens.

SpotDiagram radii for the Cooke triplet (reference tests/test_analysis.py:69-100) and
OPD RMS (tests/test_wavefront.py:135-139), recomputed from the reference here
(tests/golden/index.json "_analysis"). Reductions run on the device in a different
order than NumPy's pairwise sums: rtol 1e-12 (radii) / 1e-10 (OPD in waves).
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("needs the MI355X")
    return torch


def test_cooke_spot_diagram(gpu, golden_index):
    from optiland_pr_amd.analysis import SpotDiagram
    from optiland_pr_amd.samples import CookeTriplet

    ref = golden_index["_analysis"]
    spot = SpotDiagram(CookeTriplet())
    geo = [[float(v) for v in row] for row in spot.geometric_spot_radius()]
    rms = [[float(v) for v in row] for row in spot.rms_spot_radius()]
    np.testing.assert_allclose(geo, ref["cooke_geo_radius"], rtol=1e-12)
    np.testing.assert_allclose(rms, ref["cooke_rms_radius"], rtol=1e-12)
    cen = [[float(a), float(b)] for a, b in spot.centroid()]
    np.testing.assert_allclose(cen, ref["cooke_centroid"], rtol=1e-12, atol=1e-14)
    # the reference test's hard-coded values (rtol 1e-5 there)
    np.testing.assert_allclose(geo[0][0], 0.00597244087781, rtol=1e-5)
    np.testing.assert_allclose(rms[2][2], 0.013596802321537, rtol=1e-5)


@pytest.mark.parametrize("case", [("cooke", (0, 1), 0.55, "cooke_opd_rms_0_1_055"),
                                  ("dg", (0, 1), 0.5876, "dg_opd_rms_0_1_05876"),
                                  ("dg", (0, 0), 0.5876, "dg_opd_rms_0_0_05876")])
def test_opd_rms(gpu, golden_index, case):
    from optiland_pr_amd.analysis import OPD
    from optiland_pr_amd.samples import CookeTriplet, DoubleGauss

    name, field, wl, key = case
    lens = CookeTriplet() if name == "cooke" else DoubleGauss()
    rms = float(OPD(lens, field, wl).rms())
    np.testing.assert_allclose(rms, golden_index["_analysis"][key], rtol=1e-10)
    if key == "cooke_opd_rms_0_1_055":
        np.testing.assert_allclose(rms, 0.9709788038168692, rtol=1e-5)  # test_wavefront.py:139


@pytest.mark.parametrize("key, rms_key", [("cooke_0_1", None),
                                          ("cooke_0_07_notilt", None),
                                          ("dg_0_1", None),
                                          ("finite_pih_03_07", None)])
def test_wavefront_per_ray(gpu, key, rms_key):
    """The fused wavefront kernel (ort_wavefront_opd) per ray against the reference's
    WavefrontData (strategy.py:168-239): pupil points and OPD in waves bit-exact (same
    IEEE operations in the same order on bit-identical traced rays); with the piston /
    tilt removed (wavefront.py:97-143) to 1e-9 waves (the fit's sums are reduced in a
    different order)."""
    import os

    from optiland_pr_amd.analysis import OPD
    from optiland_pr_amd.samples import CookeTriplet, DoubleGauss, FiniteTripletImageHeight

    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                             "wavefront.npz"), allow_pickle=False)
    builders = {"cooke_0_1": (CookeTriplet, (0, 1), 0.55, {}),
                "cooke_0_07_notilt": (CookeTriplet, (0, 0.7), 0.48, {"remove_tilt": True}),
                "dg_0_1": (DoubleGauss, (0, 1), 0.5876, {"num_rays": 20}),
                "finite_pih_03_07": (FiniteTripletImageHeight, (0.3, 0.7), 0.55, {})}
    builder, field, wl, kw = builders[key]
    w = OPD(builder(), field, wl, **kw)
    d = w.get_data(w.fields[0], w.wavelengths[0])
    assert d.radius == float(g[f"{key}/radius"])
    for a in ("pupil_x", "pupil_y", "pupil_z"):
        np.testing.assert_array_equal(getattr(d, a).cpu().numpy(), g[f"{key}/{a}"], err_msg=a)
    # intensity: the trace's stated rel 1e-12 (absorption exponent accumulated per ray)
    np.testing.assert_allclose(d.intensity.cpu().numpy(), g[f"{key}/intensity"], rtol=1e-12)
    got = d.opd.cpu().numpy()
    if kw.get("remove_tilt"):
        np.testing.assert_allclose(got, g[f"{key}/opd"], rtol=0, atol=1e-9)
    else:
        np.testing.assert_array_equal(got, g[f"{key}/opd"])


@pytest.mark.parametrize("case", [("cooke", (0, 1), 0.55, "cooke_opd_rms_0_1_055_notilt"),
                                  ("dg", (0, 1), 0.5876, "dg_opd_rms_0_1_05876_notilt")])
def test_opd_rms_remove_tilt(gpu, golden_index, case):
    from optiland_pr_amd.analysis import OPD
    from optiland_pr_amd.samples import CookeTriplet, DoubleGauss

    name, field, wl, key = case
    lens = CookeTriplet() if name == "cooke" else DoubleGauss()
    rms = float(OPD(lens, field, wl, remove_tilt=True).rms())
    np.testing.assert_allclose(rms, golden_index["_analysis"][key], rtol=1e-10)
