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
