"""Wavefront reference-sphere strategies "centroid_sphere" and "best_fit_sphere"
(wavefront/strategy.py:242-479) against the reference's WavefrontData
(tests/golden/wavefront_strategies.npz, made by gen_golden.py --wavefront-strategies).

Stated parity: pupil points, OPD in waves and the sphere radius (and the best-fit centre)
BIT-EXACT -- the per-ray chain is the reference's IEEE operations in its order and the
sphere comes from the same NumPy reductions / LAPACK least squares on a bit-identical point
set; with the tilt removed 1e-12 waves; OPD.rms() relative 1e-12 (a device mean).

The CPU test drives the strategies' host logic with rays traced by the oracle (tests
only); its per-ray chain then runs on torch's CPU kernels, whose float64 sqrt is not
always correctly rounded (SLEEF; 98 of 721 rays 1 ulp off for dg_0_0_bestfit), so there
the pupil points are held to 1e-12 mm, the OPD to 1e-9 waves and the sphere to exact
equality (rms and the tilt-removed OPD to 1e-9). The GPU test runs
the whole path (HIP trace + device per-ray chain, IEEE sqrt) and is bit-exact."""

import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {  # as gen_golden.WAVEFRONT_STRATEGY_CASES
    "cooke_0_1_centroid": ("cooke", (0, 1), 0.55, {"strategy": "centroid_sphere"}),
    "cooke_0_07_bestfit": ("cooke", (0, 0.7), 0.48, {"strategy": "best_fit_sphere"}),
    "cooke_0_1_centroid_notrim": ("cooke", (0, 1), 0.55,
                                  {"strategy": "centroid_sphere", "robust_trim_std": 0.0}),
    "dg_0_1_centroid": ("dg", (0, 1), 0.5876, {"strategy": "centroid_sphere", "num_rays": 20}),
    "dg_0_0_bestfit": ("dg", (0, 0), 0.5876, {"strategy": "best_fit_sphere"}),
    "dg_0_1_bestfit_notilt": ("dg", (0, 1), 0.5876,
                              {"strategy": "best_fit_sphere", "remove_tilt": True}),
    "finite_pih_03_07_centroid": ("finite_pih", (0.3, 0.7), 0.55,
                                  {"strategy": "centroid_sphere"}),
}


def _golden():
    return np.load(os.path.join(HERE, "golden", "wavefront_strategies.npz"), allow_pickle=False)


def _lens(name):
    from optiland_pr_amd.samples import CookeTriplet, DoubleGauss, FiniteTripletImageHeight

    return {"cooke": CookeTriplet, "dg": DoubleGauss,
            "finite_pih": FiniteTripletImageHeight}[name]()


def _equal(got, want, exact, msg):
    if exact:
        np.testing.assert_array_equal(got, want, err_msg=msg)
    else:
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-12, err_msg=msg)


def _check(key, w, g, exact=True):
    d = w.get_data(w.fields[0], w.wavelengths[0])
    assert d.radius == float(g[f"{key}/radius"]), key
    if f"{key}/center" in g.files:
        assert list(w.strategy.center) == [float(v) for v in g[f"{key}/center"]]
    for a in ("pupil_x", "pupil_y", "pupil_z"):
        _equal(getattr(d, a).cpu().numpy(), g[f"{key}/{a}"], exact, f"{key}.{a}")
    np.testing.assert_allclose(d.intensity.cpu().numpy(), g[f"{key}/intensity"], rtol=1e-12)
    got = d.opd.cpu().numpy()
    if CASES[key][3].get("remove_tilt"):
        np.testing.assert_allclose(got, g[f"{key}/opd"], rtol=0, atol=1e-12 if exact else 1e-9)
    elif exact:
        np.testing.assert_array_equal(got, g[f"{key}/opd"], err_msg=f"{key}.opd")
    else:  # OPD in waves: a difference of near-equal path lengths / 5.5e-4 mm
        np.testing.assert_allclose(got, g[f"{key}/opd"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(float(w.rms()), float(g[f"{key}/rms"]),
                               rtol=1e-12 if exact else 1e-9)


class _OracleRays:
    """What the strategies read from a traced RealRays, from the oracle (CPU tensors)."""

    def __init__(self, rays, torch):
        for a in ("x", "y", "z", "L", "M", "N", "i", "opd"):
            setattr(self, a, torch.as_tensor(np.asarray(getattr(rays, a), dtype=np.float64)))


@pytest.mark.parametrize("key", sorted(CASES))
def test_strategies_host_logic_with_oracle_rays(key, monkeypatch):
    torch = pytest.importorskip("torch")
    from oracle import trace_np
    from optiland_pr_amd.analysis import OPD
    from optiland_pr_amd.lowering import lower_surface_group, segment_params

    name, field, wl, kw = CASES[key]
    lens = _lens(name)

    def oracle_trace(hx, hy, wavelength, num_rays, distribution):
        table = lower_surface_group(lens.surface_group, [wavelength])
        seg = segment_params(lens, hx, hy, 0)
        px = np.asarray(distribution.x, dtype=np.float64)
        py = np.asarray(distribution.y, dtype=np.float64)
        with np.errstate(all="ignore"):
            r = trace_np.trace_segment(table, trace_np.generate_rays(seg, px, py), 0).rays
        return _OracleRays(r, torch)

    monkeypatch.setattr(lens, "trace", oracle_trace)
    _check(key, OPD(lens, field, wl, **kw), _golden(), exact=False)


def test_unknown_strategy_and_small_point_sets(monkeypatch):
    from optiland_pr_amd.analysis import BestFitSphereStrategy, create_strategy
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    with pytest.raises(ValueError, match="Unknown wavefront strategy"):
        create_strategy("nope", lens, None)
    s = BestFitSphereStrategy(lens, None)
    h = {a: np.zeros(3) for a in ("x", "y", "z", "L", "M", "N")}
    h["i"] = np.ones(3)
    with pytest.raises(ValueError, match="at least 4 valid ray samples"):
        s._calculate_reference_sphere(h, np.zeros(3))
    h["i"] = np.zeros(3)
    with pytest.raises(ValueError, match="No valid ray samples"):
        s._calculate_reference_sphere(h, np.zeros(3))


@pytest.mark.gpu
@pytest.mark.parametrize("key", sorted(CASES))
def test_strategies_on_gpu(key):
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need the MI355X (torch.cuda.is_available() is False)")
    from optiland_pr_amd.analysis import OPD

    name, field, wl, kw = CASES[key]
    _check(key, OPD(_lens(name), field, wl, **kw), _golden())
