"""Pin the gradient goldens (tests/golden/autograd_tma.npz, the reference's torch-CPU
autograd of the TMA trace w.r.t. its Zernike coefficients, gen_autograd_golden.py)
against the oracle: central finite differences of the NumPy restatement
(oracle/trace_np.py) of the same losses. Agreement to ~1e-6 relative says the golden
gradients belong to the traced function the oracle (and hence the HIP path) computes.
Also checks the host-side parameter map of the autograd op.
"""

import numpy as np
import pytest

from oracle import trace_np
from optiland_pr_amd.autodiff import parameter_map
from optiland_pr_amd.lowering import lower_surface_group, segment_params
from optiland_pr_amd.samples import ThreeMirrorAnastigmat
from tests.conftest import load_golden

WSUM_FIELDS = ("x", "y", "z", "L", "M", "N", "opd")


def _golden():
    return load_golden("autograd_tma")


def _trace(coeffs, hy, px, py, normal_skip=()):
    """Oracle trace of the TMA with per-mirror coefficients. normal_skip: (mirror, term)
    pairs whose coefficient the Zernike NORMAL treats as zero -- the reference's normal
    skips every term whose coefficient is 0 (zernike.py:213-214: `if c == 0: continue`),
    so its autograd derivative w.r.t. a zero coefficient has no normal contribution."""
    lens = ThreeMirrorAnastigmat()
    for k, si in enumerate((1, 2, 3)):
        lens.surface_group.surfaces[si].geometry.coefficients = np.array(coeffs[k])
    table = lower_surface_group(lens.surface_group, [0.587])
    skip_rad = {int(table.zern[int(table.surfaces[m]["coef_off"]) + j]["rad_off"])
                for m, j in normal_skip}
    seg = segment_params(lens, 0.0, hy, 0)
    r = trace_np.generate_rays(seg, px, py)
    orig = trace_np.normal_zernike

    def normal(x, y, R, k, terms, coef, nr):
        t2 = terms.copy()
        for row in range(len(t2)):
            if int(t2[row]["rad_off"]) in skip_rad:
                t2[row]["c"] = 0.0
        return orig(x, y, R, k, t2, coef, nr)

    trace_np.normal_zernike = normal
    try:
        return trace_np.trace_segment(table, r, 0).rays
    finally:
        trace_np.normal_zernike = orig


def _rms(coeffs, g, skip=()):
    r = _trace(coeffs, 1.0, g["Px"], g["Py"], skip)
    return np.sqrt(np.mean((r.x - np.mean(r.x)) ** 2 + (r.y - np.mean(r.y)) ** 2))


def _wsum(coeffs, g, skip=()):
    r = _trace(coeffs, -1.0, g["Px"], g["Py"], skip)
    return sum(np.sum(g[f"wsum_w_{f}"] * getattr(r, f)) for f in WSUM_FIELDS)


def _fd(fn, g, h=1e-7):
    c0 = np.stack([ThreeMirrorAnastigmat().surface_group.surfaces[si].geometry.coefficients
                   for si in (1, 2, 3)]).astype(np.float64)
    grad = np.zeros_like(c0)
    for i in range(c0.shape[0]):
        for j in range(c0.shape[1]):
            cp, cm = c0.copy(), c0.copy()
            cp[i, j] += h
            cm[i, j] -= h
            skip = [(i, j)] if c0[i, j] == 0 else []
            grad[i, j] = (fn(cp, g, skip) - fn(cm, g, skip)) / (2 * h)
    return c0, grad


@pytest.mark.parametrize("loss", ["rms", "wsum"])
def test_oracle_fd_matches_reference_autograd(loss):
    g = _golden()
    fn = _rms if loss == "rms" else _wsum
    c0, fd = _fd(fn, g)
    # the oracle's forward value is the reference's (bit-exact trace, NumPy reductions)
    assert fn(c0, g) == pytest.approx(float(g[f"{loss}_value"]), rel=1e-12)
    ref = g[f"{loss}_grad"]
    scale = np.max(np.abs(ref))
    np.testing.assert_allclose(fd, ref, rtol=1e-5, atol=1e-6 * scale)


def test_parameter_map():
    lens = ThreeMirrorAnastigmat()
    table = lower_surface_group(lens.surface_group, [0.587])

    class _C:  # stands in for a coefficient tensor: only numel() is read
        def __init__(self, n):
            self.n = n

        def numel(self):
            return self.n

    zp, n = parameter_map(table, [(0, _C(10)), (2, _C(10))])
    assert n == 20
    assert zp.shape == (30,)
    np.testing.assert_array_equal(zp[:10], np.arange(10))
    np.testing.assert_array_equal(zp[10:20], -1)
    np.testing.assert_array_equal(zp[20:], np.arange(10, 20))
    with pytest.raises(ValueError):
        parameter_map(table, [(1, _C(9))])


def _cooke_rms(radius, conic5, thick, thick_surface, g=None):
    """Oracle rms spot of the Cooke triplet at (0, 1), uniform 24, lambda 0.55 with the
    given radii of surfaces 1, 3, 6, conic of surface 5 and thickness after
    `thick_surface`; the rays are generated from the UNPERTURBED lens (the reference
    builds ray-generation inputs from detached copies, surface_group.py:143-153)."""
    from optiland_pr_amd.distribution import create_distribution
    from optiland_pr_amd.samples import CookeTriplet

    base = CookeTriplet()
    seg = segment_params(base, 0.0, 1.0, 0)
    lens = CookeTriplet()
    for si, r in zip((1, 3, 6), radius, strict=True):
        lens.set_radius(r, si)
    lens.set_conic(conic5, 5)
    lens.set_thickness(thick, thick_surface)
    table = lower_surface_group(lens.surface_group, [0.55])
    d = create_distribution("uniform")
    d.generate_points(24)
    r = trace_np.trace_segment(table, trace_np.generate_rays(seg, d.x, d.y), 0).rays
    return np.sqrt(np.mean((r.x - np.mean(r.x)) ** 2 + (r.y - np.mean(r.y)) ** 2))


@pytest.mark.parametrize("th", [2, 6])
def test_oracle_fd_matches_reference_shape_gradients(th):
    """Radius / conic / thickness gradients of the reference (autograd_cooke.npz) against
    central differences of the oracle with fixed ray generation."""
    from optiland_pr_amd.samples import CookeTriplet

    g = load_golden("autograd_cooke")
    base = CookeTriplet()
    R0 = [base.surface_group.surfaces[si].geometry.radius for si in (1, 3, 6)]
    t0 = base.surface_group.surfaces[th].thickness
    x0 = np.array(R0 + [0.0, t0])

    def f(x):
        return _cooke_rms(list(x[:3]), x[3], x[4], th)

    assert f(x0) == pytest.approx(float(g[f"t{th}_value"]), rel=1e-12)
    fd = np.zeros(5)
    for i in range(5):
        h = 1e-6 * max(1.0, abs(x0[i]))
        xp, xm = x0.copy(), x0.copy()
        xp[i] += h
        xm[i] -= h
        fd[i] = (f(xp) - f(xm)) / (2 * h)
    np.testing.assert_allclose(fd, g[f"t{th}_grad"], rtol=1e-5, atol=1e-9)
