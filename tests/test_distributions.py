"""Pupil distributions (host, NumPy) vs the reference's own samples
(tests/golden/distributions.npz from gen_golden.py --distributions): bit-exact."""

import numpy as np
import pytest

from optiland_pr_amd.distribution import (
    GaussianQuadrature,
    RandomDistribution,
    create_distribution,
)
from tests.conftest import load_golden

CASES = [("random", 1000), ("uniform", 33), ("uniform", 128), ("hexapolar", 6),
         ("hexapolar", 17), ("ring", 13), ("line_x", 21), ("line_y", 20),
         ("positive_line_x", 9), ("positive_line_y", 10), ("cross", 21), ("cross", 20)]


@pytest.fixture(scope="module")
def g():
    return load_golden("distributions")


@pytest.mark.parametrize("kind,n", CASES)
def test_distribution_matches_reference(g, kind, n):
    d = RandomDistribution(seed=7) if kind == "random" else create_distribution(kind)
    d.generate_points(n)
    assert np.array_equal(np.asarray(d.x), g[f"{kind}_{n}_x"])
    assert np.array_equal(np.asarray(d.y), g[f"{kind}_{n}_y"])


@pytest.mark.parametrize("sym", [False, True])
@pytest.mark.parametrize("rings", range(1, 7))
def test_gaussian_quadrature_matches_reference(g, sym, rings):
    q = GaussianQuadrature(is_symmetric=sym)
    q.generate_points(rings)
    key = f"gq_{int(sym)}_{rings}"
    assert np.array_equal(q.x, g[key + "_x"])
    assert np.array_equal(q.y, g[key + "_y"])
    assert np.array_equal(q.get_weights(rings), g[key + "_w"])


def test_gaussian_quadrature_ring_range():
    with pytest.raises(ValueError):
        GaussianQuadrature().generate_points(7)


def test_unknown_distribution():
    with pytest.raises(ValueError):
        create_distribution("spiral")
