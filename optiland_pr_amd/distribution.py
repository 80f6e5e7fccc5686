"""Pupil sampling distributions (host, NumPy).

Mirrors optiland/distribution.py:19-408 (create_distribution + the distributions
SpotDiagram / Wavefront / Optic.trace use). Samples are generated on the host with
NumPy exactly as the reference does, then copied to HBM once.
"""

from __future__ import annotations

import numpy as np


class BaseDistribution:
    x: np.ndarray
    y: np.ndarray

    def generate_points(self, num_points):
        raise NotImplementedError


class RandomDistribution(BaseDistribution):
    """distribution.py:128-158: r = sqrt(U), theta = 2 pi U (numpy default_rng)."""

    def __init__(self, seed=None):
        self.rng = np.random.default_rng(seed)

    def generate_points(self, num_points: int):
        r = self.rng.uniform(size=num_points)
        theta = self.rng.uniform(0, 2 * np.pi, size=num_points)
        self.x = np.sqrt(r) * np.cos(theta)
        self.y = np.sqrt(r) * np.sin(theta)


class UniformDistribution(BaseDistribution):
    """distribution.py:161-186: linspace grid masked to r^2 <= 1 (xy indexing)."""

    def generate_points(self, num_points: int):
        x = np.linspace(-1, 1, num_points)
        x, y = np.meshgrid(x, x)
        r2 = x**2 + y**2
        self.x = x[r2 <= 1]
        self.y = y[r2 <= 1]


class HexagonalDistribution(BaseDistribution):
    """distribution.py:189-220: 1 + 3 n (n+1) points on hexapolar rings."""

    def generate_points(self, num_rings: int = 6):
        x = np.zeros([1])
        y = np.zeros([1])
        r = np.linspace(0, 1, num_rings + 1)
        for i in range(num_rings):
            num_theta = 6 * (i + 1)
            theta = np.linspace(0, 2 * np.pi, num_theta + 1)[:-1]
            x = np.concatenate([x, r[i + 1] * np.cos(theta)])
            y = np.concatenate([y, r[i + 1] * np.sin(theta)])
        self.x = x
        self.y = y


class LineXDistribution(BaseDistribution):
    """distribution.py:223-255."""

    def __init__(self, positive_only=False):
        self.positive_only = positive_only

    def generate_points(self, num_points: int):
        self.x = np.linspace(0, 1, num_points) if self.positive_only else np.linspace(-1, 1, num_points)
        self.y = np.zeros([num_points])


class LineYDistribution(BaseDistribution):
    """distribution.py:258-290."""

    def __init__(self, positive_only=False):
        self.positive_only = positive_only

    def generate_points(self, num_points: int):
        self.x = np.zeros([num_points])
        self.y = np.linspace(0, 1, num_points) if self.positive_only else np.linspace(-1, 1, num_points)


class CrossDistribution(BaseDistribution):
    """distribution.py:293-345: x and y arms, origin not duplicated."""

    def generate_points(self, num_points: int):
        y_line_x = np.zeros([num_points])
        y_line_y = np.linspace(-1, 1, num_points)
        x_line_x = np.linspace(-1, 1, num_points)
        x_line_y = np.zeros([num_points])
        if num_points % 2 == 1:
            mid = num_points // 2
            x_line_x = np.concatenate((x_line_x[:mid], x_line_x[mid + 1:]))
            x_line_y = np.concatenate((x_line_y[:mid], x_line_y[mid + 1:]))
        self.x = np.concatenate((y_line_x, x_line_x))
        self.y = np.concatenate((y_line_y, x_line_y))


class RingDistribution(BaseDistribution):
    """distribution.py:348-375: num_points on the unit circle."""

    def generate_points(self, num_points: int):
        theta = np.linspace(0, 2 * np.pi, num_points + 1)[:-1]
        self.x = np.cos(theta)
        self.y = np.sin(theta)


class GaussianQuadrature(BaseDistribution):
    """distribution.py:268-355: Gaussian-quadrature rings (G. W. Forbes, JOSA A 5, 1988),
    3 azimuths (-60, 0, 60 deg) per ring, or 1 with is_symmetric; weights per ring."""

    _RADIUS = {
        1: [0.70711],
        2: [0.45970, 0.88807],
        3: [0.33571, 0.70711, 0.94196],
        4: [0.26350, 0.57446, 0.81853, 0.96466],
        5: [0.21659, 0.48038, 0.70711, 0.87706, 0.97626],
        6: [0.18375, 0.41158, 0.61700, 0.78696, 0.91138, 0.98300],
    }
    _WEIGHTS = {
        1: [0.5],
        2: [0.25, 0.25],
        3: [0.13889, 0.22222, 0.13889],
        4: [0.08696, 0.16304, 0.16304, 0.08696],
        5: [0.059231, 0.11966, 0.14222, 0.11966, 0.059231],
        6: [0.04283, 0.09019, 0.11698, 0.11698, 0.09019, 0.04283],
    }

    def __init__(self, is_symmetric=False):
        self.is_symmetric = is_symmetric

    def _get_radius(self, num_rings: int):
        if num_rings not in self._RADIUS:
            raise ValueError("Gaussian quadrature must have between 1 and 6 rings.")
        return np.array(self._RADIUS[num_rings])

    def generate_points(self, num_rings: int):
        radius = self._get_radius(num_rings)
        theta = np.array([0.0]) if self.is_symmetric else np.array(
            [-1.04719755, 0.0, 1.04719755])
        self.x = np.outer(radius, np.cos(theta)).flatten()
        self.y = np.outer(radius, np.sin(theta)).flatten()

    def get_weights(self, num_rings: int):
        if num_rings not in self._WEIGHTS:
            raise ValueError("Gaussian quadrature must have between 1 and 6 rings.")
        w = np.array(self._WEIGHTS[num_rings])
        return w * 6.0 if self.is_symmetric else w * 2.0


def create_distribution(distribution_type) -> BaseDistribution:
    """distribution.py:378-408."""
    classes = {
        "line_x": LineXDistribution,
        "line_y": LineYDistribution,
        "positive_line_x": lambda: LineXDistribution(positive_only=True),
        "positive_line_y": lambda: LineYDistribution(positive_only=True),
        "random": RandomDistribution,
        "uniform": UniformDistribution,
        "hexapolar": HexagonalDistribution,
        "cross": CrossDistribution,
        "ring": RingDistribution,
    }
    if distribution_type not in classes:
        raise ValueError("Invalid distribution type.")
    return classes[distribution_type]()
