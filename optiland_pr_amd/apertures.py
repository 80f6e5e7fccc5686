"""Physical apertures (physical_apertures/*.py): the reference's aperture classes, lowered
to the trace kernels' clip step.

RadialAperture keeps the kernels' dedicated radial test (ORT_SURF_APERTURE). Every other
aperture -- offset radial, elliptical, rectangular, polygon (and FileAperture), and the
boolean combinations a | b, a & b, a - b (base.py:155-340) -- is lowered to a short
postfix program (ORT_SURF_APERTURE_PROG, include/optiland_rt.h ort_aperture_op) that the
kernel evaluates on the ray's local (x, y) after propagation, clipping the ray
(intensity 0) outside, exactly where Surface.trace calls aperture.clip
(standard_surface.py:221). Each primitive's test is the reference's expression with the
same operand order (e.g. r_max**2 formed once on the host as the reference does).
"""

from __future__ import annotations

import numpy as np

from . import _abi


class BaseAperture:
    """base.py:30-172."""

    def __or__(self, other):
        return UnionAperture(self, other)

    def __add__(self, other):
        return UnionAperture(self, other)

    def __and__(self, other):
        return IntersectionAperture(self, other)

    def __sub__(self, other):
        return DifferenceAperture(self, other)

    def program(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def to_dict(self):
        return {"type": type(self).__name__}

    @classmethod
    def from_dict(cls, data):
        t = data.get("type")
        sub = _REGISTRY.get(t)
        if sub is None:
            raise ValueError(f"Unknown aperture type: {t}")
        return sub._from_dict(data)


class RadialAperture(BaseAperture):
    """radial.py:31-103: r_min <= r <= r_max."""

    def __init__(self, r_max, r_min=0):
        self.r_max = float(r_max)
        self.r_min = float(r_min)

    @property
    def extent(self):
        return -self.r_max, self.r_max, -self.r_max, self.r_max

    def scale(self, scale_factor):
        self.r_max = self.r_max * scale_factor
        self.r_min = self.r_min * scale_factor

    def program(self):
        return [_abi.AP_RADIAL, self.r_min**2, self.r_max**2, 0.0, 0.0]

    def to_dict(self):
        d = super().to_dict()
        d.update(r_max=self.r_max, r_min=self.r_min)
        return d

    @classmethod
    def _from_dict(cls, d):
        return cls(d["r_max"], d.get("r_min", 0))


class OffsetRadialAperture(RadialAperture):
    """offset_radial.py:16-95: (x - ox)^2 + (y - oy)^2 between r_min^2 and r_max^2."""

    def __init__(self, r_max, r_min=0, offset_x=0, offset_y=0):
        super().__init__(r_max, r_min)
        self.offset_x = float(offset_x)
        self.offset_y = float(offset_y)

    @property
    def extent(self):
        return (self.offset_x - self.r_max, self.offset_x + self.r_max,
                self.offset_y - self.r_max, self.offset_y + self.r_max)

    def scale(self, scale_factor):
        super().scale(scale_factor)
        self.offset_x *= scale_factor
        self.offset_y *= scale_factor

    def program(self):
        return [_abi.AP_RADIAL, self.r_min**2, self.r_max**2, self.offset_x, self.offset_y]

    def to_dict(self):
        d = super().to_dict()
        d.update(offset_x=self.offset_x, offset_y=self.offset_y)
        return d

    @classmethod
    def _from_dict(cls, d):
        return cls(d["r_max"], d.get("r_min", 0), d.get("offset_x", 0), d.get("offset_y", 0))


class EllipticalAperture(BaseAperture):
    """elliptical.py:14-95: (x - ox)^2 / a^2 + (y - oy)^2 / b^2 <= 1."""

    def __init__(self, a, b, offset_x=0, offset_y=0):
        self.a = float(a)
        self.b = float(b)
        self.offset_x = float(offset_x)
        self.offset_y = float(offset_y)

    @property
    def extent(self):
        return -self.a, self.a, -self.b, self.b

    def scale(self, scale_factor):
        self.a *= scale_factor
        self.b *= scale_factor
        self.offset_x *= scale_factor
        self.offset_y *= scale_factor

    def program(self):
        return [_abi.AP_ELLIPSE, self.offset_x, self.offset_y, self.a**2, self.b**2]

    def to_dict(self):
        d = super().to_dict()
        d.update(a=self.a, b=self.b, offset_x=self.offset_x, offset_y=self.offset_y)
        return d

    @classmethod
    def _from_dict(cls, d):
        return cls(d["a"], d["b"], d.get("offset_x", 0), d.get("offset_y", 0))


class RectangularAperture(BaseAperture):
    """rectangular.py:14-95: x_min <= x <= x_max and y_min <= y <= y_max."""

    def __init__(self, x_min, x_max, y_min, y_max):
        self.x_min, self.x_max = float(x_min), float(x_max)
        self.y_min, self.y_max = float(y_min), float(y_max)

    @property
    def extent(self):
        return self.x_min, self.x_max, self.y_min, self.y_max

    def scale(self, scale_factor):
        self.x_min *= scale_factor
        self.x_max *= scale_factor
        self.y_min *= scale_factor
        self.y_max *= scale_factor

    def program(self):
        return [_abi.AP_RECT, self.x_min, self.x_max, self.y_min, self.y_max]

    def to_dict(self):
        d = super().to_dict()
        d.update(x_min=self.x_min, x_max=self.x_max, y_min=self.y_min, y_max=self.y_max)
        return d

    @classmethod
    def _from_dict(cls, d):
        return cls(d["x_min"], d["x_max"], d["y_min"], d["y_max"])


class PolygonAperture(BaseAperture):
    """polygon.py:19-104: inside the (implicitly closed) polygon of vertices (x, y),
    even-odd rule as matplotlib's Path.contains_points (numpy backend)."""

    def __init__(self, x, y):
        self.x = np.asarray(x, dtype=np.float64).ravel()
        self.y = np.asarray(y, dtype=np.float64).ravel()
        if self.x.shape != self.y.shape:
            raise ValueError("x and y must have the same length")
        self.vertices = np.column_stack((self.x, self.y))

    @property
    def extent(self):
        return self.x.min(), self.x.max(), self.y.min(), self.y.max()

    def scale(self, scale_factor):
        self.vertices = self.vertices * scale_factor
        self.x = self.vertices[:, 0]
        self.y = self.vertices[:, 1]

    def program(self):
        return [_abi.AP_POLYGON, float(len(self.x))] + self.vertices.ravel().tolist()

    def to_dict(self):
        d = super().to_dict()
        d.update(x=self.x.tolist(), y=self.y.tolist())
        return d

    @classmethod
    def _from_dict(cls, d):
        return cls(d["x"], d["y"])


class FileAperture(PolygonAperture):
    """polygon.py:107-212: polygon vertices read from a two-column text file ('//'
    comments, optional delimiter and header lines, several text encodings)."""

    ENCODINGS = ("utf-8", "utf-16", "utf-16le", "utf-16be", "utf-32", "utf-32le",
                 "utf-32be", "latin1", "ascii")

    def __init__(self, filepath, delimiter=None, skip_header=0):
        self.filepath = filepath
        self.delimiter = delimiter
        self.skip_header = skip_header
        data = None
        for enc in self.ENCODINGS:
            try:
                with open(filepath, encoding=enc) as f:
                    data = np.genfromtxt(f, delimiter=delimiter if delimiter is not None else " ",
                                         comments="//", skip_header=skip_header)
                if data is not None:
                    break
            except UnicodeDecodeError:
                continue
        if data is None or data.ndim != 2 or data.shape[1] != 2:
            raise ValueError(f'Error reading aperture file "{filepath}"')
        super().__init__(data[:, 0], data[:, 1])

    def to_dict(self):
        d = super().to_dict()
        d.update(filepath=self.filepath, delimiter=self.delimiter,
                 skip_header=self.skip_header)
        return d

    @classmethod
    def _from_dict(cls, d):
        return PolygonAperture(d["x"], d["y"]) if "x" in d else cls(
            d["filepath"], d.get("delimiter"), d.get("skip_header", 0))


class _Boolean(BaseAperture):
    OP = 0

    def __init__(self, a, b):
        self.a = a
        self.b = b

    @property
    def extent(self):  # base.py:187-199: the bounding box of both operands
        a, b = self.a.extent, self.b.extent
        return min(a[0], b[0]), max(a[1], b[1]), min(a[2], b[2]), max(a[3], b[3])

    def scale(self, scale_factor):
        self.a.scale(scale_factor)
        self.b.scale(scale_factor)

    def program(self):
        return self.a.program() + self.b.program() + [self.OP]

    def to_dict(self):
        d = super().to_dict()
        d.update(a=self.a.to_dict(), b=self.b.to_dict())
        return d

    @classmethod
    def _from_dict(cls, d):
        return cls(BaseAperture.from_dict(d["a"]), BaseAperture.from_dict(d["b"]))


class UnionAperture(_Boolean):
    """base.py:255-279: a | b."""

    OP = _abi.AP_UNION


class IntersectionAperture(_Boolean):
    """base.py:282-306: a & b."""

    OP = _abi.AP_INTERSECT


class DifferenceAperture(_Boolean):
    """base.py:309-340: a & ~b."""

    OP = _abi.AP_DIFFERENCE


_REGISTRY = {c.__name__: c for c in (
    RadialAperture, OffsetRadialAperture, EllipticalAperture, RectangularAperture,
    PolygonAperture, FileAperture, UnionAperture, IntersectionAperture, DifferenceAperture)}


def program_depth(prog):
    """Maximum stack depth of an aperture program (the kernel's stack holds 32)."""
    depth = best = 0
    q = 0
    while q < len(prog):
        op = int(prog[q])
        if op == _abi.AP_POLYGON:
            q += 2 + 2 * int(prog[q + 1])
            depth += 1
        elif op in (_abi.AP_RADIAL, _abi.AP_ELLIPSE, _abi.AP_RECT):
            q += 5
            depth += 1
        else:
            q += 1
            depth -= 1
        best = max(best, depth)
    return best
