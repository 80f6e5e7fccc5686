"""Pupil apodization: the intensity a generated ray starts with, as a function of its
normalised pupil coordinates (optiland/apodization/*.py, applied in
rays/ray_generator.py:91-95).

The classes keep the reference's names, constructor arguments, validation errors,
registry and to_dict / from_dict schema. `get_intensity` is the reference's NumPy
expression (host use: tests, analysis); the traced rays get theirs on the device
(ort::apodize, csrc/ort_core.h) from the record `lower()` returns, whose lens-constant
subexpressions (2 sigma**2, 2 R, D / 2, ...) are formed here with the reference's own
Python operations.
"""

from __future__ import annotations

import numpy as np

from . import _abi


class BaseApodization:
    """apodization/base.py:15-66."""

    _registry: dict = {}
    kind = _abi.APOD_UNIFORM

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        BaseApodization._registry[cls.__name__] = cls

    def get_intensity(self, Px, Py):  # pragma: no cover - abstract
        raise NotImplementedError

    def params(self):
        return ()

    def lower(self):
        """-> one _abi.APODIZATION record (ort_apodization)."""
        rec = np.zeros((), dtype=_abi.APODIZATION)
        rec["kind"] = self.kind
        p = [float(v) for v in self.params()]
        rec["p"][: len(p)] = p
        return rec

    def to_dict(self):
        return {"type": self.__class__.__name__}

    @classmethod
    def from_dict(cls, data):
        kind = data.get("type")
        if kind not in cls._registry:
            raise ValueError(f"Unknown apodization type: {kind}")
        return cls._registry[kind].from_dict(data)


class UniformApodization(BaseApodization):
    """apodization/uniform.py: every ray starts with intensity 1."""

    kind = _abi.APOD_UNIFORM

    def get_intensity(self, Px, Py):
        return np.ones_like(np.asarray(Px, dtype=np.float64))

    @classmethod
    def from_dict(cls, data):
        return cls()


class GaussianApodization(BaseApodization):
    """apodization/gaussian.py: exp(-(Px**2 + Py**2) / (2 sigma**2))."""

    kind = _abi.APOD_GAUSSIAN

    def __init__(self, sigma: float = 1.0):
        if sigma <= 0:
            raise ValueError("Sigma must be positive for GaussianApodization.")
        self.sigma = sigma

    def get_intensity(self, Px, Py):
        return np.exp(-(Px**2 + Py**2) / (2 * self.sigma**2))

    def params(self):
        return (2 * self.sigma**2,)

    def to_dict(self):
        return {**super().to_dict(), "sigma": self.sigma}

    @classmethod
    def from_dict(cls, data):
        return cls(sigma=data.get("sigma", 1.0))


class CosineSquaredApodization(BaseApodization):
    """apodization/cosine_squared.py: cos(pi r / (2 R))**2 inside r < R."""

    kind = _abi.APOD_COSINE_SQUARED

    def __init__(self, R: float = 1.0):
        if R <= 0:
            raise ValueError("R must be positive for CosineSquaredApodization.")
        self.R = R

    def get_intensity(self, Px, Py):
        r = (Px**2 + Py**2) ** 0.5
        cos_arg = (np.pi * r) / (2 * self.R)
        intensity = np.cos(cos_arg) ** 2
        return np.where(r < self.R, intensity, 0.0)

    def params(self):
        return (self.R, 2 * self.R)

    def to_dict(self):
        return {**super().to_dict(), "R": self.R}

    @classmethod
    def from_dict(cls, data):
        return cls(R=data.get("R", 1.0))


class HannApodization(BaseApodization):
    """apodization/hann.py: 0.5 (1 - cos(2 pi r / D)) inside r < D / 2."""

    kind = _abi.APOD_HANN

    def __init__(self, D: float = 2.0):
        if D <= 0:
            raise ValueError("D must be positive for HannApodization.")
        self.D = D

    def get_intensity(self, Px, Py):
        r = (Px**2 + Py**2) ** 0.5
        R = self.D / 2
        cos_arg = (2 * np.pi * r) / self.D
        intensity = 0.5 * (1 - np.cos(cos_arg))
        return np.where(r < R, intensity, 0.0)

    def params(self):
        return (self.D / 2, self.D)

    def to_dict(self):
        return {**super().to_dict(), "D": self.D}

    @classmethod
    def from_dict(cls, data):
        return cls(D=data.get("D", 2.0))


class PolynomialApodization(BaseApodization):
    """apodization/polynomial.py: (1 - (r / R)**2)**p inside r < R."""

    kind = _abi.APOD_POLYNOMIAL

    def __init__(self, R: float = 1.0, p: float = 1.0):
        if R <= 0:
            raise ValueError("R must be positive for PolynomialApodization.")
        if p < 0:
            raise ValueError("p must be non-negative for PolynomialApodization.")
        self.R = R
        self.p = p

    def get_intensity(self, Px, Py):
        r = (Px**2 + Py**2) ** 0.5
        r_norm_sq = (r / self.R) ** 2
        intensity = (1 - r_norm_sq) ** self.p
        return np.where(r < self.R, intensity, 0.0)

    def params(self):
        return (self.R, self.p)

    def to_dict(self):
        return {**super().to_dict(), "R": self.R, "p": self.p}

    @classmethod
    def from_dict(cls, data):
        return cls(R=data.get("R", 1.0), p=data.get("p", 1.0))


class SuperGaussianApodization(BaseApodization):
    """apodization/super_gaussian.py: exp(-((r / w)**n))."""

    kind = _abi.APOD_SUPER_GAUSSIAN

    def __init__(self, w: float = 1.0, n: float = 2.0):
        if w <= 0:
            raise ValueError("w must be positive for SuperGaussianApodization.")
        if n < 2:
            raise ValueError("n must be >= 2 for SuperGaussianApodization.")
        self.w = w
        self.n = n

    def get_intensity(self, Px, Py):
        r_squared = Px**2 + Py**2
        return np.exp(-((r_squared**0.5 / self.w) ** self.n))

    def params(self):
        return (self.w, self.n)

    def to_dict(self):
        return {**super().to_dict(), "w": self.w, "n": self.n}

    @classmethod
    def from_dict(cls, data):
        return cls(w=data.get("w", 1.0), n=data.get("n", 2.0))


class TukeyApodization(BaseApodization):
    """apodization/tukey.py: flat to R (1 - alpha / 2), cosine taper to R."""

    kind = _abi.APOD_TUKEY

    def __init__(self, R: float = 1.0, alpha: float = 0.5):
        if R <= 0:
            raise ValueError("R must be positive for TukeyApodization.")
        if not (0 <= alpha <= 1):
            raise ValueError("alpha must be between 0 and 1 for TukeyApodization.")
        self.R = R
        self.alpha = alpha

    def get_intensity(self, Px, Py):
        r = (Px**2 + Py**2) ** 0.5
        flat_region_end = self.R * (1 - self.alpha / 2)
        with np.errstate(divide="ignore", invalid="ignore"):
            cos_arg = np.pi * (r - flat_region_end) / (self.R * self.alpha / 2)
        taper_intensity = 0.5 * (1 + np.cos(cos_arg))
        cond1 = r <= flat_region_end
        cond2 = (r > flat_region_end) & (r < self.R)
        intensity = np.where(cond1, 1.0, 0.0)
        return np.where(cond2, taper_intensity, intensity)

    def params(self):
        return (self.R, self.R * (1 - self.alpha / 2), self.R * self.alpha / 2)

    def to_dict(self):
        return {**super().to_dict(), "R": self.R, "alpha": self.alpha}

    @classmethod
    def from_dict(cls, data):
        return cls(R=data.get("R", 1.0), alpha=data.get("alpha", 0.5))


def resolve(apodization=None, **kwargs):
    """optic_updater.py:312-350 (set_apodization): an instance, a registry name plus
    constructor keywords, a to_dict() dict, or None."""
    if apodization is None:
        return None
    if isinstance(apodization, BaseApodization):
        return apodization
    if isinstance(apodization, str):
        if apodization in BaseApodization._registry:
            return BaseApodization._registry[apodization](**kwargs)
        raise ValueError(f"Unknown apodization type: {apodization}")
    if isinstance(apodization, dict):
        return BaseApodization.from_dict(apodization)
    raise TypeError("apodization must be a string, a dict, a BaseApodization "
                    "instance, or None.")
