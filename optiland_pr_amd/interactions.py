"""Interaction models and phase profiles (host side: parameters lowered for the kernels).

Mirrors optiland/interactions/{refractive_reflective_model,thin_lens_interaction_model,
phase_interaction_model,diffractive_model}.py and optiland/phase/{constant,
linear_grating,radial}.py: the same class names, constructor arguments, validation and
to_dict / from_dict keys. What each model does to a ray runs only in the HIP kernels
(csrc/ort_interact.h); `lower()` packs the parameter block described at
`enum ort_interaction` in include/optiland_rt.h.
"""

from __future__ import annotations

import numpy as np

from . import _abi


# --------------------------------------------------------------------------------------
# phase profiles (optiland/phase)
# --------------------------------------------------------------------------------------
class BasePhaseProfile:
    """phase/base.py:14-108 (registry by phase_type for from_dict)."""

    _registry: dict = {}
    phase_type = None

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        if cls.phase_type:
            BasePhaseProfile._registry[cls.phase_type] = cls

    @property
    def efficiency(self):
        return 1.0

    def to_dict(self):
        return {"phase_type": self.phase_type}

    @classmethod
    def from_dict(cls, data):
        t = data.get("phase_type")
        if t not in cls._registry:
            raise ValueError(f"Unknown phase profile type: {t}")
        return cls._registry[t].from_dict(data)

    def lower(self):
        """-> [kind, efficiency, parameters...]"""
        raise NotImplementedError


class ConstantPhaseProfile(BasePhaseProfile):
    """phase/constant.py: constant phase, zero gradient."""

    phase_type = "constant"

    def __init__(self, phase: float = 0.0):
        self.phase = phase

    def to_dict(self):
        return {**super().to_dict(), "phase": self.phase}

    @classmethod
    def from_dict(cls, data):
        return cls(phase=data.get("phase", 0.0))

    def lower(self):
        return [_abi.PHASE_CONSTANT, float(self.efficiency), float(self.phase)]


class LinearGratingPhaseProfile(BasePhaseProfile):
    """phase/linear_grating.py:11-140: phi = K_x x + K_y y, K = order 2 pi / period."""

    phase_type = "linear_grating"

    def __init__(self, period: float, angle: float = 0.0, order: int = 1,
                 efficiency: float = 1.0):
        if period <= 0:
            raise ValueError("Grating period must be positive.")
        if not (0.0 <= efficiency <= 1.0):
            raise ValueError("Efficiency must be between 0 and 1.")
        self.period = period
        self.angle = angle
        self.order = order
        self._efficiency = efficiency
        K = self.order * 2 * np.pi / self.period  # linear_grating.py:52-54
        self._K_x = K * np.cos(self.angle)
        self._K_y = K * np.sin(self.angle)

    @property
    def efficiency(self):
        return self._efficiency

    def to_dict(self):
        return {**super().to_dict(), "period": self.period, "angle": self.angle,
                "order": self.order, "efficiency": self.efficiency}

    @classmethod
    def from_dict(cls, data):
        return cls(period=data["period"], angle=data.get("angle", 0.0),
                   order=data.get("order", 1), efficiency=data.get("efficiency", 1.0))

    def lower(self):
        return [_abi.PHASE_LINEAR, float(self.efficiency), float(self._K_x), float(self._K_y)]


class RadialPhaseProfile(BasePhaseProfile):
    """phase/radial.py:11-119: phi = sum_i a_i r^(2(i+1))."""

    phase_type = "radial"

    def __init__(self, coefficients):
        self.coefficients = coefficients

    def to_dict(self):
        return {**super().to_dict(), "coefficients": self.coefficients}

    @classmethod
    def from_dict(cls, data):
        return cls(coefficients=data["coefficients"])

    def lower(self):
        c = [float(v) for v in self.coefficients]
        return [_abi.PHASE_RADIAL, float(self.efficiency), float(len(c)), *c]


# --------------------------------------------------------------------------------------
# interaction models (optiland/interactions)
# --------------------------------------------------------------------------------------
class BaseInteractionModel:
    """interactions/base.py:24-128 (coatings and BSDFs are out of scope)."""

    interaction_id = _abi.IA_REFRACT_REFLECT
    _registry: dict = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        BaseInteractionModel._registry[cls.__name__] = cls

    def __init__(self, parent_surface=None, is_reflective=False, coating=None, bsdf=None):
        if coating is not None or bsdf is not None:
            raise ValueError("coatings and BSDF scattering are out of scope for the trace core")
        self.parent_surface = parent_surface
        self.is_reflective = bool(is_reflective)
        self.coating = None
        self.bsdf = None

    def flip(self):
        pass

    def to_dict(self):
        return {"type": type(self).__name__, "is_reflective": self.is_reflective,
                "coating": None, "bsdf": None}

    @classmethod
    def from_dict(cls, data, parent_surface=None):
        sub = cls._registry.get(data.get("type"))
        if sub is None:
            raise ValueError(f"Unknown interaction model type: {data.get('type')}")
        kw = {k: v for k, v in data.items() if k not in ("type", "material_pre")}
        if kw.get("coating") or kw.get("bsdf"):
            raise ValueError("coatings and BSDF scattering are out of scope for the trace core")
        kw.pop("coating", None)
        kw.pop("bsdf", None)
        return sub._from_kwargs(parent_surface, kw)

    @classmethod
    def _from_kwargs(cls, parent_surface, kw):
        return cls(parent_surface=parent_surface, **kw)

    def lower(self, geometry):
        """-> the parameter block in lens.coef (ort_interaction)."""
        return []


class RefractiveReflectiveModel(BaseInteractionModel):
    """interactions/refractive_reflective_model.py:32-55."""


class ThinLensInteractionModel(BaseInteractionModel):
    """interactions/thin_lens_interaction_model.py:24-134 (focal length f)."""

    interaction_id = _abi.IA_THIN_LENS

    def __init__(self, parent_surface=None, focal_length=None, is_reflective=False,
                 coating=None, bsdf=None):
        super().__init__(parent_surface, is_reflective, coating, bsdf)
        self.f = np.asarray(focal_length, dtype=np.float64)

    def to_dict(self):
        return {**super().to_dict(), "focal_length": float(self.f)}

    def lower(self, geometry):
        return [float(self.f)]


class PhaseInteractionModel(BaseInteractionModel):
    """interactions/phase_interaction_model.py:18-207 (generalised Snell's law)."""

    interaction_id = _abi.IA_PHASE

    def __init__(self, parent_surface=None, phase_profile=None, is_reflective=False,
                 coating=None, bsdf=None):
        super().__init__(parent_surface, is_reflective, coating, bsdf)
        if phase_profile is None:
            raise ValueError("phase_profile is required for phase interaction.")
        self.phase_profile = phase_profile

    def to_dict(self):
        return {**super().to_dict(), "phase_profile": self.phase_profile.to_dict()}

    @classmethod
    def _from_kwargs(cls, parent_surface, kw):
        kw = dict(kw)
        prof = BasePhaseProfile.from_dict(kw.pop("phase_profile"))
        return cls(parent_surface=parent_surface, phase_profile=prof, **kw)

    def lower(self, geometry):
        return [float(v) for v in self.phase_profile.lower()]


class DiffractiveInteractionModel(RefractiveReflectiveModel):
    """interactions/diffractive_model.py:23-92: the grating geometry's order, period and
    grating vector (plane_grating.py:105-124, standard_grating.py:93-146, 224-247)."""

    interaction_id = _abi.IA_DIFFRACTIVE

    def lower(self, geometry):
        from .geometries import PlaneGrating, StandardGratingGeometry

        m = float(np.asarray(geometry.grating_order))
        period = float(np.asarray(geometry.grating_period))
        alfa = np.asarray(geometry.groove_orientation_angle, dtype=np.float64)
        if isinstance(geometry, PlaneGrating):
            return [m, period, 0.0, float(-np.sin(alfa)), float(np.cos(alfa))]
        if isinstance(geometry, StandardGratingGeometry):
            R = np.asarray(geometry.radius, dtype=np.float64)
            k = np.asarray(geometry.k, dtype=np.float64)
            # the scalars the reference forms per call (NumPy 0-d array arithmetic)
            return [m, period, 1.0, float(np.tan(alfa)), float(R**2), float(R**3),
                    float(k + 1)]
        raise ValueError("the diffractive interaction needs a grating geometry")


def make_interaction(interaction_type, is_reflective, focal_length=None, phase_profile=None):
    """surfaces/factories/interaction_model_factory.py:29-90."""
    if interaction_type == "refractive_reflective":
        return RefractiveReflectiveModel(is_reflective=is_reflective)
    if interaction_type == "thin_lens":
        return ThinLensInteractionModel(focal_length=focal_length, is_reflective=is_reflective)
    if interaction_type == "diffractive":
        return DiffractiveInteractionModel(is_reflective=is_reflective)
    if interaction_type == "phase":
        if phase_profile is None:
            raise ValueError("phase_profile is required for phase interaction.")
        return PhaseInteractionModel(phase_profile=phase_profile, is_reflective=is_reflective)
    raise ValueError(f"Unknown interaction_type: {interaction_type}")
