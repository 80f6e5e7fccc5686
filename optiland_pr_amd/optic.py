"""Optic: the lens system object (host side).

Mirrors the slice of optiland/optic/optic.py the ray-trace path uses:
add_surface / set_aperture / set_field_type / add_field / add_wavelength /
update_paraxial / trace (optic.py:584-609) / trace_generic (:611-632), plus
paraxial, fields, wavelengths, surface_group, object_surface, image_surface,
primary_wavelength, n().

Optic.trace and trace_generic run on the MI355X: rays are generated and traced by the
HIP kernels; the returned RealRays hold device (torch) tensors.
"""

from __future__ import annotations

import numpy as np

from .fields import Aperture, Field, FieldGroup, WavelengthGroup
from .paraxial import Paraxial
from .surfaces import ObjectSurface, SurfaceGroup


class Optic:
    def __init__(self, name: str | None = None):
        self.name = name
        self.surface_group = SurfaceGroup()
        self.fields = FieldGroup()
        self.wavelengths = WavelengthGroup()
        self.aperture = None
        self.field_type = None
        self.paraxial = Paraxial(self)
        self.obj_space_telecentric = False
        self.polarization = "ignore"
        self.apodization = None
        self._lowered = None  # lowering cache (raytrace.LoweredLens), reset on edits
        # Newton schedule verification of trace(): "reference" checks each launch's
        # schedule on the host (one read per launch); "device" checks warm schedules on
        # the device (ort_newton_fixup: same schedules, same results, no host round trip;
        # a range error or an unsettled schedule is raised at the next trace call or
        # raytrace.check_all_pending) -- for optimisation loops
        self.newton_mode = "reference"

    # -- building ---------------------------------------------------------------------
    def add_surface(self, new_surface=None, surface_type="standard", comment="",
                    index=None, is_stop=False, material="air", **kwargs):
        self._lowered = None
        self.surface_group.add_surface(new_surface=new_surface, surface_type=surface_type,
                                       comment=comment, index=index, is_stop=is_stop,
                                       material=material, **kwargs)

    def add_field(self, y, x=0.0, vx=0.0, vy=0.0):
        self.fields.add_field(Field(x, y, vx, vy))

    def add_wavelength(self, value, is_primary=False, unit="um"):
        self.wavelengths.add_wavelength(value=value, is_primary=is_primary, unit=unit)

    def set_aperture(self, aperture_type, value):
        self._lowered = None
        self.aperture = Aperture(aperture_type, value)

    def set_apodization(self, apodization=None, **kwargs):
        """optic.py:401-419 -> optic_updater.py:312-350: an apodization instance, a
        class name plus its keyword arguments, a to_dict() dict, or None."""
        from .apodization import resolve

        self.apodization = resolve(apodization, **kwargs)

    def image_solve(self):
        """optic_updater.py:258-270: move the image surface to the paraxial focus of the
        marginal ray."""
        ya, ua = self.paraxial.marginal_ray()
        offset = float(ya[-1, 0] / ua[-1, 0])
        surfs = self.surface_group.surfaces
        surfs[-1].geometry.cs.z -= offset
        surfs[-2].thickness = surfs[-1].geometry.cs.z - surfs[-2].geometry.cs.z
        self._lowered = None

    def set_field_type(self, field_type):
        """optic.py:298-318: 'angle' | 'object_height' | 'paraxial_image_height'."""
        if field_type not in ("angle", "object_height", "paraxial_image_height"):
            raise ValueError(f"field type {field_type!r} is not supported by the trace core")
        self.field_type = field_type

    # -- parameter setters (optic_updater.py:37-86: what the optimisation variables call;
    #    torch tensors are kept as given so they can be autograd leaves, autodiff.py) ----
    def set_radius(self, value, surface_number):
        self.surface_group.surfaces[surface_number].geometry.radius = value

    def set_conic(self, value, surface_number):
        self.surface_group.surfaces[surface_number].geometry.k = value

    def set_thickness(self, value, surface_number):
        """optic_updater.py:67-85: move every later vertex by the change, keep surface 1
        at z = 0, store the thickness."""
        from .geometries import scalar

        surfs = self.surface_group.surfaces
        pos = [float(s.geometry.cs.z) for s in surfs]
        delta = scalar(value) - pos[surface_number + 1] + pos[surface_number]
        pos = [p + delta if k > surface_number else p for k, p in enumerate(pos)]
        z1 = pos[1]
        for k, s in enumerate(surfs):
            s.geometry.cs.z = pos[k] - z1
        if surface_number < len(surfs):
            surfs[surface_number].thickness = value

    def invalidate(self):
        """Drop cached device tables after editing surfaces in place."""
        self._lowered = None

    # -- properties -------------------------------------------------------------------
    @property
    def primary_wavelength(self):
        return self.wavelengths.primary_wavelength.value

    @property
    def object_surface(self):
        for s in self.surface_group.surfaces:
            if isinstance(s, ObjectSurface):
                return s
        return None

    @property
    def image_surface(self):
        return self.surface_group.surfaces[-1] if self.surface_group.surfaces else None

    def n(self, wavelength="primary"):
        if wavelength == "primary":
            wavelength = self.primary_wavelength
        return self.surface_group.n(wavelength)

    # -- optic_updater.py:192-240 --
    def update_paraxial(self):
        ya, _ = self.paraxial.marginal_ray()
        yb, _ = self.paraxial.chief_ray()
        ya = np.abs(np.ravel(ya))
        yb = np.abs(np.ravel(yb))
        for k, s in enumerate(self.surface_group.surfaces):
            s.set_semi_aperture(r_max=ya[k] + yb[k])
            # optic_updater.py:205-240 update_normalization
            if hasattr(s.geometry, "norm_x"):
                s.geometry.norm_x = float(s.semi_aperture * 1.25)
            if hasattr(s.geometry, "norm_y"):
                s.geometry.norm_y = float(s.semi_aperture * 1.25)
            if s.surface_type == "zernike":
                s.geometry.norm_radius = float(s.semi_aperture * 1.25)
        self._lowered = None

    # -- serialisation (optic.py:649-713; lensio.py) -----------------------------------
    def to_dict(self):
        from .lensio import optic_to_dict

        return optic_to_dict(self)

    @classmethod
    def from_dict(cls, data):
        from .lensio import optic_from_dict

        return optic_from_dict(data)

    # -- tracing ----------------------------------------------------------------------
    def trace(self, Hx, Hy, wavelength, num_rays=100, distribution="hexapolar"):
        """optic.py:584-609 -> RealRayTracer.trace (HIP)."""
        from .raytrace import RealRayTracer

        return RealRayTracer(self).trace(Hx, Hy, wavelength, num_rays, distribution)

    def trace_generic(self, Hx, Hy, Px, Py, wavelength):
        """optic.py:611-632 -> RealRayTracer.trace_generic (HIP)."""
        from .raytrace import RealRayTracer

        return RealRayTracer(self).trace_generic(Hx, Hy, Px, Py, wavelength)
