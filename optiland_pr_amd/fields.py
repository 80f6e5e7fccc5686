"""Fields, aperture and wavelengths (host scalars for ray generation).

Mirrors optiland/fields/{field,field_group,field_types}.py, optiland/aperture.py and
optiland/wavelength.py: the pieces RayGenerator.generate_rays reads
(ray_generator.py:49-106): max field, vignetting factors, field type, EPD/EPL.
"""

from __future__ import annotations

import numpy as np


class Field:
    """fields/field.py: one field point with vignetting factors."""

    def __init__(self, x=0.0, y=0.0, vx=0.0, vy=0.0):
        self.x, self.y, self.vx, self.vy = float(x), float(y), float(vx), float(vy)


class FieldGroup:
    """fields/field_group.py:14-153."""

    def __init__(self):
        self.fields: list[Field] = []
        self.telecentric = False

    def add_field(self, field):
        self.fields.append(field)

    @property
    def x_fields(self):
        return np.array([f.x for f in self.fields])

    @property
    def y_fields(self):
        return np.array([f.y for f in self.fields])

    @property
    def max_x_field(self):
        return np.max(self.x_fields)

    @property
    def max_y_field(self):
        return np.max(self.y_fields)

    @property
    def max_field(self):
        return np.max(np.sqrt(self.x_fields**2 + self.y_fields**2))

    @property
    def num_fields(self):
        return len(self.fields)

    def get_field_coords(self):
        """field_group.py:111-131."""
        max_field = self.max_field
        if max_field == 0:
            return [(0, 0)]
        return [(float(x / max_field), float(y / max_field))
                for x, y in zip(self.x_fields, self.y_fields, strict=True)]

    def get_vig_factor(self, Hx, Hy):
        """field_group.py:80-109: nearest-neighbour interpolation of (vx, vy) in
        normalised field space (scipy NearestNDInterpolator semantics for one query)."""
        max_field = self.max_field
        xf = self.x_fields if max_field == 0 else self.x_fields / max_field
        yf = self.y_fields if max_field == 0 else self.y_fields / max_field
        vx = np.array([f.vx for f in self.fields])
        vy = np.array([f.vy for f in self.fields])
        d2 = (xf - float(Hx)) ** 2 + (yf - float(Hy)) ** 2
        j = int(np.argmin(d2))
        return float(vx[j]), float(vy[j])


class Aperture:
    """aperture.py: aperture type in {EPD, imageFNO, objectNA, float_by_stop_size}."""

    def __init__(self, aperture_type, value):
        if aperture_type not in ("EPD", "imageFNO", "objectNA", "float_by_stop_size"):
            raise ValueError("Aperture type must be one of EPD, imageFNO, objectNA, "
                             "float_by_stop_size.")
        self.ap_type = aperture_type
        self.value = float(value)


class Wavelength:
    def __init__(self, value, is_primary=False, unit="um"):
        scale = {"nm": 1e-3, "um": 1.0, "mm": 1e3, "cm": 1e4, "m": 1e6}[unit]
        self.value = float(value) * scale
        self.is_primary = is_primary


class WavelengthGroup:
    """wavelength.py:180-260."""

    def __init__(self):
        self.wavelengths: list[Wavelength] = []

    def add_wavelength(self, value, is_primary=False, unit="um"):
        if is_primary:
            for w in self.wavelengths:
                w.is_primary = False
        if self.num_wavelengths == 0:
            is_primary = True
        self.wavelengths.append(Wavelength(value, is_primary, unit))

    @property
    def num_wavelengths(self):
        return len(self.wavelengths)

    @property
    def primary_index(self):
        for i, w in enumerate(self.wavelengths):
            if w.is_primary:
                return i
        return 0

    @property
    def primary_wavelength(self):
        return self.wavelengths[self.primary_index]

    def get_wavelengths(self):
        return [w.value for w in self.wavelengths]
