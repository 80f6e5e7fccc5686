"""First-order (paraxial y-u) quantities needed to build rays: EPL, EPD, f2, XPL,
marginal / chief rays (for update_paraxial).

Restates optiland/paraxial.py:62-450 and raytrace/paraxial_ray_tracer.py:60-148 with the
same NumPy operations on shape-(1,) arrays, so the host scalars that feed the kernel's
ray generator are the reference's to the last bit (pinned in tests/test_host_lens.py).
Host-only: a handful of scalar operations per lens.
"""

from __future__ import annotations

import numpy as np


class Paraxial:
    def __init__(self, optic):
        self.optic = optic

    @property
    def surfaces(self):
        return self.optic.surface_group

    # -- paraxial_ray_tracer.py:60-133 --
    def _trace_generic(self, y, u, z, wavelength, reverse=False, skip=0):
        from .surfaces import ObjectSurface

        def proc(v):
            if isinstance(v, (int, float)):
                return np.array([v])
            return np.array(v)

        y_, u_, z_ = proc(y), proc(u), proc(z)
        R = self.surfaces.radii
        n = self.surfaces.n(wavelength)
        pos = np.ravel(self.surfaces.positions)
        surfs = self.surfaces.surfaces
        if reverse:
            R = -np.flip(R)
            n = np.roll(n, shift=1)
            n = np.flip(n)
            pos = pos[-1] - np.flip(pos)
            surfs = surfs[::-1]
        with np.errstate(invalid="ignore", divide="ignore"):
            power = np.diff(n, prepend=np.array([n[0]])) / R
        heights, slopes = [], []
        for k in range(skip, len(R)):
            if isinstance(surfs[k], ObjectSurface):
                heights.append(np.copy(y_))
                slopes.append(np.copy(u_))
                continue
            t = pos[k] - z_
            z_ = pos[k]
            y_ = y_ + t * u_
            thin = getattr(surfs[k], "surface_type", None) == "paraxial"
            if surfs[k].is_reflective:
                if thin:  # paraxial_ray_tracer.py:118-120
                    u_ = -u_ - y_ / surfs[k].interaction_model.f
                else:
                    u_ = -u_ - 2 * y_ / R[k]
            elif thin:  # :124-126
                u_ = (n[k - 1] * u_ - y_ / surfs[k].interaction_model.f) / n[k]
            else:
                u_ = (n[k - 1] * u_ - y_ * power[k]) / n[k]
            heights.append(np.copy(y_))
            slopes.append(np.copy(u_))
        return np.array(heights).reshape(-1, 1), np.array(slopes).reshape(-1, 1)

    # -- paraxial.py:75-87 --
    def f2(self):
        z_start = self.surfaces.positions[1] - 1
        y, u = self._trace_generic(1.0, 0.0, z_start, self.optic.primary_wavelength)
        with np.errstate(divide="ignore"):  # an afocal system: inf, as the reference returns
            f2 = -y[0] / u[-1]
        return np.abs(f2[0])

    # -- paraxial.py:207-230 --
    def EPL(self):
        stop_index = self.surfaces.stop_index
        if stop_index == 1:
            return self.surfaces.positions[1, 0]
        pos = self.surfaces.positions
        z0 = pos[-1] - pos[stop_index]
        skip = self.surfaces.num_surfaces - stop_index
        y, u = self._trace_generic(0, 0.1, z0[0], self.optic.primary_wavelength,
                                   reverse=True, skip=skip)
        loc_relative = y[-1] / u[-1]
        return loc_relative[0]

    # -- paraxial.py:232-297 --
    def EPD(self):
        ap = self.optic.aperture
        if ap is None:
            raise ValueError()
        if ap.ap_type == "EPD":
            return ap.value
        if ap.ap_type == "imageFNO":
            return self.f2() / ap.value
        if ap.ap_type == "objectNA":
            obj_z = self.optic.object_surface.geometry.cs.z
            n0 = self.optic.object_surface.material_post.n_scalar(self.optic.primary_wavelength)
            u0 = np.arcsin(ap.value / n0)
            z = self.EPL() - obj_z
            return 2 * z * np.tan(u0)
        if ap.ap_type == "float_by_stop_size":
            stop_index = self.surfaces.stop_index
            wl = self.optic.primary_wavelength
            if self.optic.object_surface.is_infinite:
                y, _ = self._trace_generic(1.0, 0.0, -1, wl)
                return ap.value / y[stop_index]
            obj_z = self.optic.object_surface.geometry.cs.z
            EPL = self.EPL()
            y, _ = self._trace_generic(0.0, 0.1, obj_z, wl)
            u0 = 0.1 * ap.value / y[stop_index]
            return u0 * (EPL - obj_z)
        raise NotImplementedError()

    # -- paraxial.py:318-335 --
    def XPL(self):
        stop_index = self.surfaces.stop_index
        z_start = self.surfaces.positions[stop_index]
        y, u = self._trace_generic(0.0, 0.1, z_start, self.optic.primary_wavelength,
                                   skip=stop_index + 1)
        loc_relative = -y[-1] / u[-1]
        return loc_relative[0]

    # -- paraxial.py:387-417 --
    def marginal_ray(self):
        EPD = self.EPD()
        obj_z = self.surfaces.positions[1] - 10
        if self.optic.object_surface.is_infinite:
            ya = EPD / 2
            ua = 0
        else:
            obj_z = self.optic.object_surface.geometry.cs.z
            z = self.EPL() - obj_z
            ya = 0
            ua = EPD / (2 * z)
        return self._trace_generic(ya, ua, obj_z, self.optic.primary_wavelength)

    # -- paraxial.py:419-482 --
    def chief_ray(self):
        sg = self.surfaces
        stop_index = sg.stop_index
        pos = sg.positions
        wl = self.optic.primary_wavelength
        num_surf = sg.num_surfaces
        y_fwd_unit, _ = self._trace_generic(0.0, 0.1, pos[stop_index], wl, skip=stop_index)
        y_img_unit = y_fwd_unit[-1]
        z_rev = pos[-1] - pos[stop_index]
        y_rev_unit, u_rev_unit = self._trace_generic(0.0, 0.1, z_rev, wl, reverse=True,
                                                     skip=num_surf - stop_index)
        y_obj_unit = y_rev_unit[-1]
        u_obj_unit = u_rev_unit[-1]
        fd = self.optic.field_type
        if fd == "angle":
            target_slope = np.tan(np.deg2rad(self.optic.fields.max_y_field))
            scaling_factor = target_slope / u_obj_unit
        elif fd == "object_height":
            scaling_factor = self.optic.fields.max_y_field / y_obj_unit
        elif fd == "paraxial_image_height":  # field_types.py:423-440
            scaling_factor = self.optic.fields.max_y_field / y_img_unit
        else:
            raise NotImplementedError(fd)
        if fd == "paraxial_image_height":
            y_obj_start = y_obj_unit * scaling_factor
        else:
            y_obj_start = -(y_obj_unit * scaling_factor)
        u_obj_start = u_obj_unit * scaling_factor
        if self.optic.object_surface.is_infinite:
            EPL = self.EPL()
            z_surf1 = sg.positions[1, 0]
            y1_start = u_obj_start * (z_surf1 - EPL)
            return self._trace_generic(y1_start, u_obj_start, z_surf1, wl)
        z_start = self.optic.object_surface.geometry.cs.z
        return self._trace_generic(y_obj_start, u_obj_start, z_start, wl)
