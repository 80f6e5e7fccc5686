"""Surfaces and the surface group.

Mirrors optiland/surfaces/{standard_surface,object_surface,surface_group}.py and the
factories in optiland/surfaces/factories/*.py (add_surface keyword semantics:
radius / conic / thickness / dx / dy / x / y / z / rx / ry / rz / material /
surface_type / coefficients / aperture / tol / max_iter / norm_radius / zernike_type).

`SurfaceGroup.trace(rays, skip=0)` is the drop-in seam (surface_group.py:232-244): it
lowers the group into the kernel's surface table and runs the HIP trace; there is no
per-surface Python loop and no CPU path.
"""

from __future__ import annotations

import numpy as np

from .coordinate_system import CoordinateSystem
from .apertures import BaseAperture, RadialAperture  # noqa: F401 (re-export)
from .geometries import (
    BiconicGeometry,
    ChebyshevPolynomialGeometry,
    EvenAsphere,
    ForbesQ2dGeometry,
    ForbesQbfsGeometry,
    ForbesSolverConfig,
    ForbesSurfaceConfig,
    OddAsphere,
    Plane,
    GridSagGeometry,
    NurbsGeometry,
    PlaneGrating,
    PolynomialGeometry,
    StandardGratingGeometry,
    StandardGeometry,
    ToroidalGeometry,
    ZernikePolynomialGeometry,
    scalar,
)
from .interactions import RefractiveReflectiveModel, make_interaction
from .materials import BaseMaterial, IdealMaterial, configure_material


def _torch_or_none():
    try:
        import torch

        return torch
    except ImportError:  # pragma: no cover
        return None


def configure_aperture(aperture):
    """physical_apertures/radial.py:16-28: a number is a diameter (RadialAperture of half
    of it), an aperture object is used as is."""
    if aperture is None:
        return None
    if isinstance(aperture, (int, float)) and not isinstance(aperture, bool):
        return RadialAperture(r_max=aperture / 2)
    if isinstance(aperture, BaseAperture):
        return aperture
    raise ValueError(
        f"Invalid `aperture` provided: {aperture}. Must be scalar or of type `BaseAperture`."
    )


class Surface:
    """standard_surface.py:32-233 (the real-ray branch of Surface.trace runs in HIP)."""

    def __init__(self, previous_surface, material_post, geometry, is_stop=False,
                 aperture=None, surface_type=None, comment="", is_reflective=False,
                 interaction_model=None):
        self.geometry = geometry
        # standard_surface.py:74-83 (refractive / reflective unless given)
        if interaction_model is None:
            interaction_model = RefractiveReflectiveModel(is_reflective=is_reflective)
        self.interaction_model = interaction_model
        interaction_model.parent_surface = self
        self.previous_surface = previous_surface
        self._material_post = material_post
        self.is_stop = is_stop
        self.aperture = configure_aperture(aperture)
        self.semi_aperture = None
        self.surface_type = surface_type
        self.comment = comment
        self.thickness = 0.0
        self.reset()

    @property
    def material_pre(self):
        return (self.previous_surface.material_post if self.previous_surface is not None
                else self.material_post)

    @property
    def material_post(self):
        if self._material_post is None:  # mirror: material_post = material_pre
            return self.material_pre
        return self._material_post

    @material_post.setter
    def material_post(self, m):
        self._material_post = m

    @property
    def is_reflective(self):
        return self.interaction_model.is_reflective

    @is_reflective.setter
    def is_reflective(self, value):
        self.interaction_model.is_reflective = bool(value)

    def set_semi_aperture(self, r_max):
        self.semi_aperture = r_max

    def reset(self):
        for a in ("x", "y", "z", "L", "M", "N", "intensity", "opd"):
            setattr(self, a, np.empty(0))


class ObjectSurface(Surface):
    """object_surface.py:19-72: records only, no intersection."""

    def __init__(self, geometry, material_post, comment=""):
        super().__init__(None, material_post, geometry, comment=comment)

    @property
    def is_infinite(self):
        return bool(np.isinf(self.geometry.cs.z))


def _make_geometry(surface_type, cs, kw):
    """surfaces/factories/geometry_factory.py:58-389 with geometry_configs.py defaults."""
    st = surface_type or "standard"
    radius = kw.get("radius", np.inf)
    conic = kw.get("conic", 0.0)
    if st == "standard":
        if np.isinf(radius):
            return Plane(cs)
        return StandardGeometry(cs, radius, conic)
    if st in ("plane", "paraxial"):  # geometry_factory.py:352-367: a paraxial surface is a plane
        return Plane(cs)
    if st == "grating":  # geometry_factory.py:154-180 with GratingConfig defaults
        order = kw.get("grating_order", 0)
        period = kw.get("grating_period", np.inf)
        angle = kw.get("groove_orientation_angle", 0.0)
        if np.isinf(radius):
            return PlaneGrating(cs, order, period, angle)
        return StandardGratingGeometry(cs, radius, order, period, angle, conic)
    if st == "even_asphere":
        return EvenAsphere(cs, radius, conic, kw.get("tol", 1e-6), kw.get("max_iter", 100),
                           kw.get("coefficients", []))
    if st == "odd_asphere":
        return OddAsphere(cs, radius, conic, kw.get("tol", 1e-6), kw.get("max_iter", 100),
                          kw.get("coefficients", []))
    if st == "zernike":
        return ZernikePolynomialGeometry(
            cs, radius, conic, kw.get("tol", 1e-6), kw.get("max_iter", 100),
            kw.get("coefficients", []), kw.get("zernike_type", "fringe"),
            kw.get("norm_radius", 1.0))
    tol, max_iter = kw.get("tol", 1e-6), kw.get("max_iter", 100)
    if st == "polynomial":
        return PolynomialGeometry(cs, radius, conic, tol, max_iter, kw.get("coefficients", []))
    if st == "chebyshev":
        return ChebyshevPolynomialGeometry(cs, radius, conic, tol, max_iter,
                                           kw.get("coefficients", []), kw.get("norm_x", 1.0),
                                           kw.get("norm_y", 1.0))
    if st == "biconic":
        rx, ry = kw.get("radius_x", np.inf), kw.get("radius_y", np.inf)
        kx, ky = kw.get("conic_x", 0.0), kw.get("conic_y", 0.0)
        if np.isinf(rx) and np.isinf(ry) and kx == 0.0 and ky == 0.0:
            return Plane(cs)  # geometry_factory.py _create_biconic
        return BiconicGeometry(cs, rx, ry, kx, ky, tol, max_iter)
    if st == "toroidal":
        return ToroidalGeometry(cs, kw.get("radius_x", np.inf), kw.get("radius_y", np.inf),
                                kw.get("conic", 0.0), kw.get("toroidal_coeffs_poly_y", []),
                                tol, max_iter)
    if st == "grid_sag":  # geometry_factory.py:340-349, GridSagConfig defaults
        return GridSagGeometry(cs, kw.get("x_coordinates", []), kw.get("y_coordinates", []),
                               kw.get("sag_values", []), kw.get("tol", 1e-6),
                               kw.get("max_iter", 100))
    if st == "nurbs":  # geometry_factory.py:316-337, NurbsConfig defaults
        return NurbsGeometry(cs, radius, conic, kw.get("nurbs_norm_x", 0.0),
                             kw.get("nurbs_norm_y", 0.0), kw.get("nurbs_x_center", 0.0),
                             kw.get("nurbs_y_center", 0.0), kw.get("control_points"),
                             kw.get("weights"), kw.get("u_degree", 3), kw.get("v_degree", 3),
                             kw.get("u_knots"), kw.get("v_knots"), kw.get("n_points_u", 5),
                             kw.get("n_points_v", 5), tol, max_iter)
    if st in ("forbes_qbfs", "forbes_q2d"):  # geometry_factory.py:282-314
        cfg = ForbesSurfaceConfig(
            radius=radius, conic=conic, norm_radius=kw.get("norm_radius", 1.0),
            terms=kw.get("radial_terms" if st == "forbes_qbfs" else "freeform_coeffs", {}))
        cls = ForbesQbfsGeometry if st == "forbes_qbfs" else ForbesQ2dGeometry
        return cls(cs, cfg, ForbesSolverConfig(tol=tol, max_iter=max_iter))
    raise ValueError(
        f"Surface type {st!r} is not lowered to the MI355X trace core (supported: "
        "standard, plane, paraxial, grating, even_asphere, odd_asphere, zernike, "
        "polynomial, chebyshev, biconic, toroidal, forbes_qbfs, forbes_q2d, grid_sag, "
        "nurbs).")


_NAN_ROWS: dict = {}


def _nan_rows(k, n, device):
    """A [k][n] float64 NaN block (never handed out: only read by torch.cat)."""
    import torch

    key = (k, n, str(device))
    t = _NAN_ROWS.get(key)
    if t is None:
        if len(_NAN_ROWS) >= 4:
            _NAN_ROWS.clear()
        t = torch.full((k, n), float("nan"), dtype=torch.float64, device=device)
        _NAN_ROWS[key] = t
    return t


class SurfaceGroup:
    """surface_group.py:30-330."""

    def __init__(self):
        self.surfaces: list[Surface] = []
        self.use_absolute_cs = False
        # per-surface snapshots (standard_surface.py:266-286): None = image surface only,
        # "all" = every surface (8 x 8 B per ray per surface of HBM writes)
        self.record = None

    # -- properties (surface_group.py:95-217) --
    @property
    def num_surfaces(self):
        return len(self.surfaces)

    @property
    def positions(self):
        return np.array([s.geometry.cs.position_in_gcs[2] for s in self.surfaces]).reshape(-1, 1)

    @property
    def radii(self):
        return np.array([scalar(s.geometry.radius) for s in self.surfaces], dtype=np.float64)

    @property
    def stop_index(self):
        for i, s in enumerate(self.surfaces):
            if s.is_stop:
                return i
        raise ValueError("No stop surface found.")

    def n(self, wavelength):
        return np.array([s.material_post.n_scalar(wavelength) for s in self.surfaces])

    def _stack(self, attr):
        vals = [getattr(s, attr) for s in self.surfaces]
        torch = _torch_or_none()
        if torch is not None and any(torch.is_tensor(v) for v in vals):
            n = max(int(v.numel()) if torch.is_tensor(v) else len(v) for v in vals)
            dev = next(v.device for v in vals if torch.is_tensor(v))
            last = vals[-1]
            if (torch.is_tensor(last) and last.numel() == n and last.dtype == torch.float64
                    and not any(torch.is_tensor(v) and v.numel() == n for v in vals[:-1])):
                # the default: only the image surface is recorded -- one copy of a cached
                # NaN block instead of a fill per unrecorded surface
                return torch.cat((_nan_rows(len(vals) - 1, n, dev), last.reshape(1, n)))
            # surfaces without a record (only the image surface is recorded by default)
            rows = [v if torch.is_tensor(v) and v.numel() == n
                    else torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
                    for v in vals]
            return torch.stack(rows)
        return np.stack([np.asarray(v) for v in vals])

    @property
    def x(self):
        return self._stack("x")

    @property
    def y(self):
        return self._stack("y")

    @property
    def z(self):
        return self._stack("z")

    @property
    def L(self):
        return self._stack("L")

    @property
    def M(self):
        return self._stack("M")

    @property
    def N(self):
        return self._stack("N")

    @property
    def intensity(self):
        return self._stack("intensity")

    @property
    def opd(self):
        return self._stack("opd")

    def reset(self):
        for s in self.surfaces:
            s.reset()

    # -- building (surface_group.py:246-330 + factories) --
    def add_surface(self, new_surface=None, surface_type="standard", comment="",
                    index=None, is_stop=False, material="air", **kwargs):
        if new_surface is None:
            if index is None:
                raise ValueError("Must define index when defining surface.")
            if index > len(self.surfaces):
                raise IndexError("Surface index cannot be greater than number of surfaces.")
            new_surface = self._create(surface_type, comment, index, is_stop, material, kwargs)
        new_surface.thickness = kwargs.get("thickness", 0.0)
        if index is None:
            index = len(self.surfaces)
        if index < 0:
            raise IndexError(f"Index {index} cannot be negative.")
        if index == 0 and len(self.surfaces) > 0:
            raise ValueError("Surface index cannot be zero after first surface is created.")
        self.surfaces.insert(index, new_surface)
        self._relink()
        if not self.use_absolute_cs and index < len(self.surfaces) - 1:
            self._update_coordinate_systems(index)
        if new_surface.is_stop:
            for i, s in enumerate(self.surfaces):
                s.is_stop = i == index

    def _relink(self):
        for i, s in enumerate(self.surfaces):
            s.previous_surface = self.surfaces[i - 1] if i > 0 else None

    def _update_coordinate_systems(self, start_index):
        for i in range(max(start_index, 1), len(self.surfaces)):
            if i == 1:
                z = 0.0
            else:
                prev = self.surfaces[i - 1]
                z = prev.geometry.cs.z + scalar(prev.thickness)
            self.surfaces[i].geometry.cs.z = z

    def _create(self, surface_type, comment, index, is_stop, material, kw):
        # coordinate_system_factory.py:28-93
        if "z" in kw:
            if "thickness" in kw:
                raise ValueError('Cannot define both "thickness" and "z".')
            if "dx" in kw or "dy" in kw:
                raise ValueError('Cannot define "dx" or "dy" when using absolute "x", "y", "z".')
            x, y, z = kw.get("x", 0), kw.get("y", 0), kw["z"]
            self.use_absolute_cs = True
        else:
            if self.use_absolute_cs:
                raise ValueError('Cannot pass "thickness" after defining "x", "y", "z" '
                                 "position for a previous surface.")
            thickness = kw.get("thickness", 0)
            x, y = kw.get("dx", 0), kw.get("dy", 0)
            if index == 0:
                z = -thickness
            elif index == 1:
                z = 0
            else:
                prev = self.surfaces[index - 1]
                z = prev.geometry.cs.z + scalar(prev.thickness)
        cs = CoordinateSystem(x=x, y=y, z=z, rx=kw.get("rx", 0), ry=kw.get("ry", 0),
                              rz=kw.get("rz", 0))
        # material_factory.py:22-62
        is_reflective = isinstance(material, str) and material == "mirror"
        material_post = configure_material(material)
        geometry = _make_geometry(surface_type, cs, kw)
        if index == 0:
            s = ObjectSurface(geometry, material_post, comment)
            s.thickness = kw.get("thickness", 0.0)
            return s
        if surface_type == "paraxial" and index == 0:
            raise ValueError("Paraxial surface cannot be the object surface.")
        # surface_factory.py:117-140: the interaction model follows the surface type
        interaction_type = kw.get("interaction_type", "refractive_reflective")
        if surface_type == "paraxial":
            interaction_type = "thin_lens"
        elif surface_type == "grating":
            interaction_type = "diffractive"
        elif kw.get("phase_profile") is not None:
            interaction_type = "phase"
        for key in ("coating", "bsdf"):
            if kw.get(key) is not None:
                raise ValueError(f"{key} is out of scope for the trace core")
        model = make_interaction(interaction_type, is_reflective, focal_length=kw.get("f"),
                                 phase_profile=kw.get("phase_profile"))
        return Surface(None, material_post, geometry, is_stop=is_stop,
                       aperture=kw.get("aperture"), surface_type=surface_type,
                       comment=comment, interaction_model=model)

    def trace(self, rays, skip=0):
        """surface_group.py:232-244: trace `rays` (RealRays, device) in place."""
        from .raytrace import trace_surface_group

        return trace_surface_group(self, rays, skip=skip)
