"""Golden-vector generator: runs the REFERENCE (Optiland, /root/reference) in this
container and writes small fixtures under tests/golden/ plus the baked glass table
optiland_pr_amd/data/glasses.json.

This script is test infrastructure. It is never imported by the product, by the GPU
tests, by smoke() or by bench.py; /root/reference does not exist on the GPU box.

Invocation (from the repo root):

    PYTHONPATH=tests/golden/shims:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_golden.py

`tests/golden/shims` holds two stand-in modules (numba, vtk) that the reference
imports off the ray-trace path (scatter.py:17, nurbs_basis_functions.py:3,
huygens_fresnel_strategies.py:20, visualization/system/utils.py:11). They do not
touch any arithmetic on the traced path.

What is recorded per case (see CASES below):
  * inputs: field points, wavelengths, pupil samples Px/Py
  * reference host scalars: EPL, EPD, surface z positions, n/k per surface per lambda
  * generated rays (RayGenerator.generate_rays, ray_generator.py:28-106)
  * image-plane rays after Optic.trace (real_ray_tracer.py:37-97): x,y,z,L,M,N,i,opd
  * Newton update counts per surface (newton_raphson.py:137-166)
  * per-surface records (standard_surface.py:266-286) for the DoubleGauss case
"""

from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

import optiland.backend as be  # noqa: E402
from optiland import optic as ref_optic  # noqa: E402
from optiland.analysis import SpotDiagram  # noqa: E402
from optiland.distribution import RandomDistribution, create_distribution  # noqa: E402
from optiland.geometries.grid_sag import GridSagGeometry  # noqa: E402
from optiland.geometries.newton_raphson import NewtonRaphsonGeometry  # noqa: E402
from optiland.materials.ideal import IdealMaterial  # noqa: E402
from optiland.materials.material import Material  # noqa: E402
from optiland.samples.objectives import (  # noqa: E402
    CookeTriplet,
    DoubleGauss,
    ReverseTelephoto,
)
from optiland.rays import RayGenerator  # noqa: E402
from optiland.wavefront import OPD  # noqa: E402

be.set_backend("numpy")


# --------------------------------------------------------------------------------------
# lens builders (reference API). The native package restates each of these in
# optiland_pr_amd/samples.py with its own API.
# --------------------------------------------------------------------------------------
def rt_asph():
    """ReverseTelephoto with surfaces 2 and 13 turned into even aspheres."""
    lens = ReverseTelephoto()
    sg = lens.surface_group
    specs = {2: [0.02, -0.01, 0.005], 13: [0.01, 0.005, -0.002]}
    return _replace_with_asphere(lens, specs, "even_asphere")


def rt_odd():
    """ReverseTelephoto with surface 4 as an odd asphere (covers odd_asphere.py:73-130)."""
    lens = ReverseTelephoto()
    specs = {4: [0.0, 0.003, -0.002, 0.001]}
    return _replace_with_asphere(lens, specs, "odd_asphere")


def _replace_with_asphere(lens, specs, kind):
    sg = lens.surface_group
    rows = []
    for k, s in enumerate(sg.surfaces):
        rows.append(
            dict(
                radius=float(s.geometry.radius) if hasattr(s.geometry, "radius") else np.inf,
                thickness=float(s.thickness),
                material=s.material_post,
                is_stop=s.is_stop,
            )
        )
    new = ref_optic.Optic()
    for k, r in enumerate(rows):
        kw = dict(index=k, radius=r["radius"], thickness=r["thickness"], is_stop=r["is_stop"])
        if k == 0:
            kw["thickness"] = np.inf
        if k > 0 and not isinstance(r["material"], IdealMaterial):
            kw["material"] = r["material"]
        if k in specs:
            kw["surface_type"] = kind
            kw["conic"] = 0.0
            kw["coefficients"] = specs[k]
        if k == len(rows) - 1:
            kw = dict(index=k)
        new.add_surface(**kw)
    new.set_aperture(aperture_type="EPD", value=0.3)
    new.set_field_type(field_type="angle")
    new.add_field(y=0)
    new.add_field(y=21)
    new.add_field(y=30)
    new.add_wavelength(value=0.4861)
    new.add_wavelength(value=0.5876, is_primary=True)
    new.add_wavelength(value=0.6563)
    return new


def tma(zernike_type="fringe", coeffs=(0, 0, 0, 1e-4, 2e-4, -1e-4, 5e-5, 0, 0, 3e-5)):
    """Three-mirror anastigmat, docs/examples/Tutorial_7d_Three_Mirror_Anastigmat.ipynb
    cell 1, with fixed Zernike coefficients."""
    lens = ref_optic.Optic(name="TMA")
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=+1.5)
    lens.add_field(y=-1.5)
    lens.add_wavelength(value=0.486)
    lens.add_wavelength(value=0.587, is_primary=True)
    lens.add_wavelength(value=0.656)
    lens.add_surface(index=0, radius=np.inf, thickness=np.inf)
    common = dict(conic=0, material="mirror", surface_type="zernike",
                  coefficients=list(coeffs), zernike_type=zernike_type)
    lens.add_surface(index=1, radius=-100, thickness=-20, rx=np.radians(-15.0),
                     is_stop=True, **common)
    lens.add_surface(index=2, radius=-100, thickness=+20, rx=np.radians(-10.0),
                     dy=-11.5, **common)
    lens.add_surface(index=3, radius=-100, thickness=-22, rx=np.radians(-1.0),
                     dy=-15, **common)
    lens.add_surface(index=4, dy=-19.3)
    lens.update_paraxial()
    return lens


def cooke_aperture():
    """Cooke triplet with a radial clear aperture on surface 3 (diameter 9 mm, clips the
    edge of the 20 deg beam) and an annular one on surface 5: covers
    physical_apertures/radial.py:50-63 + real_rays.py:132-139."""
    from optiland.physical_apertures.radial import RadialAperture

    lens = CookeTriplet()
    lens.surface_group.surfaces[3].aperture = RadialAperture(r_max=4.5)
    lens.surface_group.surfaces[5].aperture = RadialAperture(r_max=8.0, r_min=0.4)
    return lens


STAR = (np.array([4.2, 1.3, 1.2, -3.4, -1.9, -3.3, 1.4, 1.1]),
        np.array([0.1, 1.2, 4.0, 2.6, -0.3, -3.1, -1.5, -4.1]))  # concave polygon


def cooke_shapes():
    """Cooke triplet with every non-radial aperture kind (physical_apertures/*.py):
    rectangular (s1), elliptical with offset (s2), offset annulus (s3), a concave polygon
    on the stop (s4) and (rectangle | ellipse) minus an offset central obscuration (s6)."""
    from optiland.physical_apertures import (
        EllipticalAperture,
        OffsetRadialAperture,
        PolygonAperture,
        RectangularAperture,
    )

    lens = CookeTriplet()
    sg = lens.surface_group.surfaces
    sg[1].aperture = RectangularAperture(-5.5, 5.0, -4.8, 5.2)
    sg[2].aperture = EllipticalAperture(5.5, 4.6, 0.2, -0.1)
    sg[3].aperture = OffsetRadialAperture(4.6, 0.3, 0.1, -0.2)
    sg[4].aperture = PolygonAperture(*STAR)
    sg[6].aperture = ((RectangularAperture(-6, 6, -2.5, 2.5) | EllipticalAperture(3.5, 6.5))
                      - OffsetRadialAperture(0.6, 0, 0.1, 0.0))
    return lens


def decentered():
    """Cooke triplet with a tilted + decentred second element and an ry/rz tilt chain,
    covering coordinate_system.py:73-107 rotate_x/y/z + translate on refracting surfaces."""
    lens = ref_optic.Optic()
    lens.add_surface(index=0, radius=np.inf, thickness=np.inf)
    lens.add_surface(index=1, radius=22.01359, thickness=3.25896, material="SK16")
    lens.add_surface(index=2, radius=-435.76044, thickness=6.00755)
    lens.add_surface(index=3, radius=-22.21328, thickness=0.99997, material=("F2", "schott"),
                     dx=0.05, dy=-0.1, rx=0.01, ry=-0.02, rz=0.3)
    lens.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True,
                     dy=-0.1, rx=0.01)
    lens.add_surface(index=5, radius=79.68360, thickness=2.95208, material="SK16",
                     conic=-0.5)
    lens.add_surface(index=6, radius=-18.39533, thickness=42.20778, conic=1.2)
    lens.add_surface(index=7)
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=14)
    lens.add_field(x=5, y=20)
    lens.add_wavelength(value=0.55, is_primary=True)
    return lens


def freeform():
    """Cooke-triplet layout with a biconic, a toroidal, an XY-polynomial and a Chebyshev
    surface (covers biconic.py, toroidal.py, polynomial.py, chebyshev.py on the trace)."""
    lens = ref_optic.Optic()
    lens.add_surface(index=0, radius=np.inf, thickness=np.inf)
    lens.add_surface(index=1, surface_type="biconic", radius_x=22.01359, radius_y=23.5,
                     conic_x=-0.2, conic_y=0.1, thickness=3.25896, material="SK16")
    lens.add_surface(index=2, surface_type="toroidal", radius_x=-300.0, radius_y=-435.76044,
                     conic=0.5, toroidal_coeffs_poly_y=[2e-6], thickness=6.00755)
    lens.add_surface(index=3, radius=-22.21328, thickness=0.99997, material=("F2", "schott"))
    lens.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True)
    lens.add_surface(index=5, surface_type="polynomial", radius=79.68360, conic=0.0,
                     coefficients=[[0.0, 0.0, 2e-4], [0.0, 1e-5, 0.0], [1.5e-4, 0.0, 0.0]],
                     thickness=2.95208, material="SK16")
    lens.add_surface(index=6, surface_type="chebyshev", radius=-18.39533, conic=0.0,
                     coefficients=[[0.0, 1e-3, 2e-3], [5e-4, 0.0, 0.0], [1e-3, 0.0, 0.0]],
                     thickness=42.20778)
    lens.add_surface(index=7)
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=14)
    lens.add_field(x=5, y=10)
    lens.add_wavelength(value=0.55, is_primary=True)
    lens.update_paraxial()
    return lens


def _forbes_prescription(lens, s2_type, s2_terms):
    """tests/test_geometries.py:2103-2143 (forbes_system): a plano-Forbes singlet and a
    plano-Forbes element at 1.55 um, CDGM glasses; fields added for off-axis coverage."""
    lens.set_aperture(aperture_type="EPD", value=4.0)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=3)
    lens.add_field(x=2, y=2)
    lens.add_wavelength(value=1.55, is_primary=True)
    h_k3 = Material("H-K3", reference="cdgm")
    h_zlaf = Material("H-ZLAF68C", reference="cdgm")
    lens.add_surface(index=0, thickness=0.055)
    lens.add_surface(index=1, thickness=26.5)
    lens.add_surface(index=2, thickness=4.0, radius=np.inf, material=h_k3, is_stop=True)
    kw = ({"radial_terms": s2_terms} if s2_type == "forbes_qbfs"
          else {"freeform_coeffs": s2_terms})
    lens.add_surface(index=3, thickness=25.0, radius=22, conic=-4.428, norm_radius=6.336,
                     surface_type=s2_type, **kw)
    lens.add_surface(index=4, thickness=7.0, radius=np.inf, material=h_zlaf)
    lens.add_surface(index=5, thickness=10.0, radius=-31.0, conic=0.038,
                     radial_terms={0: -0.270, 1: 0.087, 2: -0.048, 3: 0.026, 4: -0.012},
                     norm_radius=10.0, surface_type="forbes_qbfs")
    lens.add_surface(index=6)
    return lens


FORBES_S2_QBFS = {0: 1.614, 1: 0.348, 2: 0.150, 3: 0.033, 4: 0.030}
FORBES_S2_Q2D = {("a", 0, 0): 1.614, ("a", 0, 1): 0.348, ("a", 0, 2): 0.150,
                 ("a", 1, 1): 0.02, ("b", 1, 1): -0.01, ("a", 1, 3): 0.005,
                 ("a", 2, 0): 0.03, ("b", 2, 1): 0.01, ("a", 3, 0): -0.004,
                 ("b", 4, 1): 0.002}


def forbes():
    return _forbes_prescription(ref_optic.Optic(), "forbes_qbfs", FORBES_S2_QBFS)


def forbes_q2d():
    return _forbes_prescription(ref_optic.Optic(), "forbes_q2d", FORBES_S2_Q2D)


def _cooke_prescription(lens, object_thickness):
    lens.add_surface(index=0, radius=np.inf, thickness=object_thickness)
    lens.add_surface(index=1, radius=22.01359, thickness=3.25896, material="SK16")
    lens.add_surface(index=2, radius=-435.76044, thickness=6.00755)
    lens.add_surface(index=3, radius=-22.21328, thickness=0.99997, material=("F2", "schott"))
    lens.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True)
    lens.add_surface(index=5, radius=79.68360, thickness=2.95208, material="SK16")
    lens.add_surface(index=6, radius=-18.39533, thickness=42.20778)
    lens.add_surface(index=7)
    lens.set_aperture(aperture_type="EPD", value=10)


def cooke_pih():
    """Cooke triplet, fields as paraxial image heights (field_types.py:333-479), object at
    infinity."""
    lens = ref_optic.Optic()
    _cooke_prescription(lens, np.inf)
    lens.set_field_type(field_type="paraxial_image_height")
    lens.add_field(y=0)
    lens.add_field(y=10)
    lens.add_field(y=17)
    lens.add_wavelength(value=0.55, is_primary=True)
    return lens


def finite_pih():
    """The triplet with the object 200 mm in front, fields as paraxial image heights."""
    lens = ref_optic.Optic()
    _cooke_prescription(lens, 200.0)
    lens.set_field_type(field_type="paraxial_image_height")
    lens.add_field(y=0)
    lens.add_field(y=2)
    lens.add_field(y=4)
    lens.add_wavelength(value=0.55, is_primary=True)
    return lens


def paraxial_lens():
    """Two thin lenses (surface_type "paraxial", thin_lens_interaction_model.py) around a
    glass singlet, the second thin lens in a medium of index 1.2: covers the paraxial
    phase transformation and the normalisation at the next propagation."""
    lens = ref_optic.Optic()
    lens.add_surface(index=0, thickness=np.inf)
    lens.add_surface(index=1, surface_type="paraxial", f=80, thickness=10, is_stop=True)
    lens.add_surface(index=2, radius=60.0, thickness=4.0, material="SK16")
    lens.add_surface(index=3, radius=-200.0, thickness=10.0)
    lens.add_surface(index=4, surface_type="paraxial", f=-150, thickness=40,
                     material=IdealMaterial(1.2, 0))
    lens.add_surface(index=5)
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=5)
    lens.add_field(x=2, y=3)
    lens.add_wavelength(value=0.55, is_primary=True)
    return lens


def paraxial_mirror():
    """A reflective thin lens (n2 = -n1; paraxial_ray_tracer.py:118-120)."""
    lens = ref_optic.Optic()
    lens.add_surface(index=0, thickness=np.inf)
    lens.add_surface(index=1, surface_type="paraxial", f=-60, thickness=-50, material="mirror",
                     is_stop=True)
    lens.add_surface(index=2)
    lens.set_aperture(aperture_type="EPD", value=12)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=4)
    lens.add_wavelength(value=0.6, is_primary=True)
    return lens


def phase_plate():
    """Phase surfaces (phase_interaction_model.py): a linear grating on a plane, a radial
    profile on a sphere, a constant phase, a metalens-like radial profile on a plane."""
    from optiland.phase import ConstantPhaseProfile, LinearGratingPhaseProfile, RadialPhaseProfile

    lens = ref_optic.Optic()
    lens.add_surface(index=0, thickness=np.inf)
    lens.add_surface(index=1, thickness=5, is_stop=True,
                     phase_profile=LinearGratingPhaseProfile(period=5.0, angle=0.4, order=1,
                                                             efficiency=0.8))
    lens.add_surface(index=2, radius=60.0, thickness=4.0, material="SK16",
                     phase_profile=RadialPhaseProfile([-0.02, 1e-5, -2e-8]))
    lens.add_surface(index=3, radius=-200.0, thickness=3.0,
                     phase_profile=ConstantPhaseProfile(0.7))
    lens.add_surface(index=4, thickness=60.0, phase_profile=RadialPhaseProfile([-0.15]))
    lens.add_surface(index=5)
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=5)
    lens.add_field(x=1.5, y=-3)
    lens.add_wavelength(value=0.48)
    lens.add_wavelength(value=0.55, is_primary=True)
    lens.add_wavelength(value=0.65)
    return lens


def _grating_common(lens):
    lens.set_aperture(aperture_type="EPD", value=15)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=10)
    lens.add_field(y=0, x=10)
    lens.add_wavelength(value=0.587, is_primary=True)
    lens.update_paraxial()
    return lens


def grating(kind, angle=0.0):
    """The reference's grating test systems (tests/test_grating.py:7-117): flat and
    curved transmission gratings behind an N-BK7 plate, a curved reflective grating;
    `angle` rotates the grooves (groove_orientation_angle)."""
    lens = ref_optic.Optic()
    lens.add_surface(index=0, radius=np.inf, thickness=np.inf)
    if kind == "reflective":
        lens.add_surface(index=1, radius=70, thickness=-30, material="mirror",
                         surface_type="grating", is_stop=True, grating_period=5.0,
                         grating_order=1, groove_orientation_angle=angle)
        lens.add_surface(index=2)
        return _grating_common(lens)
    lens.add_surface(index=1, radius=np.inf, thickness=10)
    lens.add_surface(index=2, radius=np.inf, thickness=5, material="N-BK7")
    kw = dict(radius=np.inf) if kind == "flat" else dict(radius=50.0, conic=1.0)
    lens.add_surface(index=3, thickness=30, surface_type="grating", grating_order=-1,
                     grating_period=5.0, groove_orientation_angle=angle, is_stop=True, **kw)
    lens.add_surface(index=4)
    return _grating_common(lens)


def grid_sag_values():
    """A 17 x 13 sag grid over [-7, 7] x [-6, 6] mm: a weak sphere-like bowl, an xy term
    and a y tilt (shared with optiland_pr_amd.samples.GridSagLens)."""
    gx = np.linspace(-7, 7, 17)
    gy = np.linspace(-6, 6, 13)
    X, Y = np.meshgrid(gx, gy)
    return gx, gy, (X**2 + Y**2) / 80.0 + 0.003 * X * Y - 0.02 * Y


def grid_lens():
    """A singlet whose front surface is a bilinear sag grid (grid_sag.py), behind it a
    sphere: covers the grid Newton loop (t from 0, global max|dt| < tol)."""
    gx, gy, z = grid_sag_values()
    lens = ref_optic.Optic()
    lens.add_surface(index=0, thickness=np.inf)
    lens.add_surface(index=1, surface_type="grid_sag", x_coordinates=gx.tolist(),
                     y_coordinates=gy.tolist(), sag_values=z.tolist(), thickness=4.0,
                     material="SK16", is_stop=True)
    lens.add_surface(index=2, radius=-60.0, thickness=45.0)
    lens.add_surface(index=3)
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=5)
    lens.add_field(x=3, y=2)
    lens.add_wavelength(value=0.55, is_primary=True)
    return lens


def nurbs_back_net():
    """The explicit rational back surface of nurbs_lens (shared with
    optiland_pr_amd.samples.NurbsLens): a 7 x 6 net over [-8, 8] x [-8, 8], a concave bowl
    with an xy twist, non-uniform weights, u degree 3 / v degree 2 on clamped non-uniform
    knots."""
    xs = np.linspace(-8.0, 8.0, 7)
    ys = np.linspace(-8.0, 8.0, 6)
    X, Y = np.meshgrid(xs, ys, indexing="ij")
    Z = -(X**2 + Y**2) / 140.0 + 0.002 * X * Y
    W = 1.0 + 0.1 * np.cos(0.5 * X) * np.sin(0.4 * Y + 0.2)
    U = [0.0, 0.0, 0.0, 0.0, 0.3, 0.5, 0.75, 1.0, 1.0, 1.0, 1.0]
    V = [0.0, 0.0, 0.0, 0.2, 0.55, 0.8, 1.0, 1.0, 1.0]
    return np.stack([X, Y, Z]), W, U, V


def nurbs_lens():
    """A singlet whose front surface is a bicubic NURBS fit of a conic and whose back surface
    is an explicit rational NURBS net (nurbs_geometry.py): covers the (u, v) solves of
    distance and surface_normal inside a trace."""
    np.random.seed(11)  # the reference's restarts draw from numpy.random
    P, W, U, V = nurbs_back_net()
    lens = ref_optic.Optic()
    lens.add_surface(index=0, thickness=np.inf)
    lens.add_surface(index=1, surface_type="nurbs", radius=40.0, conic=-0.5,
                     nurbs_norm_x=8.0, nurbs_norm_y=8.0, n_points_u=8, n_points_v=8,
                     thickness=4.0, material="SK16", is_stop=True)
    lens.add_surface(index=2, surface_type="nurbs", radius=-70.0, control_points=P.tolist(),
                     weights=W.tolist(), u_degree=3, v_degree=2, u_knots=U, v_knots=V,
                     thickness=45.0)
    lens.add_surface(index=3)
    lens.surface_group.surfaces[1].geometry.fit_surface()
    for si in (1, 2):  # the reference's NurbsGeometry keeps P / W / knots as given
        g = lens.surface_group.surfaces[si].geometry
        g.P, g.W = np.asarray(g.P, dtype=np.float64), np.asarray(g.W, dtype=np.float64)
        g.U, g.V = np.asarray(g.U, dtype=np.float64), np.asarray(g.V, dtype=np.float64)
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=5)
    lens.add_field(x=3, y=2)
    lens.add_wavelength(value=0.55, is_primary=True)
    return lens


def cooke_apod(kind, **kwargs):
    """CookeTriplet with a pupil apodization (optic.set_apodization, optic.py:401-419;
    applied in ray_generator.py:91-95)."""
    def build():
        lens = CookeTriplet()
        lens.set_apodization(kind, **kwargs)
        return lens
    return build


def uv_projection():
    """samples/lithography.py: 43-surface object-space telecentric projection lens."""
    from optiland.samples.lithography import UVProjectionLens

    return UVProjectionLens()


def cooke_abbe():
    """The Cooke triplet prescription with AbbeMaterial model glasses (materials/abbe.py)
    in place of its catalog glasses (SK16 ~ 1.62041 / 60.32, F2 ~ 1.62004 / 36.37)."""
    from optiland.materials.abbe import AbbeMaterial

    lens = ref_optic.Optic()
    sk16 = AbbeMaterial(1.62041, 60.32)
    f2 = AbbeMaterial(1.62004, 36.37)
    lens.add_surface(index=0, radius=be.inf, thickness=be.inf)
    lens.add_surface(index=1, radius=22.01359, thickness=3.25896, material=sk16)
    lens.add_surface(index=2, radius=-435.76044, thickness=6.00755)
    lens.add_surface(index=3, radius=-22.21328, thickness=0.99997, material=f2)
    lens.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True)
    lens.add_surface(index=5, radius=79.68360, thickness=2.95208, material=sk16)
    lens.add_surface(index=6, radius=-18.39533, thickness=42.20778)
    lens.add_surface(index=7)
    lens.set_aperture(aperture_type="EPD", value=10)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=14)
    lens.add_field(y=20)
    lens.add_wavelength(value=0.48)
    lens.add_wavelength(value=0.55, is_primary=True)
    lens.add_wavelength(value=0.65)
    return lens


def json_lens(name):
    """A lens file from the reference's docs/samples (copied as data to tests/golden/lenses),
    loaded with the reference's own Optic.from_dict (optic.py:674-713)."""
    def build():
        with open(os.path.join(HERE, "lenses", name + ".json")) as f:
            return ref_optic.Optic.from_dict(json.load(f))
    return build


CASES = {
    # name: (builder, fields [(Hx,Hy)], wavelengths, distribution, num)
    "cooke": (CookeTriplet, [(0, 0), (0, 0.7), (0, 1)], [0.48, 0.55, 0.65], "uniform", 32),
    "dg": (DoubleGauss, [(0, 0), (0, 1)], [0.4861, 0.5876, 0.6563], "uniform", 32),
    "rt": (ReverseTelephoto, [(0, h) for h in np.linspace(0, 1, 7)],
           list(np.linspace(0.4861, 0.6563, 7)), "uniform", 12),
    "rt_asph": (rt_asph, [(0, h) for h in np.linspace(0, 1, 5)],
                [0.4861, 0.5876, 0.6563], "uniform", 24),
    "rt_odd": (rt_odd, [(0, 0), (0, 0.5), (0, 1)], [0.5876], "uniform", 24),
    "tma_fringe": (lambda: tma("fringe"), [(0, 0), (0, 1), (0, -1)], [0.587], "uniform", 24),
    "tma_standard": (lambda: tma("standard"), [(0, 0), (0, 1)], [0.587], "uniform", 24),
    "tma_noll": (lambda: tma("noll"), [(0, 1)], [0.587], "uniform", 24),
    "cooke_aperture": (cooke_aperture, [(0, 0), (0, 1)], [0.55], "uniform", 32),
    "cooke_shapes": (cooke_shapes, [(0, 0), (0, 1), (0.4, -0.6)], [0.55], "uniform", 32),
    "decentered": (decentered, [(0, 0), (0, 1), (0.5, -0.5)], [0.55], "hexapolar", 8),
    "freeform": (freeform, [(0, 0), (0, 1), (0.5, 0.7)], [0.48, 0.55, 0.65], "uniform", 24),
    "json_cooke": (json_lens("cooke_triplet"), [(0, 0), (0, 1)], [0.55], "uniform", 24),
    "json_heliar": (json_lens("heliar"), [(0, 0), (0, 0.7), (0, 1)], [0.4861, 0.5876],
                    "uniform", 24),
    "json_rt": (json_lens("reverse_telephoto"), [(0, 0), (0, 1)], [0.5876], "uniform", 24),
    "cooke_pih": (cooke_pih, [(0, 0), (0, 0.6), (0.3, 1)], [0.55], "uniform", 24),
    "forbes": (forbes, [(0, 0), (0, 1), (0.7, 0.7)], [1.55], "uniform", 24),
    "forbes_q2d": (forbes_q2d, [(0, 0), (0, 1), (0.7, 0.7)], [1.55], "uniform", 24),
    "finite_pih": (finite_pih, [(0, 0), (0, 1), (-0.4, 0.7)], [0.48, 0.55], "uniform", 24),
    "paraxial_lens": (paraxial_lens, [(0, 0), (0, 1), (0.4, 0.6)], [0.48, 0.55], "uniform", 24),
    "paraxial_mirror": (paraxial_mirror, [(0, 0), (0, 1)], [0.6], "uniform", 24),
    "phase_plate": (phase_plate, [(0, 0), (0, 1), (0.3, -0.6)], [0.48, 0.55, 0.65],
                    "uniform", 24),
    "grating_flat": (lambda: grating("flat"), [(0, 0), (0, 1), (1, 0), (0.2, 0.8)], [0.587],
                     "uniform", 24),
    "grating_curved": (lambda: grating("curved"), [(0, 0), (0, 1), (1, 0), (0.2, 0.8)],
                       [0.55, 0.587], "uniform", 24),
    "grating_reflective": (lambda: grating("reflective"), [(0, 0), (0, 1), (0.2, 0.8)],
                           [0.587], "uniform", 24),
    "grating_tilted": (lambda: grating("curved", angle=0.35), [(0, 0), (0.2, 0.8)], [0.587],
                       "uniform", 24),
    "grid_lens": (grid_lens, [(0, 0), (0, 1), (0.6, 0.6)], [0.48, 0.55], "uniform", 24),
    "nurbs_lens": (nurbs_lens, [(0, 0), (0, 1), (0.6, 0.6)], [0.48, 0.55], "uniform", 24),
    "cooke_abbe": (cooke_abbe, [(0, 0), (0, 1)], [0.48, 0.55, 0.65], "uniform", 24),
    "uv_projection": (uv_projection, [(0, 0), (0, 0.7), (0, 1)], [0.248], "uniform", 24),
    "apod_gaussian": (cooke_apod("GaussianApodization", sigma=0.6), [(0, 0), (0, 1)], [0.55],
                      "uniform", 24),
    "apod_cos2": (cooke_apod("CosineSquaredApodization", R=0.9), [(0, 0), (0, 1)], [0.55],
                  "uniform", 24),
    "apod_hann": (cooke_apod("HannApodization", D=1.8), [(0, 0), (0, 1)], [0.55], "uniform", 24),
    "apod_poly": (cooke_apod("PolynomialApodization", R=0.95, p=1.5), [(0, 0), (0, 1)], [0.55],
                  "uniform", 24),
    "apod_supergauss": (cooke_apod("SuperGaussianApodization", w=0.7, n=3.5), [(0, 0), (0, 1)],
                        [0.55], "uniform", 24),
    "apod_tukey": (cooke_apod("TukeyApodization", R=0.9, alpha=0.6), [(0, 0), (0, 1)], [0.55],
                   "uniform", 24),
    "apod_uniform": (cooke_apod("UniformApodization"), [(0, 0), (0, 1)], [0.55], "uniform", 24),
}


# --------------------------------------------------------------------------------------
# instrumentation: count Newton updates per surface (newton_raphson.py:137-166)
# --------------------------------------------------------------------------------------
_newton_counts: dict[int, int] = {}


def _instrument_grid(si, g):
    """GridSagGeometry.distance (grid_sag.py:108-140) calls _interpolate once per update:
    the number of those calls inside one distance() is its update count."""
    orig_distance = g.distance
    orig_interp = g._interpolate

    def distance(rays, _g=g, _si=si, _od=orig_distance, _oi=orig_interp):
        count = [0]

        def counting_interp(x, y):
            count[0] += 1
            return _oi(x, y)

        _g._interpolate = counting_interp
        try:
            t = _od(rays)
        finally:
            _g._interpolate = _oi
        _newton_counts[_si] = count[0]
        return t

    g.distance = distance


def _instrument_newton(lens):
    for si, s in enumerate(lens.surface_group.surfaces):
        g = s.geometry
        if isinstance(g, GridSagGeometry):
            _instrument_grid(si, g)
            continue
        if not isinstance(g, NewtonRaphsonGeometry):
            continue
        orig_distance = g.distance
        orig_normal = g._surface_normal

        def distance(rays, _g=g, _si=si, _od=orig_distance, _on=orig_normal):
            count = [0]

            def counting_normal(x, y):
                count[0] += 1
                return _on(x, y)

            _g._surface_normal = counting_normal
            try:
                t = _od(rays)
            finally:
                _g._surface_normal = _on
            _newton_counts[_si] = count[0]
            return t

        g.distance = distance


def material_table(lens, wavelengths):
    """n and k of material_post for every surface, at each wavelength (host scalars)."""
    S = len(lens.surface_group.surfaces)
    n = np.zeros((len(wavelengths), S))
    k = np.zeros((len(wavelengths), S))
    for j, w in enumerate(wavelengths):
        for si, s in enumerate(lens.surface_group.surfaces):
            m = s.material_post
            if m is None:
                n[j, si] = np.nan
                continue
            n[j, si] = float(np.ravel(m.n(np.array([w])))[0])
            k[j, si] = float(np.ravel(m.k(np.array([w])))[0])
    return n, k


def _paraxial_or_nan(fn):
    """A paraxial scalar for the metadata, or NaN where the reference's paraxial tracer
    cannot run (a grid sag surface has no radius: surface_group.py:153)."""
    try:
        return float(fn())
    except AttributeError:
        return float("nan")


def generate_case(name, builder, fields, wavelengths, dist, num):
    lens = builder()
    _instrument_newton(lens)
    sg = lens.surface_group
    S = len(sg.surfaces)
    if isinstance(dist, str):
        d = create_distribution(dist)
        d.generate_points(num)
    else:
        d = dist
    Px = np.asarray(d.x, dtype=np.float64)
    Py = np.asarray(d.y, dtype=np.float64)
    out = {k: [] for k in ("x0", "y0", "z0", "L0", "M0", "N0", "x", "y", "z", "L", "M", "N", "i", "opd")}
    newton = []
    records = []
    pair_field = []
    pair_wl = []
    for fi, (hx, hy) in enumerate(fields):
        for wi, w in enumerate(wavelengths):
            rays0 = RayGenerator(lens).generate_rays(
                np.full(Px.shape, float(hx)), np.full(Px.shape, float(hy)), Px, Py, float(w)
            )
            for a, b in (("x0", "x"), ("y0", "y"), ("z0", "z"), ("L0", "L"), ("M0", "M"), ("N0", "N")):
                out[a].append(np.array(getattr(rays0, b), dtype=np.float64))
            _newton_counts.clear()
            rays = lens.trace(float(hx), float(hy), float(w), num_rays=num, distribution=d)
            for a in ("x", "y", "z", "L", "M", "N", "i", "opd"):
                out[a].append(np.array(getattr(rays, a), dtype=np.float64))
            newton.append([_newton_counts.get(si, -1) for si in range(S)])
            if name == "dg":
                rec = np.stack([
                    np.stack([np.asarray(getattr(s, a), dtype=np.float64) for a in
                              ("x", "y", "z", "L", "M", "N", "intensity", "opd")])
                    for s in sg.surfaces
                ])
                records.append(rec)
            pair_field.append(fi)
            pair_wl.append(wi)
    arrays = {k: np.concatenate(v) for k, v in out.items()}
    arrays["Px"] = Px
    arrays["Py"] = Py
    arrays["newton_updates"] = np.array(newton, dtype=np.int32)
    arrays["pair_field"] = np.array(pair_field, dtype=np.int32)
    arrays["pair_wl"] = np.array(pair_wl, dtype=np.int32)
    if records:
        arrays["records"] = np.stack(records)  # [pair][surface][8][N_p]
    n_tab, k_tab = material_table(lens, wavelengths)
    arrays["n_post"] = n_tab
    arrays["k_post"] = k_tab
    arrays["positions"] = np.ravel(np.asarray(sg.positions, dtype=np.float64))
    meta = dict(
        fields=[[float(a), float(b)] for a, b in fields],
        wavelengths=[float(w) for w in wavelengths],
        distribution=dist if isinstance(dist, str) else type(dist).__name__,
        num_rays=int(num),
        n_pupil=int(Px.size),
        num_surfaces=S,
        EPL=float(lens.paraxial.EPL()),
        EPD=float(lens.paraxial.EPD()),
        f2=_paraxial_or_nan(lens.paraxial.f2),
        XPL=_paraxial_or_nan(lens.paraxial.XPL),
        primary_wavelength=float(lens.primary_wavelength),
        norm_radius=[float(getattr(s.geometry, "norm_radius", np.nan)) for s in sg.surfaces],
        semi_aperture=[None if s.semi_aperture is None else float(np.ravel(s.semi_aperture)[0])
                       for s in sg.surfaces],
    )
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
    return meta


def glass_table():
    """Bake the dispersion data of every catalog glass the sample lenses use."""
    specs = [("SK16", None), ("F2", "schott"), ("N-SSK2", None), ("N-SK2", None),
             ("F5", "schott"), ("N-SK16", None), ("N-SK10", None), ("SK15", None),
             ("BASF2", None), ("FK3", None), ("SF15", "hikari"), ("N-LAK12", None),
             ("E-LLF6", None), ("H-K3", "cdgm"), ("H-ZLAF68C", "cdgm"), ("N-BK7", None)]
    out = {}
    for name, ref in specs:
        m = Material(name, ref) if ref else Material(name)
        key = name if ref is None else f"{name}|{ref}"
        rel = m.filename.split("database" + os.sep)[-1]
        entry = dict(
            name=name,
            reference=ref,
            source=rel,
            formula=m._n_formula,
            coefficients=[float(np.ravel(c)[0]) for c in m.coefficients]
            if m.coefficients is not None else None,
            k_wavelength=None if m._k_wavelength is None else [float(v) for v in np.ravel(m._k_wavelength)],
            k=None if m._k is None else [float(v) for v in np.ravel(m._k)],
            n_wavelength=None if m._n_wavelength is None else [float(v) for v in np.ravel(m._n_wavelength)],
            n=None if m._n is None else [float(v) for v in np.ravel(m._n)],
        )
        # golden n/k values at a few wavelengths, to pin the restated formulas
        wl = np.array([0.4, 0.4861, 0.55, 0.5876, 0.6563, 0.7])
        entry["check_wavelength"] = wl.tolist()
        entry["check_n"] = [float(np.ravel(m.n(np.array([w])))[0]) for w in wl]
        entry["check_k"] = [float(np.ravel(m.k(np.array([w])))[0]) for w in wl]
        out[key] = entry
    with open(os.path.join(REPO, "optiland_pr_amd", "data", "glasses.json"), "w") as f:
        json.dump(out, f, indent=1)


ABBE_GLASSES = [(1.5168, 64.17), (1.62, 36.37), (1.7552, 27.58), (1.4875, 70.4), (1.8, 46.5)]


def abbe_table():
    """Bake the AbbeMaterial model-glass fit (materials/abbe.py:67-98: the coefficient
    matrix of database/glass_model_coefficients.npy, read without pickle) into
    optiland_pr_amd/data/abbe_coefficients.json, with n(w) of a few (nd, vd) pairs on a
    wavelength sweep as golden values."""
    from optiland.materials.abbe import AbbeMaterial

    import optiland

    path = os.path.join(os.path.dirname(optiland.__file__), "database",
                        "glass_model_coefficients.npy")
    coef = np.load(path, allow_pickle=False)
    sweep = np.linspace(0.38, 0.75, 38)
    checks = []
    for nd, vd in ABBE_GLASSES:
        m = AbbeMaterial(nd, vd)
        checks.append(dict(index=nd, abbe=vd, p=[float(v) for v in np.ravel(m._p)],
                           n=[float(v) for v in np.ravel(m.n(sweep))],
                           k=float(np.ravel(m.k(sweep))[0])))
    out = dict(source="optiland/database/glass_model_coefficients.npy",
               coefficients=coef.tolist(), check_wavelength=sweep.tolist(), checks=checks)
    with open(os.path.join(REPO, "optiland_pr_amd", "data", "abbe_coefficients.json"), "w") as f:
        json.dump(out, f, indent=1)


def analysis_goldens():
    """SpotDiagram radii (tests/test_analysis.py:69-100 goldens) and OPD rms
    (tests/test_wavefront.py:135-139) recomputed from the reference."""
    lens = CookeTriplet()
    spot = SpotDiagram(lens)
    res = dict(
        cooke_geo_radius=[[float(v) for v in row] for row in spot.geometric_spot_radius()],
        cooke_rms_radius=[[float(v) for v in row] for row in spot.rms_spot_radius()],
        cooke_centroid=[[float(a), float(b)] for a, b in spot.centroid()],
    )
    opd = OPD(CookeTriplet(), (0, 1), 0.55)
    res["cooke_opd_rms_0_1_055"] = float(opd.rms())
    dg = DoubleGauss()
    res["dg_opd_rms_0_1_05876"] = float(OPD(dg, (0, 1), 0.5876).rms())
    res["dg_opd_rms_0_0_05876"] = float(OPD(DoubleGauss(), (0, 0), 0.5876).rms())
    # piston / tilt removal (wavefront.py:97-143, 164-165)
    res["cooke_opd_rms_0_1_055_notilt"] = float(
        OPD(CookeTriplet(), (0, 1), 0.55, remove_tilt=True).rms())
    res["dg_opd_rms_0_1_05876_notilt"] = float(
        OPD(DoubleGauss(), (0, 1), 0.5876, remove_tilt=True).rms())
    # per-ray wavefront data (pupil points, OPD in waves, intensity) of a few cases
    arrays = {}
    for key, (builder, field, wl, kw) in WAVEFRONT_CASES.items():
        w = OPD(builder(), field, wl, **kw)
        d = w.get_data(w.fields[0], w.wavelengths[0])
        for a in ("pupil_x", "pupil_y", "pupil_z", "opd", "intensity"):
            arrays[f"{key}/{a}"] = np.asarray(getattr(d, a), dtype=np.float64)
        arrays[f"{key}/radius"] = np.array(float(d.radius))
    np.savez_compressed(os.path.join(HERE, "wavefront.npz"), **arrays)
    return res


WAVEFRONT_CASES = {  # name -> (lens builder, field, wavelength, OPD keywords)
    "cooke_0_1": (CookeTriplet, (0, 1), 0.55, {}),
    "cooke_0_07_notilt": (CookeTriplet, (0, 0.7), 0.48, {"remove_tilt": True}),
    "dg_0_1": (DoubleGauss, (0, 1), 0.5876, {"num_rays": 20}),
    "finite_pih_03_07": (None, (0.3, 0.7), 0.55, {}),  # paraxial image height: no tilt
}


WAVEFRONT_STRATEGY_CASES = {  # name -> (lens builder, field, wavelength, OPD keywords)
    "cooke_0_1_centroid": (CookeTriplet, (0, 1), 0.55, {"strategy": "centroid_sphere"}),
    "cooke_0_07_bestfit": (CookeTriplet, (0, 0.7), 0.48, {"strategy": "best_fit_sphere"}),
    "cooke_0_1_centroid_notrim": (CookeTriplet, (0, 1), 0.55,
                                  {"strategy": "centroid_sphere", "robust_trim_std": 0.0}),
    "dg_0_1_centroid": (DoubleGauss, (0, 1), 0.5876,
                        {"strategy": "centroid_sphere", "num_rays": 20}),
    "dg_0_0_bestfit": (DoubleGauss, (0, 0), 0.5876, {"strategy": "best_fit_sphere"}),
    "dg_0_1_bestfit_notilt": (DoubleGauss, (0, 1), 0.5876,
                              {"strategy": "best_fit_sphere", "remove_tilt": True}),
    "finite_pih_03_07_centroid": (None, (0.3, 0.7), 0.55, {"strategy": "centroid_sphere"}),
}


def wavefront_strategy_goldens():
    """Per-ray WavefrontData of the centroid-anchored and best-fit reference spheres
    (wavefront/strategy.py:242-479) -> wavefront_strategies.npz: pupil points, OPD in
    waves, intensity, radius and (best fit) the fitted centre, plus OPD.rms()."""
    arrays = {}
    for key, (builder, field, wl, kw) in WAVEFRONT_STRATEGY_CASES.items():
        builder = builder or finite_pih
        w = OPD(builder(), field, wl, **kw)
        d = w.get_data(w.fields[0], w.wavelengths[0])
        for a in ("pupil_x", "pupil_y", "pupil_z", "opd", "intensity"):
            arrays[f"{key}/{a}"] = np.asarray(getattr(d, a), dtype=np.float64)
        arrays[f"{key}/radius"] = np.array(float(d.radius))
        arrays[f"{key}/rms"] = np.array(float(w.rms()))
        center = getattr(w.strategy, "center", None)
        if center is not None:
            arrays[f"{key}/center"] = np.array([float(c) for c in center])
    np.savez_compressed(os.path.join(HERE, "wavefront_strategies.npz"), **arrays)


def full_size_summaries():
    """Size-independent checks at the BASELINE sizes: DoubleGauss 1M random rays (seed 0)
    and the Cooke config-1 workload (uniform 128, 3 fields)."""
    res = {}
    lens = DoubleGauss()
    d = RandomDistribution(seed=0)
    d.generate_points(1_000_000)
    t0 = time.perf_counter()
    rays = lens.trace(0.0, 1.0, 0.5876, num_rays=1_000_000, distribution=d)
    res["dg_1m_ref_seconds"] = time.perf_counter() - t0
    x, y, opd = (np.asarray(getattr(rays, a)) for a in ("x", "y", "opd"))
    res["dg_1m"] = dict(
        n=int(x.size), nan=int(np.isnan(x).sum()),
        sum_x=float(np.sum(x)), sum_y=float(np.sum(y)), sum_opd=float(np.sum(opd)),
        sum_x2=float(np.sum(x * x)), sum_y2=float(np.sum(y * y)),
        mean_y=float(np.mean(y)), std_y=float(np.std(y)),
        first=[float(x[0]), float(y[0]), float(opd[0])],
        last=[float(x[-1]), float(y[-1]), float(opd[-1])],
    )
    lens = CookeTriplet()
    stats = []
    for hy in (0.0, 0.7, 1.0):
        r = lens.trace(0.0, hy, 0.55, num_rays=128, distribution="uniform")
        x, y = np.asarray(r.x), np.asarray(r.y)
        stats.append(dict(n=int(x.size), sum_x=float(np.sum(x)), sum_y=float(np.sum(y)),
                          mean_y=float(np.mean(y)), std_y=float(np.std(y))))
    res["cooke_uniform128"] = stats
    return res


def full_size_newton():
    """Size-independent checks of the Newton lenses at the BASELINE ray count: RT-asph
    (config 3's lens, Hy = 1, 0.5876 um) and the fringe-Zernike TMA (config 5's, Hy = 1,
    0.587 um), 1M random pupil rays (seed 0) each: NumPy sums of the image x, y, opd, the
    NaN count, the first / last ray and the Newton update count of every surface."""
    res = {}
    for key, builder, hy, wl in (("rt_asph_1m", rt_asph, 1.0, 0.5876),
                                 ("tma_1m", tma, 1.0, 0.587)):
        lens = builder()
        _instrument_newton(lens)
        _newton_counts.clear()
        d = RandomDistribution(seed=0)
        d.generate_points(1_000_000)
        t0 = time.perf_counter()
        rays = lens.trace(0.0, hy, wl, num_rays=1_000_000, distribution=d)
        secs = time.perf_counter() - t0
        x, y, opd = (np.asarray(getattr(rays, a)) for a in ("x", "y", "opd"))
        res[key] = dict(
            n=int(x.size), nan=int(np.isnan(x).sum()), seconds=secs,
            sum_x=float(np.sum(x)), sum_y=float(np.sum(y)), sum_opd=float(np.sum(opd)),
            sum_x2=float(np.sum(x * x)),
            first=[float(x[0]), float(y[0]), float(opd[0])],
            last=[float(x[-1]), float(y[-1]), float(opd[-1])],
            newton_updates={str(k): int(v) for k, v in sorted(_newton_counts.items())},
        )
    return res


MIXED_W_CASES = {  # name -> (builder, field (Hx, Hy), pupil n, wavelength range)
    "cooke": (CookeTriplet, (0.0, 0.7), 24, (0.42, 0.75)),
    "dg": (DoubleGauss, (0.0, 1.0), 24, (0.45, 0.70)),
    "freeform": (None, (0.3, 0.6), 20, (0.45, 0.70)),
    "paraxial_lens": (paraxial_lens, (0.3, 0.6), 20, (0.45, 0.70)),
    "phase_plate": (phase_plate, (0.3, -0.6), 20, (0.45, 0.70)),
    "grating_curved": (lambda: grating("curved"), (0.2, 0.8), 20, (0.45, 0.70)),
    "grating_reflective": (lambda: grating("reflective"), (0.2, 0.8), 20, (0.45, 0.70)),
    "cooke_abbe": (cooke_abbe, (0.0, 0.7), 24, (0.42, 0.74)),
    "nurbs_lens": (nurbs_lens, (0.3, 0.6), 20, (0.45, 0.70)),
}


def mixed_wavelength_goldens():
    """SurfaceGroup.trace (surface_group.py:232-244) of RealRays whose every ray has its
    own wavelength: the materials evaluate n(rays.w) and k(rays.w) per ray. Rays are
    generated at the primary wavelength, then given seeded random wavelengths. Also
    n(w), k(w) of every baked catalog glass on a wavelength sweep."""
    from optiland.rays import RealRays

    out = {}
    rng = np.random.default_rng(123)
    for name, (builder, (hx, hy), num, (w0, w1)) in MIXED_W_CASES.items():
        lens = freeform() if builder is None else builder()
        wl = float(lens.primary_wavelength)
        d = create_distribution("uniform")
        d.generate_points(num)
        rays = RayGenerator(lens).generate_rays(hx, hy, d.x, d.y, wl)
        n = np.asarray(rays.x).size
        w = rng.uniform(w0, w1, n)
        r = RealRays(np.asarray(rays.x), np.asarray(rays.y), np.asarray(rays.z),
                     np.asarray(rays.L), np.asarray(rays.M), np.asarray(rays.N),
                     np.asarray(rays.i), w)
        for a in ("x", "y", "z", "L", "M", "N", "i"):
            out[f"{name}/in_{a}"] = np.array(getattr(r, a), dtype=np.float64)
        out[f"{name}/w"] = w
        lens.surface_group.trace(r)
        for a in ("x", "y", "z", "L", "M", "N", "i", "opd"):
            out[f"{name}/{a}"] = np.array(getattr(r, a), dtype=np.float64)
    sweep = np.linspace(0.36, 1.6, 157)
    with open(os.path.join(REPO, "optiland_pr_amd", "data", "glasses.json")) as f:
        glasses = json.load(f)
    for key, e in glasses.items():
        m = Material(e["name"], e["reference"]) if e["reference"] else Material(e["name"])
        out[f"glass/{key}/n"] = np.asarray(m.n(sweep), dtype=np.float64) * np.ones_like(sweep)
        out[f"glass/{key}/k"] = np.asarray(m.k(sweep), dtype=np.float64) * np.ones_like(sweep)
    out["glass/w"] = sweep
    np.savez_compressed(os.path.join(HERE, "mixed_w.npz"), **out)


DIST_CASES = [("random", 1000, {"seed": 7}), ("uniform", 33, {}), ("uniform", 128, {}),
              ("hexapolar", 6, {}), ("hexapolar", 17, {}), ("ring", 13, {}),
              ("line_x", 21, {}), ("line_y", 20, {}), ("positive_line_x", 9, {}),
              ("positive_line_y", 10, {}), ("cross", 21, {}), ("cross", 20, {})]


def aperture_goldens():
    """contains(x, y) of every reference aperture kind on 6000 points (random, a grid
    through the vertices, the vertices themselves) -> tests/golden/apertures.npz, with
    the apertures' to_dict() in apertures.json."""
    from optiland.physical_apertures import (
        EllipticalAperture,
        OffsetRadialAperture,
        PolygonAperture,
        RadialAperture,
        RectangularAperture,
    )

    aps = {
        "radial": RadialAperture(3.0, 0.5),
        "offset_radial": OffsetRadialAperture(2.5, 0.4, 0.7, -0.3),
        "ellipse": EllipticalAperture(3.5, 2.0, -0.4, 0.6),
        "rect": RectangularAperture(-2.0, 3.0, -1.5, 2.5),
        "polygon": PolygonAperture(*STAR),
        "union": RectangularAperture(-2.0, 3.0, -1.5, 2.5) | EllipticalAperture(3.5, 2.0),
        "intersection": RadialAperture(3.0) & PolygonAperture(*STAR),
        "difference": RectangularAperture(-2.0, 3.0, -1.5, 2.5) - OffsetRadialAperture(1.0, 0, 0.5, 0.5),
        "nested": ((RectangularAperture(-4, 4, -1, 1) + EllipticalAperture(1.5, 4.0))
                   - RadialAperture(0.8)) & PolygonAperture(*STAR),
    }
    rng = np.random.default_rng(17)
    pts = [rng.uniform(-5, 5, size=(5000, 2))]
    g = np.linspace(-5, 5, 21)
    gx, gy = np.meshgrid(g, g)
    pts.append(np.column_stack((gx.ravel(), gy.ravel())))
    pts.append(np.column_stack(STAR))
    pts = np.concatenate(pts)
    out = {"x": pts[:, 0].copy(), "y": pts[:, 1].copy()}
    dicts = {}
    for name, ap in aps.items():
        out[name] = np.asarray(ap.contains(out["x"], out["y"]), dtype=bool)
        dicts[name] = json.loads(json.dumps(ap.to_dict(), default=lambda o: np.asarray(o).tolist()))
    np.savez_compressed(os.path.join(HERE, "apertures.npz"), **out)
    with open(os.path.join(HERE, "apertures.json"), "w") as f:
        json.dump(dicts, f, indent=1)


def distribution_goldens():
    """Pupil samples of every reference distribution (distribution.py:72-408), incl.
    GaussianQuadrature (not in create_distribution) -> tests/golden/distributions.npz."""
    from optiland.distribution import GaussianQuadrature

    out = {}
    for kind, n, kw in DIST_CASES:
        d = RandomDistribution(**kw) if kind == "random" else create_distribution(kind)
        d.generate_points(n)
        out[f"{kind}_{n}_x"] = np.asarray(d.x, dtype=np.float64)
        out[f"{kind}_{n}_y"] = np.asarray(d.y, dtype=np.float64)
    for sym in (False, True):
        for rings in range(1, 7):
            g = GaussianQuadrature(is_symmetric=sym)
            g.generate_points(rings)
            key = f"gq_{int(sym)}_{rings}"
            out[key + "_x"] = np.asarray(g.x, dtype=np.float64)
            out[key + "_y"] = np.asarray(g.y, dtype=np.float64)
            out[key + "_w"] = np.asarray(g.get_weights(rings), dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "distributions.npz"), **out)


def main():
    # --only NAME [NAME ...]: regenerate just those cases, keep the rest of index.json
    if "--distributions" in sys.argv:
        distribution_goldens()
        return
    if "--mixed-w" in sys.argv:
        mixed_wavelength_goldens()
        return
    if "--apertures" in sys.argv:
        aperture_goldens()
        return
    if "--glasses" in sys.argv:  # re-bake optiland_pr_amd/data/glasses.json only
        glass_table()
        return
    if "--abbe" in sys.argv:  # re-bake optiland_pr_amd/data/abbe_coefficients.json only
        abbe_table()
        return
    if "--full-newton" in sys.argv:  # index.json "_full" Newton entries only
        with open(os.path.join(HERE, "index.json")) as f:
            index = json.load(f)
        index["_full"].update(full_size_newton())
        with open(os.path.join(HERE, "index.json"), "w") as f:
            json.dump(index, f, indent=1)
        return
    if "--wavefront-strategies" in sys.argv:  # wavefront_strategies.npz only
        wavefront_strategy_goldens()
        return
    if "--analysis" in sys.argv:  # index.json "_analysis" + wavefront.npz only
        WAVEFRONT_CASES["finite_pih_03_07"] = (finite_pih,) + WAVEFRONT_CASES["finite_pih_03_07"][1:]
        with open(os.path.join(HERE, "index.json")) as f:
            index = json.load(f)
        index["_analysis"] = analysis_goldens()
        with open(os.path.join(HERE, "index.json"), "w") as f:
            json.dump(index, f, indent=1)
        return
    only = sys.argv[sys.argv.index("--only") + 1:] if "--only" in sys.argv else None
    if only:
        with open(os.path.join(HERE, "index.json")) as f:
            index = json.load(f)
        for name in only:
            builder, fields, wls, dist, num = CASES[name]
            index[name] = generate_case(name, builder, fields, wls, dist, num)
        with open(os.path.join(HERE, "index.json"), "w") as f:
            json.dump(index, f, indent=1)
        return
    glass_table()
    abbe_table()
    index = {}
    for name, (builder, fields, wls, dist, num) in CASES.items():
        t0 = time.perf_counter()
        index[name] = generate_case(name, builder, fields, wls, dist, num)
        print(f"{name}: {index[name]['n_pupil']} pupil pts, {time.perf_counter() - t0:.2f}s",
              file=sys.stderr)
    distribution_goldens()
    aperture_goldens()
    mixed_wavelength_goldens()
    WAVEFRONT_CASES["finite_pih_03_07"] = (finite_pih,) + WAVEFRONT_CASES["finite_pih_03_07"][1:]
    index["_analysis"] = analysis_goldens()
    wavefront_strategy_goldens()
    index["_full"] = full_size_summaries()
    index["_full"].update(full_size_newton())
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
