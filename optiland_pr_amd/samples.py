"""Sample lenses (prescriptions restated from optiland/samples/objectives.py:46-173 and
docs/examples/Tutorial_7d_Three_Mirror_Anastigmat.ipynb), plus the synthetic variants
the benchmark configs and parity fixtures use (BASELINE.json configs).

Each builder mirrors tests/golden/gen_golden.py's reference-API builder of the same name.
"""

from __future__ import annotations

import numpy as np

from .optic import Optic
from .surfaces import RadialAperture


class CookeTriplet(Optic):
    """samples/objectives.py:46-72."""

    def __init__(self):
        super().__init__()
        self.add_surface(index=0, radius=np.inf, thickness=np.inf)
        self.add_surface(index=1, radius=22.01359, thickness=3.25896, material="SK16")
        self.add_surface(index=2, radius=-435.76044, thickness=6.00755)
        self.add_surface(index=3, radius=-22.21328, thickness=0.99997, material=("F2", "schott"))
        self.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True)
        self.add_surface(index=5, radius=79.68360, thickness=2.95208, material="SK16")
        self.add_surface(index=6, radius=-18.39533, thickness=42.20778)
        self.add_surface(index=7)
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=14)
        self.add_field(y=20)
        self.add_wavelength(value=0.48)
        self.add_wavelength(value=0.55, is_primary=True)
        self.add_wavelength(value=0.65)


class DoubleGauss(Optic):
    """samples/objectives.py:75-114 (8 spheres + 3 planes + image; S = 12)."""

    def __init__(self):
        super().__init__()
        self.add_surface(index=0, radius=np.inf, thickness=np.inf)
        self.add_surface(index=1, radius=56.20238, thickness=8.75, material="N-SSK2")
        self.add_surface(index=2, radius=152.28580, thickness=0.5)
        self.add_surface(index=3, radius=37.68262, thickness=12.5, material="N-SK2")
        self.add_surface(index=4, radius=np.inf, thickness=3.8, material=("F5", "schott"))
        self.add_surface(index=5, radius=24.23130, thickness=16.369445)
        self.add_surface(index=6, radius=np.inf, thickness=13.747957, is_stop=True)
        self.add_surface(index=7, radius=-28.37731, thickness=3.8, material=("F5", "schott"))
        self.add_surface(index=8, radius=np.inf, thickness=11, material="N-SK16")
        self.add_surface(index=9, radius=-37.92546, thickness=0.5)
        self.add_surface(index=10, radius=177.41176, thickness=7, material="N-SK16")
        self.add_surface(index=11, radius=-79.41143, thickness=61.487536)
        self.add_surface(index=12)
        self.set_aperture(aperture_type="imageFNO", value=5)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=10)
        self.add_field(y=14)
        self.add_wavelength(value=0.4861)
        self.add_wavelength(value=0.5876, is_primary=True)
        self.add_wavelength(value=0.6563)


_RT_ROWS = [
    # radius, thickness, material, is_stop  (samples/objectives.py:117-173)
    (np.inf, np.inf, None, False),
    (1.69111096, 0.08259680, "N-SK10", False),
    (0.94414496, 0.8, None, False),
    (4.32100401, 0.080256, "SK15", False),
    (1.78117621, 0.5, None, False),
    (2.64050282, 0.27638160, "BASF2", False),
    (-3.86177348, 0.1, None, False),
    (1.05627661, 0.2, "FK3", False),
    (-4.06933311, 0.2001384, None, False),
    (np.inf, 0.06688, None, True),
    (-2.61246583, 0.064372, ("SF15", "hikari"), False),
    (0.99117409, 0.3, None, False),
    (9.03045960, 0.18743120, "N-LAK12", False),
    (-1.35680743, 2.35130547, None, False),
]


def _reverse_telephoto(lens: Optic, aspheres=None, kind="even_asphere"):
    aspheres = aspheres or {}
    for k, (R, t, mat, stop) in enumerate(_RT_ROWS):
        kw = dict(index=k, radius=R, thickness=t, is_stop=stop)
        if mat is not None:
            kw["material"] = mat
        if k in aspheres:
            kw.update(surface_type=kind, conic=0.0, coefficients=aspheres[k])
        lens.add_surface(**kw)
    lens.add_surface(index=len(_RT_ROWS))
    lens.set_aperture(aperture_type="EPD", value=0.3)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=21)
    lens.add_field(y=30)
    lens.add_wavelength(value=0.4861)
    lens.add_wavelength(value=0.5876, is_primary=True)
    lens.add_wavelength(value=0.6563)
    return lens


class ReverseTelephoto(Optic):
    """samples/objectives.py:117-173 (S = 14)."""

    def __init__(self):
        super().__init__()
        _reverse_telephoto(self)


class ReverseTelephotoAsphere(Optic):
    """Config 3 "even-asphere wide-angle" (SURVEY 8d.3): ReverseTelephoto with surfaces 2
    and 13 as even aspheres (k = 0, C = [0.02, -0.01, 0.005] / [0.01, 0.005, -0.002])."""

    def __init__(self):
        super().__init__()
        _reverse_telephoto(self, {2: [0.02, -0.01, 0.005], 13: [0.01, 0.005, -0.002]})


class ReverseTelephotoOddAsphere(Optic):
    """ReverseTelephoto with surface 4 an odd asphere (odd_asphere.py coverage)."""

    def __init__(self):
        super().__init__()
        _reverse_telephoto(self, {4: [0.0, 0.003, -0.002, 0.001]}, kind="odd_asphere")


class ThreeMirrorAnastigmat(Optic):
    """Tutorial_7d_Three_Mirror_Anastigmat.ipynb cell 1: three tilted/decentred Zernike
    mirrors (config 5), fixed coefficients."""

    def __init__(self, zernike_type="fringe",
                 coefficients=(0, 0, 0, 1e-4, 2e-4, -1e-4, 5e-5, 0, 0, 3e-5)):
        super().__init__(name="TMA")
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=+1.5)
        self.add_field(y=-1.5)
        self.add_wavelength(value=0.486)
        self.add_wavelength(value=0.587, is_primary=True)
        self.add_wavelength(value=0.656)
        self.add_surface(index=0, radius=np.inf, thickness=np.inf)
        common = dict(conic=0, material="mirror", surface_type="zernike",
                      coefficients=list(coefficients), zernike_type=zernike_type)
        self.add_surface(index=1, radius=-100, thickness=-20, rx=np.radians(-15.0),
                         is_stop=True, **common)
        self.add_surface(index=2, radius=-100, thickness=+20, rx=np.radians(-10.0),
                         dy=-11.5, **common)
        self.add_surface(index=3, radius=-100, thickness=-22, rx=np.radians(-1.0), dy=-15,
                         **common)
        self.add_surface(index=4, dy=-19.3)
        self.update_paraxial()


class CookeTripletApertures(CookeTriplet):
    """CookeTriplet with radial clear apertures on surfaces 3 and 5 (clip coverage)."""

    def __init__(self):
        super().__init__()
        self.surface_group.surfaces[3].aperture = RadialAperture(r_max=4.5)
        self.surface_group.surfaces[5].aperture = RadialAperture(r_max=8.0, r_min=0.4)


STAR = (np.array([4.2, 1.3, 1.2, -3.4, -1.9, -3.3, 1.4, 1.1]),
        np.array([0.1, 1.2, 4.0, 2.6, -0.3, -3.1, -1.5, -4.1]))  # concave polygon


class CookeTripletShapes(CookeTriplet):
    """CookeTriplet with every non-radial aperture kind: rectangular (s1), offset ellipse
    (s2), offset annulus (s3), a concave polygon on the stop (s4) and (rectangle |
    ellipse) minus an offset central obscuration (s6)."""

    def __init__(self):
        from .apertures import (
            EllipticalAperture,
            OffsetRadialAperture,
            PolygonAperture,
            RectangularAperture,
        )

        super().__init__()
        sg = self.surface_group.surfaces
        sg[1].aperture = RectangularAperture(-5.5, 5.0, -4.8, 5.2)
        sg[2].aperture = EllipticalAperture(5.5, 4.6, 0.2, -0.1)
        sg[3].aperture = OffsetRadialAperture(4.6, 0.3, 0.1, -0.2)
        sg[4].aperture = PolygonAperture(*STAR)
        sg[6].aperture = ((RectangularAperture(-6, 6, -2.5, 2.5) | EllipticalAperture(3.5, 6.5))
                          - OffsetRadialAperture(0.6, 0, 0.1, 0.0))


class DecenteredTriplet(Optic):
    """Cooke-like triplet with a tilted/decentred element (rotate_x/y/z coverage)."""

    def __init__(self):
        super().__init__()
        self.add_surface(index=0, radius=np.inf, thickness=np.inf)
        self.add_surface(index=1, radius=22.01359, thickness=3.25896, material="SK16")
        self.add_surface(index=2, radius=-435.76044, thickness=6.00755)
        self.add_surface(index=3, radius=-22.21328, thickness=0.99997,
                         material=("F2", "schott"), dx=0.05, dy=-0.1, rx=0.01, ry=-0.02,
                         rz=0.3)
        self.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True, dy=-0.1,
                         rx=0.01)
        self.add_surface(index=5, radius=79.68360, thickness=2.95208, material="SK16",
                         conic=-0.5)
        self.add_surface(index=6, radius=-18.39533, thickness=42.20778, conic=1.2)
        self.add_surface(index=7)
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=14)
        self.add_field(x=5, y=20)
        self.add_wavelength(value=0.55, is_primary=True)


# name -> builder, matching tests/golden/gen_golden.py CASES
class FreeformTriplet(Optic):
    """Cooke-triplet layout with freeform surfaces (SURVEY 8f.3 coverage): a biconic
    front, a toroidal rear of element 1, an XY-polynomial and a Chebyshev surface on
    element 3 (normalisation set by update_paraxial, optic_updater.py:205-240)."""

    def __init__(self):
        super().__init__()
        self.add_surface(index=0, radius=np.inf, thickness=np.inf)
        self.add_surface(index=1, surface_type="biconic", radius_x=22.01359, radius_y=23.5,
                         conic_x=-0.2, conic_y=0.1, thickness=3.25896, material="SK16")
        self.add_surface(index=2, surface_type="toroidal", radius_x=-300.0,
                         radius_y=-435.76044, conic=0.5, toroidal_coeffs_poly_y=[2e-6],
                         thickness=6.00755)
        self.add_surface(index=3, radius=-22.21328, thickness=0.99997, material=("F2", "schott"))
        self.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True)
        self.add_surface(index=5, surface_type="polynomial", radius=79.68360, conic=0.0,
                         coefficients=[[0.0, 0.0, 2e-4], [0.0, 1e-5, 0.0], [1.5e-4, 0.0, 0.0]],
                         thickness=2.95208, material="SK16")
        self.add_surface(index=6, surface_type="chebyshev", radius=-18.39533, conic=0.0,
                         coefficients=[[0.0, 1e-3, 2e-3], [5e-4, 0.0, 0.0], [1e-3, 0.0, 0.0]],
                         thickness=42.20778)
        self.add_surface(index=7)
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=14)
        self.add_field(x=5, y=10)
        self.add_wavelength(value=0.55, is_primary=True)
        self.update_paraxial()


def _forbes_prescription(lens, s2_type, s2_terms):
    """The reference's Forbes test system (tests/test_geometries.py:2103-2143): a
    plano / Forbes Q-bfs singlet in H-K3 and a plano / Q-bfs element in H-ZLAF68C at
    1.55 um; surface 3 as Q-bfs or Q-2D, fields added for off-axis coverage."""
    lens.set_aperture(aperture_type="EPD", value=4.0)
    lens.set_field_type(field_type="angle")
    lens.add_field(y=0)
    lens.add_field(y=3)
    lens.add_field(x=2, y=2)
    lens.add_wavelength(value=1.55, is_primary=True)
    lens.add_surface(index=0, thickness=0.055)
    lens.add_surface(index=1, thickness=26.5)
    lens.add_surface(index=2, thickness=4.0, radius=np.inf, material=("H-K3", "cdgm"),
                     is_stop=True)
    kw = ({"radial_terms": s2_terms} if s2_type == "forbes_qbfs"
          else {"freeform_coeffs": s2_terms})
    lens.add_surface(index=3, thickness=25.0, radius=22, conic=-4.428, norm_radius=6.336,
                     surface_type=s2_type, **kw)
    lens.add_surface(index=4, thickness=7.0, radius=np.inf, material=("H-ZLAF68C", "cdgm"))
    lens.add_surface(index=5, thickness=10.0, radius=-31.0, conic=0.038,
                     radial_terms={0: -0.270, 1: 0.087, 2: -0.048, 3: 0.026, 4: -0.012},
                     norm_radius=10.0, surface_type="forbes_qbfs")
    lens.add_surface(index=6)


class ForbesSinglets(Optic):
    """Two Forbes Q-bfs elements (forbes/geometry.py:183-330)."""

    def __init__(self):
        super().__init__()
        _forbes_prescription(self, "forbes_qbfs",
                             {0: 1.614, 1: 0.348, 2: 0.150, 3: 0.033, 4: 0.030})


class ForbesFreeform(Optic):
    """The same system with a Q-2D freeform first surface (forbes/geometry.py:333-640):
    rotationally symmetric terms plus m = 1..4 cosine / sine terms."""

    Q2D = {("a", 0, 0): 1.614, ("a", 0, 1): 0.348, ("a", 0, 2): 0.150,
           ("a", 1, 1): 0.02, ("b", 1, 1): -0.01, ("a", 1, 3): 0.005,
           ("a", 2, 0): 0.03, ("b", 2, 1): 0.01, ("a", 3, 0): -0.004,
           ("b", 4, 1): 0.002}

    def __init__(self):
        super().__init__()
        _forbes_prescription(self, "forbes_q2d", dict(self.Q2D))


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


class CookeTripletImageHeight(Optic):
    """Cooke triplet with fields given as paraxial image heights (ParaxialImageHeightField,
    field_types.py:333-479), object at infinity."""

    def __init__(self):
        super().__init__()
        _cooke_prescription(self, np.inf)
        self.set_field_type(field_type="paraxial_image_height")
        self.add_field(y=0)
        self.add_field(y=10)
        self.add_field(y=17)
        self.add_wavelength(value=0.55, is_primary=True)


class FiniteTripletImageHeight(Optic):
    """The same triplet imaging an object 200 mm in front of it, fields as paraxial image
    heights (the finite-conjugate branch of ParaxialImageHeightField)."""

    def __init__(self):
        super().__init__()
        _cooke_prescription(self, 200.0)
        self.set_field_type(field_type="paraxial_image_height")
        self.add_field(y=0)
        self.add_field(y=2)
        self.add_field(y=4)
        self.add_wavelength(value=0.55, is_primary=True)


class ParaxialLens(Optic):
    """Two thin lenses (surface_type "paraxial") around a glass singlet, the second in a
    medium of index 1.2 (thin_lens_interaction_model.py)."""

    def __init__(self):
        from .materials import IdealMaterial

        super().__init__()
        self.add_surface(index=0, thickness=np.inf)
        self.add_surface(index=1, surface_type="paraxial", f=80, thickness=10, is_stop=True)
        self.add_surface(index=2, radius=60.0, thickness=4.0, material="SK16")
        self.add_surface(index=3, radius=-200.0, thickness=10.0)
        self.add_surface(index=4, surface_type="paraxial", f=-150, thickness=40,
                         material=IdealMaterial(1.2, 0))
        self.add_surface(index=5)
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=5)
        self.add_field(x=2, y=3)
        self.add_wavelength(value=0.55, is_primary=True)


class ParaxialMirror(Optic):
    """A reflective thin lens (n2 = -n1)."""

    def __init__(self):
        super().__init__()
        self.add_surface(index=0, thickness=np.inf)
        self.add_surface(index=1, surface_type="paraxial", f=-60, thickness=-50,
                         material="mirror", is_stop=True)
        self.add_surface(index=2)
        self.set_aperture(aperture_type="EPD", value=12)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=4)
        self.add_wavelength(value=0.6, is_primary=True)


class PhasePlate(Optic):
    """Phase surfaces (phase_interaction_model.py): a linear grating on a plane, a radial
    profile on a sphere, a constant phase, a metalens-like radial profile on a plane."""

    def __init__(self):
        from .interactions import (ConstantPhaseProfile, LinearGratingPhaseProfile,
                                   RadialPhaseProfile)

        super().__init__()
        self.add_surface(index=0, thickness=np.inf)
        self.add_surface(index=1, thickness=5, is_stop=True,
                         phase_profile=LinearGratingPhaseProfile(period=5.0, angle=0.4, order=1,
                                                                 efficiency=0.8))
        self.add_surface(index=2, radius=60.0, thickness=4.0, material="SK16",
                         phase_profile=RadialPhaseProfile([-0.02, 1e-5, -2e-8]))
        self.add_surface(index=3, radius=-200.0, thickness=3.0,
                         phase_profile=ConstantPhaseProfile(0.7))
        self.add_surface(index=4, thickness=60.0, phase_profile=RadialPhaseProfile([-0.15]))
        self.add_surface(index=5)
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=5)
        self.add_field(x=1.5, y=-3)
        self.add_wavelength(value=0.48)
        self.add_wavelength(value=0.55, is_primary=True)
        self.add_wavelength(value=0.65)


class Grating(Optic):
    """The reference's grating test systems (tests/test_grating.py:7-117): "flat" / "curved"
    transmission gratings behind an N-BK7 plate or a "reflective" curved grating; `angle`
    rotates the grooves."""

    def __init__(self, kind="flat", angle=0.0):
        super().__init__()
        self.add_surface(index=0, radius=np.inf, thickness=np.inf)
        if kind == "reflective":
            self.add_surface(index=1, radius=70, thickness=-30, material="mirror",
                             surface_type="grating", is_stop=True, grating_period=5.0,
                             grating_order=1, groove_orientation_angle=angle)
            self.add_surface(index=2)
        else:
            self.add_surface(index=1, radius=np.inf, thickness=10)
            self.add_surface(index=2, radius=np.inf, thickness=5, material="N-BK7")
            kw = dict(radius=np.inf) if kind == "flat" else dict(radius=50.0, conic=1.0)
            self.add_surface(index=3, thickness=30, surface_type="grating", grating_order=-1,
                             grating_period=5.0, groove_orientation_angle=angle, is_stop=True,
                             **kw)
            self.add_surface(index=4)
        self.set_aperture(aperture_type="EPD", value=15)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=10)
        self.add_field(y=0, x=10)
        self.add_wavelength(value=0.587, is_primary=True)
        self.update_paraxial()


def nurbs_back_net():
    """The explicit rational back surface of NurbsLens: a 7 x 6 net over [-8, 8] x [-8, 8],
    a concave bowl with an xy twist, non-uniform weights, u degree 3 / v degree 2 on
    clamped non-uniform knots."""
    xs = np.linspace(-8.0, 8.0, 7)
    ys = np.linspace(-8.0, 8.0, 6)
    X, Y = np.meshgrid(xs, ys, indexing="ij")
    Z = -(X**2 + Y**2) / 140.0 + 0.002 * X * Y
    W = 1.0 + 0.1 * np.cos(0.5 * X) * np.sin(0.4 * Y + 0.2)
    U = [0.0, 0.0, 0.0, 0.0, 0.3, 0.5, 0.75, 1.0, 1.0, 1.0, 1.0]
    V = [0.0, 0.0, 0.0, 0.2, 0.55, 0.8, 1.0, 1.0, 1.0]
    return np.stack([X, Y, Z]), W, U, V


class NurbsLens(Optic):
    """A singlet with a bicubic NURBS fit of a conic in front (fit_surface) and an explicit
    rational NURBS net behind (geometries/nurbs/nurbs_geometry.py)."""

    def __init__(self):
        super().__init__()
        P, W, U, V = nurbs_back_net()
        self.add_surface(index=0, thickness=np.inf)
        self.add_surface(index=1, surface_type="nurbs", radius=40.0, conic=-0.5,
                         nurbs_norm_x=8.0, nurbs_norm_y=8.0, n_points_u=8, n_points_v=8,
                         thickness=4.0, material="SK16", is_stop=True)
        self.add_surface(index=2, surface_type="nurbs", radius=-70.0, control_points=P,
                         weights=W, u_degree=3, v_degree=2, u_knots=U, v_knots=V,
                         thickness=45.0)
        self.add_surface(index=3)
        self.surface_group.surfaces[1].geometry.fit_surface()
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=5)
        self.add_field(x=3, y=2)
        self.add_wavelength(value=0.55, is_primary=True)


class GridSagLens(Optic):
    """A singlet whose front surface is a 17 x 13 bilinear sag grid (grid_sag.py)."""

    def __init__(self):
        super().__init__()
        gx = np.linspace(-7, 7, 17)
        gy = np.linspace(-6, 6, 13)
        X, Y = np.meshgrid(gx, gy)
        z = (X**2 + Y**2) / 80.0 + 0.003 * X * Y - 0.02 * Y
        self.add_surface(index=0, thickness=np.inf)
        self.add_surface(index=1, surface_type="grid_sag", x_coordinates=gx.tolist(),
                         y_coordinates=gy.tolist(), sag_values=z.tolist(), thickness=4.0,
                         material="SK16", is_stop=True)
        self.add_surface(index=2, radius=-60.0, thickness=45.0)
        self.add_surface(index=3)
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=5)
        self.add_field(x=3, y=2)
        self.add_wavelength(value=0.55, is_primary=True)




_UV_PRESCRIPTION = (  # (radius, thickness, glass) of surfaces 1-42, lithography.py:23-64
    (-737.7847, 27.484, True), (-235.2891, 0.916, False), (211.1786, 36.646, True),
    (-461.3986, 0.916, False), (412.6778, 21.071, True), (160.5391, 16.197, False),
    (-604.1283, 7.215, True), (218.1877, 23.941, False), (-3586.063, 11.978, True),
    (251.8168, 47.506, False), (-85.2817, 11.961, True), (584.8597, 9.968, False),
    (4074.801, 35.291, True), (-162.0185, 0.923, False), (629.544, 41.227, True),
    (-226.7397, 0.916, False), (522.2739, 27.842, True), (-582.424, 0.916, False),
    (423.729, 22.904, True), (-1385.36, 0.916, False), (212.039, 33.646, True),
    (802.3695, 55.304, False), (-776.5697, 8.703, True), (106.1728, 24.09, False),
    (-200.683, 11.452, True), (311.8264, 59.54, False), (-77.2276, 11.772, True),
    (2317.8032, 11.862, False), (-290.8859, 22.904, True), (-148.3577, 1.373, False),
    (-5658.5043, 41.227, True), (-151.9858, 0.916, False), (678.1005, 32.981, True),
    (-358.554, 0.916, False), (264.2734, 32.814, True), (2309.6884, 0.916, False),
    (171.2681, 29.015, True), (364.7765, 0.918, False), (113.37, 76.259, True),
    (78.6982, 54.304, False), (49.5443, 18.65, True), (109.8136, 13.07647896, False),
)


class UVProjectionLens(Optic):
    """samples/lithography.py:8-84: 248 nm projection lens, 42 spheres (S = 43),
    object-space telecentric (objectNA 0.133, object-height fields), image_solve."""

    def __init__(self):
        from .materials import IdealMaterial

        super().__init__()
        sio2 = IdealMaterial(n=1.5084, k=0)
        self.add_surface(index=0, radius=np.inf, thickness=110.85883544)
        for k, (r, t, glass) in enumerate(_UV_PRESCRIPTION, start=1):
            self.add_surface(index=k, radius=r, thickness=t, is_stop=(k == 20),
                             **({"material": sio2} if glass else {}))
        self.add_surface(index=43, radius=np.inf)
        self.set_aperture(aperture_type="objectNA", value=0.133)
        self.set_field_type(field_type="object_height")
        self.add_field(y=0)
        self.add_field(y=32)
        self.add_field(y=48)
        self.add_wavelength(value=0.248, is_primary=True)
        self.obj_space_telecentric = True
        self.image_solve()


class CookeTripletApodized(CookeTriplet):
    """CookeTriplet with a pupil apodization (optic.set_apodization): every apodization
    kind of optiland/apodization is exercised by the parity fixtures through this lens."""

    def __init__(self, apodization="GaussianApodization", **kwargs):
        super().__init__()
        self.set_apodization(apodization, **kwargs)


class CookeTripletAbbe(Optic):
    """The Cooke triplet prescription with AbbeMaterial model glasses (materials/abbe.py)
    in place of SK16 / F2 (tests/golden/gen_golden.py cooke_abbe)."""

    def __init__(self):
        from .materials import AbbeMaterial

        super().__init__()
        sk16 = AbbeMaterial(1.62041, 60.32)
        f2 = AbbeMaterial(1.62004, 36.37)
        self.add_surface(index=0, radius=np.inf, thickness=np.inf)
        self.add_surface(index=1, radius=22.01359, thickness=3.25896, material=sk16)
        self.add_surface(index=2, radius=-435.76044, thickness=6.00755)
        self.add_surface(index=3, radius=-22.21328, thickness=0.99997, material=f2)
        self.add_surface(index=4, radius=20.29192, thickness=4.75041, is_stop=True)
        self.add_surface(index=5, radius=79.68360, thickness=2.95208, material=sk16)
        self.add_surface(index=6, radius=-18.39533, thickness=42.20778)
        self.add_surface(index=7)
        self.set_aperture(aperture_type="EPD", value=10)
        self.set_field_type(field_type="angle")
        self.add_field(y=0)
        self.add_field(y=14)
        self.add_field(y=20)
        self.add_wavelength(value=0.48)
        self.add_wavelength(value=0.55, is_primary=True)
        self.add_wavelength(value=0.65)


GOLDEN_LENSES = {
    "cooke": CookeTriplet,
    "dg": DoubleGauss,
    "rt": ReverseTelephoto,
    "rt_asph": ReverseTelephotoAsphere,
    "rt_odd": ReverseTelephotoOddAsphere,
    "tma_fringe": lambda: ThreeMirrorAnastigmat("fringe"),
    "tma_standard": lambda: ThreeMirrorAnastigmat("standard"),
    "tma_noll": lambda: ThreeMirrorAnastigmat("noll"),
    "cooke_aperture": CookeTripletApertures,
    "cooke_shapes": CookeTripletShapes,
    "decentered": DecenteredTriplet,
    "freeform": FreeformTriplet,
    "cooke_pih": CookeTripletImageHeight,
    "finite_pih": FiniteTripletImageHeight,
    "forbes": ForbesSinglets,
    "forbes_q2d": ForbesFreeform,
    "paraxial_lens": ParaxialLens,
    "paraxial_mirror": ParaxialMirror,
    "phase_plate": PhasePlate,
    "grating_flat": lambda: Grating("flat"),
    "grating_curved": lambda: Grating("curved"),
    "grating_reflective": lambda: Grating("reflective"),
    "grating_tilted": lambda: Grating("curved", angle=0.35),
    "grid_lens": GridSagLens,
    "nurbs_lens": NurbsLens,
    "uv_projection": UVProjectionLens,
    "apod_gaussian": lambda: CookeTripletApodized("GaussianApodization", sigma=0.6),
    "apod_cos2": lambda: CookeTripletApodized("CosineSquaredApodization", R=0.9),
    "apod_hann": lambda: CookeTripletApodized("HannApodization", D=1.8),
    "apod_poly": lambda: CookeTripletApodized("PolynomialApodization", R=0.95, p=1.5),
    "apod_supergauss": lambda: CookeTripletApodized("SuperGaussianApodization", w=0.7, n=3.5),
    "apod_tukey": lambda: CookeTripletApodized("TukeyApodization", R=0.9, alpha=0.6),
    "apod_uniform": lambda: CookeTripletApodized("UniformApodization"),
    "cooke_abbe": CookeTripletAbbe,
}
