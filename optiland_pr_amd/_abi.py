"""NumPy mirrors of the C structs in include/optiland_rt.h.

The host builds the lowered lens as NumPy structured arrays with exactly the C
layout, so `arr.tobytes()` is the device image of the table. Offsets are asserted
against the header sizes in tests/test_abi.py.
"""

from __future__ import annotations

import numpy as np

ABI_VERSION = 20
VJP_UNROLLED = 0
VJP_ADJOINT = 1
AP_RADIAL = 1
AP_ELLIPSE = 2
AP_RECT = 3
AP_POLYGON = 4
AP_UNION = 5
AP_INTERSECT = 6
AP_DIFFERENCE = 7
PUPIL_UNIFORM = 0
PUPIL_HEXAPOLAR = 1
PUPIL_RANDOM = 2
PUPIL_RING = 3
PUPIL_LINE_X = 4
PUPIL_LINE_Y = 5
PUPIL_CROSS = 6
MAX_SURFACES = 64

# enum ort_geometry
GEOM_PLANE = 0
GEOM_STANDARD = 1
GEOM_EVEN_ASPHERE = 2
GEOM_ODD_ASPHERE = 3
GEOM_ZERNIKE = 4
GEOM_POLYNOMIAL = 5
GEOM_CHEBYSHEV = 6
GEOM_BICONIC = 7
GEOM_TOROIDAL = 8
GEOM_FORBES_QBFS = 9
GEOM_FORBES_Q2D = 10
GEOM_GRID_SAG = 11
GEOM_NURBS = 12  # ABI v20: own (u, v) solve per ray, not a Newton-in-t surface
FREEFORM_GEOMETRIES = (GEOM_POLYNOMIAL, GEOM_CHEBYSHEV, GEOM_BICONIC, GEOM_TOROIDAL,
                       GEOM_FORBES_QBFS, GEOM_FORBES_Q2D, GEOM_GRID_SAG)
NEWTON_GEOMETRIES = (GEOM_EVEN_ASPHERE, GEOM_ODD_ASPHERE, GEOM_ZERNIKE) + FREEFORM_GEOMETRIES

# enum ort_surface_flags
SURF_REFLECTIVE = 1 << 0
SURF_RADIUS_INF = 1 << 1
SURF_APERTURE = 1 << 2
SURF_RECORD = 1 << 3
SURF_TRANSLATE = 1 << 4
SURF_APERTURE_PROG = 1 << 5
SURF_INV_R2 = 1 << 6
SURF_ALPHA_ALL = 1 << 7
SURF_ALPHA_NONE = 1 << 8
SURF_SLOPE_INEXACT = 1 << 9  # (v19) the Newton slope is not the sag's derivative
LENS_AXIAL = 1 << 0  # ort_lens.frame_flags

# enum ort_interaction / ort_phase_kind
IA_REFRACT_REFLECT = 0
IA_THIN_LENS = 1
IA_PHASE = 2
IA_DIFFRACTIVE = 3
PHASE_CONSTANT = 0
PHASE_LINEAR = 1
PHASE_RADIAL = 2

# enum ort_cs_kind
CS_TRANSLATE = 0
CS_ROT_X = 1
CS_ROT_Y = 2
CS_ROT_Z = 3

# enum ort_gen_mode
GEN_INFINITE = 0
GEN_FINITE = 1
GEN_TELECENTRIC = 2

# enum ort_apod_kind
APOD_UNIFORM = 0
APOD_GAUSSIAN = 1
APOD_COSINE_SQUARED = 2
APOD_HANN = 3
APOD_POLYNOMIAL = 4
APOD_SUPER_GAUSSIAN = 5
APOD_TUKEY = 6

# enum ort_newton_mode
NEWTON_SCHEDULE = 0
NEWTON_WAVE = 1

# enum ort_status
STATUS_ZERNIKE_RANGE = 1 << 0
STATUS_CHEBYSHEV_RANGE = 1 << 1
STATUS_BAD_GEOMETRY = 1 << 2
STATUS_BAD_APODIZATION = 1 << 3

CS_OP = np.dtype(
    [("kind", "<i4"), ("reserved", "<i4"), ("p", "<f8", (3,))], align=True
)
assert CS_OP.itemsize == 32

SURFACE = np.dtype(
    [
        ("radius", "<f8"),
        ("conic", "<f8"),
        ("tol", "<f8"),
        ("norm_radius", "<f8"),
        ("ap_rmax2", "<f8"),
        ("ap_rmin2", "<f8"),
        ("geometry", "<i4"),
        ("flags", "<i4"),
        ("max_iter", "<i4"),
        ("n_coef", "<i4"),
        ("coef_off", "<i4"),
        ("mat_pre", "<i4"),
        ("mat_post", "<i4"),
        ("cs_loc_off", "<i4"),
        ("n_cs_loc", "<i4"),
        ("cs_glob_off", "<i4"),
        ("n_cs_glob", "<i4"),
        ("rec_slot", "<i4"),
        ("cs_t", "<f8", (3,)),
        ("ap_off", "<i4"),
        ("ap_len", "<i4"),
        ("interaction", "<i4"),
        ("ia_off", "<i4"),
        ("inv_r2", "<f8"),
        ("two_r", "<f8"),
        ("one_plus_k", "<f8"),
        ("r_sq", "<f8"),
        ("zm_off", "<i4"),
        ("zm_deg", "<i4"),
    ],
    align=True,
)
assert SURFACE.itemsize == 176

SURFACE_OPTICS = np.dtype(
    [("n_pre", "<f8"), ("u", "<f8"), ("alpha_pre", "<f8"), ("n_post", "<f8"), ("u_sq", "<f8")],
    align=True,
)
assert SURFACE_OPTICS.itemsize == 40

ZERNIKE_TERM = np.dtype(
    [
        ("c", "<f8"),
        ("norm", "<f8"),
        ("n", "<i4"),
        ("m", "<i4"),
        ("rad_off", "<i4"),
        ("n_rad", "<i4"),
    ],
    align=True,
)
assert ZERNIKE_TERM.itemsize == 32

SEGMENT = np.dtype(
    [
        ("epd", "<f8"),
        ("epl", "<f8"),
        ("vx", "<f8"),
        ("vy", "<f8"),
        ("x_off", "<f8"),
        ("y_off", "<f8"),
        ("z0", "<f8"),
        ("lambda_idx", "<i4"),
        ("mode", "<i4"),
    ],
    align=True,
)
assert SEGMENT.itemsize == 64

APODIZATION = np.dtype(
    [
        ("kind", "<i4"),
        ("reserved", "<i4"),
        ("p", "<f8", (4,)),
    ],
    align=True,
)
assert APODIZATION.itemsize == 40

# enum ort_material_kind
MAT_IDEAL = 0
MAT_TABULATED = 10
MAT_ABBE = 11

MATERIAL = np.dtype(
    [
        ("kind", "<i4"),
        ("n_coef", "<i4"),
        ("coef_off", "<i4"),
        ("k_len", "<i4"),
        ("k_off", "<i4"),
        ("reserved", "<i4"),
        ("n_const", "<f8"),
        ("k_const", "<f8"),
    ],
    align=True,
)
assert MATERIAL.itemsize == 40

NEWTON_STAT = np.dtype(
    [("conv_mask", "<u8", (2,)), ("last_bad", "<i4"), ("max_updates", "<i4")], align=True
)
assert NEWTON_STAT.itemsize == 24
OPT_NO_INIT = 1  # ort_options.flags: ORT_OPT_NO_INIT
OPT_EXACT = 2  # ort_options.flags: ORT_OPT_EXACT (no deferred-check pass)
CONV_WINDOW = 128  # stop indices per conv_mask window (ort_options.conv_base)

RAY_FIELDS = ("x", "y", "z", "L", "M", "N", "i", "opd")

VJP_ADJOINT_MAX_SLOTS = 512
ADJ_HIST = 4  # ort_sweep.h kHist: Newton iterates the adjoint tape keeps per surface  # ORT_VJP_ADJOINT_MAX_SLOTS: 3 S + n_zern + 1 at most
