"""Lowering: SurfaceGroup + wavelengths -> the kernel's packed lens table (host, NumPy).

The reference walks Python objects per surface per call (surface_group.py:232-244) and
evaluates n/k per ray with a cache keyed on the whole wavelength array
(materials/base.py:73-119). Here a lens is lowered ONCE per (surface group,
wavelength set) into a few KB of structured arrays (include/optiland_rt.h layout):

  surfaces  [S]            ort_surface    geometry id, R, k, tol, flags, offsets
  cs_ops    [n_ops]        ort_cs_op      localize/globalize translate/rotate ops
  coef      [n_coef]       double         asphere C_i; Zernike radial a_k / d_k
  zern      [n_terms]      ort_zernike_term
  n_tab     [n_lambda][M]  double         n(material, lambda)
  alpha_tab [n_lambda][M]  double         4*pi*k/lambda (homogeneous.py:49-54)

and segment descriptors (ort_segment) carrying the ray-generation scalars
(ray_generator.py:49-106, field_types.py:139-181) per (field, wavelength).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _abi
from .apertures import RadialAperture, program_depth
from .geometries import (NewtonRaphsonGeometry, ZernikePolynomialGeometry, scalar,
                         zernike_monomial_block)
from .surfaces import ObjectSurface


@dataclass
class LensTable:
    surfaces: np.ndarray
    cs_ops: np.ndarray
    coef: np.ndarray
    zern: np.ndarray
    n_tab: np.ndarray
    alpha_tab: np.ndarray
    wavelengths: list
    final_mat: int
    final_thickness: float
    materials: list = field(default_factory=list)
    mat_table: np.ndarray = None  # _abi.MATERIAL [n_mat] (per-ray wavelengths)
    n_rec: int = 0
    rec_surfaces: list = field(default_factory=list)  # traced-surface indices recorded
    # Zernike coefficients held in device tensors: (first zern row, tensor). Their rows
    # carry c = 0 placeholders here (the table structure does not depend on the values)
    # and the uploaded table is patched on the device (raytrace.lens_for), so an
    # optimisation loop over device-resident coefficients never waits on the GPU.
    device_coeffs: list = field(default_factory=list)
    # pupil apodization of generated rays (_abi.APODIZATION record; None: intensity 1).
    # An Optic-level property (optic.py:137): set by raytrace.lens_for from the Optic.
    apod: np.ndarray = None

    @property
    def n_surfaces(self):
        return int(self.surfaces.shape[0])

    @property
    def u_tab(self):
        """[n_lambda][S] n_pre / n_post: the refraction ratio u of real_rays.py:152,
        one IEEE division per (wavelength, surface) instead of one per ray."""
        pre = self.n_tab[:, self.surfaces["mat_pre"]]
        post = self.n_tab[:, self.surfaces["mat_post"]]
        return np.ascontiguousarray(pre / post)

    @property
    def optics(self):
        """[n_lambda][S] ort_surface_optics: n_pre, u, alpha_pre per (lambda, surface)."""
        o = np.zeros((self.n_tab.shape[0], self.n_surfaces), dtype=_abi.SURFACE_OPTICS)
        o["n_pre"] = self.n_tab[:, self.surfaces["mat_pre"]]
        o["u"] = self.u_tab
        o["alpha_pre"] = self.alpha_tab[:, self.surfaces["mat_pre"]]
        o["n_post"] = self.n_tab[:, self.surfaces["mat_post"]]
        o["u_sq"] = o["u"] * o["u"]
        return o

    @property
    def frame_flags(self):
        """ort_lens.frame_flags: ORT_LENS_AXIAL when every surface frame is a +z
        translation (no rotation / reference-cs ops, cs_t[0] = cs_t[1] = +0)."""
        s = self.surfaces
        t = s["cs_t"][:, :2]
        axial = (np.all(s["n_cs_loc"] == 0) and np.all(s["n_cs_glob"] == 0)
                 and np.all(t == 0.0) and not np.any(np.signbit(t)))
        return _abi.LENS_AXIAL if axial else 0

    @property
    def interaction_mask(self):
        m = 0
        for v in np.unique(self.surfaces["interaction"]):
            m |= 1 << int(v)
        return m

    @property
    def newton_surfaces(self):
        return [i for i, s in enumerate(self.surfaces)
                if int(s["geometry"]) in _abi.NEWTON_GEOMETRIES]

    @property
    def has_zernike(self):
        return bool(np.any(self.surfaces["geometry"] == _abi.GEOM_ZERNIKE))

    @property
    def has_range_check(self):
        """Surfaces whose sag raises on out-of-range normalised coordinates."""
        g = self.surfaces["geometry"]
        return bool(np.any((g == _abi.GEOM_ZERNIKE) | (g == _abi.GEOM_CHEBYSHEV)))

    def fingerprint(self):
        """Bytes of everything the device reads: equal fingerprints trace identically."""
        parts = [np.ascontiguousarray(a).tobytes() for a in
                 (self.surfaces, self.cs_ops, self.coef, self.zern, self.n_tab, self.alpha_tab,
                  self.mat_table)]
        parts.append(np.array([self.final_mat], dtype=np.int64).tobytes())
        parts.append(np.array([self.final_thickness], dtype=np.float64).tobytes())
        if self.apod is not None:
            parts.append(np.ascontiguousarray(self.apod).tobytes())
        return b"".join(parts)


def lower_apodization(optic):
    """optic.apodization (optiland/apodization) -> one _abi.APODIZATION record, or None
    (no apodization, or an Optic-less surface group)."""
    apod = getattr(optic, "apodization", None)
    return None if apod is None else apod.lower()


def _device_tensor(v):
    return hasattr(v, "is_cuda") and bool(v.is_cuda)


# Material lowering results by material key (BaseMaterial.key(): the formula source or
# the constants themselves, so equal keys mean equal materials) and by (key, wavelength):
# the dispersion records and n / alpha at the lens's wavelengths are the same from one
# trace call to the next. Keys that name an object rather than its parameters (the
# adapter's ("ref", id(m)) for a custom reference material, which may be mutated, or a new
# material created at a recycled id) are never cached: those are recomputed on every
# lowering.
_MAT_LOWER: dict = {}
_MAT_N_ALPHA: dict = {}


def _cacheable(key):
    return not (isinstance(key, tuple) and key[:1] == ("ref",))


def _material_lower(m):
    key = m.key()
    if not _cacheable(key):
        return m.lower()
    hit = _MAT_LOWER.get(key)
    if hit is None:
        if len(_MAT_LOWER) > 4096:
            _MAT_LOWER.clear()
        hit = _MAT_LOWER[key] = m.lower()
    return hit


def _material_n_alpha(m, w):
    key = (m.key(), w)
    hit = _MAT_N_ALPHA.get(key) if _cacheable(key[0]) else None
    if hit is None:
        if len(_MAT_N_ALPHA) > 65536:
            _MAT_N_ALPHA.clear()
        kv = m.k_scalar(w)
        # homogeneous.py:49-54: applied only when k > 0; alpha = 4*pi*k/w
        hit = (m.n_scalar(w), (4 * np.pi * np.float64(kv) / np.float64(w)) if kv > 0 else 0.0)
        if _cacheable(key[0]):
            _MAT_N_ALPHA[key] = hit
    return hit


def lower_surface_group(surface_group, wavelengths, record=False, skip_object=True):
    """Lower every traced surface (index >= 1) of `surface_group`.

    record: False, True (all traced surfaces) or an iterable of traced-surface
    indices (0-based within the traced surfaces) to snapshot (standard_surface.py:266-286).
    """
    surfs = [s for s in surface_group.surfaces if not isinstance(s, ObjectSurface)]
    if len(surfs) > _abi.MAX_SURFACES:
        raise ValueError(f"at most {_abi.MAX_SURFACES} surfaces are supported")
    wavelengths = [float(w) for w in np.atleast_1d(wavelengths)]

    mats, mat_index = [], {}

    def mat_id(m):
        key = m.key()
        if key not in mat_index:
            mat_index[key] = len(mats)
            mats.append(m)
        return mat_index[key]

    if record is True:
        rec_set = list(range(len(surfs)))
    elif record:
        rec_set = sorted(int(i) for i in record)
    else:
        rec_set = []

    # per-surface fields gathered in plain dicts and written column by column at the end
    # (numpy structured-row assignment costs ~1 us per field: most of a lowering)
    rows = [{} for _ in surfs]
    ops, coef, zern = [], [], []
    ap_progs = []
    ia_blocks = []
    device_coeffs = []
    for si, s in enumerate(surfs):
        g = s.geometry
        R, k, tol, max_iter, norm_radius, cc = g.lower_params()
        row = rows[si]
        row["zm_deg"] = -1
        row["geometry"] = g.geometry_id
        row["radius"] = R
        row["conic"] = k
        row["tol"] = tol
        row["max_iter"] = max_iter
        row["norm_radius"] = norm_radius
        # lens-constant subexpressions of the conic formulas (the same IEEE operations the
        # kernels would repeat per ray): 2 R, 1 + k, R * R
        row["two_r"] = np.float64(2.0) * np.float64(R)
        row["one_plus_k"] = np.float64(1.0) + np.float64(k)
        row["r_sq"] = np.float64(R) * np.float64(R)
        flags = 0
        if s.is_reflective:
            flags |= _abi.SURF_REFLECTIVE
        if isinstance(g, NewtonRaphsonGeometry) or g.geometry_id == _abi.GEOM_STANDARD:
            if np.isinf(R):
                flags |= _abi.SURF_RADIUS_INF
        if g.geometry_id == _abi.GEOM_STANDARD:
            # the conic normal's divisor R * R with its correctly rounded reciprocal
            # (ort_surface.inv_r2), when both are normal finite numbers
            rr = np.float64(R) * np.float64(R)
            if np.isfinite(rr) and 2.0**-300 <= rr <= 2.0**300:
                row["inv_r2"] = np.float64(1.0) / rr
                flags |= _abi.SURF_INV_R2
        if s.aperture is not None:
            if type(s.aperture) is RadialAperture:  # dedicated radial test
                flags |= _abi.SURF_APERTURE
                row["ap_rmax2"] = s.aperture.r_max**2  # radial.py:62
                row["ap_rmin2"] = s.aperture.r_min**2
            else:  # any other aperture: a postfix program in coef
                prog = [float(v) for v in s.aperture.program()]
                if program_depth(prog) > 32:
                    raise ValueError("aperture expression nests too deeply (32 levels)")
                flags |= _abi.SURF_APERTURE_PROG
                ap_progs.append((si, prog))
        if si in rec_set:
            flags |= _abi.SURF_RECORD
            row["rec_slot"] = rec_set.index(si)
        else:
            row["rec_slot"] = -1
        row["flags"] = flags
        if isinstance(g, ZernikePolynomialGeometry):
            on_device = _device_tensor(g.coefficients)
            terms = g.zernike_terms(values=not on_device)
            if on_device:
                device_coeffs.append((len(zern), g.coefficients))
            row["coef_off"] = len(zern)
            row["n_coef"] = len(terms)
            for (c, norm, n, m, a, d) in terms:
                zern.append((c, norm, n, m, len(coef), len(a)))
                coef.extend(a)
                coef.extend(d)
            if any(t[1] != 1.0 for t in terms):
                # the normal omits the normalisation (zernike.py:163-231): the Newton slope
                # is not the sag's derivative, the adjoint replays every update
                row["flags"] |= _abi.SURF_SLOPE_INEXACT
            blk = zernike_monomial_block(terms, on_device)
            if blk is not None:
                row["zm_off"] = len(coef)
                row["zm_deg"] = blk[0]
                coef.extend(blk[1])
        else:
            row["coef_off"] = len(coef)
            row["n_coef"] = len(cc)
            coef.extend(cc)
        im = getattr(s, "interaction_model", None)
        if im is not None:
            row["interaction"] = im.interaction_id
            if im.interaction_id != _abi.IA_REFRACT_REFLECT:
                ia_blocks.append((si, [float(v) for v in im.lower(g)]))
        row["mat_pre"] = mat_id(s.material_pre)
        row["mat_post"] = mat_id(s.material_post)
        loc = g.cs.localize_ops()
        glob = g.cs.globalize_ops()
        # localize starts with translate(-t) of the root frame and globalize ends with
        # translate(+t) (coordinate_system.py:73-107): that pair lives in cs_t (the kernel
        # adds -cs_t / +cs_t unconditionally), the op lists hold the rest
        t = glob[-1][1]
        assert loc[0][0] == _abi.CS_TRANSLATE and glob[-1][0] == _abi.CS_TRANSLATE
        assert tuple(loc[0][1]) == (-t[0], -t[1], -t[2])
        loc, glob = loc[1:], glob[:-1]
        row["cs_t"] = t
        row["cs_loc_off"] = len(ops)
        row["n_cs_loc"] = len(loc)
        ops.extend(loc)
        row["cs_glob_off"] = len(ops)
        row["n_cs_glob"] = len(glob)
        ops.extend(glob)
        if not loc and not glob:
            row["flags"] = int(row["flags"]) | _abi.SURF_TRANSLATE

    for si, prog in ap_progs:  # after every geometry block (coef offsets fixed above)
        rows[si]["ap_off"] = len(coef)
        rows[si]["ap_len"] = len(prog)
        coef.extend(prog)
    for si, blk in ia_blocks:  # interaction parameter blocks (ort_interaction)
        rows[si]["ia_off"] = len(coef)
        coef.extend(blk)

    final = surfs[-1]
    final_mat = mat_id(final.material_post)

    # per-ray dispersion records (used only when a batch carries per-ray wavelengths),
    # their coefficient / tabulated-k blocks after everything else in coef
    mat_table = np.zeros(len(mats), dtype=_abi.MATERIAL)
    for mi, m in enumerate(mats):
        kind, cc, kw, kv, n_const, k_const = _material_lower(m)
        row = mat_table[mi]
        row["kind"] = kind
        row["n_coef"] = len(cc) // 2 if kind == _abi.MAT_TABULATED else len(cc)
        row["coef_off"] = len(coef)
        coef.extend(cc)
        row["k_len"] = len(kw)
        row["k_off"] = len(coef)
        coef.extend(kw)
        coef.extend(kv)
        row["n_const"] = n_const
        row["k_const"] = k_const

    cs = np.zeros(max(1, len(ops)), dtype=_abi.CS_OP)
    if ops:
        cs["kind"] = [kind for kind, _ in ops]
        cs["p"] = [p for _, p in ops]
    z = np.zeros(max(1, len(zern)), dtype=_abi.ZERNIKE_TERM)
    if zern:
        z[:] = zern  # (c, norm, n, m, rad_off, n_rad) rows in field order

    n_tab = np.zeros((len(wavelengths), len(mats)))
    alpha_tab = np.zeros((len(wavelengths), len(mats)))
    for j, w in enumerate(wavelengths):
        for mi, m in enumerate(mats):
            n_tab[j, mi], alpha_tab[j, mi] = _material_n_alpha(m, w)
    for row in rows:  # absorption decided per surface when every wavelength row agrees
        a = alpha_tab[:, row["mat_pre"]]
        if np.all(a > 0):
            row["flags"] |= _abi.SURF_ALPHA_ALL
        elif np.all(a == 0):
            row["flags"] |= _abi.SURF_ALPHA_NONE
    table = np.zeros(len(surfs), dtype=_abi.SURFACE)
    for name in {k for row in rows for k in row}:
        table[name] = [row.get(name, 0) for row in rows]
    return LensTable(
        surfaces=table,
        cs_ops=cs,
        coef=np.array(coef if coef else [0.0], dtype=np.float64),
        zern=z,
        n_tab=n_tab,
        alpha_tab=alpha_tab,
        wavelengths=wavelengths,
        final_mat=final_mat,
        final_thickness=scalar(final.thickness),
        materials=mats,
        mat_table=mat_table,
        n_rec=len(rec_set),
        rec_surfaces=rec_set,
        device_coeffs=device_coeffs,
    )


def lower_geometry(geometry):
    """One-surface table for a bare geometry (the per-geometry API: sag / surface_normal /
    distance in the geometry's local frame; materials are placeholders)."""
    from types import SimpleNamespace

    from .materials import IdealMaterial
    from .surfaces import Surface

    surf = Surface(None, IdealMaterial(1.0), geometry)
    return lower_surface_group(SimpleNamespace(surfaces=[surf]), [0.55])


# --------------------------------------------------------------------------------------
# ray-generation scalars per (field, wavelength) segment
# --------------------------------------------------------------------------------------
def _unit_chief_rays(optic):
    """ParaxialImageHeightField._trace_unit_chief_ray (field_types.py:461-479): y at the
    image of a (y=0, u=1) ray from the stop, and y, u at the object of the same ray traced
    backwards."""
    sg = optic.surface_group
    stop = sg.stop_index
    pos = sg.positions
    wl = optic.primary_wavelength
    y, _ = optic.paraxial._trace_generic(y=0, u=1, z=pos[stop], wavelength=wl, skip=stop)
    y_img = y[-1]
    y, u = optic.paraxial._trace_generic(y=0, u=1, z=pos[-1] - pos[stop], wavelength=wl,
                                         reverse=True, skip=sg.num_surfaces - stop)
    return y_img, y[-1], u[-1]


def _starting_z_offset(optic):
    """field_types.py:223-235."""
    z = optic.surface_group.positions[1:-1]
    offset = optic.paraxial.EPD()
    return offset - np.min(z)


def pupil_scalars(optic):
    """(EPL, EPD) for ray generation (paraxial.py:207-297), computed once per trace call.
    Object-space telecentric systems aim at the object-space NA instead and the reference
    computes neither (ray_generator.py:56-73): (None, None)."""
    if optic.obj_space_telecentric:
        return None, None
    return optic.paraxial.EPL(), optic.paraxial.EPD()


def _telecentric_checks(optic):
    """ray_generator.py:56-68."""
    if optic.field_type == "angle":
        raise ValueError('Field type cannot be "angle" for telecentric object space.')
    if optic.aperture.ap_type == "EPD":
        raise ValueError('Aperture type cannot be "EPD" for telecentric object space.')
    if optic.aperture.ap_type == "imageFNO":
        raise ValueError('Aperture type cannot be "imageFNO" for telecentric object space.')


def segment_params(optic, Hx, Hy, lambda_idx, EPL=None, EPD=None):
    """One ort_segment for field (Hx, Hy): ray_generator.py:49-89 + AngleField /
    ObjectHeightField / ParaxialImageHeightField.get_ray_origins (field_types.py:139-181,
    255-275, 336-390); object-space telecentric aiming ray_generator.py:56-73."""
    seg = np.zeros((), dtype=_abi.SEGMENT)
    vxf, vyf = optic.fields.get_vig_factor(Hx, Hy)
    vx = 1 - np.array(vxf)
    vy = 1 - np.array(vyf)
    telecentric = bool(optic.obj_space_telecentric)
    if telecentric:
        if optic.field_type == "angle":
            _telecentric_checks(optic)  # raises (the angle origins would need EPL first)
        EPL = EPD = 0.0
    else:
        EPL = optic.paraxial.EPL() if EPL is None else EPL
        EPD = optic.paraxial.EPD() if EPD is None else EPD
    max_field = optic.fields.max_field
    field_x = max_field * Hx
    field_y = max_field * Hy
    obj = optic.object_surface
    if optic.field_type == "angle":
        if obj.is_infinite:
            offset = _starting_z_offset(optic)
            x = -np.tan(np.radians(field_x)) * (offset + EPL)
            y = -np.tan(np.radians(field_y)) * (offset + EPL)
            z = optic.surface_group.positions[1] - offset
            seg["mode"] = _abi.GEN_INFINITE
            seg["x_off"], seg["y_off"] = float(x), float(y)
            seg["z0"] = float(np.ravel(z)[0])
        else:
            z0 = float(np.ravel(optic.surface_group.positions[0])[0])
            seg["mode"] = _abi.GEN_FINITE
            seg["x_off"] = float(-np.tan(np.radians(field_x)) * (EPL - z0))
            seg["y_off"] = float(-np.tan(np.radians(field_y)) * (EPL - z0))
            seg["z0"] = z0
    elif optic.field_type == "object_height":
        if obj.is_infinite:
            raise ValueError("Object surface is at infinity.")
        seg["mode"] = _abi.GEN_FINITE
        seg["x_off"] = float(np.array(field_x))
        seg["y_off"] = float(np.array(field_y))
        seg["z0"] = float(0.0 + obj.geometry.cs.z)  # plane object: sag 0 (field_types.py:273)
    elif optic.field_type == "paraxial_image_height":
        # ParaxialImageHeightField.get_ray_origins (field_types.py:336-390): the object-side
        # chief-ray slope / height that lands the paraxial chief ray at the target image
        # height, from unit chief rays traced forward and backward from the stop
        y_img_unit, y_obj_unit, u_obj_unit = _unit_chief_rays(optic)
        if obj.is_infinite:
            u_obj_y = u_obj_unit * (field_y / y_img_unit)
            u_obj_x = u_obj_unit * (field_x / y_img_unit)
            offset = _starting_z_offset(optic)
            x = -u_obj_x * (offset + EPL)
            y = -u_obj_y * (offset + EPL)
            z = optic.surface_group.positions[1] - offset
            seg["mode"] = _abi.GEN_INFINITE
            seg["x_off"], seg["y_off"] = float(np.ravel(x)[0]), float(np.ravel(y)[0])
            seg["z0"] = float(np.ravel(z)[0])
        else:
            y_obj = y_obj_unit * (field_y / y_img_unit)
            x_obj = y_obj_unit * (field_x / y_img_unit)
            seg["mode"] = _abi.GEN_FINITE
            seg["x_off"] = float(np.ravel(x_obj)[0])
            seg["y_off"] = float(np.ravel(y_obj)[0])
            seg["z0"] = float(0.0 + obj.geometry.cs.z)  # plane object: sag 0
    else:
        raise ValueError(f"field type {optic.field_type!r} not supported")
    if telecentric:  # ray_generator.py:56-73: aim at z = sqrt(1 - NA^2) / NA + z0
        _telecentric_checks(optic)
        if int(seg["mode"]) != _abi.GEN_FINITE:
            # ORT_GEN_TELECENTRIC takes the origin as (x_off, y_off, z0), the finite-object
            # origin; an infinite object's origin also depends on the pupil point (the
            # Px EPD / 2 vx term), which this mode does not carry -- refuse, never trace
            # it from the wrong origins
            raise ValueError("object-space telecentric ray generation needs a finite "
                             "object (object_height / paraxial_image_height field)")
        sin = optic.aperture.value
        seg["mode"] = _abi.GEN_TELECENTRIC
        seg["epd"] = 0.0
        seg["epl"] = float(np.sqrt(1 - sin**2) / sin + seg["z0"])
    else:
        seg["epd"] = float(EPD)
        seg["epl"] = float(EPL)
    seg["vx"] = float(vx)
    seg["vy"] = float(vy)
    seg["lambda_idx"] = int(lambda_idx)
    return seg
