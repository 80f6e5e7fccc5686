"""Consumers of the trace: SpotDiagram (analysis/spot_diagram.py:40-438) and
Wavefront / OPD with the chief-ray reference sphere (wavefront/wavefront.py:56-167,
wavefront/strategy.py:68-239, wavefront/opd.py:71-157).

MI355X-first: SpotDiagram traces EVERY (field, wavelength) pair of the analysis in one
fused launch (each pair its own Newton group = one reference Optic.trace call) and
reduces centroid / RMS / max radius on the device; only the statistics leave HBM.
The elementwise post-processing uses torch ops on the device (one IEEE operation each,
in the reference's order); reductions differ from NumPy's pairwise order by ulps.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _abi
from .distribution import BaseDistribution, create_distribution
from .pupil import pupil_arrays
from .lowering import pupil_scalars, segment_params
from .raytrace import RealRays, lens_for, trace_pupil

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def resolve_fields(optic, fields):
    """utils.py:113-135."""
    if isinstance(fields, str):
        if fields == "all":
            return optic.fields.get_field_coords()
        raise ValueError("Invalid field string. Must be 'all'.")
    if isinstance(fields, list):
        return fields
    raise TypeError("Fields must be a string ('all') or a list.")


def resolve_wavelengths(optic, wavelengths):
    """utils.py:67-88."""
    if isinstance(wavelengths, str):
        if wavelengths == "all":
            return optic.wavelengths.get_wavelengths()
        if wavelengths == "primary":
            return [optic.primary_wavelength]
        raise ValueError("Invalid wavelength string. Must be 'all' or 'primary'.")
    if isinstance(wavelengths, list):
        return wavelengths
    raise TypeError("Wavelengths must be a string ('all', 'primary') or a list.")


def localize_points(x, y, z, surface):
    """visualization/system/utils.py:16-46 (transform, is_global=True): apply the surface's
    localize ops to points (direction cosines zero)."""
    for kind, p in surface.geometry.cs.localize_ops():
        if kind == _abi.CS_TRANSLATE:
            x, y, z = x + p[0], y + p[1], z + p[2]
        elif kind == _abi.CS_ROT_X:
            c, s = p[0], p[1]
            y, z = y * c - z * s, y * s + z * c
        elif kind == _abi.CS_ROT_Y:
            c, s = p[0], p[1]
            x, z = x * c + z * s, -x * s + z * c
        else:
            c, s = p[0], p[1]
            x, y = x * c - y * s, x * s + y * c
    return x, y, z


@dataclass
class SpotData:
    x: object
    y: object
    intensity: object


class SpotStatistics:
    """ort_spot_stats for a fixed layout: per (field, wavelength) pair of a pair-major
    ray batch (n_pupil rays each) -> device tensor [n_fields * n_wl][5] = count,
    centroid x, centroid y, rms radius, max radius; the radii about the centroid of the
    field's ref_wl pair (spot_diagram.py:317-357), points with i > 0 (:425-427), taken
    into `surface`'s frame when given (coordinates="local").

    The constructor uploads the image frame's ops and allocates the workspace and the
    output; run() only launches (three small kernels, no host sync, no allocation), so
    it can be captured in a HIP graph."""

    def __init__(self, n_fields, n_wl, n_pupil, ref_wl, surface=None, device=None):
        import ctypes as C

        from . import _native

        self._lib = _native.load()
        dev = device if device is not None else torch.device("cuda")
        ops = surface.geometry.cs.localize_ops() if surface is not None else []
        self._ops = None
        if ops:
            cs = np.zeros(len(ops), dtype=_abi.CS_OP)
            for k, (kind, p) in enumerate(ops):
                cs[k]["kind"] = kind
                cs[k]["p"] = p
            self._ops = torch.tensor(np.frombuffer(cs.tobytes(), dtype=np.uint8), device=dev)
        self._lay = _native.ort_spot_layout(
            int(n_pupil), int(n_fields), int(n_wl), int(ref_wl), len(ops),
            None if self._ops is None else self._ops.data_ptr())
        size = int(self._lib.ort_spot_workspace_size(C.byref(self._lay)))
        _native.check(size if size < 0 else 0, "ort_spot_workspace_size")
        self._size = size
        self._ws = torch.empty(max(size, 8) // 8, dtype=torch.float64, device=dev)
        self.out = torch.empty((n_fields * n_wl, 5), dtype=torch.float64, device=dev)

    def run(self, rays):
        import ctypes as C

        from . import _native
        from .raytrace import _stream_handle

        rc = self._lib.ort_spot_stats(C.byref(rays.c_struct()), C.byref(self._lay),
                                      C.c_void_p(self._ws.data_ptr()), self._size,
                                      C.c_void_p(self.out.data_ptr()), _stream_handle())
        _native.check(rc, "ort_spot_stats")
        return self.out


def spot_statistics(rays, n_fields, n_wl, n_pupil, ref_wl, surface=None):
    """One-shot SpotStatistics(...).run(rays)."""
    return SpotStatistics(n_fields, n_wl, n_pupil, ref_wl, surface, rays.x.device).run(rays)


class SpotDiagram:
    """analysis/spot_diagram.py:40-438 (data generation + statistics; plotting is out
    of scope)."""

    def __init__(self, optic, fields="all", wavelengths="all", num_rings=6,
                 distribution="hexapolar", coordinates="local", newton_mode="reference"):
        self.optic = optic
        self.fields = resolve_fields(optic, fields)
        if coordinates not in ("global", "local"):
            raise ValueError("Coordinates must be 'global' or 'local'.")
        self.coordinates = coordinates
        self.num_rings = num_rings
        self.distribution = distribution
        self.wavelengths = resolve_wavelengths(optic, wavelengths)
        self.newton_mode = newton_mode
        primary = optic.primary_wavelength
        self._analysis_ref_wavelength_index = (
            self.wavelengths.index(primary) if primary in self.wavelengths else 0)
        self._data = None
        self._stats = None
        self._trace()

    def _trace(self):
        """Every (field, wavelength) pair in ONE fused launch, then the statistics kernel
        (ort_spot_stats) on the image rays: nothing is copied to the host here."""
        optic = self.optic
        for hx, hy in self.fields:  # real_ray_tracer.py:59 validation
            if not (-1 <= hx <= 1 and -1 <= hy <= 1):
                raise ValueError("Normalized field coordinates must be within (-1, 1)")
        dl = lens_for(optic, self.wavelengths)
        EPL, EPD = pupil_scalars(optic)
        segs = np.stack([segment_params(optic, float(hx), float(hy), wi, EPL, EPD)
                         for hx, hy in self.fields for wi in range(len(self.wavelengths))])
        dev = dl.device
        px, py = pupil_arrays(self.distribution, self.num_rings, dev)
        n_p = px.numel()
        n = n_p * len(segs)
        out = RealRays.empty(n, 0.0, device=dev)
        keys = [("trace", (float(hx),), (float(hy),), float(w), n_p)
                for hx, hy in self.fields for w in self.wavelengths]
        trace_pupil(dl, segs, px, py, out, n, n_p, n_p, keys=keys, newton_mode=self.newton_mode)
        self.rays = out
        self._n_p = n_p
        self._stats = spot_statistics(
            out, len(self.fields), len(self.wavelengths), n_p,
            self._analysis_ref_wavelength_index,
            optic.image_surface if self.coordinates == "local" else None)

    @property
    def data(self):
        """spot_diagram.py:381-438: [field][wavelength] SpotData of the i > 0 points
        (device tensors, built on first use: boolean masking synchronises)."""
        if self._data is None:
            self._data = self._generate_data()
        return self._data

    def _generate_data(self):
        out, n_p = self.rays, self._n_p
        data = []
        k = 0
        img = self.optic.image_surface
        for _ in self.fields:
            row = []
            for _ in self.wavelengths:
                sl = slice(k * n_p, (k + 1) * n_p)
                x, y, z, i = out.x[sl], out.y[sl], out.z[sl], out.i[sl]
                mask = i > 0  # spot_diagram.py:425-427
                x, y, z, i = x[mask], y[mask], z[mask], i[mask]
                if self.coordinates == "local":
                    x, y, _ = localize_points(x, y, z, img)
                row.append(SpotData(x=x, y=y, intensity=i))
                k += 1
            data.append(row)
        return data

    # -- statistics (spot_diagram.py:317-379), from the device statistics kernel --
    def _stat(self, col):
        nw = len(self.wavelengths)
        st = self._stats
        return [[st[f * nw + w, col] for w in range(nw)] for f in range(len(self.fields))]

    def centroid(self):
        """Centroid of each field's reference-wavelength spot (spot_diagram.py:317-328)."""
        ref = self._analysis_ref_wavelength_index
        nw = len(self.wavelengths)
        st = self._stats
        return [(st[f * nw + ref, 1], st[f * nw + ref, 2]) for f in range(len(self.fields))]

    def geometric_spot_radius(self):
        """spot_diagram.py:330-343 (be.max over an empty spot raises, as NumPy does)."""
        if bool((self._stats[:, 0] == 0).any()):
            raise ValueError("zero-size array to reduction operation maximum which has no "
                             "identity")
        return self._stat(4)

    def rms_spot_radius(self):
        """spot_diagram.py:345-357."""
        return self._stat(3)


# --------------------------------------------------------------------------------------
# wavefront
# --------------------------------------------------------------------------------------
@dataclass
class WavefrontData:
    pupil_x: object
    pupil_y: object
    pupil_z: object
    opd: object
    intensity: object
    radius: float


class ChiefRayStrategy:
    """wavefront/strategy.py:168-239."""

    def __init__(self, optic, distribution):
        self.optic = optic
        self.distribution = distribution
        self.n_image = optic.n()[-1]
        self.pupil_z = optic.paraxial.XPL() + optic.surface_group.positions[-1]

    def _opd_image_to_xp(self, rays, xc, yc, zc, R):
        """strategy.py:68-116: ray to reference-sphere distance from the image plane."""
        xr, yr, zr = rays.x, rays.y, rays.z
        L, M, N = -rays.L, -rays.M, -rays.N
        a = L**2 + M**2 + N**2
        b = 2 * (L * (xr - xc) + M * (yr - yc) + N * (zr - zc))
        c = (xr**2 + yr**2 + zr**2 - 2 * (xr * xc + yr * yc + zr * zc)
             + xc**2 + yc**2 + zc**2 - R**2)
        d = b**2 - 4 * a * c
        d = torch.where(d < 0, torch.zeros_like(d), d)
        t = (-b - torch.sqrt(d)) / (2 * a)
        mask = t < 0
        t = torch.where(mask, (-b + torch.sqrt(d)) / (2 * a), t)
        return self.n_image * t

    def _correct_tilt(self, field, opd, x=None, y=None):
        """strategy.py:118-166 (angle fields only)."""
        if self.optic.field_type != "angle":
            return opd
        hx, hy = field
        max_field_deg = self.optic.fields.max_field
        fx_rad = np.deg2rad(hx * max_field_deg)
        fy_rad = np.deg2rad(hy * max_field_deg)
        tx, ty = np.tan(fx_rad), np.tan(fy_rad)
        uz = 1.0 / np.sqrt(1.0 + tx**2 + ty**2)
        ux, uy = tx * uz, ty * uz
        dev = opd.device
        xs = torch.as_tensor(np.asarray(self.distribution.x if x is None else x, dtype=np.float64),
                             device=dev)
        ys = torch.as_tensor(np.asarray(self.distribution.y if y is None else y, dtype=np.float64),
                             device=dev)
        epd = self.optic.paraxial.EPD()
        X_m = xs * epd / 2
        Y_m = ys * epd / 2
        tilt = float(ux) * X_m + float(uy) * Y_m
        return opd + tilt

    def compute_wavefront_data(self, field, wavelength):
        optic = self.optic
        chief = optic.trace_generic(*field, Px=0.0, Py=0.0, wavelength=wavelength)
        x, y, z = chief.x, chief.y, chief.z
        if x.numel() != 1:
            raise ValueError("Chief ray cannot be determined. It must be traced alone.")
        R = float(torch.sqrt(x**2 + y**2 + (z - float(np.ravel(self.pupil_z)[0])) ** 2).item())
        xc, yc, zc = x, y, z
        opd_img_ref = self._opd_image_to_xp(chief, xc, yc, zc, R)
        opd_ref = chief.opd - opd_img_ref
        opd_ref = self._correct_tilt(field, opd_ref, x=0.0, y=0.0)
        rays = optic.trace(*field, wavelength, None, self.distribution)
        intensity = rays.i
        opd_img = self._opd_image_to_xp(rays, xc, yc, zc, R)
        opd = rays.opd - opd_img
        opd = self._correct_tilt(field, opd)
        opd_wv = (opd_ref - opd) / (wavelength * 1e-3)
        t = opd_img / self.n_image
        return WavefrontData(pupil_x=rays.x - t * rays.L, pupil_y=rays.y - t * rays.M,
                             pupil_z=rays.z - t * rays.N, opd=opd_wv, intensity=intensity,
                             radius=R)


class Wavefront:
    """wavefront/wavefront.py:56-167 (chief_ray strategy)."""

    def __init__(self, optic, fields="all", wavelengths="all", num_rays=12,
                 distribution="hexapolar", strategy="chief_ray", remove_tilt=False):
        if strategy != "chief_ray":
            raise ValueError(f"strategy {strategy!r} is not implemented on the trace core")
        self.optic = optic
        self.fields = resolve_fields(optic, fields)
        self.wavelengths = resolve_wavelengths(optic, wavelengths)
        self.num_rays = num_rays
        if isinstance(distribution, str):
            d = create_distribution(distribution)
            d.generate_points(num_rays)
            distribution = d
        if not isinstance(distribution, BaseDistribution) and not hasattr(distribution, "x"):
            raise ValueError("Invalid distribution")
        self.distribution = distribution
        self.strategy = ChiefRayStrategy(optic, distribution)
        self.remove_tilt = remove_tilt
        self.data = {}
        for f in self.fields:
            for wl in self.wavelengths:
                self.data[(tuple(f), wl)] = self.strategy.compute_wavefront_data(tuple(f), wl)

    def get_data(self, field, wl):
        return self.data[(tuple(field), wl)]


class OPD(Wavefront):
    """wavefront/opd.py:19-157."""

    def __init__(self, optic, field, wavelength, num_rays=15, distribution="hexapolar",
                 strategy="chief_ray", remove_tilt=False):
        if isinstance(wavelength, str):
            if wavelength != "primary":
                raise ValueError("Invalid wavelength string. For a single wavelength, it "
                                 "must be 'primary'.")
            wavelength = optic.primary_wavelength
        super().__init__(optic, fields=[tuple(field)], wavelengths=[float(wavelength)],
                         num_rays=num_rays, distribution=distribution, strategy=strategy,
                         remove_tilt=remove_tilt)

    def rms(self):
        """opd.py:143-157."""
        data = self.get_data(self.fields[0], self.wavelengths[0])
        mask = data.intensity > 0
        if not bool(torch.any(mask)):
            raise ValueError("No valid rays with non-zero intensity for RMS calculation.")
        opd = data.opd[mask]
        return torch.sqrt(torch.mean(opd**2))
