"""Consumers of the trace: SpotDiagram (analysis/spot_diagram.py:40-438) and
Wavefront / OPD with the chief-ray, centroid-anchored and best-fit reference spheres
(wavefront/wavefront.py:56-167, wavefront/strategy.py:68-514, wavefront/opd.py:71-157).

MI355X-first: SpotDiagram traces EVERY (field, wavelength) pair of the analysis in one
fused launch (each pair its own Newton group = one reference Optic.trace call) and
reduces centroid / RMS / max radius on the device (ort_spot_stats); the wavefront's
per-ray OPD, exit-pupil points, rms and tilt-fit sums are one fused kernel
(ort_wavefront_opd) in the reference's operation order. Only statistics leave HBM;
reductions run in a fixed order that differs from NumPy's pairwise sums by ulps.
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

    def trace(self, dlens, segments, px, py, rays):
        """Trace the pairs of a lens without Newton geometries into `rays` and run the
        statistics, the first pass fused into the trace kernel (ort_trace_spot): the same
        numbers as trace_pupil + run(rays), one launch fewer. Capturable like run()."""
        from .raytrace import trace_spot

        n_p = int(self._lay.n_pupil)
        return trace_spot(dlens, segments, px, py, rays, len(rays), n_p, self)


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
        self.rays = out
        self._n_p = n_p
        spot = SpotStatistics(len(self.fields), len(self.wavelengths), n_p,
                              self._analysis_ref_wavelength_index,
                              optic.image_surface if self.coordinates == "local" else None, dev)
        if dl.newton:
            trace_pupil(dl, segs, px, py, out, n, n_p, n_p, keys=keys,
                        newton_mode=self.newton_mode)
            self._stats = spot.run(out)
        else:  # statistics pass 1 in the trace kernel's epilogue (ort_trace_spot)
            self._stats = spot.trace(dl, segs, px, py, out)

    @property
    def data(self):
        """spot_diagram.py:381-438: [field][wavelength] SpotData of the i > 0 points
        (device tensors, built on first use: boolean masking synchronises)."""
        if self._data is None:
            self._data = self._generate_data()
        return self._data

    @data.setter
    def data(self, value):
        """The reference's SpotDiagram.data is a plain attribute its helpers may reassign
        (e.g. re-centred spots). Assigned data is kept as given; the device statistics
        (centroid / rms / geometric radius) keep describing the traced rays."""
        self._data = value

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


def _tilt_direction(optic, field):
    """strategy.py:141-153: (ux, uy) of an angle field, None otherwise."""
    if optic.field_type != "angle":
        return None
    hx, hy = field
    max_field_deg = optic.fields.max_field
    tx, ty = np.tan(np.deg2rad(hx * max_field_deg)), np.tan(np.deg2rad(hy * max_field_deg))
    uz = 1.0 / np.sqrt(1.0 + tx**2 + ty**2)
    return tx * uz, ty * uz


class ChiefRayStrategy:
    """wavefront/strategy.py:168-239 on the device: the chief ray and the full ray set
    are traced by the HIP kernels; the chief ray's reference sphere is formed on the
    host from its 7 doubles (the reference reads R with .item() too), and the per-ray
    OPD, exit-pupil points, rms and tilt-fit sums come from one fused kernel
    (ort_wavefront_opd) instead of a chain of elementwise array operations."""

    def __init__(self, optic, distribution, **kwargs):
        self.optic = optic
        self.distribution = distribution
        self.n_image = optic.n()[-1]
        self.pupil_z = optic.paraxial.XPL() + optic.surface_group.positions[-1]

    # -- host restatements for the single chief ray (NumPy, the reference's order) --
    def _opd_image_to_xp_np(self, c, xc, yc, zc, R):
        """strategy.py:68-116 on the chief ray's 1-element arrays."""
        xr, yr, zr = c["x"], c["y"], c["z"]
        L, M, N = -c["L"], -c["M"], -c["N"]
        a = L**2 + M**2 + N**2
        b = 2 * (L * (xr - xc) + M * (yr - yc) + N * (zr - zc))
        cc = (xr**2 + yr**2 + zr**2 - 2 * (xr * xc + yr * yc + zr * zc)
              + xc**2 + yc**2 + zc**2 - R**2)
        d = b**2 - 4 * a * cc
        d = np.where(d < 0, 0, d)
        with np.errstate(invalid="ignore", divide="ignore"):
            t = (-b - np.sqrt(d)) / (2 * a)
            t = np.where(t < 0, (-b + np.sqrt(d)) / (2 * a), t)
        return self.n_image * t

    def _tilt_direction(self, field):
        return _tilt_direction(self.optic, field)

    def compute_wavefront_data(self, field, wavelength):
        import ctypes as C

        from . import _native
        from .raytrace import _stream_handle

        optic = self.optic
        chief = optic.trace_generic(*field, Px=0.0, Py=0.0, wavelength=wavelength)
        if chief.x.numel() != 1:
            raise ValueError("Chief ray cannot be determined. It must be traced alone.")
        c = {a: chief_v for a, chief_v in zip(
            ("x", "y", "z", "L", "M", "N", "opd"),
            torch.stack([chief.x, chief.y, chief.z, chief.L, chief.M, chief.N,
                         chief.opd]).reshape(7, 1).cpu().numpy(), strict=True)}
        xc, yc, zc = c["x"], c["y"], c["z"]
        R = float(np.sqrt(xc**2 + yc**2 + (zc - self.pupil_z) ** 2).item())  # :236-241
        opd_ref = c["opd"] - self._opd_image_to_xp_np(c, xc, yc, zc, R)
        tilt = self._tilt_direction(field)
        epd = optic.paraxial.EPD() if tilt is not None else 0.0
        if tilt is not None:  # _correct_tilt(field, opd_ref, x=0, y=0)
            X_m = np.array(0.0) * epd / 2
            Y_m = np.array(0.0) * epd / 2
            opd_ref = opd_ref + (tilt[0] * X_m + tilt[1] * Y_m)

        rays = optic.trace(*field, wavelength, None, self.distribution)
        n = len(rays)
        dev = rays.x.device
        px = py = None
        if tilt is not None:
            px = torch.as_tensor(np.ascontiguousarray(self.distribution.x, dtype=np.float64),
                                 device=dev)
            py = torch.as_tensor(np.ascontiguousarray(self.distribution.y, dtype=np.float64),
                                 device=dev)
        f1 = lambda v: float(np.ravel(v)[0])  # noqa: E731
        ref = _native.ort_wavefront_ref(
            f1(xc), f1(yc), f1(zc), f1(xc**2), f1(yc**2), f1(zc**2), R**2,
            float(self.n_image), f1(opd_ref), 0.0 if tilt is None else float(tilt[0]),
            0.0 if tilt is None else float(tilt[1]), float(np.ravel(epd)[0]),
            float(wavelength * 1e-3), int(tilt is not None), 0)
        lib = _native.load()
        opd_wv = torch.empty(n, dtype=torch.float64, device=dev)
        pup = [torch.empty(n, dtype=torch.float64, device=dev) for _ in range(3)]
        size = int(lib.ort_wavefront_workspace_size(n))
        _native.check(size if size < 0 else 0, "ort_wavefront_workspace_size")
        ws = torch.empty(max(size, 8) // 8, dtype=torch.float64, device=dev)
        sums = torch.empty(11, dtype=torch.float64, device=dev)
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        rc = lib.ort_wavefront_opd(C.byref(rays.c_struct()), ptr(px), ptr(py), n, C.byref(ref),
                                   ptr(opd_wv), ptr(pup[0]), ptr(pup[1]), ptr(pup[2]),
                                   ptr(ws), size, ptr(sums), _stream_handle())
        _native.check(rc, "ort_wavefront_opd")
        data = WavefrontData(pupil_x=pup[0], pupil_y=pup[1], pupil_z=pup[2], opd=opd_wv,
                             intensity=rays.i, radius=R)
        data.sums = sums
        return data


def _full(like, v):
    """A divisor as a device tensor: torch divides by a Python scalar as a multiplication
    by its reciprocal (not the IEEE quotient the reference's NumPy forms)."""
    return torch.full_like(like, float(np.ravel(v)[0]))


class CentroidReferenceSphereStrategy:
    """strategy.py:242-402: the reference sphere centred on the (optionally outlier-
    trimmed) centroid of the image-plane points, its radius the mean distance from that
    centre to the wavefront points p - (opd / n_image) d; OPD relative to the mean over
    the rays with i > 0.

    The traced rays and every per-ray array stay on the device (the trace is the HIP
    kernel, the elementwise chain -- launch-plane tilt, the image-to-sphere distance, OPD
    in waves, exit-pupil points -- runs there in the reference's operation order). The
    few reductions that fix the sphere (centroid, mean / std of the distances, the
    radius, the mean OPD; the best-fit sphere's 4-column least squares) read host copies
    of the point set and use NumPy exactly as the reference does, so the sphere and
    every per-ray output are bit-identical to the reference's."""

    def __init__(self, optic, distribution, robust_trim_std=3.0):
        self.optic = optic
        self.distribution = distribution
        self.n_image = optic.n()[-1]
        self.robust_trim_std = robust_trim_std

    def _points_from_rays(self, h, opd):
        """strategy.py:325-351 (host arrays)."""
        valid = (np.isfinite(h["x"]) & np.isfinite(h["y"]) & np.isfinite(h["z"])
                 & np.isfinite(h["L"]) & np.isfinite(h["M"]) & np.isfinite(h["N"])
                 & np.isfinite(opd) & (h["i"] != 0))
        if not np.any(valid):
            raise ValueError("No valid ray samples found for best-fit sphere.")
        p = np.stack((h["x"], h["y"], h["z"]), axis=1)[valid]
        d = np.stack((h["L"], h["M"], h["N"]), axis=1)[valid]
        s = opd[valid] / self.n_image
        return p - s[:, None] * d, valid

    def _calculate_reference_sphere(self, h, opd):
        """strategy.py:353-402 (host arrays)."""
        wavefront_points, valid_mask = self._points_from_rays(h, opd)
        image_points = np.stack((h["x"], h["y"], h["z"]), axis=1)[valid_mask]
        weights = h["i"][valid_mask]
        weights = np.where(weights < 0.0, 0.0, weights)
        total_weight = np.sum(weights)
        if total_weight == 0:
            weights = np.ones_like(weights)
        else:  # the reference then weighs every valid point equally (:377-379)
            weights = np.ones((image_points.shape[0],))
        total_weight = np.sum(weights)
        centroid = np.sum(image_points * weights[:, None], axis=0) / total_weight
        if self.robust_trim_std and self.robust_trim_std > 0:
            distances_img = np.linalg.norm(image_points - centroid, axis=1)
            mean_d = np.mean(distances_img)
            std_d = np.std(distances_img)
            if std_d > 0:
                keep_mask = distances_img <= (mean_d + self.robust_trim_std * std_d)
                if np.sum(keep_mask) >= 4:
                    weights = weights * np.array(keep_mask)
                    total_weight = np.sum(weights)
                    centroid = np.sum(image_points * weights[:, None], axis=0) / total_weight
        distances_wf = np.linalg.norm(wavefront_points - centroid, axis=1)
        radius = float(np.sum(weights * distances_wf) / np.sum(weights))
        return float(centroid[0]), float(centroid[1]), float(centroid[2]), radius

    def _opd_image_to_xp(self, rays, xc, yc, zc, R):
        """strategy.py:68-116 on the device (tensor ops in the reference's order; the
        centre's squares formed as the reference forms them, from Python floats)."""
        xr, yr, zr = rays.x, rays.y, rays.z
        L, M, N = -rays.L, -rays.M, -rays.N
        a = L**2 + M**2 + N**2
        b = 2 * (L * (xr - xc) + M * (yr - yc) + N * (zr - zc))
        c = (xr**2 + yr**2 + zr**2 - 2 * (xr * xc + yr * yc + zr * zc)
             + xc**2 + yc**2 + zc**2 - R**2)
        d = b**2 - 4 * a * c
        d = torch.where(d < 0, torch.zeros_like(d), d)
        t = (-b - torch.sqrt(d)) / (2 * a)
        t = torch.where(t < 0, (-b + torch.sqrt(d)) / (2 * a), t)
        return float(self.n_image) * t

    def _correct_tilt(self, field, opd, dev):
        """strategy.py:118-166 over the whole pupil (device)."""
        tilt = _tilt_direction(self.optic, field)
        if tilt is None:
            return opd
        ux, uy = (float(v) for v in tilt)
        epd = float(np.ravel(self.optic.paraxial.EPD())[0])
        xs = torch.as_tensor(np.asarray(self.distribution.x, dtype=np.float64), device=dev)
        ys = torch.as_tensor(np.asarray(self.distribution.y, dtype=np.float64), device=dev)
        X_m = xs * epd / 2
        Y_m = ys * epd / 2
        return opd + (ux * X_m + uy * Y_m)

    def compute_wavefront_data(self, field, wavelength):
        """strategy.py:273-323."""
        rays = self.optic.trace(*field, wavelength, None, self.distribution)
        dev = rays.x.device
        opd_c = self._correct_tilt(field, rays.opd, dev)
        h = {a: getattr(rays, a).cpu().numpy() for a in ("x", "y", "z", "L", "M", "N", "i")}
        xc, yc, zc, radius = self._calculate_reference_sphere(h, opd_c.cpu().numpy())
        opd_img = self._opd_image_to_xp(rays, xc, yc, zc, radius)
        opd = opd_c - opd_img
        valid = h["i"] > 0
        if not np.any(valid):
            raise ValueError("No valid rays with non-zero intensity for OPD calculation.")
        mean_opd = float(np.mean(opd.cpu().numpy()[valid]))
        opd_waves = (mean_opd - opd) / _full(opd, wavelength * 1e-3)
        t = opd_img / _full(opd_img, self.n_image)
        data = WavefrontData(pupil_x=rays.x - t * rays.L, pupil_y=rays.y - t * rays.M,
                             pupil_z=rays.z - t * rays.N, opd=opd_waves, intensity=rays.i,
                             radius=radius)
        data.sums = None
        return data


class BestFitSphereStrategy(CentroidReferenceSphereStrategy):
    """strategy.py:405-479: the sphere through the wavefront points in the least-squares
    sense, 2 x xc + 2 y yc + 2 z zc + (R^2 - |c|^2) = |p|^2, solved by the same LAPACK
    least squares (numpy.linalg.lstsq) on the same bit-identical point set."""

    def __init__(self, optic, distribution, **kwargs):
        super().__init__(optic, distribution, **kwargs)
        self.center = None

    def _calculate_reference_sphere(self, h, opd):
        wavefront_points, _ = self._points_from_rays(h, opd)
        if wavefront_points.shape[0] < 4:
            raise ValueError("Need at least 4 valid ray samples for a best-fit sphere.")
        x, y, z = wavefront_points[:, 0], wavefront_points[:, 1], wavefront_points[:, 2]
        A = np.stack([x, y, z, np.ones_like(x)], axis=1)
        b = x**2 + y**2 + z**2
        try:
            c, _, _, _ = np.linalg.lstsq(A, b, rcond=None)
        except np.linalg.LinAlgError as e:
            raise RuntimeError(f"Least-squares sphere fit failed: {e}") from e
        xc, yc, zc = c[0] / 2, c[1] / 2, c[2] / 2
        radius = np.sqrt(c[3] + xc**2 + yc**2 + zc**2)
        self.center = (float(xc), float(yc), float(zc))
        return self.center[0], self.center[1], self.center[2], float(radius)


STRATEGIES = {"chief_ray": ChiefRayStrategy,
              "centroid_sphere": CentroidReferenceSphereStrategy,
              "best_fit_sphere": BestFitSphereStrategy}


def create_strategy(strategy_name, optic, distribution, **kwargs):
    """strategy.py:489-514."""
    cls = STRATEGIES.get(strategy_name)
    if cls is None:
        raise ValueError(f"Unknown wavefront strategy: {strategy_name}")
    return cls(optic, distribution, **kwargs)


def fit_and_remove_tilt(data, remove_piston=False, ridge=1e-12):
    """wavefront.py:97-143: weighted least-squares piston / tilt plane removed from the
    OPD. Chief-ray data carries the normal equations' sums from the wavefront kernel
    (data.sums): the 3 x 3 solve on the host and the plane subtracted on the device.
    Otherwise the reference's own NumPy expressions on host copies (a few hundred rays)."""
    if getattr(data, "sums", None) is None:
        x, y, w, opd = (t.cpu().numpy() for t in (data.pupil_x, data.pupil_y, data.intensity,
                                                   data.opd))
        one = np.ones_like(x)
        X = np.stack([one, x, y], axis=1)
        W = np.sqrt(w)[:, None]
        Xw = X * W
        yw = opd * np.sqrt(w)
        XT_X = np.matmul(Xw.T, Xw) + ridge * np.eye(3)
        XT_y = np.matmul(Xw.T, yw)
        coeffs = np.linalg.solve(XT_X, XT_y)
        if not remove_piston:
            coeffs = coeffs.copy()
            coeffs[0] = 0.0
        return torch.as_tensor(opd - X @ coeffs, device=data.opd.device)
    s = data.sums.cpu().numpy()
    _, _, w, wx, wy, wxx, wxy, wyy, wz, wxz, wyz = s
    XT_X = np.array([[w, wx, wy], [wx, wxx, wxy], [wy, wxy, wyy]]) + ridge * np.eye(3)
    coeffs = np.linalg.solve(XT_X, np.array([wz, wxz, wyz]))
    if not remove_piston:
        coeffs = coeffs.copy()
        coeffs[0] = 0.0
    return data.opd - (coeffs[0] + data.pupil_x * coeffs[1] + data.pupil_y * coeffs[2])


class Wavefront:
    """wavefront/wavefront.py:56-167 ("chief_ray", "centroid_sphere", "best_fit_sphere";
    keyword arguments go to the strategy, e.g. robust_trim_std)."""

    def __init__(self, optic, fields="all", wavelengths="all", num_rays=12,
                 distribution="hexapolar", strategy="chief_ray", remove_tilt=False,
                 **kwargs):
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
        self.strategy = create_strategy(strategy, optic, distribution, **kwargs)
        self.remove_tilt = remove_tilt
        self.data = {}
        for f in self.fields:
            for wl in self.wavelengths:
                data = self.strategy.compute_wavefront_data(tuple(f), wl)
                if remove_tilt:  # wavefront.py:164-165
                    data.opd = fit_and_remove_tilt(data)
                    data.sums = None
                self.data[(tuple(f), wl)] = data

    def get_data(self, field, wl):
        return self.data[(tuple(field), wl)]


class OPD(Wavefront):
    """wavefront/opd.py:19-157."""

    def __init__(self, optic, field, wavelength, num_rays=15, distribution="hexapolar",
                 strategy="chief_ray", remove_tilt=False, **kwargs):
        if isinstance(wavelength, str):
            if wavelength != "primary":
                raise ValueError("Invalid wavelength string. For a single wavelength, it "
                                 "must be 'primary'.")
            wavelength = optic.primary_wavelength
        super().__init__(optic, fields=[tuple(field)], wavelengths=[float(wavelength)],
                         num_rays=num_rays, distribution=distribution, strategy=strategy,
                         remove_tilt=remove_tilt, **kwargs)

    def rms(self):
        """opd.py:143-157 (from the wavefront kernel's sums unless the tilt was removed)."""
        data = self.get_data(self.fields[0], self.wavelengths[0])
        if getattr(data, "sums", None) is not None:
            cnt, s2 = (float(v) for v in data.sums[:2].cpu())
            if cnt == 0:
                raise ValueError("No valid rays with non-zero intensity for RMS calculation.")
            return torch.sqrt(data.sums[1] / data.sums[0])
        mask = data.intensity > 0
        if not bool(torch.any(mask)):
            raise ValueError("No valid rays with non-zero intensity for RMS calculation.")
        opd = data.opd[mask]
        return torch.sqrt(torch.mean(opd**2))
