"""Host (CPU) side of the trace core: the CPU dispatch key of torch.ops.ort.trace_sequential
and of its VJP (include/optiland_host.h, liboptiland_host.so).

The reference runs its torch backend on the CPU by default (backend/torch_backend.py:66-77)
and its own tests force it there (tests/conftest.py:5-19), so `SurfaceGroup.trace`
(surfaces/surface_group.py:232-244) reaches the op with CPU tensors as often as with device
ones. A HostLens is the lowered lens in host memory (the same LensTable bytes a DeviceLens
uploads); the calls below hand host pointers to the C ABI of the host library, which runs
the GPU kernels' per-ray source compiled with g++ (csrc/ort_host.cpp). This is not a
fallback of the device path: device tensors never come here, and host tensors never reach
the HIP library.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _abi, _native


def _p(a):
    """Host address of a numpy array or CPU tensor (None: NULL)."""
    if a is None:
        return None
    if torch.is_tensor(a):
        return a.data_ptr()
    return a.ctypes.data


class HostLens:
    """A LensTable held in host memory for liboptiland_host.so (the counterpart of
    raytrace.DeviceLens for CPU tensors)."""

    def __init__(self, table):
        self.table = table
        self.device = torch.device("cpu")
        keep = []

        def arr(a, dtype=None):
            a = np.ascontiguousarray(a if dtype is None else np.asarray(a, dtype=dtype))
            keep.append(a)
            return a

        surfaces = arr(table.surfaces)
        cs_ops = arr(table.cs_ops)
        coef = arr(table.coef, np.float64)
        zern = arr(table.zern)
        n_tab = arr(table.n_tab, np.float64)
        alpha_tab = arr(table.alpha_tab, np.float64)
        optics = arr(table.optics)
        mats = arr(table.mat_table if table.mat_table is not None else np.zeros(1, _abi.MATERIAL))
        lambdas = arr(np.asarray(table.wavelengths, dtype=np.float64))
        mask = 0
        for g in np.unique(table.surfaces["geometry"]):
            mask |= 1 << int(g)
        self.geometry_mask = mask
        self.c = _native.ort_lens(
            _p(surfaces), _p(cs_ops), _p(coef), _p(zern), _p(n_tab), _p(alpha_tab), _p(optics),
            table.n_surfaces, len(table.wavelengths), table.n_tab.shape[1], table.final_mat,
            mask, table.interaction_mask, table.final_thickness, _p(mats), _p(lambdas),
            table.frame_flags)
        self._keep = keep
        # the same nine tables as torch CPU tensors sharing these arrays' memory (the lens as
        # the torch ops take it: ops.lens_args)
        self._tensors = [torch.from_numpy(a.view(np.uint8) if a.dtype.fields else a)
                         for a in (surfaces, cs_ops, coef, zern, n_tab.reshape(-1),
                                   alpha_tab.reshape(-1), optics.reshape(-1), mats, lambdas)]
        self.newton = table.newton_surfaces
        self.last_schedule = None
        self.last_schedule_dev = None
        self.last_schedule_private = False
        self._resident: dict = {}

    def lens_tensors(self):
        """[surfaces, cs_ops, coef, zern, n_tab, alpha_tab, optics, materials, wavelengths]
        as CPU tensors (structured tables as their bytes)."""
        return self._tensors

    def resident(self, slot, arr):
        """A CPU tensor copy of a small host table, reused while its bytes are unchanged
        (DeviceLens.resident's counterpart)."""
        a = np.ascontiguousarray(arr)
        raw = a.tobytes()
        hit = self._resident.get(slot)
        if hit is not None and hit[0] == raw and hit[1] == a.dtype:
            return hit[2]
        t = torch.from_numpy(a.copy())
        self._resident[slot] = (raw, a.dtype, t)
        return t


def _rays_c(ts):
    return _native.ort_rays(*(0 if t is None else t.data_ptr() for t in ts))


def trace_sequential(hl: HostLens, rays_in, w, per_ray_w, start_surface, rec):
    """ort_host_trace_sequential of resident CPU rays (8 contiguous float64 tensors):
    returns the 8 output tensors and the Newton update counts [S] (int32 tensor) the
    reference's stop rule made."""
    from .raytrace import _raise_status_value

    lib = _native.load_host()
    n = rays_in[0].numel()
    outs = [torch.empty(n, dtype=torch.float64) for _ in range(8)]
    batch = _native.ort_batch(n, max(n, 1), max(n, 1), 0, 0, None)
    w_keep = None
    if per_ray_w:
        w_keep = w.detach().to(dtype=torch.float64).reshape(-1)
        w_keep = w_keep.expand(n).contiguous() if w_keep.numel() == 1 else w_keep.contiguous()
        if w_keep.numel() != n:
            raise ValueError("rays.w must hold one wavelength per ray")
        mt = hl.table.mat_table
        if mt is not None and np.any(mt["kind"] == _abi.MAT_ABBE):
            # abbe.py:47-48 raises before any n is used
            if bool(((w_keep < 0.380) | (w_keep > 0.750)).any()):
                raise ValueError("Wavelength out of range for this model.")
        batch.w = w_keep.data_ptr()
    S = hl.table.n_surfaces
    updates = torch.zeros(S, dtype=torch.int32)
    status = np.zeros(1, dtype=np.int32)
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, int(start_surface), None)
    rin_c, out_c = _rays_c(rays_in), _rays_c(outs)
    rc = lib.ort_host_trace_sequential(C.byref(hl.c), C.byref(rin_c), C.byref(out_c),
                                       C.byref(batch), C.byref(opt), _p(rec),
                                       _p(updates), _p(status))
    _native.check(rc, "ort_host_trace_sequential")
    _raise_status_value(int(status[0]))
    return outs, updates


def trace_sequential_vjp(hl: HostLens, rays_in, w, per_ray_w, start_surface, sched, tabs,
                         need, n_param, mode, cot, rec_cot, rec, grad, gin):
    """ort_host_trace_sequential_vjp: grad += J^T cot, gin = input-ray cotangents.
    tabs: (zern_param, surf_tangent, final_tangent) CPU tensors or None."""
    lib = _native.load_host()
    n = rays_in[0].numel()
    batch = _native.ort_batch(n, max(n, 1), max(n, 1), 0, 0, None)
    w_keep = None
    if per_ray_w:
        w_keep = w.to(dtype=torch.float64).reshape(-1)
        w_keep = w_keep.expand(n).contiguous() if w_keep.numel() == 1 else w_keep.contiguous()
        batch.w = w_keep.data_ptr()
    sched_c = sched if sched is not None and sched.numel() else None
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, int(start_surface), _p(sched_c))
    zp, st, ft = tabs
    params = _native.ort_vjp_params(int(n_param), int(mode), _p(zp), _p(st), _p(ft),
                                    0 if zp is None else int(zp.numel()), 0, None, 0, _p(need))
    from .ops import mono_slot_count

    params.n_mono = mono_slot_count(hl.table, None if zp is None else zp.numpy())
    rc = lib.ort_host_trace_sequential_vjp(
        C.byref(hl.c), C.byref(_rays_c(rays_in)), C.byref(batch), C.byref(opt),
        C.byref(params), C.byref(_rays_c(cot)), _p(rec_cot),
        _p(rec if rec_cot is not None else None), _p(grad),
        C.byref(_rays_c(gin if gin is not None else [None] * 8)))
    _native.check(rc, "ort_host_trace_sequential_vjp")
    del w_keep


def trace_pupil(hl: HostLens, seg, px, py, n, seg_len, pupil_per_ray, apod=None):
    """ort_host_trace_pupil: rays generated from the pupil samples by the segments (SEGMENT
    records as a uint8 CPU tensor) and traced as one reference trace call (one Newton
    group); returns the 8 output tensors and the update counts [S] (int32)."""
    from .raytrace import _raise_status_value

    lib = _native.load_host()
    n_seg = seg.numel() // _abi.SEGMENT.itemsize
    outs = [torch.empty(n, dtype=torch.float64) for _ in range(8)]
    # one Newton group: the whole call, as RealRayTracer.trace traces every field of a
    # wavelength in one SurfaceGroup.trace (real_ray_tracer.py:37-97)
    batch = _native.ort_batch(n, max(seg_len, 1), max(n, 1), n_seg, int(pupil_per_ray),
                              seg.data_ptr())
    batch.apod = None if apod is None else apod.data_ptr()
    S = hl.table.n_surfaces
    n_groups = 1 if n else 0
    updates = torch.zeros(max(1, n_groups) * S, dtype=torch.int32)
    status = np.zeros(1, dtype=np.int32)
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, 0, None)
    out_c = _rays_c(outs)
    rc = lib.ort_host_trace_pupil(C.byref(hl.c), _p(px), _p(py), C.byref(out_c), C.byref(batch),
                                  C.byref(opt), _p(updates), _p(status))
    _native.check(rc, "ort_host_trace_pupil")
    _raise_status_value(int(status[0]))
    return outs, updates[:n_groups * S]


def trace_pupil_vjp(hl: HostLens, seg, px, py, n, seg_len, pupil_per_ray, sched, tabs, need,
                    n_param, mode, cot, grad, apod=None, rms=None):
    """ort_host_trace_pupil_vjp: grad = J^T cot of the pupil trace (grad overwritten).
    rms: (stats[5], g[1]) of an rms spot size of the outputs, folded into the x, y
    cotangents (ort_vjp_params.rms_stats / rms_grad; the adjoint mode)."""
    from .ops import mono_slot_count

    lib = _native.load_host()
    n_seg = seg.numel() // _abi.SEGMENT.itemsize
    batch = _native.ort_batch(n, max(seg_len, 1), max(n, 1), n_seg, int(pupil_per_ray),
                              seg.data_ptr())
    batch.apod = None if apod is None else apod.data_ptr()
    sched_c = sched if sched is not None and sched.numel() else None
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, 0, _p(sched_c))
    zp, st, ft = tabs
    params = _native.ort_vjp_params(int(n_param), int(mode), _p(zp), _p(st), _p(ft),
                                    0 if zp is None else int(zp.numel()), 1, None, 0, _p(need))
    params.n_mono = mono_slot_count(hl.table, None if zp is None else zp.numpy())
    if rms is not None:
        params.rms_stats, params.rms_grad = _p(rms[0]), _p(rms[1])
    rc = lib.ort_host_trace_pupil_vjp(C.byref(hl.c), _p(px), _p(py), C.byref(batch), C.byref(opt),
                                      C.byref(params), C.byref(_rays_c(cot)), _p(grad))
    _native.check(rc, "ort_host_trace_pupil_vjp")


def rms_spot(x, y):
    """ort_host_rms_spot: (rms scalar, stats[5]) of contiguous float64 CPU tensors."""
    lib = _native.load_host()
    stats = torch.empty(5, dtype=torch.float64)
    rms = torch.empty((), dtype=torch.float64)
    rc = lib.ort_host_rms_spot(_p(x), _p(y), x.numel(), _p(stats), _p(rms))
    _native.check(rc, "ort_host_rms_spot")
    return rms, stats


def rms_spot_vjp(x, y, stats, g):
    lib = _native.load_host()
    gx, gy = torch.empty_like(x), torch.empty_like(y)
    rc = lib.ort_host_rms_spot_vjp(_p(x), _p(y), x.numel(), _p(stats), _p(g), _p(gx), _p(gy))
    _native.check(rc, "ort_host_rms_spot_vjp")
    return gx, gy
