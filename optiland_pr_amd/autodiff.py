"""Autograd through the MI355X trace: d(image rays) / d(Zernike coefficients).

Reference behaviour (config 5): under the torch backend the
coefficients of a ZernikePolynomialGeometry are torch tensors written in place by
ZernikeCoefficientVariable.update_value (optimization/variable/zernike_coeff.py:71-95);
Optic.trace builds a torch graph through every be.* op of the sequential trace,
including the unrolled Newton iterations (geometries/newton_raphson.py:137-166), and
TorchOptimizer.optimize (optimization/optimizer/torch/base.py:95-154) calls
loss.backward() on an operand such as RayOperand.rms_spot_size (operand/ray.py:300-340).

Here the forward is the fused HIP trace (ort_trace_pupil) and the backward is one
forward-mode derivative launch per chunk of coefficients (ort_trace_pupil_vjp): the rays
carry dual numbers through exactly the Newton update counts the primal ran, and the
kernel contracts them with the incoming cotangents on the device. No torch graph is
built over the per-ray arithmetic; torch only sees one autograd node per trace.

Scope: Zernike coefficients of ZernikePolynomialGeometry surfaces (the reference's
ZernikeCoefficientVariable). The image-surface record (surface_group.x[-1], ...) and
the returned rays are differentiable; records of other surfaces are not.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def zernike_parameters(optic):
    """[(traced-surface index, coefficient tensor)] for every Zernike surface whose
    coefficients are a torch tensor that requires grad (index into the lowered table)."""
    from .geometries import ZernikePolynomialGeometry
    from .surfaces import ObjectSurface

    if torch is None:
        return []
    sg = getattr(optic, "surface_group", optic)
    traced = [s for s in sg.surfaces if not isinstance(s, ObjectSurface)]
    out = []
    for si, s in enumerate(traced):
        g = s.geometry
        if isinstance(g, ZernikePolynomialGeometry):
            c = g.coefficients
            if torch.is_tensor(c) and c.requires_grad:
                out.append((si, c))
    return out


def wants_grad(optic):
    return torch is not None and torch.is_grad_enabled() and bool(zernike_parameters(optic))


def parameter_map(table, params):
    """zern_param[j] for every Zernike term row j of the lowered table: index into the
    concatenation of the parameter tensors, or -1."""
    zp = np.full(max(1, len(table.zern)), -1, dtype=np.int32)
    off = 0
    for si, c in params:
        row = table.surfaces[si]
        n = int(row["n_coef"])
        if n != c.numel():
            raise ValueError(f"surface {si}: {c.numel()} coefficients, lowered {n}")
        base = int(row["coef_off"])
        zp[base:base + n] = np.arange(off, off + n, dtype=np.int32)
        off += n
    return zp, off


class _TracePupilFn(torch.autograd.Function if torch is not None else object):
    """outputs (x, y, z, L, M, N, i, opd) of ort_trace_pupil as functions of the
    coefficient tensors."""

    @staticmethod
    def forward(ctx, plan, *coeffs):
        from .raytrace import RealRays, trace_pupil

        dl = plan["dlens"]
        out = RealRays.empty(plan["n"], plan["wavelength"], device=dl.device)
        trace_pupil(dl, plan["seg_dev"], plan["px"], plan["py"], out, plan["n"],
                    plan["seg_len"], plan["n"], keys=plan["keys"])
        sched = dl.last_schedule
        ctx.plan = plan
        ctx.set_materialize_grads(False)
        ctx.sched_dev = (None if sched is None else
                         torch.from_numpy(np.ascontiguousarray(sched.reshape(-1))).to(dl.device))
        ctx.shapes = [(c.numel(), c.shape, c.device, c.dtype) for c in coeffs]
        outs = tuple(getattr(out, a) for a in _abi.RAY_FIELDS)
        return outs

    @staticmethod
    def backward(ctx, *grads):
        plan = ctx.plan
        dl = plan["dlens"]
        n_param = plan["n_param"]
        g = torch.zeros(n_param, dtype=torch.float64, device=dl.device)
        cot = []
        for gr in grads:
            cot.append(None if gr is None else gr.to(torch.float64).contiguous())
        vjp(dl, plan["seg_dev"], plan["px"], plan["py"], plan["n"], plan["seg_len"],
            ctx.sched_dev, plan["zparam_dev"], n_param, cot, g)
        res = [None]
        off = 0
        for numel, shape, dev, dtype in ctx.shapes:
            res.append(g[off:off + numel].reshape(shape).to(device=dev, dtype=dtype))
            off += numel
        return tuple(res)


def vjp(dlens, seg_dev, px, py, n, seg_len, sched_dev, zparam_dev, n_param, cot, grad,
        pupil_per_ray=False):
    """grad += J^T cot through ort_trace_pupil_vjp. cot: 8 device tensors or None."""
    from .raytrace import _ptr, _stream_handle

    lib = _native.load()
    n_seg = seg_dev.numel() // _abi.SEGMENT.itemsize
    batch = _native.ort_batch(n, seg_len, n, n_seg, int(pupil_per_ray), seg_dev.data_ptr())
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, 0,
                              None if sched_dev is None else sched_dev.data_ptr())
    cot_c = _native.ort_rays(*(0 if c is None else c.data_ptr() for c in cot))
    rc = lib.ort_trace_pupil_vjp(C.byref(dlens.c), _ptr(px), _ptr(py), C.byref(batch),
                                 C.byref(opt), _ptr(zparam_dev), int(n_param),
                                 C.byref(cot_c), _ptr(grad), _stream_handle())
    _native.check(rc, "ort_trace_pupil_vjp")


def trace_pupil_grad(optic, dlens, seg_dev, px, py, n, seg_len, wavelength, keys):
    """Differentiable fused trace: returns the 8 output tensors connected to the
    coefficient tensors of zernike_parameters(optic)."""
    params = zernike_parameters(optic)
    zp, n_param = parameter_map(dlens.table, params)
    plan = dict(dlens=dlens, seg_dev=seg_dev, px=px, py=py, n=n, seg_len=seg_len,
                wavelength=wavelength, keys=keys, n_param=n_param,
                zparam_dev=torch.from_numpy(zp).to(dlens.device))
    return _TracePupilFn.apply(plan, *[c for _, c in params])
