"""Autograd through the MI355X trace: d(image rays) / d(Zernike coefficients).

Reference behaviour (config 5): under the torch backend the
coefficients of a ZernikePolynomialGeometry are torch tensors written in place by
ZernikeCoefficientVariable.update_value (optimization/variable/zernike_coeff.py:71-95);
Optic.trace builds a torch graph through every be.* op of the sequential trace,
including the unrolled Newton iterations (geometries/newton_raphson.py:137-166), and
TorchOptimizer.optimize (optimization/optimizer/torch/base.py:95-154) calls
loss.backward() on an operand such as RayOperand.rms_spot_size (operand/ray.py:300-340).

Here the forward is the fused HIP trace (ort_trace_pupil) and the backward is
ort_trace_pupil_vjp, in one of two modes (vjp_mode):
  adjoint   one reverse-mode launch whatever the number of parameters: the primal
            re-traced with a tape of per-surface states, then the adjoint of each
            surface step from the image back (ort_adjoint.h); intersection distances are
            differentiated through their implicit equation;
  unrolled  one forward-mode launch per chunk of 4 parameters: dual numbers through
            exactly the Newton update counts the primal ran (the derivative of the
            unrolled iteration, bit-for-bit the reference's semantics); used for
            standard / noll Zernike surfaces, whose Newton slope is not the sag's
            derivative (see vjp_mode).
No torch graph is built over the per-ray arithmetic; torch only sees one autograd node
per trace.

Parameters: Zernike coefficients, surface radius and conic (geometry.radius / .k) and
thickness (Optic.set_thickness moves the later vertices), i.e. what the reference's
ZernikeCoefficientVariable / RadiusVariable / ConicVariable / ThicknessVariable write.
As in the reference, ray generation (EPL, EPD, ray origins) is not differentiated: its
paraxial inputs are rebuilt from detached copies there (surface_group.py:143-153,
backend be.array). The image-surface record (surface_group.x[-1], ...) and the returned
rays are differentiable; records of other surfaces are not.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def _is_leaf_param(v):
    return torch is not None and torch.is_tensor(v) and v.requires_grad


def zernike_parameters(optic):
    """[(traced-surface index, coefficient tensor)] for every Zernike surface whose
    coefficients are a torch tensor that requires grad (index into the lowered table)."""
    return [(si, t) for kind, si, t in parameters(optic) if kind == "zernike"]


def parameters(optic):
    """[(kind, traced-surface index, tensor)]: every lens parameter that is a torch tensor
    requiring grad -- what the reference's optimisation variables write
    (variable/zernike_coeff.py:71-95, radius.py, conic.py, thickness.py through
    optic_updater.py:37-86): Zernike coefficients ("zernike"), geometry.radius
    ("radius"), geometry.k ("conic"), surface.thickness ("thickness")."""
    from .geometries import ZernikePolynomialGeometry
    from .surfaces import ObjectSurface

    if torch is None:
        return []
    sg = getattr(optic, "surface_group", optic)
    out = []
    traced = 0
    for s in sg.surfaces:
        if isinstance(s, ObjectSurface):
            if _is_leaf_param(getattr(s, "thickness", None)):
                raise NotImplementedError("the object distance is not differentiated "
                                          "(ray generation is not part of the backward)")
            continue
        g = s.geometry
        if isinstance(g, ZernikePolynomialGeometry) and _is_leaf_param(g.coefficients):
            out.append(("zernike", traced, g.coefficients))
        if _is_leaf_param(getattr(g, "radius", None)):
            out.append(("radius", traced, g.radius))
        if _is_leaf_param(getattr(g, "k", None)):
            out.append(("conic", traced, g.k))
        if _is_leaf_param(getattr(s, "thickness", None)):
            out.append(("thickness", traced, s.thickness))
        traced += 1
    return out


def wants_grad(optic):
    return torch is not None and torch.is_grad_enabled() and bool(parameters(optic))


def parameter_map(table, params):
    """zern_param[j] for every Zernike term row j of the lowered table: index into the
    concatenation of the (Zernike) parameter tensors, or -1."""
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


def vjp_mode(table, sched=None):
    """ORT_VJP_ADJOINT (one reverse-mode pass) unless the lens has more parameter slots
    than the adjoint holds (ORT_VJP_ADJOINT_MAX_SLOTS), or a surface whose Newton slope is
    not its sag's derivative (SURF_SLOPE_INEXACT: the standard / noll Zernike normal omits
    the normalisation constant, zernike.py:163-231, so the unrolled iteration converges
    linearly) ran more updates than the adjoint tape keeps (ADJ_HIST): the forward-mode
    ORT_VJP_UNROLLED then differentiates every update. With U <= ADJ_HIST the tape holds
    every iterate and the adjoint is the unrolled derivative on any surface.

    sched: the verified Newton schedule ([n_groups][S] update counts, host array or
    tensor) when known, else None -- then the adjoint runs, and a schedule the device
    raised past ADJ_HIST on such a surface poisons the gradient with NaN rather than
    truncating it (ort_sweep.h). ORT_VJP_MODE=unrolled|adjoint overrides (A/B checks)."""
    if has_interactions(table):
        return _abi.VJP_UNROLLED  # thin-lens / phase / grating: forward mode only (vjp_ray)
    env = os.environ.get("ORT_VJP_MODE", "").lower()
    if env in ("unrolled", "adjoint"):
        return _abi.VJP_UNROLLED if env == "unrolled" else _abi.VJP_ADJOINT
    from .ops import mono_slot_count

    z = table.zern
    if 3 * table.n_surfaces + len(z) + 1 + mono_slot_count(table, z) > _abi.VJP_ADJOINT_MAX_SLOTS:
        return _abi.VJP_UNROLLED  # more parameter slots than the adjoint's LDS partials hold
    if sched is not None and inexact_updates(table, sched) > _abi.ADJ_HIST:
        return _abi.VJP_UNROLLED
    return _abi.VJP_ADJOINT


def has_interactions(table):
    """The lens has thin-lens, phase or grating surfaces: its gradient is the forward-mode
    VJP's (their interactions are carried in duals by vjp_ray; the adjoint has no reverse
    for them)."""
    return bool(table.interaction_mask & ~(1 << _abi.IA_REFRACT_REFLECT))


def inexact_surfaces(table):
    """bool [S]: the surfaces whose Newton slope is not the sag's derivative"""
    return (table.surfaces["flags"] & _abi.SURF_SLOPE_INEXACT) != 0


def inexact_updates(table, sched):
    """The most Newton updates any SURF_SLOPE_INEXACT surface ran under `sched` (0: none)"""
    mask = inexact_surfaces(table)
    if not mask.any() or sched is None:
        return 0
    if torch is not None and torch.is_tensor(sched):
        sched = sched.detach().cpu().numpy()
    s = np.asarray(sched).reshape(-1, table.n_surfaces)
    return int(s[:, mask].max()) if s.size else 0


def schedule_for_mode(table, sched_t, hint=None):
    """The schedule vjp_mode should see for a backward: nothing to read when the lens has
    no SURF_SLOPE_INEXACT surface; else the saved schedule tensor (a host tensor, or a
    device one copied back -- one small synchronising read, only for such lenses), or
    while a HIP graph is being captured (no synchronisation allowed) `hint`, the host's
    cached schedule the captured trace starts from."""
    if not inexact_surfaces(table).any():
        return None
    if sched_t is None or sched_t.numel() == 0:
        return hint
    if sched_t.device.type == "cpu":
        return sched_t
    if torch.cuda.is_current_stream_capturing():
        return hint
    return sched_t.cpu()


_WORKSPACE = {}

# the forward of a differentiable Newton-lens trace writes the adjoint tape (F_TAPE), so
# the backward skips its re-trace; ORT_TAPED_FORWARD=0 keeps the re-trace (A/B checks)
TAPED_FORWARD = os.environ.get("ORT_TAPED_FORWARD", "1") != "0"

# Measurement hook (bench.py config 5): when a list, every vjp() appends a pair of
# timing events recorded on the launch stream around ort_trace_pupil_vjp
VJP_EVENTS = None


def _workspace(device, nbytes):
    """Device scratch for the adjoint VJP, grown on demand and reused (per device)."""
    ws = _WORKSPACE.get(device)
    if ws is None or ws.numel() < nbytes:
        _WORKSPACE.pop(device, None)
        ws = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
        _WORKSPACE[device] = ws
    return ws


def vjp(dlens, seg_dev, px, py, n, seg_len, sched_dev, tables, n_param, cot, grad,
        pupil_per_ray=False, mode=None, tape=None, primal=None, overwrite=False, rms=None):
    """grad += J^T cot through ort_trace_pupil_vjp (overwrite: grad = J^T cot, grad need
    not be initialised). tables: device tensors (zern_param, surf_tangent,
    final_tangent), each possibly None; cot: 8 tensors / None; rms: (stats[5], g[1]) of an
    rms spot size of the outputs, folded into the x, y cotangent load (adjoint mode)."""
    from .raytrace import _ptr, _stream_handle

    if np.any(dlens.table.surfaces["geometry"] == _abi.GEOM_GRID_SAG):
        raise NotImplementedError("autograd through grid-sag surfaces is not implemented by "
                                  "the trace core (no derivative kernels)")
    mode = vjp_mode(dlens.table) if mode is None else mode
    if has_interactions(dlens.table) and mode != _abi.VJP_UNROLLED:
        raise NotImplementedError("thin-lens, phase and grating surfaces are differentiated "
                                  "by the forward-mode VJP only (ORT_VJP_UNROLLED)")
    lib = _native.load()
    n_seg = seg_dev.numel() // _abi.SEGMENT.itemsize
    batch = _native.ort_batch(n, seg_len, n, n_seg, int(pupil_per_ray), seg_dev.data_ptr())
    batch.apod = None if dlens.apod is None else dlens.apod.data_ptr()
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, 0,
                              None if sched_dev is None else sched_dev.data_ptr())
    zp, st, ft = tables[:3]
    need = tables[3] if len(tables) > 3 else None  # ort_vjp_params.slot_need (resident)
    params = _native.ort_vjp_params(int(n_param), int(mode), _ptr(zp).value, _ptr(st).value,
                                    _ptr(ft).value, 0 if zp is None else int(zp.numel()),
                                    int(bool(overwrite)), None, 0, _ptr(need).value)
    if mode == _abi.VJP_ADJOINT:
        from .ops import mono_slot_count

        params.n_mono = mono_slot_count(dlens.table, zp)
    if tape is not None and mode == _abi.VJP_ADJOINT:
        # the forward wrote the tape (ort_options.tape): reverse sweep only, the final
        # state read from the forward's outputs
        params.tape = tape.data_ptr()
        params.primal = _native.ort_rays(*(t.data_ptr() for t in primal))
    if rms is not None:
        if mode != _abi.VJP_ADJOINT:
            raise ValueError("vjp: the rms cotangent fold is the adjoint mode's")
        params.rms_stats, params.rms_grad = rms[0].data_ptr(), rms[1].data_ptr()
    # both modes take a workspace (ABI v15: the unrolled mode's block partials)
    size = lib.ort_vjp_workspace_size(C.byref(dlens.c), C.byref(batch), C.byref(params))
    _native.check(int(size) if size < 0 else 0, "ort_vjp_workspace_size")
    ws = _workspace(grad.device, size)
    params.workspace = ws.data_ptr()
    params.workspace_size = ws.numel()
    cot_c = _native.ort_rays(*(0 if c is None else c.data_ptr() for c in cot))
    timer = VJP_EVENTS
    if timer is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record(torch.cuda.current_stream())
    rc = lib.ort_trace_pupil_vjp(C.byref(dlens.c), _ptr(px), _ptr(py), C.byref(batch),
                                 C.byref(opt), C.byref(params), C.byref(cot_c), _ptr(grad),
                                 _stream_handle())
    _native.check(rc, "ort_trace_pupil_vjp")
    if timer is not None:
        ev[1].record(torch.cuda.current_stream())
        timer.append(ev)


def trace_pupil_grad(optic, dlens, seg_dev, px, py, n, seg_len, wavelength, keys,
                     newton_mode="reference", want_rms=False):
    """Differentiable fused trace: returns the 8 output tensors connected to the
    parameter tensors of parameters(optic), through the torch.ops.ort.trace_pupil custom
    op (ops.py) whose autograd formula is ort_trace_pupil_vjp, and a 9th: the rms spot size
    of the final points (a 0-dim tensor) when want_rms and the forward is taped with one
    wavelength row (F_RMS), else an empty tensor."""
    from . import ops

    params = parameters(optic)
    plan = ops.PupilPlan(dlens, seg_dev, px, py, n, seg_len, keys, newton_mode=newton_mode)
    # adjoint-mode backward of a Newton lens: let the forward write the tape
    plan.want_tape = (bool(params) and bool(dlens.newton) and TAPED_FORWARD
                      and vjp_mode(dlens.table, dlens.cached_schedule(keys)) == _abi.VJP_ADJOINT
                      and not dlens.table.interaction_mask & ~(1 << _abi.IA_REFRACT_REFLECT)
                      and not np.any(dlens.table.surfaces["geometry"] == _abi.GEOM_GRID_SAG))
    plan.want_rms = bool(want_rms and plan.want_tape and len(dlens.table.wavelengths) == 1)
    lens, meta, ft, key = ops.lens_args(dlens)
    seg, apod, pmeta, pkey = ops.plan_args(plan)
    outs = torch.ops.ort.trace_pupil(lens, meta, ft, key, seg, apod, px, py,
                                     [t for _, _, t in params],
                                     ops.encode_spec([(k, si) for k, si, _ in params]), pmeta,
                                     pkey)
    return (*outs[:8], outs[10])


class CapturedStep:
    """One optimisation step -- `loss = loss_fn(); loss.backward(); optimizer.step()` -- run
    as ONE HIP graph replay (the driver loop of optimization/optimizer/torch/base.py:
    95-154 without its per-step host work). Every op on the path is free of host
    synchronisation once warm: the coefficient patch, the taped trace with
    newton_mode="device" (its verify-and-re-trace rounds are captured as launches), the
    rms_spot reduction, the adjoint VJP and a capturable optimizer
    (`torch.optim.Adam(..., capturable=True)`).

    The first call warms the Newton schedules, workspaces and caches with `warmup` eager
    steps on a side stream, checks their pending Newton flags, and captures; every call
    (the first included) then replays the graph once. `loss` is the graph's static loss
    tensor (read it after a synchronisation). `check()` reads the last replay's Newton
    flags of `lenses` (one synchronising copy) and raises as `raytrace.check_pending`
    would: call it at the end of a run or every few steps.

    A replay traces the lens as it was lowered at capture, reading the device-resident
    parameter tensors (the optimizer's leaves) afresh each time; any other edit of the
    lens (a setter, an in-place array edit, a new surface) needs a new CapturedStep. The
    eager path (`eager()`) re-lowers the lens on every call and sees every edit."""

    def __init__(self, loss_fn, optimizer, lenses=(), warmup=3):
        self.loss_fn, self.opt, self.lenses, self.warmup = loss_fn, optimizer, list(lenses), warmup
        self.graph = None
        self.loss = None

    def eager(self):
        self.opt.zero_grad()
        loss = self.loss_fn()
        loss.backward()
        self.opt.step()
        return loss

    def _capture(self):
        import torch

        from . import raytrace

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        loss = None
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                loss = self.eager()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        raytrace.check_all_pending()  # the warm-up's Newton flags, before the capture
        self.opt.zero_grad(set_to_none=True)
        # the backward's seed d loss / d loss = 1 as a static tensor made before the capture
        # (loss.backward() would fill a fresh one inside every replay: one launch per step)
        seed = None if loss is None else torch.ones_like(loss)
        # drop the last warm-up loss before capturing: its autograd graph holds the leaves'
        # AccumulateGrad nodes, which remember the warm-up stream, and the captured backward
        # would reuse them on the capture stream (torch warns that the AccumulateGrad
        # node's stream does not match). Freed here, the capture builds its own nodes; the
        # capture also runs on the warm-up's stream.
        del loss
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            loss = self.loss_fn()
            loss.backward(seed)
            self.opt.step()
        torch.cuda.current_stream().wait_stream(side)
        self.graph, self.loss = g, loss.detach()
        del loss

    def __call__(self):
        if self.graph is None:
            self._capture()
        self.graph.replay()
        return self.loss

    def check(self):
        from . import raytrace

        for lens in self.lenses:
            for dl in getattr(lens, "_lowered", {}).values():
                raytrace.check_graph_flags(dl)
