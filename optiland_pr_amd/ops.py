"""PyTorch custom ops over the C ABI: ``torch.ops.ort.trace_sequential`` and
``torch.ops.ort.trace_pupil`` (SURVEY.md 8b "Torch custom op").

The reference differentiates a trace by running every ``be.*`` primitive of
``SurfaceGroup.trace`` (surfaces/surface_group.py:232-244) under torch autograd
(backend/torch_backend.py:45-148, driven by optimization/optimizer/torch/base.py:116-131).
Here the whole trace is ONE dispatcher op whose CUDA (HIP) kernel is the fused trace
(ort_trace_sequential / ort_trace_pupil) and whose autograd formula is the adjoint (or
forward-mode) VJP of the trace core (ort_trace_sequential_vjp / ort_trace_pupil_vjp), so
autograd sees one node per trace call:

  ort::trace_sequential(lens, rays[8], w, params, spec, start_surface, per_ray_w)
      -> (x, y, z, L, M, N, i, opd, rec, sched)
      resident rays in (SurfaceGroup.trace, the drop-in seam); rec = every traced
      surface's record [S][8][n] (standard_surface.py:266-286); differentiable w.r.t. the
      input rays, the record buffer's cotangents included, and the lens parameters in
      `params`.
  ort::trace_pupil(plan, px, py, params, spec) -> (x, y, z, L, M, N, i, opd, sched)
      rays generated from pupil samples in the same launch (Optic.trace's fused path,
      raytrace/real_ray_tracer.py:37-97); differentiable w.r.t. the lens parameters.

``lens`` / ``plan`` are integer handles of host objects (the uploaded lens tables, the
pupil samples and segment descriptors): the dispatcher passes ints, and the tables they
name are a few KB that the kernels read from HBM. ``params`` are the lens-parameter
tensors that require grad and ``spec`` says which lens value each one is, as flattened
(kind, traced-surface index) pairs with kind in SPEC_KINDS: the forward ignores their
values (the lowered lens already holds them), the backward returns d loss / d each.

ort::trace_sequential has two kernels, one per dispatch key: CUDA (HIP) runs
the fused GPU trace on a DeviceLens handle, CPU runs the host build of the same per-ray
source (host.py, liboptiland_host.so, include/optiland_host.h) on a HostLens handle, with
its VJP on the host too. Neither falls back to the other: the dispatcher picks the kernel
by the tensors' device, and a handle of the other kind raises. trace_pupil and rms_spot
are CUDA-only.
"""

from __future__ import annotations

import ctypes as C
import weakref

import numpy as np
import torch

from . import _abi, _native

SPEC_KINDS = ("zernike", "radius", "conic", "thickness", "vertex")

# handle -> host object (DeviceLens / pupil plan); weak, so a handle never keeps a lens
# alive (the autograd context holds the object itself for the backward)
_HANDLES: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()


def handle(obj) -> int:
    """Integer handle of a host object for the ops' `lens` / `plan` argument."""
    h = id(obj)
    _HANDLES[h] = obj
    return h


def _lookup(h):
    obj = _HANDLES.get(int(h))
    if obj is None:
        raise RuntimeError(f"ort op: stale handle {h} (the lens / plan object was freed)")
    return obj


class PupilPlan:
    """Everything ort::trace_pupil needs besides the parameter tensors."""

    def __init__(self, dlens, seg_dev, px, py, n, seg_len, keys=(), pupil_per_ray=False,
                 newton_mode="reference"):
        self.dlens = dlens
        self.seg_dev = seg_dev
        self.px = px
        self.py = py
        self.n = int(n)
        self.seg_len = int(seg_len)
        self.keys = list(keys)
        self.pupil_per_ray = bool(pupil_per_ray)
        self.newton_mode = newton_mode
        self.want_tape = False  # set by the caller when the backward is an adjoint sweep
        self.tape = None


def _spec_pairs(spec):
    if len(spec) % 2:
        raise ValueError("spec holds (kind, surface) pairs")
    return [(SPEC_KINDS[int(spec[i])], int(spec[i + 1])) for i in range(0, len(spec), 2)]


def encode_spec(pairs):
    """[(kind name, traced-surface index)] -> the flat int list the ops take."""
    out = []
    for kind, si in pairs:
        out += [SPEC_KINDS.index(kind), int(si)]
    return out


def tangent_tables(table, pairs, params):
    """ort_vjp_params tables for the parameter tensors: (zern_param, surf_tangent,
    final_tangent, n_param) -- numpy arrays or None. "vertex" is the vertex z of one
    surface (its coordinate system's z, coordinate_system.py:73-107); "thickness" moves
    every later vertex (optic_updater.py set_thickness)."""
    S = table.n_surfaces
    n_param = sum(int(t.numel()) for t in params)
    zp = surf = final = None
    off = 0
    for (kind, si), t in zip(pairs, params, strict=True):
        n = int(t.numel())
        row = table.surfaces[si]
        if kind == "zernike":
            if int(row["geometry"]) != _abi.GEOM_ZERNIKE:
                raise ValueError(f"surface {si}: Zernike coefficients of a non-Zernike surface")
            if zp is None:
                zp = np.full(max(1, len(table.zern)), -1, dtype=np.int32)
            if n != int(row["n_coef"]):
                raise ValueError(f"surface {si}: {n} coefficients, lowered {int(row['n_coef'])}")
            base = int(row["coef_off"])
            zp[base:base + n] = np.arange(off, off + n, dtype=np.int32)
        else:
            if n != 1:
                raise ValueError(f"surface {si}: {kind} must be a scalar tensor")
            if surf is None:
                surf = np.zeros((n_param, S, 3), dtype=np.float64)
            g = int(row["geometry"])
            if kind in ("radius", "conic"):
                if g in (_abi.GEOM_PLANE, _abi.GEOM_BICONIC, _abi.GEOM_TOROIDAL, _abi.GEOM_GRID_SAG):
                    raise NotImplementedError(f"surface {si}: {kind} of this geometry is not a "
                                              "differentiable parameter of the trace core")
                surf[off, si, 0 if kind == "radius" else 1] = 1.0
            elif kind == "vertex":
                surf[off, si, 2] = 1.0
            else:  # thickness after surface si moves every later vertex
                surf[off, si + 1:, 2] = 1.0
                if si == S - 1:  # the image surface's thickness: the final propagate
                    if final is None:
                        final = np.zeros(n_param, dtype=np.float64)
                    final[off] = 1.0
        off += n
    return zp, surf, final, n_param


def slot_need(table, zp, surf, final):
    """ort_vjp_params.slot_need of the tangent tables: nonzero for every slot (radius,
    conic, vertex z of each surface; each Zernike term; the final thickness) some
    parameter depends on. Host NumPy, kept resident with the tables."""
    S = table.n_surfaces
    n_z = 0 if zp is None else len(zp)
    need = np.zeros(3 * S + n_z + 1, dtype=np.int32)
    if surf is not None:
        need[:3 * S] = np.any(surf != 0.0, axis=0).reshape(-1)
    if zp is not None:
        need[3 * S:3 * S + n_z] = zp >= 0
    if final is not None:
        need[-1] = np.any(final != 0.0)
    return need


def tape_doubles(dl, n):
    """Doubles of the adjoint tape of an n-ray trace of this lens (ort_vjp_tape_size)."""
    lib = _native.load()
    batch = _native.ort_batch(n, max(n, 1), max(n, 1), 0, 0, None)
    size = int(lib.ort_vjp_tape_size(C.byref(dl.c), C.byref(batch)))
    _native.check(size if size < 0 else 0, "ort_vjp_tape_size")
    return size // 8


def _check_differentiable(table):
    if np.any(table.surfaces["geometry"] == _abi.GEOM_GRID_SAG):
        raise NotImplementedError("autograd through grid-sag surfaces is not implemented by "
                                  "the trace core (no derivative kernels)")
    if table.interaction_mask & ~(1 << _abi.IA_REFRACT_REFLECT):
        raise NotImplementedError("autograd through thin-lens, phase or grating surfaces is "
                                  "not implemented by the trace core (no derivative kernels)")


_WORKSPACE: dict = {}


def _workspace(device, nbytes):
    ws = _WORKSPACE.get(device)
    if ws is None or ws.numel() < nbytes:
        _WORKSPACE.pop(device, None)
        ws = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
        _WORKSPACE[device] = ws
    return ws


def _ray_struct(ts):
    return _native.ort_rays(*(0 if t is None else t.data_ptr() for t in ts))


# --------------------------------------------------------------------------------------
# ort::trace_sequential
# --------------------------------------------------------------------------------------
@torch.library.custom_op("ort::trace_sequential", mutates_args=(), device_types="cuda")
def trace_sequential(lens: int, rays: list[torch.Tensor], w: torch.Tensor | None,
                     params: list[torch.Tensor], spec: list[int], start_surface: int,
                     per_ray_w: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor,
                                               torch.Tensor, torch.Tensor, torch.Tensor,
                                               torch.Tensor, torch.Tensor, torch.Tensor,
                                               torch.Tensor]:
    from .raytrace import RealRays, trace_rays

    dl = _lookup(lens)
    if len(rays) != 8:
        raise ValueError("rays: x, y, z, L, M, N, i, opd")
    n = rays[0].numel()
    dev = dl.device
    rin = RealRays.__new__(RealRays)
    for a, t in zip(_abi.RAY_FIELDS, rays, strict=True):
        setattr(rin, a, t.detach().to(device=dev, dtype=torch.float64).reshape(-1).contiguous())
    rin.w = w.detach() if w is not None else torch.zeros(1, dtype=torch.float64, device=dev)
    rout = RealRays.__new__(RealRays)
    for a in _abi.RAY_FIELDS:
        setattr(rout, a, torch.empty(n, dtype=torch.float64, device=dev))
    n_rec = dl.table.n_rec
    rec = torch.empty(n_rec * 8 * n, dtype=torch.float64, device=dev)
    trace_rays(dl, rin, rout, rec=rec if n_rec else None, start_surface=int(start_surface),
               per_ray_w=bool(per_ray_w))
    sched = dl.last_schedule
    if dl.last_schedule_dev is not None:  # device-verified: the settled device schedule
        sched_t = (dl.last_schedule_dev if dl.last_schedule_private  # a per-call copy
                   else dl.last_schedule_dev.clone())
    elif sched is None:
        sched_t = torch.empty(0, dtype=torch.int32, device=dev)
    else:
        sched_t = torch.from_numpy(np.ascontiguousarray(sched.reshape(-1), dtype=np.int32)).to(dev)
    return (*(getattr(rout, a) for a in _abi.RAY_FIELDS), rec, sched_t)


@trace_sequential.register_kernel("cpu")
def _trace_sequential_cpu(lens, rays, w, params, spec, start_surface, per_ray_w):
    """The CPU dispatch key: the host build of the trace core on a HostLens (host.py)."""
    from . import host

    hl = _lookup(lens)
    if not isinstance(hl, host.HostLens):
        raise RuntimeError("ort::trace_sequential: CPU tensors need a HostLens handle "
                           f"(got {type(hl).__name__})")
    if len(rays) != 8:
        raise ValueError("rays: x, y, z, L, M, N, i, opd")
    n = rays[0].numel()
    rin = [t.detach().to(dtype=torch.float64).reshape(-1).contiguous() for t in rays]
    if any(t.numel() != n for t in rin):
        raise ValueError("ray fields of different sizes")
    n_rec = hl.table.n_rec
    rec = torch.empty(n_rec * 8 * n, dtype=torch.float64)
    outs, updates = host.trace_sequential(hl, rin, w, bool(per_ray_w), int(start_surface),
                                          rec if n_rec else None)
    hl.last_schedule = updates.numpy().reshape(1, -1) if hl.newton else None
    sched = updates if hl.newton else torch.empty(0, dtype=torch.int32)
    return (*outs, rec, sched)


@trace_sequential.register_fake
def _(lens, rays, w, params, spec, start_surface, per_ray_w):
    dl = _lookup(lens)
    n = rays[0].numel()
    outs = [rays[0].new_empty(n, dtype=torch.float64) for _ in range(8)]
    rec = rays[0].new_empty(dl.table.n_rec * 8 * n, dtype=torch.float64)
    ns = dl.table.n_surfaces if dl.newton else 0
    return (*outs, rec, rays[0].new_empty(ns, dtype=torch.int32))


def _seq_setup(ctx, inputs, output):
    lens, rays, w, params, spec, start_surface, per_ray_w = inputs
    ctx.dlens = _lookup(lens)  # a strong reference for the backward
    ctx.pairs = _spec_pairs(spec)
    ctx.start_surface = int(start_surface)
    ctx.per_ray_w = bool(per_ray_w)
    ctx.shapes = [(p.shape, p.dtype, p.device) for p in params]
    ctx.n_spec = len(spec)
    ctx.ray_meta = [(r.shape, r.dtype) for r in rays]
    ctx.set_materialize_grads(False)
    rec, sched = output[8], output[9]
    saved = [r.detach() for r in rays] + [rec, sched]
    if w is not None:
        saved.append(w.detach())
    ctx.has_w = w is not None
    ctx.save_for_backward(*saved)


def _seq_backward(ctx, *grads):
    saved = ctx.saved_tensors
    rays_in, rec, sched = saved[:8], saved[8], saved[9]
    w = saved[10] if ctx.has_w else None
    dl = ctx.dlens
    table = dl.table
    n = rays_in[0].numel()
    dev = dl.device
    # list inputs: needs_input_grad holds one bool per list element
    want_rays = any(ctx.needs_input_grad[1])
    want_params = any(ctx.needs_input_grad[3]) and len(ctx.shapes) > 0
    cot = [None if g is None else g.detach().to(torch.float64).reshape(-1).contiguous()
           for g in grads[:8]]
    rec_cot = grads[8]
    if rec_cot is not None:
        rec_cot = rec_cot.detach().to(torch.float64).reshape(-1).contiguous()
    # Tensor-list arguments take a list of Nones; the int list `spec` is one leaf of the
    # argument structure, except when empty (then it reads as an empty tensor list)
    none_rays, none_params = [None] * 8, [None] * len(ctx.shapes)
    none_spec = [] if ctx.n_spec == 0 else None
    if not (want_rays or want_params) or (all(c is None for c in cot) and rec_cot is None):
        return None, none_rays, None, none_params, none_spec, None, None
    _check_differentiable(table)
    params_like = [torch.empty(s, dtype=d, device="meta") for s, d, _ in ctx.shapes]
    zp, st, ft, n_param = tangent_tables(table, ctx.pairs, params_like)
    g = torch.zeros(max(1, n_param), dtype=torch.float64, device=dev)
    gin = [torch.zeros(n, dtype=torch.float64, device=dev) if want_rays else None
           for _ in range(8)]
    from .autodiff import vjp_mode

    mode = vjp_mode(table)
    if want_params and n_param:
        _seq_vjp(dl, rays_in, w, ctx.per_ray_w, ctx.start_surface, sched, zp, st, ft,
                 n_param, cot, rec_cot, rec, g, gin if mode == _abi.VJP_ADJOINT else None,
                 mode)
    if want_rays and not (want_params and n_param and mode == _abi.VJP_ADJOINT):
        # input-ray cotangents come from the reverse-mode pass (forward mode carries only
        # the parameter tangents): one adjoint launch with no parameters
        _seq_vjp(dl, rays_in, w, ctx.per_ray_w, ctx.start_surface, sched, None, None, None,
                 0, cot, rec_cot, rec, None, gin, _abi.VJP_ADJOINT)
    ray_grads = none_rays
    if want_rays:
        ray_grads = [gi.reshape(s).to(d) for gi, (s, d) in zip(gin, ctx.ray_meta, strict=True)]
    param_grads = none_params
    if want_params:
        param_grads = []
        off = 0
        for shape, dtype, pdev in ctx.shapes:
            k = int(np.prod(shape)) if len(shape) else 1
            param_grads.append(g[off:off + k].reshape(shape).to(device=pdev, dtype=dtype))
            off += k
    return None, ray_grads, None, param_grads, none_spec, None, None


def _seq_vjp(dl, rays_in, w, per_ray_w, start_surface, sched, zp, st, ft, n_param, cot,
             rec_cot, rec, grad, gin, mode):
    """One ort_trace_sequential_vjp call (grad += J^T cot, gin = input-ray cotangents); on
    a HostLens the host library's ort_host_trace_sequential_vjp."""
    from . import host
    from .raytrace import _ptr, _stream_handle

    if isinstance(dl, host.HostLens):
        tabs = [None if a is None else dl.resident(("seq_tangent", i), a)
                for i, a in enumerate((zp, st, ft))]
        need = dl.resident("seq_need", slot_need(dl.table, zp, st, ft))
        host.trace_sequential_vjp(dl, rays_in, w, per_ray_w, start_surface, sched, tabs, need,
                                  n_param, mode, cot, rec_cot, rec, grad, gin)
        return

    lib = _native.load()
    n = rays_in[0].numel()
    batch = _native.ort_batch(n, max(n, 1), max(n, 1), 0, 0, None)
    w_keep = None
    if per_ray_w:
        w_keep = w.to(device=dl.device, dtype=torch.float64).reshape(-1)
        w_keep = w_keep.expand(n).contiguous() if w_keep.numel() == 1 else w_keep.contiguous()
        batch.w = w_keep.data_ptr()
    sched_dev = sched if sched is not None and sched.numel() else None
    opt = _native.ort_options(_abi.NEWTON_SCHEDULE, int(start_surface),
                              None if sched_dev is None else sched_dev.data_ptr())
    tabs = [None if a is None else dl.resident(("seq_tangent", i), a)
            for i, a in enumerate((zp, st, ft))]
    need = dl.resident("seq_need", slot_need(dl.table, zp, st, ft))
    params = _native.ort_vjp_params(int(n_param), int(mode), _ptr(tabs[0]).value,
                                    _ptr(tabs[1]).value, _ptr(tabs[2]).value,
                                    0 if tabs[0] is None else int(tabs[0].numel()), 0, None, 0,
                                    need.data_ptr())
    # both modes take a workspace (ABI v15: the unrolled mode's block partials)
    size = lib.ort_vjp_workspace_size(C.byref(dl.c), C.byref(batch), C.byref(params))
    _native.check(int(size) if size < 0 else 0, "ort_vjp_workspace_size")
    ws = _workspace(dl.device, size)
    params.workspace = ws.data_ptr()
    params.workspace_size = ws.numel()
    rin_c = _ray_struct(rays_in)
    cot_c = _ray_struct(cot)
    gin_c = _ray_struct(gin if gin is not None else [None] * 8)
    rc = lib.ort_trace_sequential_vjp(C.byref(dl.c), C.byref(rin_c), C.byref(batch),
                                      C.byref(opt), C.byref(params), C.byref(cot_c),
                                      _ptr(rec_cot), _ptr(rec if rec_cot is not None else None),
                                      _ptr(grad), C.byref(gin_c), _stream_handle())
    _native.check(rc, "ort_trace_sequential_vjp")
    del w_keep, tabs  # ordered on the stream before any reuse of their memory


trace_sequential.register_autograd(_seq_backward, setup_context=_seq_setup)


# --------------------------------------------------------------------------------------
# ort::trace_pupil
# --------------------------------------------------------------------------------------
@torch.library.custom_op("ort::trace_pupil", mutates_args=(), device_types="cuda")
def trace_pupil(plan: int, px: torch.Tensor, py: torch.Tensor, params: list[torch.Tensor],
                spec: list[int]) -> tuple[
        torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor,
        torch.Tensor, torch.Tensor, torch.Tensor]:
    from .raytrace import RealRays
    from .raytrace import trace_pupil as _trace

    p = _lookup(plan)
    dl = p.dlens
    out = RealRays.__new__(RealRays)
    for a in _abi.RAY_FIELDS:
        setattr(out, a, torch.empty(p.n, dtype=torch.float64, device=dl.device))
    p.tape = None
    if p.want_tape:  # the forward writes the adjoint tape: the backward is the reverse sweep
        p.tape = torch.empty(tape_doubles(dl, p.n), dtype=torch.float64, device=dl.device)
    _trace(dl, p.seg_dev, px, py, out, p.n, p.seg_len, p.n, keys=p.keys,
           pupil_per_ray=p.pupil_per_ray, newton_mode=p.newton_mode, tape=p.tape)
    sched = dl.last_schedule
    if dl.last_schedule_dev is not None:  # device-verified: the settled device schedule
        sched_t = (dl.last_schedule_dev if dl.last_schedule_private  # a per-call copy
                   else dl.last_schedule_dev.clone())
    elif sched is None:
        sched_t = torch.empty(0, dtype=torch.int32, device=dl.device)
    else:
        sched_t = dl.resident("sched", sched.reshape(-1)).clone()
    return (*(getattr(out, a) for a in _abi.RAY_FIELDS), sched_t)


@trace_pupil.register_fake
def _(plan, px, py, params, spec):
    p = _lookup(plan)
    ref = px
    outs = [ref.new_empty(p.n, dtype=torch.float64) for _ in range(8)]
    ns = p.dlens.table.n_surfaces if p.dlens.newton else 0
    return (*outs, ref.new_empty(ns, dtype=torch.int32))


def _pupil_setup(ctx, inputs, output):
    plan, px, py, params, spec = inputs
    ctx.plan = _lookup(plan)
    ctx.pairs = _spec_pairs(spec)
    ctx.n_spec = len(spec)
    ctx.shapes = [(p.shape, p.dtype, p.device) for p in params]
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(output[8], *output[:8])


def _pupil_backward(ctx, *grads):
    from .autodiff import vjp

    sched, *primal = ctx.saved_tensors
    p = ctx.plan
    dl = p.dlens
    none_spec = [] if ctx.n_spec == 0 else None  # see _seq_backward
    if not any(ctx.needs_input_grad[3]) or not ctx.shapes:
        return None, None, None, [None] * len(ctx.shapes), none_spec
    _check_differentiable(dl.table)
    params_like = [torch.empty(s, dtype=d, device="meta") for s, d, _ in ctx.shapes]
    zp, st, ft, n_param = tangent_tables(dl.table, ctx.pairs, params_like)
    tables = tuple(None if a is None else dl.resident(("tangent", i), a)
                   for i, a in enumerate((zp, st, ft)))
    tables = (*tables, dl.resident("tangent_need", slot_need(dl.table, zp, st, ft)))
    g = torch.empty(n_param, dtype=torch.float64, device=dl.device)  # overwritten
    cot = [None if gr is None else gr.to(torch.float64).contiguous() for gr in grads[:8]]
    vjp(dl, p.seg_dev, p.px, p.py, p.n, p.seg_len, sched if sched.numel() else None, tables,
        n_param, cot, g, pupil_per_ray=p.pupil_per_ray,
        tape=p.tape, primal=primal if p.tape is not None else None, overwrite=True)
    p.tape = None  # one backward per forward: release the tape
    res = []
    off = 0
    for shape, dtype, pdev in ctx.shapes:
        k = int(np.prod(shape)) if len(shape) else 1
        res.append(g[off:off + k].reshape(shape).to(device=pdev, dtype=dtype))
        off += k
    return None, None, None, res, none_spec


trace_pupil.register_autograd(_pupil_backward, setup_context=_pupil_setup)


# --------------------------------------------------------------------------------------
# ort::rms_spot -- RayOperand.rms_spot_size's reduction (optimization/operand/ray.py:300-340)
# --------------------------------------------------------------------------------------
_RMS_WS: dict = {}


def _rms_workspace(device, n):
    lib = _native.load()
    size = int(lib.ort_rms_spot_workspace_size(int(n)))
    _native.check(size if size < 0 else 0, "ort_rms_spot_workspace_size")
    return _workspace_named(_RMS_WS, device, size), size


def _workspace_named(cache, device, nbytes):
    ws = cache.get(device)
    if ws is None or ws.numel() < nbytes:
        cache.pop(device, None)
        ws = torch.empty(max(int(nbytes), 8), dtype=torch.uint8, device=device)
        cache[device] = ws
    return ws


@torch.library.custom_op("ort::rms_spot", mutates_args=(), device_types="cuda")
def rms_spot(x: torch.Tensor, y: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(rms, stats[5] = n, mean x, mean y, rms, max radius): sqrt(mean((x - mean x)^2 +
    (y - mean y)^2)) as the reference's operand forms it, two deterministic passes on the
    device (ort_rms_spot), no host synchronisation."""
    from .raytrace import _ptr, _stream_handle

    lib = _native.load()
    _check_rms_inputs(x, y)
    x = x.detach().reshape(-1).contiguous()
    y = y.detach().reshape(-1).contiguous()
    n = x.numel()
    ws, size = _rms_workspace(x.device, n)
    stats = torch.empty(5, dtype=torch.float64, device=x.device)
    rms = torch.empty((), dtype=torch.float64, device=x.device)
    rc = lib.ort_rms_spot(_ptr(x), _ptr(y), n, _ptr(ws), size, _ptr(stats), _ptr(rms),
                          _stream_handle())
    _native.check(rc, "ort_rms_spot")
    return rms, stats


def _check_rms_inputs(x, y):
    """The kernels read x and y as n doubles each on one device: refuse anything else
    (a shorter y would be read past its end, a float32 record read as doubles)."""
    if x.dtype != torch.float64 or y.dtype != torch.float64:
        raise ValueError(f"ort::rms_spot: x and y must be float64 (got {x.dtype}, {y.dtype})")
    if x.numel() != y.numel():
        raise ValueError(f"ort::rms_spot: x has {x.numel()} points, y {y.numel()}")
    if x.device != y.device:
        raise ValueError(f"ort::rms_spot: x on {x.device}, y on {y.device}")


@rms_spot.register_fake
def _(x, y):
    _check_rms_inputs(x, y)
    return x.new_empty((), dtype=torch.float64), x.new_empty(5, dtype=torch.float64)


def _rms_setup(ctx, inputs, output):
    x, y = inputs
    ctx.shapes = (x.shape, y.shape)
    ctx.set_materialize_grads(False)
    # stats (n, centroid, rms, max radius) are reported, not differentiated: mark them so a
    # loss built on them raises instead of silently getting a zero gradient
    ctx.mark_non_differentiable(output[1])
    ctx.save_for_backward(x.detach(), y.detach(), output[1])


def _rms_backward(ctx, g_rms, g_stats):
    from .raytrace import _ptr, _stream_handle

    if g_rms is None:
        return None, None
    x, y, stats = ctx.saved_tensors
    xf = x.reshape(-1).contiguous()
    yf = y.reshape(-1).contiguous()
    g = g_rms.detach().to(torch.float64).contiguous()
    gx = torch.empty_like(xf)
    gy = torch.empty_like(yf)
    rc = _native.load().ort_rms_spot_vjp(_ptr(xf), _ptr(yf), xf.numel(), _ptr(stats), _ptr(g),
                                         _ptr(gx), _ptr(gy), _stream_handle())
    _native.check(rc, "ort_rms_spot_vjp")
    return gx.reshape(ctx.shapes[0]), gy.reshape(ctx.shapes[1])


rms_spot.register_autograd(_rms_backward, setup_context=_rms_setup)
