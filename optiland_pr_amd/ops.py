"""PyTorch custom ops over the C ABI: ``torch.ops.ort.trace_sequential`` and
``torch.ops.ort.trace_pupil`` (SURVEY.md 8b "Torch custom op").

The reference differentiates a trace by running every ``be.*`` primitive of
``SurfaceGroup.trace`` (surfaces/surface_group.py:232-244) under torch autograd
(backend/torch_backend.py:45-148, driven by optimization/optimizer/torch/base.py:116-131).
Here the whole trace is ONE dispatcher op whose CUDA (HIP) kernel is the fused trace
(ort_trace_sequential / ort_trace_pupil) and whose autograd formula is the adjoint (or
forward-mode) VJP of the trace core (ort_trace_sequential_vjp / ort_trace_pupil_vjp), so
autograd sees one node per trace call:

  ort::trace_sequential(lens, lens_meta, final_thickness, lens_key, rays[8], w, params,
                        spec, start_surface, per_ray_w)
      -> (x, y, z, L, M, N, i, opd, rec, sched)
      resident rays in (SurfaceGroup.trace, the drop-in seam); rec = every traced
      surface's record [S][8][n] (standard_surface.py:266-286); differentiable w.r.t. the
      input rays, the record buffer's cotangents included, and the lens parameters in
      `params`.
  ort::trace_pupil(lens, lens_meta, final_thickness, lens_key, seg, apod, px, py, params,
                   spec, plan_meta, plan_key)
      -> (x, y, z, L, M, N, i, opd, sched, tape, rms, rms_stats)
      rays generated from pupil samples in the same launch (Optic.trace's fused path,
      raytrace/real_ray_tracer.py:37-97); differentiable w.r.t. the lens parameters.

The ops are self-describing: ``lens`` is the lowered lens as tensors (lens_args: the nine
uploaded tables, a few KB the kernels read from HBM) with its scalars in ``lens_meta``;
``seg`` / ``apod`` / ``plan_meta`` describe the pupil plan the same way. ``lens_key`` /
``plan_key`` are integer cache keys only -- the handle of the live host object holding the
Newton schedule caches; a key that names no live object of these tensors makes the op
rebuild the lens from the tensors. ``params`` are the lens-parameter tensors that require
grad and ``spec`` says which lens value each one is, as flattened (kind, traced-surface
index) pairs with kind in SPEC_KINDS: the forward ignores their values (the lowered lens
already holds them), the backward returns d loss / d each.

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

import os

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
        self.want_rms = False  # the rms spot size in the taped forward's epilogue (F_RMS)
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
                if g in (_abi.GEOM_PLANE, _abi.GEOM_BICONIC, _abi.GEOM_TOROIDAL, _abi.GEOM_GRID_SAG,
                         _abi.GEOM_NURBS):
                    raise NotImplementedError(f"surface {si}: {kind} of this geometry is not a "
                                              "differentiable parameter of the trace core")
                if int(row["interaction"]) == _abi.IA_DIFFRACTIVE:
                    # the grating vector's groove-tangent constants are formed from them on
                    # the host (standard_grating.py:93-146): no tangent reaches them
                    raise NotImplementedError(f"surface {si}: {kind} of a grating surface is not "
                                              "a differentiable parameter of the trace core")
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


# ORT_ADJ_MONO=0 (A/B checks): Zernike coefficient adjoints in per-term slots instead of
# the Cartesian monomial basis (ort_vjp_params.n_mono, ABI v18)
ADJ_MONO = os.environ.get("ORT_ADJ_MONO", "1") != "0"


def mono_slot_count(table, zp):
    """ort_vjp_params.n_mono: the monomial-basis slots of the lens's Zernike surfaces with a
    Cartesian block (2 K = (zm_deg + 1)(zm_deg + 2) each, in surface order), 0 without
    Zernike parameters (or with ORT_ADJ_MONO=0)."""
    if zp is None or not ADJ_MONO:
        return 0
    s = table.surfaces
    # (blocks above ort_sweep.h kMonoMaxDeg = 6 take the per-term slots)
    d = s["zm_deg"][(s["geometry"] == _abi.GEOM_ZERNIKE) & (s["zm_deg"] >= 0)
                    & (s["zm_deg"] <= 6)].astype(np.int64)
    return int(np.sum((d + 1) * (d + 2)))


def slot_need(table, zp, surf, final):
    """ort_vjp_params.slot_need of the tangent tables: nonzero for every slot (radius,
    conic, vertex z of each surface; each Zernike term; the final thickness; the monomial
    slots of the Cartesian Zernike surfaces) some parameter depends on. Host NumPy, kept
    resident with the tables."""
    S = table.n_surfaces
    n_z = 0 if zp is None else len(zp)
    n_mono = mono_slot_count(table, zp)
    need = np.zeros(3 * S + n_z + 1 + n_mono, dtype=np.int32)
    if surf is not None:
        need[:3 * S] = np.any(surf != 0.0, axis=0).reshape(-1)
    if zp is not None:
        need[3 * S:3 * S + n_z] = zp >= 0
    if final is not None:
        need[3 * S + n_z] = np.any(final != 0.0)
    if n_mono:
        off = 3 * S + n_z + 1
        for row in table.surfaces:
            if int(row["geometry"]) != _abi.GEOM_ZERNIKE or int(row["zm_deg"]) < 0:
                continue
            d = int(row["zm_deg"])
            c0, nt = int(row["coef_off"]), int(row["n_coef"])
            if np.any(zp[c0:c0 + nt] >= 0):
                need[off:off + (d + 1) * (d + 2)] = 1
                # the per-term slots of this surface are not summed (the monomials are)
                need[3 * S + c0:3 * S + c0 + nt] = 0
            off += (d + 1) * (d + 2)
    return need


def tape_rows(table):
    """Rows of the adjoint tape per ray (ort_options.tape, ABI v19): 7 per plane / conic
    surface, 11 per Newton surface -- every one written by the taped trace."""
    g = table.surfaces["geometry"]
    closed = (g == _abi.GEOM_PLANE) | (g == _abi.GEOM_STANDARD)
    return int(7 * len(g) + 4 * np.count_nonzero(~closed))


def tape_doubles(dl, n):
    """Doubles of the adjoint tape of an n-ray trace of this lens: exactly the rows the
    taped trace writes (ort_vjp_tape_size bytes bound it for any lens of this many
    surfaces)."""
    return tape_rows(dl.table) * int(n)


def _check_differentiable(table, adjoint=False):
    """Refuse what no derivative kernel covers. adjoint: the reverse-mode pass is needed
    (input-ray cotangents), which has no reverse for thin-lens / phase / grating surfaces
    (their parameter gradients come from the forward-mode VJP, autodiff.vjp_mode)."""
    if np.any(table.surfaces["geometry"] == _abi.GEOM_GRID_SAG):
        raise NotImplementedError("autograd through grid-sag surfaces is not implemented by "
                                  "the trace core (no derivative kernels)")
    if np.any(table.surfaces["geometry"] == _abi.GEOM_NURBS):
        raise NotImplementedError("autograd through NURBS surfaces is not implemented by "
                                  "the trace core (no derivative kernels)")
    if adjoint and table.interaction_mask & ~(1 << _abi.IA_REFRACT_REFLECT):
        raise NotImplementedError("input-ray gradients through thin-lens, phase or grating "
                                  "surfaces are not implemented by the trace core (the "
                                  "forward-mode VJP carries parameter tangents only)")


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
# the lens as the ops take it (the op is self-describing)
# --------------------------------------------------------------------------------------
# lens_meta: the host-side scalars of the ort_lens struct, in this order
LENS_META = ("n_surfaces", "n_lambda", "n_mat", "final_mat", "geometry_mask",
             "interaction_mask", "frame_flags", "n_rec", "newton", "tape_rows")
NEWTON_MODES = ("reference", "device", "wave")


def lens_args(dl):
    """(lens, lens_meta, final_thickness, lens_key) of a DeviceLens / HostLens: the nine
    lowered tables as tensors on the lens's device -- surfaces, cs_ops, zern, optics and
    materials as their bytes (uint8), coef, n_tab, alpha_tab and the wavelengths as float64
    -- the ort_lens scalars, the image-space thickness and the handle of the object that
    holds the host-side state (Newton schedule caches), used only as a cache key."""
    t = dl.table
    meta = [int(t.n_surfaces), len(t.wavelengths), int(t.n_tab.shape[1]), int(t.final_mat),
            int(dl.geometry_mask), int(t.interaction_mask), int(t.frame_flags), int(t.n_rec),
            1 if dl.newton else 0, tape_rows(t)]
    return dl.lens_tensors(), meta, float(t.final_thickness), handle(dl)


# lenses rebuilt from their tensors (a handle that names no live object of those tensors:
# e.g. a traced graph run in another process), keyed by the tables' addresses
_REBUILT: "weakref.WeakValueDictionary[tuple, object]" = weakref.WeakValueDictionary()


def _table_from_tensors(lens, meta, final_thickness):
    from .lowering import LensTable

    def raw(t, dt):
        return np.frombuffer(t.detach().cpu().numpy().tobytes(), dtype=dt).copy()

    S, n_lambda, n_mat = meta[0], meta[1], meta[2]
    surfaces = raw(lens[0], _abi.SURFACE)
    rec = [i for i in range(S) if int(surfaces[i]["flags"]) & _abi.SURF_RECORD]
    mats = raw(lens[7], _abi.MATERIAL)
    return LensTable(
        surfaces=surfaces, cs_ops=raw(lens[1], _abi.CS_OP),
        coef=lens[2].detach().cpu().numpy().astype(np.float64).copy(),
        zern=raw(lens[3], _abi.ZERNIKE_TERM),
        n_tab=lens[4].detach().cpu().numpy().reshape(n_lambda, n_mat).copy(),
        alpha_tab=lens[5].detach().cpu().numpy().reshape(n_lambda, n_mat).copy(),
        wavelengths=[float(v) for v in lens[8].detach().cpu().numpy()],
        final_mat=int(meta[3]), final_thickness=float(final_thickness), mat_table=mats,
        n_rec=int(meta[7]), rec_surfaces=rec)


def _has_data(t):
    """False for tensors without storage (fake / functional tensors while tracing)."""
    try:
        t.data_ptr()
        return True
    except RuntimeError:
        return False


def _resolve(lens, meta, final_thickness, key):
    """The DeviceLens / HostLens these tensors are: the object named by `key` when it holds
    exactly these tables, else one rebuilt from the tensors (cached by their addresses).
    While tracing (fake tensors: no data to compare or rebuild from), the object the key
    names -- the backward formulas only read its host-side tables."""
    obj = _HANDLES.get(int(key))
    if not _has_data(lens[0]):
        if obj is None or not hasattr(obj, "lens_tensors"):
            raise RuntimeError("ort op traced with a lens key that names no live lens")
        return obj
    if obj is not None and hasattr(obj, "lens_tensors"):
        mine = obj.lens_tensors()
        if all(a.data_ptr() == b.data_ptr() and a.device == b.device
               for a, b in zip(mine, lens, strict=True)):
            return obj
    ck = tuple((t.device.type, t.data_ptr()) for t in lens)
    hit = _REBUILT.get(ck)
    if hit is None:
        table = _table_from_tensors(lens, meta, final_thickness)
        if lens[0].device.type == "cpu":
            from .host import HostLens

            hit = HostLens(table)
        else:
            from .raytrace import DeviceLens

            hit = DeviceLens(table, device=lens[0].device)
        hit._source_tensors = list(lens)  # the rebuilt object keeps its source alive
        _REBUILT[ck] = hit
    return hit


def _opt(t):
    return None if t is None else t


# --------------------------------------------------------------------------------------
# ort::trace_sequential
# --------------------------------------------------------------------------------------
@torch.library.custom_op("ort::trace_sequential", mutates_args=(), device_types="cuda")
def trace_sequential(lens: list[torch.Tensor], lens_meta: list[int], final_thickness: float,
                     lens_key: int, rays: list[torch.Tensor], w: torch.Tensor | None,
                     params: list[torch.Tensor], spec: list[int], start_surface: int,
                     per_ray_w: bool) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor,
                                               torch.Tensor, torch.Tensor, torch.Tensor,
                                               torch.Tensor, torch.Tensor, torch.Tensor,
                                               torch.Tensor]:
    from .raytrace import RealRays, trace_rays

    dl = _resolve(lens, lens_meta, final_thickness, lens_key)
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
def _trace_sequential_cpu(lens, lens_meta, final_thickness, lens_key, rays, w, params, spec,
                          start_surface, per_ray_w):
    """The CPU dispatch key: the host build of the trace core (host.py) on the lens's CPU
    tensors."""
    from . import host

    hl = _resolve(lens, lens_meta, final_thickness, lens_key)
    if not isinstance(hl, host.HostLens):
        raise RuntimeError("ort::trace_sequential: CPU rays need the lens's tables on the CPU "
                           f"(got a {type(hl).__name__})")
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
def _(lens, lens_meta, final_thickness, lens_key, rays, w, params, spec, start_surface,
      per_ray_w):
    n = rays[0].numel()
    outs = [rays[0].new_empty(n, dtype=torch.float64) for _ in range(8)]
    rec = rays[0].new_empty(lens_meta[7] * 8 * n, dtype=torch.float64)
    ns = lens_meta[0] if lens_meta[8] else 0
    return (*outs, rec, rays[0].new_empty(ns, dtype=torch.int32))


def _seq_setup(ctx, inputs, output):
    lens, meta, ft, key, rays, w, params, spec, start_surface, per_ray_w = inputs
    ctx.lens_meta, ctx.final_thickness, ctx.lens_key = list(meta), float(ft), int(key)
    ctx.n_lens = len(lens)
    ctx.pairs = _spec_pairs(spec)
    ctx.start_surface = int(start_surface)
    ctx.per_ray_w = bool(per_ray_w)
    ctx.shapes = [(p.shape, p.dtype, p.device) for p in params]
    ctx.n_spec = len(spec)
    ctx.ray_meta = [(r.shape, r.dtype) for r in rays]
    ctx.set_materialize_grads(False)
    rec, sched = output[8], output[9]
    saved = list(lens) + [r.detach() for r in rays] + [rec, sched]
    if w is not None:
        saved.append(w.detach())
    ctx.has_w = w is not None
    ctx.save_for_backward(*saved)


def _seq_backward(ctx, *grads):
    saved = ctx.saved_tensors
    nl = ctx.n_lens
    lens = list(saved[:nl])
    rays_in, rec, sched = list(saved[nl:nl + 8]), saved[nl + 8], saved[nl + 9]
    w = saved[nl + 10] if ctx.has_w else None
    dl = _resolve(lens, ctx.lens_meta, ctx.final_thickness, ctx.lens_key)
    table = dl.table
    want_rays = any(ctx.needs_input_grad[4])  # list inputs: one bool per element
    want_params = any(ctx.needs_input_grad[6]) and len(ctx.shapes) > 0
    cot = [None if g is None else g.detach().to(torch.float64).reshape(-1).contiguous()
           for g in grads[:8]]
    rec_cot = grads[8]
    if rec_cot is not None:
        rec_cot = rec_cot.detach().to(torch.float64).reshape(-1).contiguous()
    # Tensor-list arguments take a list of Nones; the int lists are one leaf each, except an
    # empty `spec` (then it reads as an empty tensor list)
    none_rays, none_params = [None] * 8, [None] * len(ctx.shapes)
    none_spec = [] if ctx.n_spec == 0 else None
    nothing = ([None] * ctx.n_lens, None, None, None)
    if not (want_rays or want_params) or (all(c is None for c in cot) and rec_cot is None):
        return (*nothing, none_rays, None, none_params, none_spec, None, None)
    _check_differentiable(table, adjoint=want_rays)
    params_like = [torch.empty(s, dtype=d, device="meta") for s, d, _ in ctx.shapes]
    zp, st, ft, n_param = tangent_tables(table, ctx.pairs, params_like)
    from .autodiff import schedule_for_mode, vjp_mode

    mode = vjp_mode(table, schedule_for_mode(table, sched))
    if not (want_params and n_param):
        zp = st = ft = None
        n_param = 0
        mode = _abi.VJP_ADJOINT  # input-ray cotangents: the reverse-mode pass
    tabs = _tables_cpu(zp, st, ft, slot_need(table, zp, st, ft) if mode == _abi.VJP_ADJOINT
                       else None)
    g, gin = torch.ops.ort.trace_sequential_vjp(
        lens, ctx.lens_meta, ctx.final_thickness, ctx.lens_key, rays_in, w, sched, rec, cot,
        rec_cot, tabs, n_param, int(mode), ctx.start_surface, ctx.per_ray_w, bool(want_rays))
    if want_rays and mode != _abi.VJP_ADJOINT:
        # input-ray cotangents come from the reverse-mode pass (forward mode carries only the
        # parameter tangents): one adjoint launch with no parameters
        _, gin = torch.ops.ort.trace_sequential_vjp(
            lens, ctx.lens_meta, ctx.final_thickness, ctx.lens_key, rays_in, w, sched, rec,
            cot, rec_cot, [None, None, None, None], 0, int(_abi.VJP_ADJOINT),
            ctx.start_surface, ctx.per_ray_w, True)
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
    return (*nothing, ray_grads, None, param_grads, none_spec, None, None)


def _tables_cpu(zp, st, ft, need):
    """The tangent tables as host tensors (the VJP ops' `tables` argument)."""
    return [None if a is None else torch.from_numpy(np.ascontiguousarray(a))
            for a in (zp, st, ft, need)]


trace_sequential.register_autograd(_seq_backward, setup_context=_seq_setup)


# --------------------------------------------------------------------------------------
# ort::trace_sequential_vjp -- the backward as its own op (traceable: fake + kernels)
# --------------------------------------------------------------------------------------
@torch.library.custom_op("ort::trace_sequential_vjp", mutates_args=(), device_types="cuda")
def trace_sequential_vjp(lens: list[torch.Tensor], lens_meta: list[int], final_thickness: float,
                         lens_key: int, rays_in: list[torch.Tensor], w: torch.Tensor | None,
                         sched: torch.Tensor, rec: torch.Tensor,
                         cot: list[torch.Tensor | None], rec_cot: torch.Tensor | None,
                         tables: list[torch.Tensor | None], n_param: int, mode: int,
                         start_surface: int, per_ray_w: bool,
                         want_rays: bool) -> tuple[torch.Tensor, list[torch.Tensor]]:
    """ort_trace_sequential_vjp: (grad [max(1, n_param)] = J^T cot w.r.t. the parameters of
    the tangent tables (zern_param, surf_tangent, final_tangent, slot_need), the input-ray
    cotangents [8][n] when want_rays, else [])."""
    dl = _resolve(lens, lens_meta, final_thickness, lens_key)
    return _seq_vjp_run(dl, rays_in, w, sched, rec, cot, rec_cot, tables, n_param, mode,
                        start_surface, per_ray_w, want_rays)


@trace_sequential_vjp.register_kernel("cpu")
def _trace_sequential_vjp_cpu(lens, lens_meta, final_thickness, lens_key, rays_in, w, sched, rec,
                              cot, rec_cot, tables, n_param, mode, start_surface, per_ray_w,
                              want_rays):
    dl = _resolve(lens, lens_meta, final_thickness, lens_key)
    return _seq_vjp_run(dl, rays_in, w, sched, rec, cot, rec_cot, tables, n_param, mode,
                        start_surface, per_ray_w, want_rays)


@trace_sequential_vjp.register_fake
def _(lens, lens_meta, final_thickness, lens_key, rays_in, w, sched, rec, cot, rec_cot, tables,
      n_param, mode, start_surface, per_ray_w, want_rays):
    n = rays_in[0].numel()
    g = rays_in[0].new_empty(max(1, n_param), dtype=torch.float64)
    gin = [rays_in[0].new_empty(n, dtype=torch.float64) for _ in range(8)] if want_rays else []
    return g, gin


def _seq_vjp_run(dl, rays_in, w, sched, rec, cot, rec_cot, tables, n_param, mode,
                 start_surface, per_ray_w, want_rays):
    dev = dl.device
    n = rays_in[0].numel()
    rays_in = [t.detach().to(device=dev, dtype=torch.float64).reshape(-1).contiguous()
               for t in rays_in]
    cot = [None if c is None else c.detach().to(device=dev, dtype=torch.float64).reshape(-1)
           .contiguous() for c in cot]
    g = torch.zeros(max(1, n_param), dtype=torch.float64, device=dev)
    gin = [torch.zeros(n, dtype=torch.float64, device=dev) for _ in range(8)] if want_rays else None
    zp, st, ft, need = (None if t is None else t.detach().cpu().numpy() for t in tables)
    _seq_vjp(dl, rays_in, w, per_ray_w, start_surface, sched, zp, st, ft, n_param, cot,
             rec_cot, rec, g if n_param else None, gin, mode, need)
    return g, (gin if want_rays else [])


def _seq_vjp(dl, rays_in, w, per_ray_w, start_surface, sched, zp, st, ft, n_param, cot,
             rec_cot, rec, grad, gin, mode, need=None):
    """One ort_trace_sequential_vjp call (grad += J^T cot, gin = input-ray cotangents); on
    a HostLens the host library's ort_host_trace_sequential_vjp."""
    from . import host
    from .raytrace import _ptr, _stream_handle

    if need is None and mode == _abi.VJP_ADJOINT and zp is not None:
        need = slot_need(dl.table, zp, st, ft)
    if isinstance(dl, host.HostLens):
        tabs = [None if a is None else dl.resident(("seq_tangent", i), a)
                for i, a in enumerate((zp, st, ft))]
        need_t = None if need is None else dl.resident("seq_need", need)
        host.trace_sequential_vjp(dl, rays_in, w, per_ray_w, start_surface, sched, tabs, need_t,
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
    need_t = None if need is None else dl.resident("seq_need", need)
    params = _native.ort_vjp_params(int(n_param), int(mode), _ptr(tabs[0]).value,
                                    _ptr(tabs[1]).value, _ptr(tabs[2]).value,
                                    0 if tabs[0] is None else int(tabs[0].numel()), 0, None, 0,
                                    _ptr(need_t).value)
    params.n_mono = mono_slot_count(dl.table, zp) if mode == _abi.VJP_ADJOINT else 0
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


# --------------------------------------------------------------------------------------
# ort::trace_pupil
# --------------------------------------------------------------------------------------
def plan_args(plan):
    """(seg, apod, plan_meta, plan_key) of a PupilPlan: the segment descriptors (SEGMENT
    records as bytes on the lens's device), the apodization record (or None), [n, seg_len,
    pupil_per_ray, newton mode index, want_tape, want_rms] and the plan's handle (its Newton
    schedule cache keys; a cache key only)."""
    dl = plan.dlens
    seg = plan.seg_dev
    if not torch.is_tensor(seg):
        seg = dl.resident("segments", np.asarray(seg, dtype=_abi.SEGMENT))
    apod = getattr(dl, "apod", None)
    if apod is None and getattr(dl.table, "apod", None) is not None and dl.device.type == "cpu":
        apod = dl.resident("apod", dl.table.apod)
    meta = [plan.n, plan.seg_len, int(plan.pupil_per_ray),
            NEWTON_MODES.index(plan.newton_mode), int(bool(plan.want_tape)),
            int(bool(plan.want_rms))]
    return seg, apod, meta, handle(plan)


def _want_rms(plan_meta):
    """plan_meta's want_rms entry (absent: 0)"""
    return int(plan_meta[5]) if len(plan_meta) > 5 else 0


def _plan_keys(plan_key):
    """The Newton schedule cache keys of the plan (raytrace._run falls back to per-group
    keys when there are none)."""
    p = _HANDLES.get(int(plan_key))
    return list(getattr(p, "keys", ()) or ())


@torch.library.custom_op("ort::trace_pupil", mutates_args=(), device_types="cuda")
def trace_pupil(lens: list[torch.Tensor], lens_meta: list[int], final_thickness: float,
                lens_key: int, seg: torch.Tensor, apod: torch.Tensor | None, px: torch.Tensor,
                py: torch.Tensor, params: list[torch.Tensor], spec: list[int],
                plan_meta: list[int], plan_key: int) -> tuple[
        torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor,
        torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """Optic.trace's fused generation + trace (ort_trace_pupil): outputs the 8 ray columns,
    the verified Newton schedule, the adjoint tape (empty unless plan_meta asks for it:
    the backward is then the reverse sweep only; every row written, tape_rows per ray),
    and RayOperand.rms_spot_size of the final points with its stats[5] (empty
    unless plan_meta's want_rms: the rows in the taped kernel's epilogue, ort_rms_finish;
    its gradient folds into the backward's x, y cotangents)."""
    from .raytrace import RealRays
    from .raytrace import trace_pupil as _trace

    dl = _resolve(lens, lens_meta, final_thickness, lens_key)
    n, seg_len, ppr, mode, want_tape = plan_meta[:5]
    want_rms = _want_rms(plan_meta)
    if want_rms and not want_tape:
        raise ValueError("ort::trace_pupil: want_rms needs the taped forward (want_tape)")
    out = RealRays.__new__(RealRays)
    for a in _abi.RAY_FIELDS:
        setattr(out, a, torch.empty(n, dtype=torch.float64, device=dl.device))
    tape = torch.empty(tape_doubles(dl, n) if want_tape else 0, dtype=torch.float64,
                       device=dl.device)
    rms = torch.empty(() if want_rms else 0, dtype=torch.float64, device=dl.device)
    rms_stats = torch.empty(5 if want_rms else 0, dtype=torch.float64, device=dl.device)
    if want_rms and n == 0:  # the mean over no points: NaN (no finish launch runs)
        rms.fill_(float("nan"))
        rms_stats.fill_(float("nan"))
    _trace(dl, seg, px, py, out, n, seg_len, n, keys=_plan_keys(plan_key),
           pupil_per_ray=bool(ppr), newton_mode=NEWTON_MODES[mode],
           tape=tape if want_tape else None, rms=(rms, rms_stats) if want_rms else None)
    sched = dl.last_schedule
    if dl.last_schedule_dev is not None:  # device-verified: the settled device schedule
        sched_t = (dl.last_schedule_dev if dl.last_schedule_private  # a per-call copy
                   else dl.last_schedule_dev.clone())
    elif sched is None:
        sched_t = torch.empty(0, dtype=torch.int32, device=dl.device)
    else:
        sched_t = dl.resident("sched", sched.reshape(-1)).clone()
    return (*(getattr(out, a) for a in _abi.RAY_FIELDS), sched_t, tape, rms, rms_stats)


@trace_pupil.register_kernel("cpu")
def _trace_pupil_cpu(lens, lens_meta, final_thickness, lens_key, seg, apod, px, py, params,
                     spec, plan_meta, plan_key):
    """The CPU dispatch key: rays generated and traced by the host build (host.py), the
    Newton stop rule evaluated exactly per (field, wavelength) group; no tape (the host
    backward re-traces); want_rms: ort_host_rms_spot of the outputs."""
    from . import host

    hl = _resolve(lens, lens_meta, final_thickness, lens_key)
    n, seg_len, ppr = plan_meta[:3]
    outs, updates = host.trace_pupil(hl, seg, px.detach().contiguous(), py.detach().contiguous(),
                                     n, seg_len, bool(ppr), apod)
    sched = updates if hl.newton else torch.empty(0, dtype=torch.int32)
    if _want_rms(plan_meta):
        rms, rms_stats = host.rms_spot(outs[0], outs[1])
    else:
        rms, rms_stats = (torch.empty(0, dtype=torch.float64) for _ in range(2))
    return (*outs, sched, torch.empty(0, dtype=torch.float64), rms, rms_stats)


@trace_pupil.register_fake
def _(lens, lens_meta, final_thickness, lens_key, seg, apod, px, py, params, spec, plan_meta,
      plan_key):
    n, seg_len, _, _, want_tape = plan_meta[:5]
    want_rms = _want_rms(plan_meta)
    outs = [px.new_empty(n, dtype=torch.float64) for _ in range(8)]
    S = lens_meta[0]
    ns = S if lens_meta[8] else 0  # one Newton group per call (group_len = n)
    nt = lens_meta[9] * n if (want_tape and px.device.type != "cpu") else 0  # tape_rows
    return (*outs, px.new_empty(ns, dtype=torch.int32), px.new_empty(nt, dtype=torch.float64),
            px.new_empty(() if want_rms else 0, dtype=torch.float64),
            px.new_empty(5 if want_rms else 0, dtype=torch.float64))


def _pupil_setup(ctx, inputs, output):
    lens, meta, ft, key, seg, apod, px, py, params, spec, plan_meta, plan_key = inputs
    ctx.lens_meta, ctx.final_thickness, ctx.lens_key = list(meta), float(ft), int(key)
    ctx.plan_meta, ctx.plan_key = list(plan_meta), int(plan_key)
    ctx.n_lens = len(lens)
    ctx.pairs = _spec_pairs(spec)
    ctx.n_spec = len(spec)
    ctx.shapes = [(p.shape, p.dtype, p.device) for p in params]
    ctx.has_apod = apod is not None
    ctx.set_materialize_grads(False)
    ctx.mark_non_differentiable(output[8], output[9], output[11])
    saved = [*lens, seg, px.detach(), py.detach(), output[8], output[9], output[11],
             *output[:8]]
    if apod is not None:
        saved.append(apod)
    ctx.save_for_backward(*saved)


def _pupil_backward(ctx, *grads):
    saved = ctx.saved_tensors
    nl = ctx.n_lens
    lens = list(saved[:nl])
    seg, px, py, sched, tape, rms_stats = saved[nl:nl + 6]
    primal = list(saved[nl + 6:nl + 14])
    apod = saved[nl + 14] if ctx.has_apod else None
    none_spec = [] if ctx.n_spec == 0 else None  # see _seq_backward
    nothing = ([None] * ctx.n_lens, None, None, None, None, None, None, None)
    if not any(ctx.needs_input_grad[8]) or not ctx.shapes:
        return (*nothing, [None] * len(ctx.shapes), none_spec, None, None)
    dl = _resolve(lens, ctx.lens_meta, ctx.final_thickness, ctx.lens_key)
    _check_differentiable(dl.table)
    params_like = [torch.empty(s, dtype=d, device="meta") for s, d, _ in ctx.shapes]
    zp, st, ft, n_param = tangent_tables(dl.table, ctx.pairs, params_like)
    from .autodiff import schedule_for_mode, vjp_mode

    hint = None
    if hasattr(dl, "cached_schedule"):
        hint = dl.cached_schedule(_plan_keys(ctx.plan_key))
    mode = vjp_mode(dl.table, schedule_for_mode(dl.table, sched, hint))
    tabs = _tables_cpu(zp, st, ft, slot_need(dl.table, zp, st, ft))
    cot = [None if gr is None else gr.to(torch.float64).contiguous() for gr in grads[:8]]
    g_rms = grads[10] if _want_rms(ctx.plan_meta) else None  # (AOT: zeros of an empty output)
    if g_rms is not None:
        g_rms = g_rms.detach().to(torch.float64).reshape(1)
    if all(c is None for c in cot) and g_rms is None:
        return (*nothing, [None] * len(ctx.shapes), none_spec, None, None)
    g = torch.ops.ort.trace_pupil_vjp(lens, ctx.lens_meta, ctx.final_thickness, ctx.lens_key,
                                      seg, apod, px, py, sched, tape, primal, cot, tabs,
                                      n_param, int(mode), ctx.plan_meta,
                                      rms_stats if g_rms is not None else None, g_rms)
    res = []
    off = 0
    for shape, dtype, pdev in ctx.shapes:
        k = int(np.prod(shape)) if len(shape) else 1
        res.append(g[off:off + k].reshape(shape).to(device=pdev, dtype=dtype))
        off += k
    return (*nothing, res, none_spec, None, None)


trace_pupil.register_autograd(_pupil_backward, setup_context=_pupil_setup)


@torch.library.custom_op("ort::trace_pupil_vjp", mutates_args=(), device_types="cuda")
def trace_pupil_vjp(lens: list[torch.Tensor], lens_meta: list[int], final_thickness: float,
                    lens_key: int, seg: torch.Tensor, apod: torch.Tensor | None,
                    px: torch.Tensor, py: torch.Tensor, sched: torch.Tensor, tape: torch.Tensor,
                    primal: list[torch.Tensor], cot: list[torch.Tensor | None],
                    tables: list[torch.Tensor | None], n_param: int, mode: int,
                    plan_meta: list[int], rms_stats: torch.Tensor | None = None,
                    g_rms: torch.Tensor | None = None) -> torch.Tensor:
    """ort_trace_pupil_vjp: grad [n_param] = J^T cot (the reverse sweep over `tape` when the
    forward wrote one, else with its own re-trace). rms_stats / g_rms: the forward's rms
    spot size (its stats[5]) and its upstream gradient [1], folded into the x, y cotangents
    of the adjoint (ort_vjp_params.rms_stats / rms_grad)."""
    from .autodiff import vjp

    dl = _resolve(lens, lens_meta, final_thickness, lens_key)
    n, seg_len, ppr = plan_meta[:3]
    dev = dl.device
    tabs = tuple(None if t is None else dl.resident(("tangent", i), t.detach().cpu().numpy())
                 for i, t in enumerate(tables))
    g = torch.empty(max(1, n_param), dtype=torch.float64, device=dev)  # overwritten
    cot = [None if c is None else c.detach().to(device=dev, dtype=torch.float64).contiguous()
           for c in cot]
    taped = tape.numel() > 0 and mode == _abi.VJP_ADJOINT
    rms = None
    if g_rms is not None:
        if rms_stats is None or mode != _abi.VJP_ADJOINT:
            raise ValueError("ort::trace_pupil_vjp: g_rms needs rms_stats and the adjoint mode")
        rms = (rms_stats.detach().to(dev).contiguous(), g_rms.detach().to(dev).contiguous())
    vjp(dl, seg, px, py, n, seg_len, sched if sched.numel() else None, tabs, n_param, cot, g,
        pupil_per_ray=bool(ppr), mode=mode, tape=tape if taped else None,
        primal=primal if taped else None, overwrite=True, rms=rms)
    return g


@trace_pupil_vjp.register_kernel("cpu")
def _trace_pupil_vjp_cpu(lens, lens_meta, final_thickness, lens_key, seg, apod, px, py, sched,
                         tape, primal, cot, tables, n_param, mode, plan_meta, rms_stats=None,
                         g_rms=None):
    from . import host

    hl = _resolve(lens, lens_meta, final_thickness, lens_key)
    n, seg_len, ppr = plan_meta[:3]
    zp, st, ft, need = (None if t is None else t.detach().contiguous() for t in tables)
    g = torch.empty(max(1, n_param), dtype=torch.float64)
    cot = [None if c is None else c.detach().to(torch.float64).contiguous() for c in cot]
    host.trace_pupil_vjp(hl, seg, px.detach().contiguous(), py.detach().contiguous(), n,
                         seg_len, bool(ppr), sched, (zp, st, ft),
                         need if mode == _abi.VJP_ADJOINT else None, n_param, mode, cot, g, apod,
                         rms=None if g_rms is None else (rms_stats.detach().contiguous(),
                                                         g_rms.detach().contiguous()))
    return g


@trace_pupil_vjp.register_fake
def _(lens, lens_meta, final_thickness, lens_key, seg, apod, px, py, sched, tape, primal, cot,
      tables, n_param, mode, plan_meta, rms_stats=None, g_rms=None):
    return px.new_empty(max(1, n_param), dtype=torch.float64)


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


@rms_spot.register_kernel("cpu")
def _rms_spot_cpu(x, y):
    """The CPU dispatch key: the same formula in the host library (sums in index order)."""
    from . import host

    _check_rms_inputs(x, y)
    return host.rms_spot(x.detach().reshape(-1).contiguous(), y.detach().reshape(-1).contiguous())


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
    if g_rms is None:
        return None, None
    x, y, stats = ctx.saved_tensors
    gx, gy = torch.ops.ort.rms_spot_vjp(x, y, stats, g_rms.detach().to(torch.float64))
    return gx.reshape(ctx.shapes[0]), gy.reshape(ctx.shapes[1])


rms_spot.register_autograd(_rms_backward, setup_context=_rms_setup)


@torch.library.custom_op("ort::rms_spot_vjp", mutates_args=(), device_types="cuda")
def rms_spot_vjp(x: torch.Tensor, y: torch.Tensor, stats: torch.Tensor,
                 g: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """ort_rms_spot_vjp: g (x - mean x, y - mean y) / (n rms) (one kernel)."""
    from .raytrace import _ptr, _stream_handle

    xf = x.detach().reshape(-1).contiguous()
    yf = y.detach().reshape(-1).contiguous()
    gg = g.detach().to(torch.float64).contiguous()
    gx = torch.empty_like(xf)
    gy = torch.empty_like(yf)
    rc = _native.load().ort_rms_spot_vjp(_ptr(xf), _ptr(yf), xf.numel(), _ptr(stats), _ptr(gg),
                                         _ptr(gx), _ptr(gy), _stream_handle())
    _native.check(rc, "ort_rms_spot_vjp")
    return gx, gy


@rms_spot_vjp.register_kernel("cpu")
def _rms_spot_vjp_cpu(x, y, stats, g):
    from . import host

    return host.rms_spot_vjp(x.detach().reshape(-1).contiguous(), y.detach().reshape(-1)
                             .contiguous(), stats.contiguous(), g.detach().to(torch.float64)
                             .reshape(1).contiguous())


@rms_spot_vjp.register_fake
def _(x, y, stats, g):
    return (x.new_empty(x.numel(), dtype=torch.float64),
            y.new_empty(y.numel(), dtype=torch.float64))
