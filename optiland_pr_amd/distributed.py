"""Multi-GPU: ray batches sharded across one-process-per-GPU ranks (RCCL over xGMI).

SURVEY 8e: rays are independent, so every (field, wavelength) pair's pupil samples are
split into `world` contiguous, near-equal slices (global ray index = pair*N_p + offset);
each rank traces all pairs on its slice with the same lowered lens (no broadcast: every
rank lowers the lens itself). There is no collective on the trace's data path.

Two collectives exist only for the consumers:
  * gather_image_plane: image-plane intercepts to rank 0 (SpotDiagram plots, parity),
    one all_gather of equal-size padded shards (RCCL ring over xGMI);
  * spot_statistics: centroid / RMS / max radius from per-pair partial sums, two
    all_reduce calls of a few doubles per pair -- no intercepts move.
"""

from __future__ import annotations

import numpy as np

try:
    import torch
    import torch.distributed as dist
except ImportError:  # pragma: no cover
    torch = dist = None


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """[start, stop) of rank's contiguous share of n items (sizes differ by <= 1)."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def world_info(group=None):
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def trace_sharded(optic, fields, wavelengths, px, py, group=None, newton_mode="reference"):
    """Trace this rank's slice of the pupil samples for every (field, wavelength) pair.

    Returns (RealRays of this rank's rays, laid out [pair][local pupil], local count).
    Newton semantics: each rank verifies its own schedule; the reference's global rule
    spans all ranks of a pair, so the schedule is agreed with one all_reduce(MAX) of the
    per-pair update counts when ranks disagree (rare)."""
    from .lowering import pupil_scalars, segment_params
    from .raytrace import RealRays, lens_for, trace_pupil

    rank, world = world_info(group)
    n_p = len(px)
    a, b = shard_range(n_p, rank, world)
    dl = lens_for(optic, list(wavelengths))
    dev = dl.device
    EPL, EPD = pupil_scalars(optic)
    segs = np.stack([segment_params(optic, float(hx), float(hy), wi, EPL, EPD)
                     for hx, hy in fields for wi in range(len(wavelengths))])
    n_loc = b - a
    n = n_loc * len(segs)
    out = RealRays.empty(n, 0.0, device=dev)
    pxl = torch.as_tensor(np.ascontiguousarray(px[a:b]), dtype=torch.float64, device=dev)
    pyl = torch.as_tensor(np.ascontiguousarray(py[a:b]), dtype=torch.float64, device=dev)
    keys = [("shard", k, rank, world) for k in range(len(segs))]
    if n_loc > 0:
        trace_pupil(dl, segs, pxl, pyl, out, n, n_loc, n_loc, keys=keys,
                    newton_mode=newton_mode)
        if dl.newton and world > 1 and newton_mode != "wave":
            _agree_newton_schedule(dl, keys, segs, pxl, pyl, out, n, n_loc, group)
    return out, n_loc


def _agree_newton_schedule(dl, keys, segs, px, py, out, n, n_loc, group):
    """Make every rank use the max over ranks of the per-pair schedules (the stopping
    index of the union of the shards = the reference's global rule on the whole pair)."""
    from .raytrace import trace_pupil

    S = dl.table.n_surfaces
    local = np.stack([dl.sched_cache[k] for k in keys]).astype(np.int64)
    t = torch.as_tensor(local, device=out.x.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    agreed = t.cpu().numpy().astype(np.int32)
    if not np.array_equal(agreed, local):
        # re-run with the agreed schedule, no further verification (every rank now runs
        # the pair's global stopping index, which no rank's own check can contradict)
        import ctypes as C

        from . import _abi, _native
        from .raytrace import _ptr, _stream_handle, upload_segments

        lib = _native.load()
        seg_dev = upload_segments(segs, dl.device)
        batch = _native.ort_batch(n, n_loc, n_loc, len(segs), 0, seg_dev.data_ptr())
        batch.apod = None if dl.apod is None else dl.apod.data_ptr()
        sched_dev = torch.as_tensor(agreed.reshape(-1), device=dl.device)
        opt = _native.ort_options(_abi.NEWTON_SCHEDULE, 0, sched_dev.data_ptr())
        out_c = out.c_struct()
        rc = lib.ort_trace_pupil(C.byref(dl.c), _ptr(px), _ptr(py), C.byref(out_c),
                                 C.byref(batch), C.byref(opt), None, None, None,
                                 _stream_handle())
        _native.check(rc, "ort_trace_pupil")
        for g, k in enumerate(keys):
            dl.sched_cache[k] = agreed[g].copy()
    del S


def gather_image_plane(x, y, n_loc_pairs, n_pairs, n_p, group=None):
    """All-gather image-plane (x, y) of every rank's [pair][local] rays and reassemble
    the reference order [pair][pupil] (real_ray_tracer.py:74-77). Returns (X, Y) of
    shape [n_pairs * n_p] on every rank."""
    rank, world = world_info(group)
    if world == 1:
        return x, y
    sizes = [shard_range(n_p, r, world) for r in range(world)]
    maxloc = max(b - a for a, b in sizes)
    buf = torch.full((2, n_pairs, maxloc), float("nan"), dtype=torch.float64, device=x.device)
    nl = n_loc_pairs
    if nl:
        buf[0, :, :nl] = x.view(n_pairs, nl)
        buf[1, :, :nl] = y.view(n_pairs, nl)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    X = torch.empty((n_pairs, n_p), dtype=torch.float64, device=x.device)
    Y = torch.empty_like(X)
    for r, (a, b) in enumerate(sizes):
        X[:, a:b] = parts[r][0, :, : b - a]
        Y[:, a:b] = parts[r][1, :, : b - a]
    return X.reshape(-1), Y.reshape(-1)


def spot_statistics(x, y, i, n_fields, n_wl, ref_wl_index, group=None):
    """Centroid (reference wavelength), RMS and max spot radius per (field, wl) from
    sharded image-plane rays (spot_diagram.py:317-379) with two all_reduce calls.
    x, y, i: this rank's rays laid out [field][wl][local]."""
    n_pairs = n_fields * n_wl
    X = x.view(n_pairs, -1)
    Y = y.view(n_pairs, -1)
    m = (i.view(n_pairs, -1) > 0).to(torch.float64)
    Xm = torch.where(m > 0, X, torch.zeros_like(X))
    Ym = torch.where(m > 0, Y, torch.zeros_like(Y))
    sums = torch.stack([m.sum(1), Xm.sum(1), Ym.sum(1), (Xm * Xm).sum(1), (Ym * Ym).sum(1)], 1)
    if world_info(group)[1] > 1:
        dist.all_reduce(sums, group=group)
    cnt, sx, sy, sxx, syy = sums.unbind(1)
    mx = (sx / cnt).view(n_fields, n_wl)
    my = (sy / cnt).view(n_fields, n_wl)
    cx = mx[:, ref_wl_index].repeat_interleave(n_wl)
    cy = my[:, ref_wl_index].repeat_interleave(n_wl)
    # mean((x-cx)^2 + (y-cy)^2) = E[x^2] - 2 cx E[x] + cx^2 + (same in y)
    ex, ey = sx / cnt, sy / cnt
    ms = (sxx / cnt - 2 * cx * ex + cx * cx) + (syy / cnt - 2 * cy * ey + cy * cy)
    rms = torch.sqrt(torch.clamp(ms, min=0.0))
    r = torch.sqrt((X - cx[:, None]) ** 2 + (Y - cy[:, None]) ** 2)
    r = torch.where(m > 0, r, torch.full_like(r, -1.0))
    rmax = r.max(1).values if r.shape[1] else torch.full((n_pairs,), -1.0, dtype=torch.float64,
                                                            device=x.device)
    if world_info(group)[1] > 1:
        dist.all_reduce(rmax, op=dist.ReduceOp.MAX, group=group)
    return {
        "centroid": torch.stack([mx[:, ref_wl_index], my[:, ref_wl_index]], 1),
        "rms": rms.view(n_fields, n_wl),
        "geo": rmax.view(n_fields, n_wl),
        "count": cnt.view(n_fields, n_wl),
    }
