"""Multi-GPU: ray batches sharded across one-process-per-GPU ranks (RCCL over xGMI).

SURVEY 8e: rays are independent, so every (field, wavelength) pair's pupil samples are
split into `world` contiguous, near-equal slices (global ray index = pair*N_p + offset);
each rank traces all pairs on its slice with the same lowered lens (no broadcast: every
rank lowers the lens itself). There is no collective on the trace's data path.

Two collectives exist only for the consumers:
  * ImageGather / gather_image_plane: image-plane intercepts to rank 0 (SpotDiagram
    plots, parity), one torch.distributed.gather into pre-allocated buffers (RCCL
    send / recv over xGMI: only rank 0 receives);
  * ShardedSpotStatistics / spot_statistics: centroid / RMS / max radius from per-rank
    partials of the device kernel (ort_spot_partials), two all-gathers of a few doubles
    per pair combined in rank order -- no intercepts move.
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


class ImageGather:
    """Image-plane intercepts of every rank to ONE rank (the RCCL gather of the
    final intercepts over xGMI): torch.distributed.gather (ncclSend / ncclRecv pairs under
    RCCL, each peer on its own xGMI link into rank dst), not an all-gather -- only dst
    receives. Buffers are allocated once (constructor) and reused by every gather: the
    per-rank send slab [fields][n_pairs][max local] (the tail of the shorter shards stays
    NaN) and, on dst, one receive slab per rank plus the reassembled [n_pairs][n_p] planes
    in the reference's order (real_ray_tracer.py:74-77).

    Pipelining (gather_pairs): the pairs can be gathered in chunks, each an asynchronous
    collective issued right after the launch that traced those pairs -- RCCL's stream
    waits for that launch only, so chunk k moves over xGMI while chunk k + 1 traces (a
    step costs max(trace, gather) instead of their sum). send_views() gives the send slab's
    rows as the trace's output columns (even shards), so nothing is copied before sending.

    dst is a rank of `group` (translated to the global rank the collective takes).
    Bytes: each rank sends fields x n_pairs x ceil(n_p / world) x 8; dst receives world - 1
    such slabs (config 4 at N = 8, (x, y): 196 MB out of every rank, 1.37 GB into rank 0;
    the all-gather this replaces moved 1.37 GB into EVERY rank)."""

    def __init__(self, n_pairs, n_p, device, fields=2, dst=0, group=None):
        self.rank, self.world = world_info(group)
        self.group = group
        self.dst = dst
        self.dst_global = dst
        if group is not None and self.world > 1:
            self.dst_global = dist.get_global_rank(group, dst)
        self.n_pairs, self.n_p, self.fields = n_pairs, n_p, fields
        self.sizes = [shard_range(n_p, r, self.world) for r in range(self.world)]
        self.maxloc = max(b - a for a, b in self.sizes)
        self.send = torch.full((fields, n_pairs, self.maxloc), float("nan"),
                               dtype=torch.float64, device=device)
        self.recv = None
        self.planes = None
        if self.rank == dst:
            self.recv = [torch.empty_like(self.send) for _ in range(self.world)]
            self.planes = torch.empty((fields, n_pairs, n_p), dtype=torch.float64,
                                      device=device)

    @property
    def bytes_sent(self):
        return 0 if self.world == 1 or self.rank == self.dst else self.send.numel() * 8

    @property
    def bytes_received(self):
        return (self.world - 1) * self.send.numel() * 8 if self.rank == self.dst else 0

    @property
    def local(self):
        a, b = self.sizes[self.rank]
        return b - a

    def send_views(self):
        """This rank's send rows as flat [n_pairs * local] columns (one per field) that a
        trace can write its outputs into directly, or None when this rank's shard is
        shorter than the slab rows (then gather_pairs copies)."""
        if self.local != self.maxloc:
            return None
        return [self.send[f].view(-1) for f in range(self.fields)]

    def gather_pairs(self, lo, hi, *cols, async_op=True):
        """Gather pairs [lo, hi): cols are this rank's [pair][local] columns (flat, the
        whole batch), or nothing when the trace wrote into send_views(). Returns the
        collectives' work handles (wait() them, or pass them to finish())."""
        nl = self.local
        if cols:
            for f, c in enumerate(cols):
                src = c.view(self.n_pairs, nl)[lo:hi]
                dstv = self.send[f, lo:hi, :nl]
                if src.data_ptr() != dstv.data_ptr():
                    dstv.copy_(src)
        works = []
        for f in range(self.fields):
            glist = [r[f, lo:hi] for r in self.recv] if self.rank == self.dst else None
            w = dist.gather(self.send[f, lo:hi], glist, dst=self.dst_global, group=self.group,
                            async_op=async_op)
            if w is not None:
                works.append(w)
        return works

    def finish(self, works, lo=0, hi=None, assemble=True):
        """Wait for gather_pairs' work handles; on dst, with assemble, lay pairs [lo, hi)
        out in the reference's order. Returns the [fields][n_pairs * n_p] planes on dst
        (None elsewhere)."""
        for w in works:
            w.wait()
        if self.rank != self.dst:
            return None
        hi = self.n_pairs if hi is None else hi
        if assemble:
            for r, (ra, rb) in enumerate(self.sizes):
                src = self.send if r == self.rank else self.recv[r]
                self.planes[:, lo:hi, ra:rb].copy_(src[:, lo:hi, : rb - ra])
        return self.planes.view(self.fields, -1)

    def gather(self, *cols):
        """cols: this rank's [pair][local] arrays (flat), one per field. Returns the
        [fields][n_pairs * n_p] planes on dst (None elsewhere)."""
        if self.world == 1:
            for f, c in enumerate(cols):
                self.planes[f].copy_(c.view(self.n_pairs, self.n_p))
            return self.planes.view(self.fields, -1)
        works = self.gather_pairs(0, self.n_pairs, *cols, async_op=False)
        return self.finish(works)


class PipelinedImageTrace:
    """This rank's shard of every (field, wavelength) pair traced in pair chunks, each
    chunk's image-plane x, y handed to an asynchronous ImageGather collective as soon as
    its launch is queued: RCCL gathers chunk k over xGMI while chunk k + 1 traces, so the
    step costs max(trace, gather) + one chunk instead of trace + gather (config 4 at
    N > 1). The trace writes x, y straight into the gather's send slab (even
    shards). Closed-form lenses only: a Newton lens's schedule check would synchronise
    every chunk (trace_sharded + ImageGather.gather serve those).

    px, py: this rank's pupil samples, [pair][local] on the device (pupil_per_ray);
    segs: the pairs' SEGMENT records (host)."""

    def __init__(self, dlens, segs, px, py, gather, chunks):
        from .raytrace import RealRays, upload_segments

        if dlens.newton:
            raise ValueError("PipelinedImageTrace: lenses without Newton surfaces only")
        self.dl, self.gather = dlens, gather
        n_pairs, nl = gather.n_pairs, gather.local
        n = n_pairs * nl
        self.out = RealRays.empty(n, 0.0, device=dlens.device)
        views = gather.send_views()
        self.zero_copy = views is not None
        if self.zero_copy:
            self.out.x, self.out.y = views[0], views[1]
        bounds = np.linspace(0, n_pairs, max(1, min(int(chunks), n_pairs)) + 1).astype(int)
        self.chunks = []
        for lo, hi in zip(bounds[:-1], bounds[1:], strict=True):
            if hi == lo:
                continue
            sub = RealRays.__new__(RealRays)
            for a in ("x", "y", "z", "L", "M", "N", "i", "opd"):
                setattr(sub, a, getattr(self.out, a)[lo * nl:hi * nl])
            sub.w = self.out.w
            self.chunks.append((int(lo), int(hi), upload_segments(segs[lo:hi], dlens.device),
                                px[lo * nl:hi * nl], py[lo * nl:hi * nl], sub))

    def trace_only(self):
        """The chunks' launches alone (timing)."""
        from .raytrace import trace_pupil

        nl = self.gather.local
        for lo, hi, seg_dev, pxc, pyc, sub in self.chunks:
            nc = (hi - lo) * nl
            trace_pupil(self.dl, seg_dev, pxc, pyc, sub, nc, nl, nc, pupil_per_ray=True)

    def run(self, assemble=True):
        """Trace + gather; returns the planes on the gather's dst (assembled into the
        reference's order when asked), None elsewhere."""
        from .raytrace import trace_pupil

        nl = self.gather.local
        works = []
        for lo, hi, seg_dev, pxc, pyc, sub in self.chunks:
            nc = (hi - lo) * nl
            if nc:
                trace_pupil(self.dl, seg_dev, pxc, pyc, sub, nc, nl, nc, pupil_per_ray=True)
            if self.gather.world > 1:
                cols = () if self.zero_copy else (self.out.x, self.out.y)
                works.append((lo, hi, self.gather.gather_pairs(lo, hi, *cols)))
        if self.gather.world == 1:
            return self.gather.gather(self.out.x, self.out.y)
        # chunk by chunk: the compute stream waits for chunk k's gather only, so dst lays
        # chunk k out in the reference's order while chunk k + 1 is still on xGMI
        planes = None
        for lo, hi, w in works:
            planes = self.gather.finish(w, lo, hi, assemble=assemble)
        return planes


def gather_image_plane(x, y, n_loc_pairs, n_pairs, n_p, group=None, dst=0):
    """One-shot ImageGather: (X, Y) of shape [n_pairs * n_p] on rank dst, (None, None)
    on the other ranks."""
    g = ImageGather(n_pairs, n_p, x.device, 2, dst, group)
    planes = g.gather(x, y)
    if planes is None:
        return None, None
    return planes[0], planes[1]


def combine_spot_partials(parts1, parts2=None):
    """Fixed-order (rank 0, 1, ...) combination of every rank's ort_spot_partials:
    parts1 [world][pairs][3] (count, sum x, sum y) -> sums1; parts2 [world][pairs][3]
    (sum r^2, max r, NaN flag) -> (sum r^2, max r, flag). The same order on every rank,
    so every rank holds the same bits."""
    s1 = parts1[0].clone()
    for r in range(1, parts1.shape[0]):
        s1 += parts1[r]
    if parts2 is None:
        return s1
    s2 = parts2[0].clone()
    for r in range(1, parts2.shape[0]):
        s2[:, 0] += parts2[r][:, 0]
        s2[:, 1:] = torch.maximum(s2[:, 1:], parts2[r][:, 1:])
    return s1, s2


def finalize_spot(s1, s2, n_fields, n_wl, ref_wl):
    """spot_diagram.py:317-357 from the combined sums: per pair (count, centroid x,
    centroid y, rms radius, max radius) -- the ort_spot_stats row layout -- and the
    dict of the earlier API (centroid of the reference wavelength, rms, geo, count)."""
    n = s1[:, 0]
    out = torch.empty((n_fields * n_wl, 5), dtype=torch.float64, device=s1.device)
    out[:, 0] = n
    out[:, 1] = s1[:, 1] / n
    out[:, 2] = s1[:, 2] / n
    out[:, 3] = torch.sqrt(s2[:, 0] / n)
    bad = (s2[:, 2] != 0) | torch.isnan(s2[:, 0]) | (n == 0)
    out[:, 4] = torch.where(bad, torch.full_like(n, float("nan")), s2[:, 1])
    pairs = out.view(n_fields, n_wl, 5)
    return out, {
        "centroid": pairs[:, ref_wl, 1:3],
        "rms": pairs[:, :, 3],
        "geo": pairs[:, :, 4],
        "count": pairs[:, :, 0],
    }


class ShardedSpotStatistics:
    """Spot-diagram statistics of sharded image rays (every rank holds its contiguous
    slice of every (field, wavelength) pair), with the reference's formulas
    (spot_diagram.py:317-357): two all-gathers of a few doubles per pair -- per-rank
    (count, sum x, sum y) from ort_spot_partials phase 1, combined in rank order into the
    global centroids; then per-rank (sum r^2, max r, NaN flag) about those centroids
    (phase 2) -- so no intercepts move and the rms is sqrt(sum r^2 / n) about the global
    centroid, as the reference forms it, not a one-pass E[x^2] - E[x]^2.

    phase_fn(phase, sums1) -> this rank's [pairs][3] partials (default: ort_spot_partials
    on `rays`, see run()); tests on CPU inject a NumPy restatement of it."""

    def __init__(self, n_fields, n_wl, n_loc, ref_wl, surface=None, device=None, group=None):
        self.n_fields, self.n_wl, self.n_loc, self.ref_wl = n_fields, n_wl, n_loc, ref_wl
        self.group = group
        self.rank, self.world = world_info(group)
        self.device = device
        self.pairs = n_fields * n_wl
        self._dev = None
        if device is not None and torch.device(device).type == "cuda":
            from .analysis import SpotStatistics

            # layout, image-frame ops and workspace of the local slice (no launch here)
            self._dev = SpotStatistics(n_fields, n_wl, n_loc, ref_wl, surface, device)
        dev = device if device is not None else "cpu"
        self.local = torch.zeros((2, self.pairs, 3), dtype=torch.float64, device=dev)
        self.gathered = torch.zeros((2, self.world, self.pairs, 3), dtype=torch.float64,
                                    device=dev)

    def _partials(self, rays, phase, sums1):
        import ctypes as C

        from . import _native
        from .raytrace import _ptr, _stream_handle

        d = self._dev
        out = self.local[phase - 1]
        rc = d._lib.ort_spot_partials(C.byref(rays.c_struct()), C.byref(d._lay), phase,
                                      _ptr(sums1), C.c_void_p(d._ws.data_ptr()), d._size,
                                      C.c_void_p(out.data_ptr()), _stream_handle())
        _native.check(rc, "ort_spot_partials")
        return out

    def run(self, rays=None, phase_fn=None):
        if phase_fn is None:
            if self._dev is None:
                raise RuntimeError("ShardedSpotStatistics needs the HIP device (ort_spot_partials)")
            phase_fn = lambda ph, s: self._partials(rays, ph, s)  # noqa: E731
        p1 = phase_fn(1, None)
        g1 = self._gather(0, p1)
        s1 = combine_spot_partials(g1)
        p2 = phase_fn(2, s1)
        g2 = self._gather(1, p2)
        s1, s2 = combine_spot_partials(g1, g2)
        return finalize_spot(s1, s2, self.n_fields, self.n_wl, self.ref_wl)

    def _gather(self, k, part):
        if self.world == 1:
            return part.unsqueeze(0)
        # rank r's rows land in gathered[k][r] (views of the pre-allocated buffer)
        dist.all_gather(list(self.gathered[k].unbind(0)), part.contiguous(), group=self.group)
        return self.gathered[k]


def spot_statistics(x, y, i, n_fields, n_wl, ref_wl_index, group=None, z=None):
    """Centroid (reference wavelength), RMS and max spot radius per (field, wl) of sharded
    image-plane rays (spot_diagram.py:317-379): ShardedSpotStatistics on the device.
    x, y, i: this rank's rays laid out [field][wl][local] (global image coordinates)."""
    from .raytrace import RealRays

    n_pairs = n_fields * n_wl
    n_loc = x.numel() // max(1, n_pairs)
    r = RealRays.__new__(RealRays)
    r.x, r.y, r.i = x, y, i
    r.z = z if z is not None else x
    r.L = r.M = r.N = r.opd = x
    st = ShardedSpotStatistics(n_fields, n_wl, n_loc, ref_wl_index, device=x.device,
                               group=group)
    return st.run(r)[1]
