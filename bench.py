"""Benchmark: ray-surface intersections/s, 10-surface double-Gauss, 1M pupil rays, fp64.

BASELINE.json metric "ray-surface intersections/sec at 1M pupil rays, 10-surf
double-Gauss" on configs[1] (the default, --config 2): DoubleGauss
(samples/objectives.py:75-114; S = 12 traced surfaces = len(surfaces) - 1), 1,000,000
random pupil rays (numpy default_rng, seed 0 + rank), field Hy = 1 (14 deg),
lambda = 0.5876 um, fp64.

One step = one fused launch (ort_trace_pupil) that generates the rays from the resident
pupil samples and traces them through every surface to the image plane, writing
x, y, z, L, M, N, i, opd to HBM: exactly RealRayTracer.trace's work
(real_ray_tracer.py:37-97) for one (field, wavelength) on 1M rays.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rays R] [--no-cpu]
                    [--config {1,2,3,4,5}]

N > 1: launched by torch.distributed.run, one process per GPU; every rank traces its
own 1M-ray shard (weak scaling, no collective on the data path); the elapsed time is
the max over ranks. value = N * R * S * K / time.

The other BASELINE configs are secondary measurements, same JSON shape:
  --config 1  Cooke triplet spot diagram (the reference's CPU-runnable case): 3 fields x
              1 lambda x uniform 128 pupil grid (12,644 rays per field), one step = the
              fused trace of the 3 pairs + the device spot statistics (ort_spot_stats:
              centroid, rms and max radius per pair), replayed as one HIP graph
  --config 3  RT-asph (even aspheres, Newton sag): 5 fields x 3 lambda x 4M pupil rays
              (60M rays, one launch, one Newton group per (field, lambda))
  --config 4  ReverseTelephoto 7 fields x 7 lambda x 2M rays per pair (seed = pair),
              98M rays sharded over the ranks (strong scaling) + all_gather of the image
              (x, y) over RCCL
  --config 5  TMA (3 Zernike mirrors), 1M random rays, Hy = 1: one optimisation step =
              lens update + differentiable trace + rms_spot_size + backward (VJP kernel)
              + Adam step on the 30 coefficients
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SPEC_HBM_TBPS = 8.0        # MI355X_MICROARCH.md: 8.0 TB/s spec HBM3E
SPEC_FP64_VEC_TFLOPS = 78.6  # AMD MI355X FP64 vector spec (not in the local guide)


def _flops_per_ray(table, sched=None):
    """Algorithmic fp64 operations per ray (+,-,*,/,sqrt each 1) counted from
    optiland_pr_amd/csrc/ort_core.h for the lowered surfaces (DESIGN.md 'Roofline').
    Closed-form surfaces, and even aspheres given the Newton schedule `sched` [S] (updates
    per surface; every ray makes them, plus the stop-test evaluation whose normal the
    interaction takes): the conic start (45), per evaluation the point P(t) (6), the sag +
    normal with nc coefficients (23 + 12 nc: even_asphere.py:82-129 as written in
    sagnorm_even) and f = sag - z (1), per update the step t - f / f' (8). None when a
    surface kind is not counted."""
    from optiland_pr_amd import _abi

    f = 20  # ray generation (ray_generator.py:71-89)
    for si, s in enumerate(table.surfaces):
        g = int(s["geometry"])
        f += 3 * int(s["n_cs_loc"]) + 3 * int(s["n_cs_glob"])  # translate ops (no tilts here)
        f += 6 + 2 + 33  # propagate, opd, refract
        if g == _abi.GEOM_STANDARD:
            f += 45 + 20  # conic distance + normal
        elif g == _abi.GEOM_PLANE:
            f += 1
        elif g == _abi.GEOM_EVEN_ASPHERE and sched is not None:
            U = int(sched[si])
            f += 45 + (U + 1) * (30 + 12 * int(s["n_coef"])) + 8 * U
        else:
            return None
        if table.alpha_tab[0, int(s["mat_pre"])] > 0:
            f += 3
    return f


class Workload:
    """One bench configuration: step() is the timed unit; units = intersections/step;
    ramp_steps = untimed steps that keep the GPU busy ~0.5 s before the warmup."""

    ramp_steps = 64

    def __init__(self, **kw):
        self.__dict__.update(kw)


def _pupil(seed, n, dev, torch):
    from optiland_pr_amd.distribution import RandomDistribution

    d = RandomDistribution(seed=seed)
    d.generate_points(n)
    return (torch.as_tensor(np.ascontiguousarray(d.x), device=dev),
            torch.as_tensor(np.ascontiguousarray(d.y), device=dev), d)


def config1(args, dev, rank, world, torch):
    from optiland_pr_amd.analysis import SpotStatistics
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.pupil import pupil_arrays
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil, upload_segments
    from optiland_pr_amd.samples import CookeTriplet

    wl, fields = 0.55, [(0.0, 0.0), (0.0, 0.7), (0.0, 1.0)]
    lens = CookeTriplet()
    dl = lens_for(lens, [wl])
    S = dl.table.n_surfaces
    px, py = pupil_arrays("uniform", 128, dev)
    n_p = px.numel()
    seg_dev = upload_segments(np.stack([segment_params(lens, hx, hy, 0) for hx, hy in fields]),
                              dev)
    n = n_p * len(fields)
    out = RealRays.empty(n, wl, device=dev)
    img = lens.image_surface

    spot = SpotStatistics(len(fields), 1, n_p, 0, img, dev)

    def once():  # trace + statistics pass 1 in one kernel, then the 2 other passes
        return spot.trace(dl, seg_dev, px, py, out)

    once()  # closed-form lens: one launch, no host sync, no allocation -> capturable
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        stats = once()
    state = {"stats": stats}

    def step():
        graph.replay()

    return Workload(
        metric="ray-surface intersections/sec, Cooke triplet spot diagram (3 fields x "
               "uniform-128 pupil) incl. device spot statistics",
        unit="intersections/s", units=world * n * S, step=step, scaling="weak",
        config={"workload": "CookeTriplet (samples/objectives.py:46-72), fields Hy 0 / 0.7 / 1 "
                            "(0 / 14 / 20 deg), lambda 0.55 um, uniform 128 (12,644 rays per "
                            "field): fused trace of the 3 pairs with the statistics' first "
                            "pass in its epilogue, then the second pass and the totals "
                            "(ort_trace_spot), one HIP graph replay per step",
                "rays_per_gpu": n, "surfaces": S,
                "parallelism": f"dp{world} (replicas, no collective)"},
        kernel="trace_closed_kernel<F_GEN|F_SPOT> + spot_dev + spot_final (graph)",
        launches=3,
        bytes_per_launch=None, flops_per_ray=None, pmc_file=None, rays=n, state=state,
        spot=True, data="synthetic (the reference's uniform 128 pupil grid)", ramp_steps=24000)


def config2(args, dev, rank, world, torch):
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil, upload_segments
    from optiland_pr_amd.samples import DoubleGauss

    wl, Hx, Hy = 0.5876, 0.0, 1.0
    lens = DoubleGauss()
    dl = lens_for(lens, [wl])
    S = dl.table.n_surfaces
    R = args.rays
    px, py, _ = _pupil(rank, R, dev, torch)  # rank 0 = the parity workload (seed 0)
    seg = np.stack([segment_params(lens, Hx, Hy, 0)])
    seg_dev = upload_segments(seg, dev)
    out = RealRays.empty(R, wl, device=dev)

    def step():
        trace_pupil(dl, seg_dev, px, py, out, R, R, R)

    flops = _flops_per_ray(dl.table)
    return Workload(
        metric="ray-surface intersections/sec at 1M pupil rays, 10-surf double-Gauss",
        unit="intersections/s", units=world * R * S, step=step, scaling="weak",
        config={
            "workload": "DoubleGauss (samples/objectives.py:75-114), 1 field Hy=1 (14 deg), "
                        "lambda 0.5876 um, fused ray generation + 12-surface trace to image",
            "rays_per_gpu": R, "surfaces": S, "intersections_per_step": world * R * S,
            "parallelism": f"dp{world} (ray shards, no collective)"},
        kernel="trace_closed_kernel<F_GEN> (ort_trace_pupil)", launches=1,
        bytes_per_launch=R * (16 + 64), flops_per_ray=flops, pmc_file="hbm_traffic.json",
        rays=R, ramp_steps=max(64, 90_000_000_000 // max(1, R * S)))


def config3(args, dev, rank, world, torch):
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil, upload_segments
    from optiland_pr_amd.samples import ReverseTelephotoAsphere

    wls = [0.4861, 0.5876, 0.6563]
    fields = [(0.0, float(h)) for h in np.linspace(0, 1, 5)]
    lens = ReverseTelephotoAsphere()
    dl = lens_for(lens, wls)
    S = dl.table.n_surfaces
    n_p = args.rays if args.rays != 1_000_000 else 4_000_000
    px, py, _ = _pupil(rank, n_p, dev, torch)
    EPL, EPD = lens.paraxial.EPL(), lens.paraxial.EPD()
    seg = np.stack([segment_params(lens, hx, hy, wi, EPL, EPD)
                    for hx, hy in fields for wi in range(len(wls))])
    seg_dev = upload_segments(seg, dev)
    n = n_p * len(seg)
    out = RealRays.empty(n, 0.0, device=dev)
    keys = [("bench3", k) for k in range(len(seg))]

    def step():
        trace_pupil(dl, seg_dev, px, py, out, n, n_p, n_p, keys=keys, newton_mode=args.newton_mode)

    # the verified Newton schedule fixes the work per ray: count the algorithmic flops with
    # the mean updates per surface over the (field, lambda) groups
    flops = None
    if args.newton_mode == "reference":
        step()
        sched = np.mean(np.stack([dl.sched_cache[k] for k in keys]), axis=0)
        flops = _flops_per_ray(dl.table, np.rint(sched))

    return Workload(
        metric="ray-surface intersections/sec, RT-asph even-asphere (Newton sag), 5 fields x "
               "3 lambda x 4M pupil rays",
        unit="intersections/s", units=world * n * S, step=step, scaling="weak",
        config={"workload": "ReverseTelephoto + even aspheres on surfaces 2, 13 (SURVEY 8d.3), "
                            "5 fields x 3 lambda, one launch, Newton group per pair",
                "rays_per_gpu": n, "pupil_per_pair": n_p, "surfaces": S,
                "newton_mode": args.newton_mode,
                "parallelism": f"dp{world} (ray shards, no collective)"},
        kernel="trace_kernel<F_GEN|KM_EVEN> (ort_trace_pupil)", launches=1,
        bytes_per_launch=n_p * 16 + n * 64, flops_per_ray=flops, pmc_file="hbm_traffic_c3.json",
        compute_pmc_file="r05_config3_pmc_compute.json", rays=n)


def config4(args, dev, rank, world, torch):
    from optiland_pr_amd import distributed
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil, upload_segments
    from optiland_pr_amd.samples import ReverseTelephoto

    wls = [float(w) for w in np.linspace(0.4861, 0.6563, 7)]
    fields = [(0.0, float(h)) for h in np.linspace(0, 1, 7)]
    lens = ReverseTelephoto()
    dl = lens_for(lens, wls)
    S = dl.table.n_surfaces
    n_p = args.rays if args.rays != 1_000_000 else 2_000_000
    EPL, EPD = lens.paraxial.EPL(), lens.paraxial.EPD()
    pairs = [(hx, hy, wi) for hx, hy in fields for wi in range(len(wls))]
    seg = np.stack([segment_params(lens, hx, hy, wi, EPL, EPD) for hx, hy, wi in pairs])
    a, b = distributed.shard_range(n_p, rank, world)
    n_loc = b - a
    from optiland_pr_amd.distribution import RandomDistribution

    pxs, pys = [], []
    for k in range(len(pairs)):  # seed = pair index; this rank's slice of every pair
        d = RandomDistribution(seed=k)
        d.generate_points(n_p)
        pxs.append(d.x[a:b])
        pys.append(d.y[a:b])
    px = torch.as_tensor(np.concatenate(pxs), device=dev)
    py = torch.as_tensor(np.concatenate(pys), device=dev)
    seg_dev = upload_segments(seg, dev)
    n = n_loc * len(pairs)
    out = RealRays.empty(n, 0.0, device=dev)
    # N > 1: the image-plane gather into rank 0 (send / receive buffers allocated here,
    # once), pipelined with the trace: 7 chunks of 7 pairs, each chunk's x, y traced into
    # the send slab and gathered asynchronously (RCCL on its own stream) while the next
    # chunk traces (distributed.PipelinedImageTrace); rank 0 lays each chunk out in the
    # reference's pair-major order as soon as that chunk has arrived (inside the step, as
    # in rounds 1-3; round 4 had left the reassembly out of the timed step)
    gather = pipe = None
    if world > 1:
        gather = distributed.ImageGather(len(pairs), n_p, dev)
        pipe = distributed.PipelinedImageTrace(dl, seg, px, py, gather, chunks=args.gather_chunks)

    def step():
        if pipe is not None:
            pipe.run(assemble=True)
        else:
            trace_pupil(dl, seg_dev, px, py, out, n, n_loc, n, pupil_per_ray=True)

    def trace_ms(steps):
        """Device time of the trace launches alone (at N > 1 the step also gathers): events
        on the launch stream around them, over extra steps after the timed region."""
        stream = torch.cuda.current_stream()
        spans = []
        for _ in range(steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            if pipe is not None:
                pipe.trace_only()
            else:
                trace_pupil(dl, seg_dev, px, py, out, n, n_loc, n, pupil_per_ray=True)
            e1.record(stream)
            spans.append((e0, e1))
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in spans) / steps

    def gather_report(reps=5):
        """After the timed region (every rank): bytes a rank sends, bytes rank 0
        receives, the max-over-ranks time of the gather alone (all chunks, nothing
        tracing) and of the trace alone, and the pipelined step: gather_exposed_ms =
        step - trace is what the overlap did not hide."""
        if gather is None:
            return {"gather_bytes_per_rank": 0, "gather_bytes_into_rank0": 0, "gather_ms": 0.0}
        import torch.distributed as dist

        def timed(fn):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64,
                             device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item()) * 1e3

        g_ms = timed(lambda: gather.finish(gather.gather_pairs(0, len(pairs)), assemble=False))
        a_ms = timed(lambda: gather.finish([], assemble=True))
        t_ms = timed(pipe.trace_only)
        s_ms = timed(lambda: pipe.run(assemble=True))
        recv = torch.tensor([gather.bytes_received], dtype=torch.float64, device=dev)
        dist.all_reduce(recv, op=dist.ReduceOp.MAX)
        return {"gather_bytes_per_rank": gather.send.numel() * 8,
                "gather_bytes_into_rank0": int(recv.item()), "gather_ms": g_ms,
                "assemble_ms": a_ms, "trace_ms": t_ms, "pipelined_step_ms": s_ms,
                "step_includes": "trace + gather + rank 0's reassembly into the reference's "
                                 "pair-major order",
                "gather_exposed_ms": max(0.0, s_ms - t_ms),
                "gather_hidden_ms": max(0.0, g_ms - max(0.0, s_ms - t_ms)),
                "gather_chunks": len(pipe.chunks), "gather_zero_copy": pipe.zero_copy}

    return Workload(
        metric="ray-surface intersections/sec, ReverseTelephoto 7 fields x 7 lambda x 2M rays, "
               "sharded + RCCL gather of image-plane hits",
        unit="intersections/s", units=n_p * len(pairs) * S, step=step, scaling="strong",
        config={"workload": "ReverseTelephoto (samples/objectives.py:117-173), 49 (field, "
                            "lambda) pairs x 2M rays (seed = pair), gather of image x,y to rank 0",
                "rays_total": n_p * len(pairs), "surfaces": S,
                "parallelism": f"dp{world} (pupil shards of every pair) + gather to rank 0"},
        kernel="trace_closed_kernel<F_GEN> (ort_trace_pupil)", launches=1,
        bytes_per_launch=n * (16 + 64), flops_per_ray=None, pmc_file="hbm_traffic_c4.json",
        rays=n, extra=gather_report, trace_timer=trace_ms if world > 1 else None,
        traffic_scale=n / (n_p * len(pairs)))  # the PMC pass traced all pairs on one GPU


def config5(args, dev, rank, world, torch):
    from optiland_pr_amd.autodiff import CapturedStep
    from optiland_pr_amd.operands import RayOperand
    from optiland_pr_amd.optim import ZernikeAdam
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    R = args.rays
    _, _, d = _pupil(rank, R, dev, torch)
    use_graph = not args.eager
    S = 4

    def problem(capturable):
        """The TMA with device-resident coefficient leaves, its Adam and loss."""
        lens = ThreeMirrorAnastigmat(args.zernike_scheme)
        # Newton schedules verified on the device once warm (ort_newton_fixup): the same
        # schedules and results as the host check, without its per-step host round trip;
        # range errors / unsettled schedules surface at raytrace.check_all_pending (below)
        lens.newton_mode = "device"
        leaves = []
        for si in (1, 2, 3):
            g = lens.surface_group.surfaces[si].geometry
            # device-resident parameters: the uploaded lens table is patched on the device,
            # the gradient and the Adam state stay in HBM (no per-step host round trip)
            t = torch.tensor(np.asarray(g.coefficients), dtype=torch.float64, device=dev,
                             requires_grad=True)
            g.coefficients = t
            leaves.append(t)
        # torch.optim.Adam's update fused with the lens-table patch (optim.ZernikeAdam: ONE
        # launch for torch's two fused-Adam kernels and the next trace's patch; the same bits,
        # tests/test_gpu_optim.py); --torch-adam: torch.optim.Adam(fused=True) + the patch.
        # Capturable either way: step counts on the device, so the step can be a graph replay
        if args.torch_adam:
            opt = torch.optim.Adam(leaves, lr=1e-7, fused=True, capturable=capturable)
        else:
            opt = ZernikeAdam(leaves, [lens], lr=1e-7)

        def loss_fn():
            return RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, R, 0.587, d)

        return lens, opt, loss_fn

    lens, opt, loss_fn = problem(use_graph)
    state = {}

    def eager_step_of(opt, loss_fn, keep):
        def step():
            opt.zero_grad()
            loss = loss_fn()
            loss.backward()
            opt.step()
            if keep:
                state["loss"] = loss.detach()  # read once after the timed region
        return step

    eager_step = eager_step_of(opt, loss_fn, True)
    # the backward's device time (vjp_timer) is measured on eager steps of a SECOND copy of
    # the problem: eager steps of the captured lens itself would overwrite the replays'
    # Newton flags and reuse the autograd nodes the capture's outputs keep alive
    _, opt_t, loss_t = problem(False) if use_graph else (lens, opt, loss_fn)
    timer_step = eager_step_of(opt_t, loss_t, False) if use_graph else eager_step

    # the whole optimisation step -- coefficient patch, taped trace with its device-verified
    # Newton rounds, rms_spot, the adjoint VJP, the fused Adam update -- as ONE HIP graph
    # replay (autodiff.CapturedStep): the host issues one launch per step instead of ~40
    # 
    captured = CapturedStep(loss_fn, opt, lenses=[lens])

    def graph_step():
        state["loss"] = captured()

    def check():  # the captured device-verified Newton rounds: flags of the last replay
        if captured.graph is not None:
            captured.check()

    state["check"] = check
    step = graph_step if use_graph else eager_step

    return Workload(
        metric="TMA Zernike optimisation steps: ray-surface intersections/sec of forward + "
               "backward (d rms_spot / d coeff) at 1M rays",
        unit="intersections/s", units=world * R * S, step=step, scaling="weak",
        config={"workload": f"TMA (Tutorial_7d), 3 {args.zernike_scheme}-Zernike mirrors x 10 "
                            "coefficients, 1M random rays, Hy=1, lambda 0.587: lens update + "
                            "trace + rms_spot_size + backward (VJP) + Adam",
                "zernike_scheme": args.zernike_scheme,
                "optimizer": "torch.optim.Adam(fused=True) + patch" if args.torch_adam else
                             "optim.ZernikeAdam (torch Adam's update + the lens patch, one launch)",
                "rays_per_gpu": R, "surfaces": S, "parameters": 30,
                "parallelism": f"dp{world} (independent replicas)",
                "step_issue": "one HIP graph replay per step (captured after 3 eager steps)"
                              if use_graph else "eager (torch ops + ctypes launches)"},
        kernel="adj_kernel<KM_ZERN, 2> (ort_trace_pupil_vjp, adjoint mode)", launches=None,
        bytes_per_launch=None, flops_per_ray=None, pmc_file="hbm_traffic_c5.json", rays=R,
        state=state, vjp_timer=vjp_timer, eager_step=timer_step, ramp_steps=720,
        # the taped forward writes the tape, the adjoint only reads it: per traced surface the
        # incoming ray and t (7 rows) plus, for a Newton surface, the min(U, 4) iterates it
        # replays (ort_sweep.h adj_ray), with U the verified schedule -- read after the run
        tape_bytes_per_launch=lambda: _tape_read_bytes(lens, R),
        # the adjoint launch's algorithmic HBM bytes: the tape read, the pupil samples
        # (16 B/ray), the primal outputs it reads (L, M, N, i and, for the rms gradient
        # folded into its cotangent load, x, y: 48 B/ray; no cotangent buffers) and the
        # block partials written (the monomial slots of the Zernike surfaces, per 256 rays)
        algorithmic_bytes_per_launch=lambda: (_tape_read_bytes(lens, R) + (16 + 48) * R
                                              + _mono_slots(lens) * 8 * (R // 256)))


def _mono_slots(lens):
    """The adjoint's monomial-basis slots (ops.mono_slot_count) of the lowered lens."""
    from optiland_pr_amd import ops

    dl = next(iter(getattr(lens, "_lowered", {}).values()), None)
    return 0 if dl is None else ops.mono_slot_count(dl.table, True)


def _tape_read_bytes(lens, R):
    """Tape bytes the adjoint reads per launch: 7 rows per traced surface plus min(U, kHist)
    Newton iterates per Newton surface (the rows the taped forward writes)."""
    from optiland_pr_amd import _abi

    dl = next(iter(getattr(lens, "_lowered", {}).values()), None)
    if dl is None:
        return None
    U = dl.sched_cache.get("_default")
    rows = 0
    for si, srow in enumerate(dl.table.surfaces):
        rows += 7
        if int(srow["geometry"]) in _abi.NEWTON_GEOMETRIES:
            rows += min(int(U[si]) if U is not None else 4, 4)
    return rows * 8 * R


def vjp_timer(step, steps, torch):
    """Device time of the backward's ort_trace_pupil_vjp launch sequence (adj_need +
    adj_kernel + adj_param_reduce; adj_kernel is ~97% of it): events recorded on
    the launch stream around every call (autodiff.VJP_EVENTS), over `steps` extra steps
    run after the timed region so the event pairs do not touch the timed steps."""
    from optiland_pr_amd import autodiff

    autodiff.VJP_EVENTS = []
    try:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        spans = [a.elapsed_time(b) for a, b in autodiff.VJP_EVENTS]
    finally:
        autodiff.VJP_EVENTS = None
    return sum(spans) / len(spans)


CONFIGS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--newton-mode", default="reference", choices=["reference", "wave"],
                    help="config 3: the reference's global Newton stop rule (exact) or the "
                         "per-wavefront stop (within the Newton tolerance)")
    ap.add_argument("--gather-chunks", type=int, default=7,
                    help="config 4 at N > 1: pair chunks of the pipelined trace + gather")
    ap.add_argument("--torch-adam", action="store_true",
                    help="config 5: torch.optim.Adam(fused=True) and the trace's own coefficient "
                         "patch instead of the fused optim.ZernikeAdam launch")
    ap.add_argument("--zernike-scheme", default="fringe", choices=["fringe", "standard", "noll"],
                    help="config 5: the Zernike indexing of the TMA mirrors (SURVEY 8d.5 names "
                         "fringe and standard; standard / noll normals omit the normalisation "
                         "constant, zernike.py:162-231)")
    ap.add_argument("--eager", action="store_true",
                    help="config 5: issue the optimisation step eagerly instead of as one HIP "
                         "graph replay")
    ap.add_argument("--cpu-rays", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=1.5,
                    help="wall time of the multi-process CPU baseline leg")
    ap.add_argument("--ramp-steps", type=int, default=None,
                    help="untimed steps before the warmup so the GPU clock has ramped "
                         "(MI355X power management raises the engine clock only under "
                         "sustained load: the first ~50 ms of launches run up to 15%% "
                         "slower); default: the config's own count, ~0.5 s of its steps")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N > 1 (nccl = RCCL, one GPU per rank); gloo "
                         "lets several ranks share a GPU (rank r on device r mod count) to "
                         "rehearse the multi-rank path on a one-GPU box")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU baseline runs first, before anything touches the GPU (its worker processes
    # are forked from this one)
    cpu_line = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu_line = _cpu_baseline(args)

    import torch
    import torch.distributed as dist

    dev_idx = 0
    if world > 1:
        dev_idx = local_rank if args.backend == "nccl" else local_rank % torch.cuda.device_count()
        torch.cuda.set_device(dev_idx)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", dev_idx)

    from optiland_pr_amd import _native

    _native.load()
    w = CONFIGS[args.config](args, dev, rank, world, torch)

    # clock ramp (untimed): keep the GPU busy until its engine clock has risen (~0.5 s of
    # load), then the W warmup steps. A FIXED number of ramp steps per config (not a wall
    # time), so the work before the timed region -- and config 5's optimisation trajectory,
    # hence its final_loss -- is the same on every run
    n_ramp = args.ramp_steps if args.ramp_steps is not None else w.ramp_steps
    for k in range(n_ramp):
        w.step()
        if k % 8 == 7:
            torch.cuda.synchronize()
    for _ in range(args.warmup):
        w.step()
    torch.cuda.synchronize()

    # device time of the step's kernel(s): HIP events on the stream they are launched on
    # (torch's current stream: raytrace._stream_handle) at both ends of the timed region;
    # per step = that span / K (kernel + the ~1 us launch gap between back-to-back
    # kernels; an event pair around every step would itself add ~6 us to each step)
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        w.step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = step_dev_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    value = w.units * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    # results of the timed steps themselves, read before anything else runs: the captured
    # step's device-verified Newton flags (config 5: vjp_timer's eager steps below share
    # the flag buffers and would overwrite them) and the last timed step's loss
    final_loss = None
    if getattr(w, "state", None) and not getattr(w, "spot", False):
        from optiland_pr_amd import raytrace

        raytrace.check_all_pending()  # device-verified Newton schedules: raise here
        if "check" in w.state:
            w.state["check"]()
        loss = w.state.get("loss")
        final_loss = None if loss is None else float(loss)
    extra = w.extra() if getattr(w, "extra", None) else None  # every rank (collectives)
    if getattr(w, "vjp_timer", None):
        w.vjp_ms = w.vjp_timer(getattr(w, "eager_step", w.step), max(3, min(args.steps, 20)),
                               torch)
    if getattr(w, "trace_timer", None):
        kern_ms = w.trace_timer(max(3, min(args.steps, 20)))

    if rank == 0:
        line = {
            "metric": w.metric,
            "value": value,
            "unit": w.unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": w.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": getattr(w, "data", "synthetic (random pupil rays, numpy default_rng seed = rank)"),
            "config": w.config,
            "roofline": _roofline(w, kern_ms),
            "timing": {"clock_ramp_steps": n_ramp,
                       "device_ms_per_step": step_dev_ms,
                       "kernel_time": "HIP events at both ends of the timed region / steps"
                       + ("; roofline kernel_ms = the trace launch alone (events around "
                          "each launch, after the timed region: the step also gathers)"
                          if getattr(w, "trace_timer", None) else "")},
        }
        if w.flops_per_ray is not None:
            line["roofline_fp64"] = _roofline_fp64(w, kern_ms)
        S = w.config.get("surfaces")
        if S:  # the reference notebook counts len(surfaces) = S + 1 per ray
            line["counting_convention"] = {
                "surfaces_counted_in_value": S,
                "reference_notebook_surfaces_per_ray": S + 1,
                "note": "value counts traced surfaces only; the reference's notebook counts "
                        "len(surfaces) = S + 1 per ray (the object surface computes no "
                        "intersection): multiply by (S + 1) / S to compare with its figures"}
        if getattr(w, "spot", False):
            st = w.state["stats"].cpu().numpy()
            line["config"]["rms_spot_radius_mm"] = [float(v) for v in st[:, 3]]
            line["config"]["geo_spot_radius_mm"] = [float(v) for v in st[:, 4]]
        elif getattr(w, "state", None):
            line["config"]["final_loss"] = final_loss
            line["config"]["steps_before_timed"] = n_ramp + args.warmup
        if extra:
            line["config"].update(extra)
        line["cpu_baseline"] = cpu_line
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _val(v):
    return v() if callable(v) else v


def _roofline(w, kern_ms):
    if getattr(w, "spot", False):
        return {"bound": "launch", "achieved": None, "peak": None, "unit": None, "frac": None,
                "traffic": None, "kernel": w.kernel, "step_device_ms": kern_ms,
                "note": "38K rays per step: launch / latency bound (3 kernels in one graph); "
                        "the per-intersection roofline is config 2's"}
    if getattr(w, "vjp_ms", None):
        # multi-launch optimisation step: the roofline is the backward's adjoint kernel,
        # timed live (vjp_timer); FP64 FLOPs and HBM bytes per launch from its PMC passes
        pmc = _pmc_summary(w.pmc_file)
        flops = pmc.get("fp64_flops_per_launch")
        achieved = None if flops is None else flops / (w.vjp_ms * 1e-3) / 1e12
        return {"bound": "fp64_valu", "achieved": achieved, "peak": SPEC_FP64_VEC_TFLOPS,
                "unit": "TFLOP/s",
                "frac": None if achieved is None else achieved / SPEC_FP64_VEC_TFLOPS,
                "traffic": pmc.get("bytes_per_launch"), "kernel": w.kernel,
                "kernel_ms": w.vjp_ms, "step_device_ms": kern_ms,
                "tape_bytes_per_launch": _val(w.tape_bytes_per_launch),
                "algorithmic_bytes_per_launch": _val(w.algorithmic_bytes_per_launch),
                "hbm_frac": None if pmc.get("bytes_per_launch") is None else
                pmc["bytes_per_launch"] / (w.vjp_ms * 1e-3) / 1e9 / (SPEC_HBM_TBPS * 1e3),
                "note": "achieved = hardware-counted FP64 FLOPs of adj_kernel "
                        f"(SQ_INSTS_VALU_FLOPS_FP64 x 64, profiles/{w.pmc_file}) / the live "
                        "device time of the ort_trace_pupil_vjp launch sequence; traffic = "
                        "its rocprofv3 FETCH/WRITE bytes; the taped forward writes the tape, "
                        "the adjoint only reads it (tape_bytes_per_launch)"}
    if w.bytes_per_launch is None:
        return {"bound": "fp64_valu", "achieved": None, "peak": SPEC_FP64_VEC_TFLOPS,
                "unit": "TFLOP/s", "frac": None, "traffic": None, "kernel": w.kernel,
                "step_device_ms": kern_ms,
                "note": "multi-launch step; per-kernel times in profiles/r02_*_kernel_stats.csv"}
    pmc = _pmc_summary(w.pmc_file)
    achieved = w.bytes_per_launch / (kern_ms * 1e-3) / 1e9
    return {
        "bound": "hbm",
        "achieved": achieved,
        "peak": SPEC_HBM_TBPS * 1e3,
        "unit": "GB/s",
        "frac": achieved / (SPEC_HBM_TBPS * 1e3),
        "traffic": None if pmc.get("bytes_per_launch") is None else
        pmc["bytes_per_launch"] * getattr(w, "traffic_scale", 1.0),
        "kernel": w.kernel,
        "kernel_ms": kern_ms,
        "algorithmic_bytes_per_launch": w.bytes_per_launch,
        "note": "the fused trace is FP64-VALU bound (see roofline_fp64); HBM frac is "
                "reported because BASELINE asks for it",
    }


def _roofline_fp64(w, kern_ms):
    pmc = _pmc_summary(w.pmc_file)
    hw_flops = pmc.get("fp64_flops_per_launch")
    src = w.pmc_file
    per_wave = {}
    cpmc = _pmc_summary(getattr(w, "compute_pmc_file", None))
    if cpmc.get("counters"):  # the kernel's compute counters (tools/pmc_c3.sh passes)
        c = cpmc["counters"]
        src = w.compute_pmc_file
        hw_flops = c["SQ_INSTS_VALU_FLOPS_FP64"] * 64
        per_wave = {k: cpmc["derived"][k] for k in (
            "valu_insts_per_wave", "fp64_valu_insts_per_wave", "salu_insts_per_wave")
            if k in cpmc.get("derived", {})}
    achieved_tf = w.flops_per_ray * w.rays / (kern_ms * 1e-3) / 1e12
    return {
        "bound": "fp64_valu",
        "achieved": achieved_tf,
        "peak": SPEC_FP64_VEC_TFLOPS,
        "unit": "TFLOP/s",
        "frac": achieved_tf / SPEC_FP64_VEC_TFLOPS,
        "flops_per_ray": w.flops_per_ray,
        "note": "achieved = algorithmic ops (+,-,*,/,sqrt = 1 each); the hardware "
                "executes IEEE / and sqrt as ~10-instruction FMA sequences",
        "hw_counted": None if hw_flops is None else {
            "fp64_flops_per_launch": hw_flops,
            "achieved": hw_flops / (kern_ms * 1e-3) / 1e12,
            "frac": hw_flops / (kern_ms * 1e-3) / 1e12 / SPEC_FP64_VEC_TFLOPS,
            "source": f"SQ_INSTS_VALU_FLOPS_FP64 x 64 (profiles/{src})",
            **per_wave,
        },
    }


def _pmc_summary(name):
    """Per-launch HBM bytes / FP64 FLOPs of the trace kernel from the committed
    rocprofv3 PMC summary (profiles/<name>, tools/profile_hbm.py); {} if absent."""
    if not name:
        return {}
    try:
        with open(os.path.join(HERE, "profiles", name)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _cpu_workload(args):
    """(lens table, segments, rays per pair, pairs used, label) of the bench config, host
    only: the same lowered table and ray-generation scalars the GPU gets."""
    from optiland_pr_amd.lowering import lower_surface_group, segment_params
    from optiland_pr_amd import samples

    if args.config == 1:
        lens = samples.CookeTriplet()
        table = lower_surface_group(lens.surface_group, [0.55])
        segs = np.stack([segment_params(lens, 0.0, h, 0) for h in (0.0, 0.7, 1.0)])
        return table, segs, None, "Cooke (uniform 128)"
    if args.config == 2:
        lens = samples.DoubleGauss()
        table = lower_surface_group(lens.surface_group, [0.5876])
        segs = np.stack([segment_params(lens, 0.0, 1.0, 0)])
        return table, segs, args.cpu_rays, "DoubleGauss"
    if args.config == 3:
        lens = samples.ReverseTelephotoAsphere()
        wls = [0.4861, 0.5876, 0.6563]
        table = lower_surface_group(lens.surface_group, wls)
        segs = np.stack([segment_params(lens, 0.0, float(h), wi)
                         for h in np.linspace(0, 1, 5) for wi in range(3)])[:3]
        return table, segs, max(1, args.cpu_rays // 10), "RT-asph"
    if args.config == 4:
        lens = samples.ReverseTelephoto()
        wls = [float(w) for w in np.linspace(0.4861, 0.6563, 7)]
        table = lower_surface_group(lens.surface_group, wls)
        segs = np.stack([segment_params(lens, 0.0, float(h), wi)
                         for h in np.linspace(0, 1, 7) for wi in range(7)])[:3]
        return table, segs, max(1, args.cpu_rays // 10), "ReverseTelephoto"
    lens = samples.ThreeMirrorAnastigmat(getattr(args, "zernike_scheme", "fringe"))
    table = lower_surface_group(lens.surface_group, [0.587])
    segs = np.stack([segment_params(lens, 0.0, 1.0, 0)])
    return table, segs, max(1, args.cpu_rays // 10), "TMA (forward trace only: the oracle " \
        "has no derivative path)"


_CPU = {}


def _cpu_task(k_lo_hi):
    """One worker's share: generate + trace rays [lo, hi) of pair k with the oracle."""
    from oracle import trace_np

    k, lo, hi = k_lo_hi
    table, segs, px, py = _CPU["w"]
    r = trace_np.generate_rays(segs[k], px[lo:hi], py[lo:hi])
    trace_np.trace_segment(table, r, int(segs[k]["lambda_idx"]))
    return hi - lo


def _cpu_baseline(args):
    """The oracle (NumPy restatement of the reference, oracle/trace_np.py) on this host's
    cores: a bounded sample of the bench workload (up to 3 (field, lambda) pairs) split
    into contiguous ray chunks over a pool of forked worker processes (each chunk is its
    own trace call: for Newton lenses the global stop rule then spans a chunk). As
    BASELINE.md's plan asks: one warm-up, then the median of (at least) 5 timed
    repetitions, for the pool (repeated until ~--cpu-seconds of wall time) and for one
    process. Workers: the CPUs this process may run on (sched_getaffinity), capped by the
    box's CPU share (OMP_NUM_THREADS, 16 per GPU on the GPU pool: os.cpu_count() there is
    the whole machine's 256)."""
    import multiprocessing as mp

    from optiland_pr_amd.distribution import RandomDistribution

    table, segs, n_rays, label = _cpu_workload(args)
    if n_rays is None:  # config 1: the uniform 128 grid of the reference's spot diagram
        from optiland_pr_amd.distribution import create_distribution

        d = create_distribution("uniform")
        d.generate_points(128)
        n_rays = int(np.asarray(d.x).size)
    else:
        d = RandomDistribution(seed=0)
        d.generate_points(n_rays)
    px, py = np.asarray(d.x), np.asarray(d.y)
    _CPU["w"] = (table, segs, px, py)
    S = table.n_surfaces
    units = n_rays * len(segs) * S

    def sample():
        for k in range(len(segs)):
            _cpu_task((k, 0, n_rays))

    sample()  # warm-up
    singles = []
    for _ in range(5):
        t0 = time.perf_counter()
        sample()
        singles.append(time.perf_counter() - t0)
    t_single = float(np.median(singles))
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (
        os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS") or affinity)
    workers = max(1, min(affinity, share))
    chunk = -(-n_rays // workers)
    tasks = [(k, lo, min(n_rays, lo + chunk)) for k in range(len(segs))
             for lo in range(0, n_rays, chunk)]
    with mp.get_context("fork").Pool(workers) as pool:
        pool.map(_cpu_task, tasks, chunksize=1)  # warm-up repetition
        # repeat the sample until ~args.cpu_seconds of wall time, at least 5 times
        times = []
        t_all = time.perf_counter()
        while True:
            t0 = time.perf_counter()
            pool.map(_cpu_task, tasks, chunksize=1)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() - t_all >= args.cpu_seconds and len(times) >= 5:
                break
    reps = len(times)
    t = float(np.median(times))
    ratio = _ref_over_oracle()
    value = units / t
    line = {
        "value": value,
        "unit": "intersections/s",
        "cores": workers,
        "kind": "port",
        "single_process_value": units / t_single,
        "host_cpus": os.cpu_count(),
        "affinity_cpus": affinity,
        "cpu_share": share,
        "cpu_model": _cpu_model(),
        "statistic": "median of the timed repetitions after one warm-up",
        "sample": f"{label}: {n_rays} rays x {len(segs)} (field, lambda) pair(s) x {S} "
                  f"surfaces (generation + trace), NumPy oracle; {workers} processes, median "
                  f"of {reps} repetitions {t:.3f} s (1 process: median of 5, {t_single:.3f} s); "
                  f"workers = min(CPUs in this process's affinity mask {affinity}, the box's CPU "
                  f"share OMP_NUM_THREADS {share}) of the {os.cpu_count()} host CPUs",
    }
    if ratio:
        # the reference itself (Optiland's NumPy backend) is slower than its restatement:
        # tests/golden/cpu_ratio.json times both single-process on one host
        line["ref_over_oracle"] = ratio["ref_over_oracle"]
        line["reference_estimate_value"] = value / ratio["ref_over_oracle"]
        line["ref_over_oracle_source"] = (
            f"tests/golden/cpu_ratio.json: {ratio['workload']}; reference "
            f"{ratio['reference_seconds']:.2f} s, oracle {ratio['oracle_seconds']:.2f} s on "
            f"{ratio['cpu_model']} ({ratio['method']})")
    return line


def _cpu_model():
    """The host CPU's model name (/proc/cpuinfo), as lscpu prints it."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _ref_over_oracle():
    try:
        with open(os.path.join(HERE, "tests", "golden", "cpu_ratio.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


if __name__ == "__main__":
    main()
