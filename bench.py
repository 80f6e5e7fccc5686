"""Benchmark: ray-surface intersections/s, 10-surface double-Gauss, 1M pupil rays, fp64.

BASELINE.json metric "ray-surface intersections/sec at 1M pupil rays, 10-surf
double-Gauss" on configs[1]: DoubleGauss (samples/objectives.py:75-114; S = 12 traced
surfaces = len(surfaces) - 1), 1,000,000 random pupil rays (numpy default_rng, seed 0 +
rank), field Hy = 1 (14 deg), lambda = 0.5876 um, fp64.

One step = one fused launch (ort_trace_pupil) that generates the rays from the resident
pupil samples and traces them through every surface to the image plane, writing
x, y, z, L, M, N, i, opd to HBM: exactly RealRayTracer.trace's work
(real_ray_tracer.py:37-97) for one (field, wavelength) on 1M rays.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rays R] [--no-cpu]

N > 1: launched by torch.distributed.run, one process per GPU; every rank traces its
own 1M-ray shard (weak scaling, no collective on the data path); the elapsed time is
the max over ranks. value = N * R * S / time.
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


def _flops_per_ray(table):
    """Algorithmic fp64 operations per ray (+,-,*,/,sqrt each 1) counted from
    optiland_pr_amd/csrc/ort_core.h for the lowered surfaces (DESIGN.md 'Roofline')."""
    from optiland_pr_amd import _abi

    f = 20  # ray generation (ray_generator.py:71-89)
    for s in table.surfaces:
        g = int(s["geometry"])
        f += 3 * int(s["n_cs_loc"]) + 3 * int(s["n_cs_glob"])  # translate ops (no tilts here)
        f += 6 + 2 + 33  # propagate, opd, refract
        if g == _abi.GEOM_STANDARD:
            f += 45 + 20  # conic distance + normal
        elif g == _abi.GEOM_PLANE:
            f += 1
        if table.alpha_tab[0, int(s["mat_pre"])] > 0:
            f += 3
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-rays", type=int, default=1_000_000)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank if world > 1 else 0)

    from optiland_pr_amd import _native
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.lowering import segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil, upload_segments
    from optiland_pr_amd.samples import DoubleGauss

    _native.load()
    wl, Hx, Hy = 0.5876, 0.0, 1.0
    lens = DoubleGauss()
    dl = lens_for(lens, [wl])
    S = dl.table.n_surfaces
    R = args.rays
    d = RandomDistribution(seed=rank)  # rank 0 = the parity workload (seed 0)
    d.generate_points(R)
    px = torch.as_tensor(np.ascontiguousarray(d.x), device=dev)
    py = torch.as_tensor(np.ascontiguousarray(d.y), device=dev)
    seg = np.stack([segment_params(lens, Hx, Hy, 0)])
    seg_dev = upload_segments(seg, dev)
    out = RealRays.empty(R, wl, device=dev)

    def step():
        trace_pupil(dl, seg_dev, px, py, out, R, R, R)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # per-launch kernel time with HIP events on the stream the kernel is launched on
    # (torch's current stream: raytrace._stream_handle)
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    units = world * R * S  # ray-surface intersections per step, all ranks
    value = units * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        # algorithmic HBM bytes per launch: 16 B/ray pupil in + 64 B/ray rays out
        # (+ 64 B segment descriptor, negligible)
        bytes_per_launch = R * (16 + 64)
        achieved_gbs = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        flops = _flops_per_ray(dl.table) * R
        achieved_tf = flops / (kern_ms * 1e-3) / 1e12
        pmc = _pmc_summary()
        traffic = pmc.get("bytes_per_launch")
        hw_flops = pmc.get("fp64_flops_per_launch")
        line = {
            "metric": "ray-surface intersections/sec at 1M pupil rays, 10-surf double-Gauss",
            "value": value,
            "unit": "intersections/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (random pupil rays, numpy default_rng seed = rank)",
            "config": {
                "workload": "DoubleGauss (samples/objectives.py:75-114), 1 field Hy=1 (14 deg), "
                            "lambda 0.5876 um, fused ray generation + 12-surface trace to image",
                "rays_per_gpu": R,
                "surfaces": S,
                "intersections_per_step": units,
                "parallelism": f"dp{world} (ray shards, no collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": SPEC_HBM_TBPS * 1e3,
                "unit": "GB/s",
                "frac": achieved_gbs / (SPEC_HBM_TBPS * 1e3),
                "traffic": traffic,
                "kernel": "trace_closed_kernel<F_GEN> (ort_trace_pupil)",
                "kernel_ms": kern_ms,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "note": "the fused trace is FP64-VALU bound (see roofline_fp64); HBM frac is "
                        "reported because BASELINE asks for it",
            },
            "roofline_fp64": {
                "bound": "fp64_valu",
                "achieved": achieved_tf,
                "peak": SPEC_FP64_VEC_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tf / SPEC_FP64_VEC_TFLOPS,
                "flops_per_ray": _flops_per_ray(dl.table),
                "note": "achieved = algorithmic ops (+,-,*,/,sqrt = 1 each); the hardware "
                        "executes IEEE / and sqrt as ~10-instruction FMA sequences",
                "hw_counted": None if hw_flops is None else {
                    "fp64_flops_per_launch": hw_flops,
                    "achieved": hw_flops / (kern_ms * 1e-3) / 1e12,
                    "frac": hw_flops / (kern_ms * 1e-3) / 1e12 / SPEC_FP64_VEC_TFLOPS,
                    "source": "SQ_INSTS_VALU_FLOPS_FP64 x 64 (profiles/hbm_traffic.json)",
                },
            },
            "cpu_baseline": None if args.no_cpu else _cpu_baseline(lens, dl, seg, args.cpu_rays),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _pmc_summary():
    """Per-launch HBM bytes / FP64 FLOPs of the trace kernel from the committed
    rocprofv3 PMC summary (profiles/hbm_traffic.json, tools/profile_hbm.py); {} if absent."""
    p = os.path.join(HERE, "profiles", "hbm_traffic.json")
    try:
        with open(p) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _cpu_baseline(lens, dl, seg, n_rays):
    """The oracle (NumPy restatement of the reference, oracle/trace_np.py) timed on this
    host on the same workload: n_rays rays of the DoubleGauss, one process."""
    from oracle import trace_np
    from optiland_pr_amd.distribution import RandomDistribution

    d = RandomDistribution(seed=0)
    d.generate_points(n_rays)
    px, py = np.asarray(d.x), np.asarray(d.y)
    times = []
    for _ in range(2):
        t0 = time.perf_counter()
        r = trace_np.generate_rays(seg[0], px, py)
        trace_np.trace_segment(dl.table, r, 0)
        times.append(time.perf_counter() - t0)
    t = min(times)
    S = dl.table.n_surfaces
    return {
        "value": n_rays * S / t,
        "unit": "intersections/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{n_rays} DoubleGauss rays x {S} surfaces (generation + trace), NumPy "
                  f"oracle, 1 process, best of 2: {t:.2f} s on {platform.processor() or platform.machine()}",
    }


if __name__ == "__main__":
    main()
