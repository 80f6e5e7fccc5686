"""Worker for tests/test_gpu_distributed.py: one rank of a world-size-2 job on cuda:0.

Both ranks share the one GPU of the test box, so the process group is gloo (RCCL refuses
two ranks on one device); the collectives of distributed.py run on CUDA tensors through
gloo exactly as they do through RCCL on a node. Each rank traces its slice of every
(field, wavelength) pair (trace_sharded, with the Newton schedule agreement), the image
plane is gathered into rank 0 (ImageGather) and the spot statistics are formed from the
per-rank device partials (ort_spot_partials, two all-gathers of a few doubles per pair).
"rt77" is config 4's shape (ReverseTelephoto, 7 fields x 7 wavelengths) at a few thousand
rays per pair."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from optiland_pr_amd import samples  # noqa: E402
from optiland_pr_amd.distributed import ImageGather, spot_statistics, trace_sharded  # noqa: E402

LENSES = {"dg": samples.DoubleGauss, "rt_asph": samples.ReverseTelephotoAsphere,
          "rt_asph_nan": samples.ReverseTelephotoAsphere, "rt77": samples.ReverseTelephoto}
FIELDS = [(0.0, 0.0), (0.0, 0.5), (0.0, 1.0)]
WAVELENGTHS = [0.4861, 0.5876, 0.6563]
N_P = 20011  # odd: the two shards differ in size by one


def case(name):
    """(fields, wavelengths, pupil points per pair) of a test case."""
    if name == "rt77":  # config 4: Hy = linspace(0, 1, 7), lambda = linspace(0.4861, 0.6563, 7)
        return ([(0.0, float(h)) for h in np.linspace(0, 1, 7)],
                [float(w) for w in np.linspace(0.4861, 0.6563, 7)], 3001)
    return FIELDS, WAVELENGTHS, N_P


def pupil(name):
    n_p = case(name)[2]
    rng = np.random.default_rng(0)
    r = np.sqrt(rng.uniform(size=n_p))
    th = 2 * np.pi * rng.uniform(size=n_p)
    px, py = r * np.cos(th), r * np.sin(th)
    if name.endswith("_nan"):
        # one ray that misses the lens (NaN), in the LAST shard only: that shard's Newton
        # surfaces run max_iter updates (the reference's global rule), the other shard
        # converges sooner on its own, and the schedule agreement must lift it to the
        # pair's max_iter (distributed._agree_newton_schedule's re-launch)
        px[-1] = py[-1] = 50.0
    return px, py


def run(name):
    """(rays, n_loc, schedule) of this rank's shard (the whole batch when no group is
    up); schedule = the Newton updates per (pair, surface) the trace ran (-1: none)."""
    from optiland_pr_amd.raytrace import lens_for

    fields, wls, _ = case(name)
    px, py = pupil(name)
    optic = LENSES[name]()
    rays, n_loc = trace_sharded(optic, fields, wls, px, py)
    dl = lens_for(optic, wls)  # the cached upload trace_sharded used
    keys = sorted(k for k in dl.sched_cache if k[0] == "shard")
    sched = np.stack([dl.sched_cache[k] for k in keys]) if keys else np.full((1, 1), -1)
    return rays, n_loc, sched


def main(rank, world, name, out):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fields, wls, n_p = case(name)
    rays, n_loc, sched = run(name)
    n_pairs = len(fields) * len(wls)
    g = ImageGather(n_pairs, n_p, rays.x.device)
    for _ in range(2):  # the pre-allocated buffers are reused
        planes = g.gather(rays.x, rays.y)
    extra = {}
    if name == "rt77":  # config 4's pipelined path: pair chunks traced into the send slab,
        # each chunk gathered asynchronously while the next traces
        from optiland_pr_amd.distribution import create_distribution  # noqa: F401
        from optiland_pr_amd.lowering import pupil_scalars, segment_params
        from optiland_pr_amd.distributed import PipelinedImageTrace, shard_range
        from optiland_pr_amd.raytrace import lens_for

        optic = LENSES[name]()
        dl = lens_for(optic, wls)
        EPL, EPD = pupil_scalars(optic)
        segs = np.stack([segment_params(optic, float(hx), float(hy), wi, EPL, EPD)
                         for hx, hy in fields for wi in range(len(wls))])
        px, py = pupil(name)
        a, b = shard_range(n_p, rank, world)
        pxl = torch.as_tensor(np.tile(np.asarray(px[a:b]), n_pairs), device=rays.x.device)
        pyl = torch.as_tensor(np.tile(np.asarray(py[a:b]), n_pairs), device=rays.x.device)
        g2 = ImageGather(n_pairs, n_p, rays.x.device)
        pipe = PipelinedImageTrace(dl, segs, pxl, pyl, g2, chunks=7)
        for _ in range(2):
            planes2 = pipe.run()
        if rank == 0:
            extra = {"X2": planes2[0].cpu().numpy(), "Y2": planes2[1].cpu().numpy(),
                     "zero_copy": pipe.zero_copy}
    st = spot_statistics(rays.x, rays.y, rays.i, len(fields), len(wls), len(wls) // 2)
    torch.cuda.synchronize()
    scheds = [None] * world
    dist.all_gather_object(scheds, sched)
    if rank == 0:
        np.savez(out, X=planes[0].cpu().numpy(), Y=planes[1].cpu().numpy(),
                 sched=np.stack(scheds), received=g.bytes_received,
                 **{k: v.cpu().numpy() for k, v in st.items()}, **extra)
    else:
        assert planes is None
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4])
