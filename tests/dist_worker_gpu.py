"""Worker for tests/test_gpu_distributed.py: one rank of a world-size-2 job on cuda:0.

Both ranks share the one GPU of the test box, so the process group is gloo (RCCL refuses
two ranks on one device); the collectives of distributed.py run on CUDA tensors through
gloo exactly as they do through RCCL on a node. Each rank traces its slice of every
(field, wavelength) pair (trace_sharded, with the Newton schedule agreement) and rank 0
saves the all-gathered image plane."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from optiland_pr_amd import samples  # noqa: E402
from optiland_pr_amd.distributed import gather_image_plane, spot_statistics, trace_sharded  # noqa: E402

LENSES = {"dg": samples.DoubleGauss, "rt_asph": samples.ReverseTelephotoAsphere,
          "rt_asph_nan": samples.ReverseTelephotoAsphere}
FIELDS = [(0.0, 0.0), (0.0, 0.5), (0.0, 1.0)]
WAVELENGTHS = [0.4861, 0.5876, 0.6563]
N_P = 20011  # odd: the two shards differ in size by one


def pupil(name):
    rng = np.random.default_rng(0)
    r = np.sqrt(rng.uniform(size=N_P))
    th = 2 * np.pi * rng.uniform(size=N_P)
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

    px, py = pupil(name)
    optic = LENSES[name]()
    rays, n_loc = trace_sharded(optic, FIELDS, WAVELENGTHS, px, py)
    dl = lens_for(optic, WAVELENGTHS)  # the cached upload trace_sharded used
    keys = sorted(k for k in dl.sched_cache if k[0] == "shard")
    sched = np.stack([dl.sched_cache[k] for k in keys]) if keys else np.full((1, 1), -1)
    return rays, n_loc, sched


def main(rank, world, name, out):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rays, n_loc, sched = run(name)
    n_pairs = len(FIELDS) * len(WAVELENGTHS)
    X, Y = gather_image_plane(rays.x, rays.y, n_loc, n_pairs, N_P)
    st = spot_statistics(rays.x, rays.y, rays.i, len(FIELDS), len(WAVELENGTHS), 1)
    torch.cuda.synchronize()
    scheds = [None] * world
    dist.all_gather_object(scheds, sched)
    if rank == 0:
        np.savez(out, X=X.cpu().numpy(), Y=Y.cpu().numpy(), sched=np.stack(scheds),
                 **{k: v.cpu().numpy() for k, v in st.items()})
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4])
