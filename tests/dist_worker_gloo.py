"""Worker for tests/test_distributed_cpu.py: one gloo rank (run as a subprocess).

The trace needs the GPU; here each rank's "image-plane rays" are its slice of synthetic
arrays, so the data movement (ImageGather: gather to rank 0 into pre-allocated buffers)
and the sharded statistics' collectives and rank-ordered combination
(ShardedSpotStatistics) are under test. The per-rank partials, which ort_spot_partials
computes on the GPU, come from spot_partials_np below (test-only restatement)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from optiland_pr_amd.distributed import ImageGather, ShardedSpotStatistics, shard_range  # noqa: E402

N_FIELDS, N_WL, N_P = 3, 2, 101
REF_WL = 1


def full_rays():
    rng = np.random.default_rng(7)
    x = rng.normal(size=(N_FIELDS * N_WL, N_P))
    y = rng.normal(size=(N_FIELDS * N_WL, N_P)) + 3.0
    i = (rng.uniform(size=(N_FIELDS * N_WL, N_P)) > 0.1).astype(np.float64)
    return x, y, i


def spot_partials_np(x, y, i, phase, sums1):
    """ort_spot_partials (csrc/ort_k_spot.hip) restated for [pair][local] arrays."""
    out = np.zeros((x.shape[0], 3))
    for p in range(x.shape[0]):
        m = i[p] > 0
        if phase == 1:
            out[p] = [m.sum(), x[p][m].sum(), y[p][m].sum()]
        else:
            ref = (p // N_WL) * N_WL + REF_WL
            cx, cy = sums1[ref][1] / sums1[ref][0], sums1[ref][2] / sums1[ref][0]
            r2 = (x[p][m] - cx) ** 2 + (y[p][m] - cy) ** 2
            out[p] = [r2.sum(), np.sqrt(r2).max() if r2.size else 0.0, 0.0]
    return torch.as_tensor(out)


def main(rank, world, out):
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, y, i = full_rays()
    a, b = shard_range(N_P, rank, world)
    xl, yl, il = (np.ascontiguousarray(v[:, a:b]) for v in (x, y, i))
    g = ImageGather(N_FIELDS * N_WL, N_P, "cpu")
    res = {}
    for rep in range(2):  # the buffers are reused
        planes = g.gather(torch.as_tensor(xl).reshape(-1), torch.as_tensor(yl).reshape(-1))
        if rank == 0:
            res[f"X{rep}"], res[f"Y{rep}"] = planes[0].numpy().copy(), planes[1].numpy().copy()
        else:
            assert planes is None
    res["sent"], res["received"] = g.bytes_sent, g.bytes_received
    # the pipelined form: pairs gathered in 3 chunks with asynchronous collectives, then
    # finished (and laid out) chunk by chunk
    n_pairs = N_FIELDS * N_WL
    xt, yt = torch.as_tensor(xl).reshape(-1), torch.as_tensor(yl).reshape(-1)
    bounds = [0, 2, 5, n_pairs]
    pending = [(lo, hi, g.gather_pairs(lo, hi, xt, yt)) for lo, hi in zip(bounds[:-1], bounds[1:])]
    for lo, hi, works in pending:
        planes = g.finish(works, lo, hi)
    if rank == 0:
        res["Xc"], res["Yc"] = planes[0].numpy().copy(), planes[1].numpy().copy()
    st = ShardedSpotStatistics(N_FIELDS, N_WL, b - a, REF_WL)
    rows, d = st.run(phase_fn=lambda ph, s1: spot_partials_np(
        xl, yl, il, ph, None if s1 is None else s1.numpy()))
    res["rows"] = rows.numpy()
    res.update({k: v.numpy() for k, v in d.items()})
    np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3])
