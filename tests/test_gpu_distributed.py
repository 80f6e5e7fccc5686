"""Sharded trace on the GPU (distributed.py): a world-size-2 job of two ranks on
cuda:0 (gloo: RCCL refuses two ranks on one device) traces every (field, wavelength)
pair's pupil slices, agrees the Newton schedule across the shards, gathers the image plane
into rank 0 (ImageGather; for config 4's shape also the pipelined trace + chunked
asynchronous gather, PipelinedImageTrace) and reduces the spot statistics. The gathered image plane must be bit-identical to
the unsharded trace of the whole batch: the shards are a partition of the rays, and the
agreed schedule is the reference's global stopping rule over the whole pair
(newton_raphson.py:148), so no ray may see a different number of Newton updates."""

import os
import subprocess
import sys

import numpy as np
import pytest

from tests.dist_worker_gpu import case, run
from tests.test_distributed_cpu import _free_port

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU tests need the MI355X (torch.cuda.is_available() is False)")
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dg", "rt_asph", "rt_asph_nan", "rt77"])
def test_sharded_trace_equals_unsharded(torch, tmp_path, name):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               OMP_NUM_THREADS="1")
    out = tmp_path / "r0.npz"
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_gpu.py"),
                               str(r), "2", name, str(out)], env=env) for r in range(2)]
    try:
        rcs = [p.wait(timeout=100) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0]
    got = np.load(out)

    FIELDS, WAVELENGTHS, N_P = case(name)
    rays, n, sched = run(name)  # no process group here: the whole batch in one launch
    assert n == N_P
    # every shard ran the whole pair's schedule (the agreement); with the NaN ray in the
    # last shard only, that is max_iter on the asphere surfaces for the first shard too
    for r in range(2):
        np.testing.assert_array_equal(got["sched"][r], sched)
    if name == "rt_asph_nan":
        assert sched.max() == 100
    x = rays.x.cpu().numpy()
    y = rays.y.cpu().numpy()
    np.testing.assert_array_equal(got["X"], x)  # NaNs compare equal here
    np.testing.assert_array_equal(got["Y"], y)
    if name == "rt77":  # the pipelined trace + chunked asynchronous gather (config 4, N > 1)
        assert bool(got["zero_copy"])  # 3,001 rays per pair split 1,501 / 1,500: rank 0 even
        np.testing.assert_array_equal(got["X2"], x)
        np.testing.assert_array_equal(got["Y2"], y)
    if name.endswith("_nan"):
        nf, nw = len(FIELDS), len(WAVELENGTHS)
        bad = np.isnan(x.reshape(nf * nw, N_P))
        assert bad[:, -1].all() and not bad[:, :-1].any()
        return
    assert not np.isnan(x).any()

    # spot statistics from the per-rank device partials vs ort_spot_stats on the unsharded
    # image (counts exact; sums in another order: rtol 1e-12) and the reference's formulas
    # (spot_diagram.py:317-357) on the unsharded image plane
    from optiland_pr_amd.analysis import spot_statistics as unsharded_stats

    nf, nw = len(FIELDS), len(WAVELENGTHS)
    ref_wl = nw // 2
    rows = unsharded_stats(rays, nf, nw, N_P, ref_wl).cpu().numpy().reshape(nf, nw, 5)
    np.testing.assert_array_equal(got["count"], rows[:, :, 0])
    # (small spots far off axis: a last-bit centroid difference moves the radii by
    # ~1e-16 mm, hence the absolute term)
    np.testing.assert_allclose(got["rms"], rows[:, :, 3], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["geo"], rows[:, :, 4], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(got["centroid"], rows[:, ref_wl, 1:3], rtol=1e-12)
    X, Y = x.reshape(nf * nw, N_P), y.reshape(nf * nw, N_P)
    for f in range(nf):
        cx, cy = X[f * nw + ref_wl].mean(), Y[f * nw + ref_wl].mean()
        for w in range(nw):
            p = f * nw + w
            d2 = (X[p] - cx) ** 2 + (Y[p] - cy) ** 2
            np.testing.assert_allclose(got["rms"][f, w], np.sqrt(d2.mean()), rtol=1e-12,
                                       atol=1e-15)
            np.testing.assert_allclose(got["geo"][f, w], np.sqrt(d2.max()), rtol=1e-12,
                                       atol=1e-15)
            assert got["count"][f, w] == N_P
    half = -(-N_P // 2)  # rank 0 received one padded (x, y) slab from rank 1
    assert int(got["received"]) == 2 * nf * nw * half * 8
