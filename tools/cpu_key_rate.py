"""Measurement tooling (container only: imports the reference from /root/reference, which
the GPU box does not have): the CPU dispatch key of torch.ops.ort.trace_sequential
(liboptiland_host.so) against the reference's own SurfaceGroup.trace loop on the same
CPU tensors -- the reference's torch backend on the CPU, float64 -- through
adapter.install(), as a caller of the reference would see it.

usage: PYTHONPATH=/root/reference:. python tools/cpu_key_rate.py [n_rays] [threads]
"""
import json
import os
import sys
import time

import numpy as np


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else (os.cpu_count() or 1)
    import torch

    import optiland.backend as be
    from optiland.samples.objectives import DoubleGauss

    from optiland_pr_amd import _native, adapter

    be.set_backend("torch")
    be.set_device("cpu")
    be.set_precision("float64")
    torch.set_num_threads(threads)
    _native.load_host().ort_host_set_threads(threads)
    lens = DoubleGauss()

    def run():
        t0 = time.perf_counter()
        lens.trace(0.0, 1.0, 0.5876, num_rays=n, distribution="random")
        dt = time.perf_counter() - t0
        sg = lens.surface_group
        return dt, np.asarray(sg.x[-1]).copy(), np.asarray(sg.y[-1]).copy()

    out = {}
    for mode in ("reference", "installed"):
        if mode == "installed":
            adapter.install()
        run()  # warm-up (lowering cache, material tables)
        times, x, y = [], None, None
        for _ in range(3):
            dt, x, y = run()
            times.append(dt)
        out[mode] = dict(seconds=float(np.median(times)), x=x, y=y)
        if mode == "installed":
            adapter.uninstall()
    S = len(lens.surface_group.surfaces) - 1
    rep = {
        "rays": n, "surfaces": S, "threads": threads,
        "reference_s": out["reference"]["seconds"], "installed_s": out["installed"]["seconds"],
        "speedup": out["reference"]["seconds"] / out["installed"]["seconds"],
        "installed_intersections_per_s": n * S / out["installed"]["seconds"],
        "max_abs_dx": float(np.nanmax(np.abs(out["reference"]["x"] - out["installed"]["x"]))),
        "max_abs_dy": float(np.nanmax(np.abs(out["reference"]["y"] - out["installed"]["y"]))),
        "stats": adapter.STATS,
    }
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
