"""Reference-vs-oracle CPU speed ratio (bench.py's cpu_baseline reports it beside the
oracle's rate): both run here, single process, on the config-2 workload (DoubleGauss,
1M random pupil rays seed 0, field Hy = 1, lambda 0.5876, generation + 12-surface trace),
median of 3 after one warm-up, time.perf_counter. Writes tests/golden/cpu_ratio.json.

Test infrastructure only: imports the REFERENCE (/root/reference), never runs on the GPU
box. Invocation (repo root):

    PYTHONPATH=tests/golden/shims:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_cpu_ratio.py
"""

from __future__ import annotations

import json
import os
import platform
import statistics
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.machine()


def _median(fn, reps=3):
    fn()  # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def main():
    import optiland.backend as be
    from optiland.distribution import RandomDistribution as RefRandom
    from optiland.samples.objectives import DoubleGauss as RefDG

    from oracle import trace_np
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.lowering import lower_surface_group, segment_params
    from optiland_pr_amd.samples import DoubleGauss

    be.set_backend("numpy")
    n = 1_000_000
    d_ref = RefRandom(seed=0)
    d_ref.generate_points(n)
    ref_lens = RefDG()
    t_ref = _median(lambda: ref_lens.trace(0.0, 1.0, 0.5876, num_rays=n, distribution=d_ref))

    lens = DoubleGauss()
    table = lower_surface_group(lens.surface_group, [0.5876])
    seg = segment_params(lens, 0.0, 1.0, 0)
    d = RandomDistribution(seed=0)
    d.generate_points(n)
    px, py = np.asarray(d.x), np.asarray(d.y)

    def oracle():
        trace_np.trace_segment(table, trace_np.generate_rays(seg, px, py), 0)

    t_oracle = _median(oracle)
    out = {
        "workload": "DoubleGauss 1M random rays (seed 0), Hy=1, 0.5876 um, generation + trace",
        "reference_seconds": t_ref,
        "oracle_seconds": t_oracle,
        "ref_over_oracle": t_ref / t_oracle,
        "cpu_model": _cpu_model(),
        "method": "single process, median of 3 after one warm-up",
    }
    with open(os.path.join(HERE, "cpu_ratio.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
