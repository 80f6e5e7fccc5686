"""Golden summaries at the BASELINE configs' own sizes, from the
REFERENCE run here; writes tests/golden/config_sizes.json.

  config 1  Cooke triplet, fields Hy = 0 / 0.7 / 1 (of 20 deg), 0.55 um, uniform 128
            (12,644 rays per field): SpotDiagram(num_rings=128, distribution="uniform")
            centroids, geometric and rms radii (spot_diagram.py:317-357, 381-438);
  config 3  RT-asph (ReverseTelephoto + even aspheres on surfaces 2, 13), 3 of the 15
            (field, lambda) pairs (Hy = linspace(0, 1, 5), lambda 0.4861 / 0.5876 / 0.6563)
            at the full 4M random pupil rays, seed = pair index: the same sums;
  config 4  ReverseTelephoto, 3 of the 49 (field, lambda) pairs (Hy = linspace(0, 1, 7),
            lambda = linspace(0.4861, 0.6563, 7)) at the full 2M random pupil rays,
            seed = pair index (the bench's sampling): NumPy sums of the image x, y, opd,
            sum x^2, the NaN count and the first / last ray.

Test infrastructure only: imports /root/reference, never runs on the GPU box.

    PYTHONPATH=tests/golden/shims:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_config_sizes.py
"""

from __future__ import annotations

import json
import os
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

CONFIG4_PAIRS = (0, 24, 48)  # pair = field index * 7 + wavelength index
CONFIG3_PAIRS = (0, 7, 14)  # pair = field index * 3 + wavelength index


def config1():
    from optiland.analysis import SpotDiagram
    from optiland.samples.objectives import CookeTriplet

    lens = CookeTriplet()
    t0 = time.perf_counter()
    spot = SpotDiagram(lens, wavelengths=[0.55], num_rings=128, distribution="uniform")
    secs = time.perf_counter() - t0
    return dict(
        fields=[[float(a), float(b)] for a, b in lens.fields.get_field_coords()],
        centroid=[[float(a), float(b)] for a, b in spot.centroid()],
        geo=[[float(v) for v in row] for row in spot.geometric_spot_radius()],
        rms=[[float(v) for v in row] for row in spot.rms_spot_radius()],
        seconds=secs,
    )


def config4():
    from optiland.distribution import RandomDistribution
    from optiland.samples.objectives import ReverseTelephoto

    lens = ReverseTelephoto()
    hys = np.linspace(0, 1, 7)
    wls = np.linspace(0.4861, 0.6563, 7)
    out = {}
    for k in CONFIG4_PAIRS:
        hy, wl = float(hys[k // 7]), float(wls[k % 7])
        d = RandomDistribution(seed=k)
        d.generate_points(2_000_000)
        t0 = time.perf_counter()
        r = lens.trace(0.0, hy, wl, num_rays=2_000_000, distribution=d)
        secs = time.perf_counter() - t0
        x, y, opd = (np.asarray(getattr(r, a)) for a in ("x", "y", "opd"))
        out[str(k)] = dict(
            hy=hy, wavelength=wl, n=int(x.size), nan=int(np.isnan(x).sum()), seconds=secs,
            sum_x=float(np.sum(x)), sum_y=float(np.sum(y)), sum_opd=float(np.sum(opd)),
            sum_x2=float(np.sum(x * x)),
            first=[float(x[0]), float(y[0]), float(opd[0])],
            last=[float(x[-1]), float(y[-1]), float(opd[-1])],
        )
        print(k, out[str(k)])
    return out


def _sums(r):
    x, y, opd = (np.asarray(getattr(r, a)) for a in ("x", "y", "opd"))
    return dict(
        n=int(x.size), nan=int(np.isnan(x).sum()),
        sum_x=float(np.sum(x)), sum_y=float(np.sum(y)), sum_opd=float(np.sum(opd)),
        sum_x2=float(np.sum(x * x)),
        first=[float(x[0]), float(y[0]), float(opd[0])],
        last=[float(x[-1]), float(y[-1]), float(opd[-1])],
    )


def config3():
    import sys

    sys.path.insert(0, HERE)
    from gen_golden import rt_asph
    from optiland.distribution import RandomDistribution

    lens = rt_asph()
    hys = np.linspace(0, 1, 5)
    wls = (0.4861, 0.5876, 0.6563)
    out = {}
    for k in CONFIG3_PAIRS:
        hy, wl = float(hys[k // 3]), float(wls[k % 3])
        d = RandomDistribution(seed=k)
        d.generate_points(4_000_000)
        t0 = time.perf_counter()
        r = lens.trace(0.0, hy, wl, num_rays=4_000_000, distribution=d)
        out[str(k)] = dict(hy=hy, wavelength=wl, seconds=time.perf_counter() - t0, **_sums(r))
        print(k, out[str(k)])
    return out


def main():
    import sys

    import optiland.backend as be

    be.set_backend("numpy")
    path = os.path.join(HERE, "config_sizes.json")
    if "--config3" in sys.argv:  # add config 3 to the existing file
        with open(path) as f:
            res = json.load(f)
        res["config3"] = config3()
        with open(path, "w") as f:
            json.dump(res, f, indent=1)
        return
    res = {"config1": config1(), "config3": config3(), "config4": config4()}
    with open(os.path.join(HERE, "config_sizes.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
