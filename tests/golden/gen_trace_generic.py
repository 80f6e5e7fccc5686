"""Golden vectors for Optic.trace_generic (optic.py:611-632 -> real_ray_tracer.py:99-133),
from the REFERENCE run here; writes tests/golden/trace_generic.npz.

Cases (per-ray field AND pupil coordinates, the call's array form):
  cooke       Hx = 0, Hy = 0.7 scalars, 600 random pupil points, 0.55 um
  dg          Hx, Hy, Px, Py all per-ray arrays (1,000 rays), 0.5876 um
  rt_asph     per-ray Hy and pupil, even aspheres (Newton), 0.4861 um
  cooke_vig   Cooke with vignetted fields (vx, vy per field; get_vig_factor's nearest
              field scales the pupil, real_ray_tracer.py:113-116), per-ray Hy

Test infrastructure only: imports /root/reference, never runs on the GPU box.

    PYTHONPATH=tests/golden/shims:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_trace_generic.py
"""

from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

VIG_FIELDS = [(0.0, 0.0, 0.0), (14.0, 0.1, 0.2), (20.0, 0.2, 0.35)]  # (y, vx, vy)


def inputs(case):
    rng = np.random.default_rng({"cooke": 1, "dg": 2, "rt_asph": 3, "cooke_vig": 4}[case])
    n = {"cooke": 600, "dg": 1000, "rt_asph": 800, "cooke_vig": 700}[case]
    r = np.sqrt(rng.uniform(size=n))
    th = 2 * np.pi * rng.uniform(size=n)
    px, py = r * np.cos(th), r * np.sin(th)
    if case == "cooke":
        return 0.0, 0.7, px, py, 0.55
    if case == "dg":
        return rng.uniform(-0.7, 0.7, n), rng.uniform(-0.7, 0.7, n), px, py, 0.5876
    if case == "rt_asph":
        return np.zeros(n), rng.uniform(0.0, 1.0, n), px, py, 0.4861
    return np.zeros(n), rng.uniform(0.0, 1.0, n), px, py, 0.5876


def lens(case):
    import gen_golden as g

    if case in ("cooke", "cooke_vig"):
        lens = g.CookeTriplet()
        if case == "cooke_vig":
            lens.fields.fields = []
            for y, vx, vy in VIG_FIELDS:
                lens.add_field(y=y, vx=vx, vy=vy)
        return lens
    if case == "dg":
        return g.DoubleGauss()
    return g.rt_asph()


def main():
    import sys

    sys.path.insert(0, HERE)
    import optiland.backend as be

    be.set_backend("numpy")
    out = {}
    for case in ("cooke", "dg", "rt_asph", "cooke_vig"):
        hx, hy, px, py, wl = inputs(case)
        r = lens(case).trace_generic(hx, hy, px, py, wl)
        out[f"{case}_in"] = np.stack(np.broadcast_arrays(hx, hy, px, py)).astype(np.float64)
        out[f"{case}_wl"] = np.float64(wl)
        out[f"{case}_out"] = np.stack([np.asarray(getattr(r, a), dtype=np.float64)
                                       for a in ("x", "y", "z", "L", "M", "N", "i", "opd")])
        print(case, out[f"{case}_out"].shape, int(np.isnan(out[f"{case}_out"][0]).sum()))
    np.savez_compressed(os.path.join(HERE, "trace_generic.npz"), **out)


if __name__ == "__main__":
    main()
