"""Config 1 (Cooke spot diagram, 37,932 rays) launch-overhead probe: is the step bound by the
host's graph launch or by the GPU? Times, per spot diagram,
  graph1   one HIP graph of one spot diagram, replayed (bench.py's step)
  graph10  one HIP graph of ten spot diagrams, replayed (the GPU's own rate)
  direct   the launches issued directly (ctypes -> ort_trace_spot), no graph
  replay0  replaying a graph of ONE trivial kernel (the launch floor)
    python tools/c1_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from optiland_pr_amd.analysis import SpotStatistics  # noqa: E402
from optiland_pr_amd.lowering import segment_params  # noqa: E402
from optiland_pr_amd.pupil import pupil_arrays  # noqa: E402
from optiland_pr_amd.raytrace import RealRays, lens_for, upload_segments  # noqa: E402
from optiland_pr_amd.samples import CookeTriplet  # noqa: E402


def rate(fn, reps, per):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * per) * 1e6


def main():
    dev = torch.device("cuda")
    lens = CookeTriplet()
    fields = [(0.0, 0.0), (0.0, 0.7), (0.0, 1.0)]
    dl = lens_for(lens, [0.55])
    px, py = pupil_arrays("uniform", 128, dev)
    n_p = px.numel()
    seg = upload_segments(np.stack([segment_params(lens, hx, hy, 0) for hx, hy in fields]), dev)
    out = RealRays.empty(n_p * 3, 0.55, device=dev)
    spot = SpotStatistics(3, 1, n_p, 0, lens.image_surface, dev)

    def once():
        spot.trace(dl, seg, px, py, out)

    once()
    torch.cuda.synchronize()
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        once()
    g10 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g10):
        for _ in range(10):
            once()
    x = torch.zeros(1, device=dev)
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g0):
        x.add_(1.0)
    res = {
        "graph1_us": rate(g1.replay, 2000, 1),
        "graph10_us": rate(g10.replay, 200, 10),
        "direct_us": rate(once, 2000, 1),
        "replay0_us": rate(g0.replay, 2000, 1),
    }
    print(res)


if __name__ == "__main__":
    main()
