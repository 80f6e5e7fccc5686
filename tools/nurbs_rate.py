"""Throughput of the NURBS kernels (measurement tooling, not product): the samples'
NurbsLens (a fitted conic in front, an explicit rational net behind; two (u, v) solves per
NURBS surface and ray -- distance and normal) traced at 1M pupil rays with ort_trace_pupil,
HIP events around N launches on the launch stream, against the same lens with both
surfaces replaced by the conics they approximate. Prints one JSON line.

    python tools/nurbs_rate.py [--rays 1000000] [--steps 20]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def rate(lens, n, steps):
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.lowering import pupil_scalars, segment_params
    from optiland_pr_amd.raytrace import RealRays, lens_for, trace_pupil, upload_segments

    dl = lens_for(lens, [0.55])
    EPL, EPD = pupil_scalars(lens)
    seg = upload_segments(np.stack([segment_params(lens, 0.0, 1.0, 0, EPL, EPD)]), "cuda")
    d = RandomDistribution(seed=1)
    d.generate_points(n)
    px = torch.as_tensor(np.asarray(d.x), device="cuda")
    py = torch.as_tensor(np.asarray(d.y), device="cuda")
    out = RealRays.empty(n, 0.55)
    for _ in range(3):
        trace_pupil(dl, seg, px, py, out, n, n, n)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        trace_pupil(dl, seg, px, py, out, n, n, n)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    return ms, int(np.count_nonzero(~np.isnan(out.numpy()["x"])))


def main():
    from optiland_pr_amd.samples import NurbsLens

    n = int(sys.argv[sys.argv.index("--rays") + 1]) if "--rays" in sys.argv else 1_000_000
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 20
    ms, ok = rate(NurbsLens(), n, steps)
    conic = NurbsLens()
    from optiland_pr_amd.geometries import StandardGeometry

    for si, (R, k) in ((1, (40.0, -0.5)), (2, (-70.0, 0.0))):
        s = conic.surface_group.surfaces[si]
        s.geometry = StandardGeometry(s.geometry.cs, R, k)
    conic._lowered = None
    ms_c, _ = rate(conic, n, steps)
    S = 3
    print(json.dumps({"lens": "NurbsLens (fitted conic + explicit rational net), 1 field",
                      "rays": n, "finite_rays": ok, "ms_per_trace": ms,
                      "intersections_per_s": n * S / (ms * 1e-3),
                      "conic_twin_ms_per_trace": ms_c}))


if __name__ == "__main__":
    main()
