"""Marginal device cost of one device-verified Newton round in config 5's captured step
(measurement tooling, not product): the same optimisation step (bench.py config 5: TMA,
1M rays, taped forward, verify rounds, adjoint, fused Adam) captured with R = 1, 3, 5, 7
verify rounds (raytrace.MAX_DEVICE_ROUNDS; 7 = the protocol's 2 n_newton + 1), K graph
replays timed with events on the capture's stream, two alternating repetitions. The
schedule is settled, so rounds 2.. are the no-op rounds whose cost VERDICT r05 item 3
asks about. Prints one JSON line."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from optiland_pr_amd import _native, raytrace  # noqa: E402
from optiland_pr_amd.autodiff import CapturedStep  # noqa: E402
from optiland_pr_amd.distribution import RandomDistribution  # noqa: E402
from optiland_pr_amd.operands import RayOperand  # noqa: E402
from optiland_pr_amd.optim import ZernikeAdam  # noqa: E402
from optiland_pr_amd.samples import ThreeMirrorAnastigmat  # noqa: E402

_native.load()
dev = torch.device("cuda", 0)
R_RAYS = 1_000_000
d = RandomDistribution(seed=0)
d.generate_points(R_RAYS)


def make(rounds):
    raytrace.MAX_DEVICE_ROUNDS = rounds
    lens = ThreeMirrorAnastigmat()
    lens.newton_mode = "device"
    leaves = []
    for si in (1, 2, 3):
        g = lens.surface_group.surfaces[si].geometry
        t = torch.tensor(np.asarray(g.coefficients), dtype=torch.float64, device=dev,
                         requires_grad=True)
        g.coefficients = t
        leaves.append(t)
    opt = ZernikeAdam(leaves, [lens], lr=1e-7)
    step = CapturedStep(lambda: RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, R_RAYS, 0.587, d),
                        opt, lenses=[lens])
    step()
    torch.cuda.synchronize()
    return step


def timed(step, k=200):
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(k):
        step()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1e3


steps = {r: make(r) for r in (1, 3, 5, 7)}
res = {r: [] for r in steps}
for rep in range(2):
    for r, st in steps.items():
        res[r].append(timed(st))
for st in steps.values():
    st.check()
us = {r: float(np.mean(v)) for r, v in res.items()}
slope = float(np.polyfit(list(us), list(us.values()), 1)[0])
print(json.dumps({"us_per_step": res, "mean": us, "us_per_round": slope}))
