"""Config 5 (TMA optimisation step): is the step host- or device-bound? Issues 200 steps
without synchronising and reports the host's issue time per step next to the wall time per
step once the device has drained (measurement tooling).
    python tools/host_rate_c5.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from optiland_pr_amd.distribution import RandomDistribution  # noqa: E402
from optiland_pr_amd.operands import RayOperand  # noqa: E402
from optiland_pr_amd.samples import ThreeMirrorAnastigmat  # noqa: E402

d = RandomDistribution(seed=0)
d.generate_points(1_000_000)
lens = ThreeMirrorAnastigmat()
lens.newton_mode = "device"
leaves = []
for si in (1, 2, 3):
    g = lens.surface_group.surfaces[si].geometry
    t = torch.tensor(np.asarray(g.coefficients), dtype=torch.float64, device="cuda",
                     requires_grad=True)
    g.coefficients = t
    leaves.append(t)
opt = torch.optim.Adam(leaves, lr=1e-7, fused=True)


def step():
    opt.zero_grad()
    loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 1_000_000, 0.587, d)
    loss.backward()
    opt.step()


for _ in range(20):
    step()
torch.cuda.synchronize()
for rep in range(3):
    K = 200
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e3 * (t1 - t0) / K:.3f} ms/step, wall {1e3 * (t2 - t0) / K:.3f} ms/step",
          flush=True)
