"""Host-side profile of the config-5 optimisation step in steady state (measurement
tooling): 5 warm-up steps, then cProfile over 30 steps. usage (GPU box):
    python tools/prof_host_c5.py > gpurun_out/c5_host.txt"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from optiland_pr_amd.distribution import RandomDistribution  # noqa: E402
from optiland_pr_amd.operands import RayOperand  # noqa: E402
from optiland_pr_amd.samples import ThreeMirrorAnastigmat  # noqa: E402

d = RandomDistribution(seed=0)
d.generate_points(1_000_000)
lens = ThreeMirrorAnastigmat()
lens.newton_mode = "device"  # as bench.py config 5
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


if os.environ.get("PROF_BACKWARD_MAIN_THREAD"):  # let cProfile see the backward's Python
    torch.autograd.set_multithreading_enabled(False)
for _ in range(5):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(30):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(45)
