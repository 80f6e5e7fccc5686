"""The REFERENCE's rms-spot gradients through thin-lens, phase and grating surfaces
(tests/golden/gen_autograd_golden.py ia_params: radius leaves and the thickness after
surface 1 of gen_golden.py's paraxial_lens, phase_plate and grating_curved) with the drop-in
installed: the reference's torch-backend traces served by the op's CPU kernel, its
backward by the forward-mode VJP of the host build (ort_sweep.h vjp_ray with the
interactions in duals). Prints one JSON line {case: {value, grad}, stats}. Launched by
tests/test_reference_install.py in the build container:

    python tests/refrun/ia_grad_run.py
"""

import json
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "tests", "golden", "shims"),
          "/root/reference", REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

import gen_golden  # noqa: E402
import optiland.backend as be  # noqa: E402
from gen_autograd_golden import IA_CASES  # noqa: E402
from optiland.optimization.operand.ray import RayOperand  # noqa: E402

from optiland_pr_amd import adapter  # noqa: E402


def main():
    adapter.install()
    be.set_backend("torch")
    be.set_precision("float64")
    builders = {"paraxial_lens": gen_golden.paraxial_lens, "phase_plate": gen_golden.phase_plate,
                "grating_curved": lambda: gen_golden.grating("curved")}
    out = {}
    for name, (rsurf, wl) in IA_CASES.items():
        lens = builders[name]()
        leaves = []
        for si in rsurf:
            t = torch.tensor(float(lens.surface_group.surfaces[si].geometry.radius),
                             dtype=torch.float64, requires_grad=True)
            lens.set_radius(t, si)
            leaves.append(t)
        t = torch.tensor(float(lens.surface_group.surfaces[1].thickness), dtype=torch.float64,
                         requires_grad=True)
        lens.set_thickness(t, 1)
        leaves.append(t)
        rms = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 16, wl, "uniform")
        rms.backward()
        out[name] = {"value": float(rms), "grad": [float(v.grad) for v in leaves]}
    print(json.dumps({"cases": out, "stats": adapter.STATS}))


if __name__ == "__main__":
    main()
