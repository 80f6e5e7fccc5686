"""A few steps of the REFERENCE's TorchAdamOptimizer (optimization/optimizer/torch/base.py:
95-154) on a reference lens, with or without the drop-in installed; prints one JSON line
(per-step losses, final parameters, final loss, adapter.STATS). Launched by
tests/test_reference_install.py in the build container (the reference is not on the GPU
box):

    python tests/refrun/optimize_run.py {installed|reference} {tma_zernike|cooke}

tma_zernike  ZernikeCoeffVariables (variable/zernike_coeff.py:71-95) of the three mirrors
             of the TMA, operand rms_spot_size (operand/ray.py:300-340)
cooke        RadiusVariables of surfaces 1 and 3, the ConicVariable of surface 5 and the
             ThicknessVariable of surface 2 of the Cooke triplet, same operand

installed  TorchAdamOptimizer.optimize as it is (be.grad_mode on: every be.array a
           requires-grad leaf, so the adapter must find the nn.Parameters through the graph,
           adapter._grad_params), the traces served by the op's CPU kernel.
reference  the same loop (base.py:116-131: update_value, update_optics, sum_squared,
           backward, Adam step, bounds, scheduler) through the reference's own trace, on a
           FRESHLY BUILT lens every step, be.grad_mode off.

Why the reference run cannot be TorchOptimizer.optimize itself: on its own it raises at the
second step ("Trying to backward through the graph a second time") for every variable tried
here with a ray operand -- the persistent lens keeps tensors from the previous step's freed
graph -- and its Zernike backward with be.grad_mode on fails on aten::floor_divide
(zernike/base.py:289; tests/golden/gen_autograd_golden.py records it). A fresh lens holding
the same variable values is the same optical state, so the two trajectories must agree.
ZernikeCoeffVariable.update_value writes the coefficient in place (zernike_coeff.py:71-95),
so the installed run's coefficient tensor would keep the previous step's graph as well: its
step callback re-detaches the coefficient arrays after every step.
"""

import contextlib
import json
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "tests", "golden", "shims"),
          "/root/reference", REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import gen_golden  # noqa: E402
import optiland.backend as be  # noqa: E402
from optiland.optimization import OptimizationProblem, TorchAdamOptimizer  # noqa: E402
from optiland.samples.objectives import CookeTriplet  # noqa: E402

from optiland_pr_amd import adapter  # noqa: E402


def build(case):
    """-> (lens, OptimizationProblem, lr, Zernike surfaces) of one case, freshly built."""
    problem = OptimizationProblem()
    if case == "tma_zernike":
        lens = gen_golden.tma("fringe")
        zsurf = (1, 2, 3)
        for si in zsurf:
            for k in (3, 4, 5, 6):
                problem.add_variable(lens, "zernike_coeff", surface_number=si, coeff_index=k)
        op = dict(optic=lens, surface_number=-1, Hx=0.0, Hy=1.0, num_rays=16,
                  wavelength=0.587, distribution="uniform")
        lr = 1e-5
    else:
        lens = CookeTriplet()
        zsurf = ()
        problem.add_variable(lens, "radius", surface_number=1)
        problem.add_variable(lens, "radius", surface_number=3)
        problem.add_variable(lens, "conic", surface_number=5)
        problem.add_variable(lens, "thickness", surface_number=2)
        op = dict(optic=lens, surface_number=-1, Hx=0.0, Hy=1.0, num_rays=12,
                  wavelength=0.55, distribution="uniform")
        lr = 1e-3
    problem.add_operand(operand_type="rms_spot_size", target=0.0, weight=1.0, input_data=op)
    return lens, problem, lr, zsurf


N_STEPS = 5


def run_installed(case):
    lens, problem, lr, zsurf = build(case)
    adapter.install()
    opt = TorchAdamOptimizer(problem)
    losses = []

    def step_done(i, loss):
        losses.append(loss)
        for si in zsurf:
            g = lens.surface_group.surfaces[si].geometry
            g.coefficients = g.coefficients.detach().clone()

    res = opt.optimize(n_steps=N_STEPS, lr=lr, disp=False, callback=step_done)
    return losses, [float(v) for v in res.x], float(res.fun)


def run_reference(case):
    _, problem, lr, _ = build(case)
    be.grad_mode.temporary_enable = contextlib.nullcontext
    opt = TorchAdamOptimizer(problem)  # its nn.Parameters, optimizer and scheduler
    be.grad_mode.disable()
    optimizer, scheduler = opt._create_optimizer_and_scheduler(lr, 0.99)
    losses = []

    def fresh():
        _, pb, _, _ = build(case)
        be.grad_mode.disable()  # OptimizationProblem() turns it on
        for k, param in enumerate(opt.params):
            pb.variables[k].variable.update_value(param)
        pb.update_optics()
        opt.problem = pb  # _apply_bounds reads the variables' bounds
        return pb

    for _ in range(N_STEPS):
        optimizer.zero_grad()
        loss = fresh().sum_squared()
        loss.backward()
        optimizer.step()
        opt._apply_bounds()
        scheduler.step()
        losses.append(loss.item())
    fun = fresh().sum_squared().item()
    return losses, [p.item() for p in opt.params], fun


def main(mode, case):
    be.set_backend("torch")
    be.set_device("cpu")
    be.set_precision("float64")
    losses, x, fun = (run_installed if mode == "installed" else run_reference)(case)
    print(json.dumps({"losses": losses, "x": x, "fun": fun, "stats": adapter.STATS}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
