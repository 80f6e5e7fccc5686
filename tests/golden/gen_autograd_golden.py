"""Gradient golden vectors (config 5): the REFERENCE's torch backend (CPU, float64)
differentiating the Three-Mirror Anastigmat trace w.r.t. its Zernike coefficients.

Test infrastructure only, run in the build container (never on the GPU box):

    PYTHONPATH=tests/golden/shims:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/gen_autograd_golden.py

With --ia: tests/golden/autograd_ia.npz, d rms / d (radius, thickness) through the
thin-lens, phase and grating surfaces of gen_golden.py's paraxial_lens, phase_plate and
grating_curved (ia_params).

Writes tests/golden/autograd_tma.npz (fringe) and autograd_tma_standard.npz /
autograd_tma_noll.npz (the same loss and weights with the standard and noll schemes,
whose Newton slope omits the normalisation constant, zernike.py:162-231; SURVEY 8d.5's
"standard" variant), and with --full autograd_tma_1m.json (fringe; --full --scheme
standard|noll: autograd_tma_{scheme}_1m.json), config 5's own 1M-ray loss and gradient,
see full_size:
  rms_*      RayOperand.rms_spot_size(optic, -1, 0, 1, 32, 0.587, "uniform")
             (operand/ray.py:300-340) and d rms / d c for the coefficients of the three
             Zernike mirrors (surfaces 1-3, 10 fringe coefficients each)
  wsum_*     loss = sum_f sum_rays w_f * out_f over the image rays of Optic.trace at field
             (0, -1) with seeded weights w_f (x, y, z, L, M, N, opd), and its gradient:
             exercises every output's cotangent
  Px, Py     the pupil samples (uniform 32 -> 812 points)

Reference quirk recorded here: with be.grad_mode enabled (what TorchOptimizer does,
optimizer/torch/base.py:50-53) the Zernike normal's factorial weights are built from
requires-grad tensors and backward() fails with "derivative for aten::floor_divide is
not implemented" (zernike/base.py:289). The gradients below are therefore taken with
grad_mode off and the coefficient tensors as the only leaves requiring grad -- the same
graph over the same values.
"""

from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import gen_golden  # noqa: E402  (sets the numpy backend at import)
import optiland.backend as be  # noqa: E402
from optiland.distribution import create_distribution  # noqa: E402
from optiland.optimization.operand.ray import RayOperand  # noqa: E402

FIELDS = ("x", "y", "z", "L", "M", "N", "opd")


def _leaf_coefficients(lens):
    leaves = []
    for si in (1, 2, 3):
        geo = lens.surface_group.surfaces[si].geometry
        c = geo.coefficients
        c = c.detach() if torch.is_tensor(c) else torch.as_tensor(np.asarray(c))
        t = c.clone().to(torch.float64).requires_grad_(True)
        geo.coefficients = t
        leaves.append(t)
    return leaves


def main(scheme="fringe"):
    be.set_backend("torch")
    be.set_precision("float64")
    out = {}

    lens = gen_golden.tma(scheme)
    leaves = _leaf_coefficients(lens)
    rms = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 32, 0.587, "uniform")
    rms.backward()
    out["rms_value"] = np.array(float(rms))
    out["rms_grad"] = np.stack([t.grad.numpy().copy() for t in leaves])

    lens = gen_golden.tma(scheme)
    leaves = _leaf_coefficients(lens)
    d = create_distribution("uniform")
    d.generate_points(32)
    px = np.asarray(d.x.detach() if torch.is_tensor(d.x) else d.x, dtype=np.float64)
    py = np.asarray(d.y.detach() if torch.is_tensor(d.y) else d.y, dtype=np.float64)
    rng = np.random.default_rng(1234)
    w = {f: rng.standard_normal(px.size) for f in FIELDS}
    rays = lens.trace(0.0, -1.0, 0.587, num_rays=32, distribution="uniform")
    loss = 0.0
    for f in FIELDS:
        loss = loss + torch.sum(torch.as_tensor(w[f]) * getattr(rays, f))
    loss.backward()
    out["wsum_value"] = np.array(float(loss))
    out["wsum_grad"] = np.stack([t.grad.numpy().copy() for t in leaves])
    for f in FIELDS:
        out[f"wsum_w_{f}"] = w[f]
    out["Px"] = px
    out["Py"] = py
    name = "autograd_tma" if scheme == "fringe" else f"autograd_tma_{scheme}"
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(scheme, "rms", out["rms_value"], "wsum", out["wsum_value"])
    print(out["rms_grad"])
    if scheme == "fringe":
        shape_params()


def _cooke_leaves(thickness_surface):
    """Cooke triplet with radius (surfaces 1, 3, 6), conic (5) and one thickness variable
    as torch leaves, written the way the reference's variables write them
    (optic_updater.py:37-86). Only one thickness variable: every set_thickness rebuilds
    the positions from detached values (surface_group.py:143-148), so in the reference
    only the last one written keeps its graph."""
    from optiland.samples.objectives import CookeTriplet

    lens = CookeTriplet()
    leaves = {}
    for si in (1, 3, 6):
        t = torch.tensor(float(lens.surface_group.surfaces[si].geometry.radius),
                         dtype=torch.float64, requires_grad=True)
        lens.set_radius(t, si)
        leaves[f"radius{si}"] = t
    t = torch.tensor(0.0, dtype=torch.float64, requires_grad=True)
    lens.set_conic(t, 5)
    leaves["conic5"] = t
    th = float(lens.surface_group.surfaces[thickness_surface].thickness)
    t = torch.tensor(th, dtype=torch.float64, requires_grad=True)
    lens.set_thickness(t, thickness_surface)
    leaves[f"thickness{thickness_surface}"] = t
    return lens, leaves


def shape_params():
    """d rms / d (radius, conic, thickness) for the Cooke triplet at field (0, 1),
    uniform 24, lambda 0.55 (autograd_cooke.npz), with the thickness variable after
    surface 2 (moves surfaces 3-7) or after surface 6 (moves the image plane)."""
    out = {}
    for th in (2, 6):
        lens, leaves = _cooke_leaves(th)
        rms = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 24, 0.55, "uniform")
        rms.backward()
        out[f"t{th}_value"] = np.array(float(rms))
        out[f"t{th}_names"] = np.array(list(leaves))
        out[f"t{th}_grad"] = np.array([float(v.grad) for v in leaves.values()])
        print(th, float(rms), dict(zip(leaves, out[f"t{th}_grad"])))
    np.savez_compressed(os.path.join(HERE, "autograd_cooke.npz"), **out)


# lenses with thin-lens / phase / grating surfaces (gen_golden.py builders): radius leaves
# of their refractive (or grating) surfaces and the thickness after surface 1, rms spot
# size at field (0, 1), uniform 16 -- the gradient flows through the interaction models
# (thin_lens_interaction_model.py:55-113, phase_interaction_model.py:45-132,
# diffractive_model.py:28-61)
IA_CASES = {
    "paraxial_lens": ((2, 3), 0.55),
    "phase_plate": ((2, 3), 0.55),
    "grating_curved": ((), 0.587),  # (a grating's own radius: not a core parameter)
}


def ia_params():
    """d rms / d (radii, thickness 1) through thin-lens, phase and grating surfaces
    (autograd_ia.npz)."""
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
        out[f"{name}_value"] = np.array(float(rms))
        out[f"{name}_grad"] = np.array([float(v.grad) for v in leaves])
        print(name, float(rms), out[f"{name}_grad"])
    np.savez_compressed(os.path.join(HERE, "autograd_ia.npz"), **out)


def full_size(scheme="fringe"):
    """Config 5 at its own size (VERDICT r02 item 6 for config 5): the TMA loss
    rms_spot_size(optic, -1, 0, 1, 1M, 0.587, RandomDistribution(seed=0)) -- the bench's
    workload -- and d rms / d c for the 30 coefficients, from the reference's torch
    backend; the pupil points are drawn with the NumPy backend (PCG64, seed 0) as the
    native package draws them. Writes tests/golden/autograd_tma_1m.json."""
    import json
    import time

    from optiland.distribution import RandomDistribution

    be.set_backend("numpy")
    d = RandomDistribution(seed=0)
    d.generate_points(1_000_000)
    px, py = np.asarray(d.x, dtype=np.float64), np.asarray(d.y, dtype=np.float64)
    be.set_backend("torch")
    be.set_precision("float64")
    d.x, d.y = torch.as_tensor(px), torch.as_tensor(py)
    lens = gen_golden.tma(scheme)
    leaves = _leaf_coefficients(lens)
    t0 = time.perf_counter()
    rms = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 1_000_000, 0.587, d)
    rms.backward()
    res = dict(rms=float(rms), grad=[[float(v) for v in t.grad.numpy()] for t in leaves],
               seconds=time.perf_counter() - t0, n=int(px.size),
               px_sum=float(np.sum(px)), py_sum=float(np.sum(py)))
    name = "autograd_tma_1m" if scheme == "fringe" else f"autograd_tma_{scheme}_1m"
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(res, f, indent=1)
    print(res["rms"], res["seconds"])


if __name__ == "__main__":
    if "--ia" in sys.argv:  # autograd_ia.npz only
        ia_params()
        sys.exit(0)
    schemes = ("fringe", "standard", "noll")
    if "--scheme" in sys.argv:
        schemes = (sys.argv[sys.argv.index("--scheme") + 1],)
    for sc in schemes:
        if "--full" in sys.argv:
            full_size(sc)
        else:
            main(sc)
