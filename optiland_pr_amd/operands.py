"""Ray operands of the optimisation layer that sit directly on the trace.

RayOperand.rms_spot_size (optimization/operand/ray.py:300-340) is the loss of config 5
(torch-autograd step): it reads the image record after Optic.trace. With torch-tensor
Zernike coefficients that require grad, Optic.trace runs the differentiable trace
(autodiff.py) and the value returned here back-propagates to the coefficients through
ort_trace_pupil_vjp. On the image surface of a taped single-wavelength trace the
reduction runs inside the trace: the taped kernel's epilogue writes per-workgroup rows
(count, sums, second moment about the workgroup centroid), one ort_rms_finish launch
combines them, and the gradient folds into the adjoint's x, y cotangent load
(raytrace.fused_rms; ORT_FUSED_RMS=0 turns it off). Otherwise the reduction is the custom
op torch.ops.ort.rms_spot (ops.py: ort_rms_spot's two deterministic passes,
ort_rms_spot_vjp for its gradient).
"""

from __future__ import annotations

import os

FUSED_RMS = os.environ.get("ORT_FUSED_RMS", "1") != "0"

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


class RayOperand:
    @staticmethod
    def rms_spot_size(optic, surface_number, Hx, Hy, num_rays, wavelength,
                      distribution="hexapolar"):
        """operand/ray.py:300-340: sqrt(mean((x - mean x)^2 + (y - mean y)^2)) on the
        record of surface_number; wavelength "all" pools every wavelength around the
        primary wavelength's centroid."""
        if wavelength == "all":
            xs, ys = [], []
            for w in optic.wavelengths.get_wavelengths():
                optic.trace(Hx, Hy, w, num_rays, distribution)
                xs.append(optic.surface_group.x[surface_number, :].flatten())
                ys.append(optic.surface_group.y[surface_number, :].flatten())
            k = optic.wavelengths.primary_index
            mx, my = torch.mean(xs[k]), torch.mean(ys[k])
            r2 = [(x - mx) ** 2 + (y - my) ** 2 for x, y in zip(xs, ys, strict=True)]
            return torch.sqrt(torch.mean(torch.cat(r2)))
        if FUSED_RMS and surface_number in (-1, len(optic.surface_group.surfaces) - 1):
            from . import raytrace

            with raytrace.fused_rms() as req:
                optic.trace(Hx, Hy, wavelength, num_rays, distribution)
            if req.get("rms") is not None:
                return req["rms"]
        else:
            optic.trace(Hx, Hy, wavelength, num_rays, distribution)
        x = _record_row(optic.surface_group, "x", surface_number)
        y = _record_row(optic.surface_group, "y", surface_number)
        if torch.is_tensor(x) and x.is_cuda:
            # the reduction (and its gradient) as one custom op: ort_rms_spot's two
            # deterministic passes on the device instead of ~10 eager kernels
            from . import ops

            return torch.ops.ort.rms_spot(x, y)[0]
        r2 = (x - torch.mean(x)) ** 2 + (y - torch.mean(y)) ** 2
        return torch.sqrt(torch.mean(r2))


def _record_row(sg, name, index):
    """surface_group.x[index, :] (surface_group.py:95-140; the reference records every
    surface it traces, so row k is surface k) read from the surface's own record without
    building the [S+1][n] stack; surfaces without a record fall back to the stack (NaN
    rows, SurfaceGroup._stack)."""
    v = getattr(sg.surfaces[index], name)
    n = v.numel() if torch is not None and torch.is_tensor(v) else len(v)
    if n == 0:
        return getattr(sg, name)[index, :].flatten()
    return v.flatten()


rms_spot_size = RayOperand.rms_spot_size
