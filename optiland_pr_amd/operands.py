"""Ray operands of the optimisation layer that sit directly on the trace.

RayOperand.rms_spot_size (optimization/operand/ray.py:300-340) is the loss of config 5
(torch-autograd step): it reads the image record after Optic.trace. With torch-tensor
Zernike coefficients that require grad, Optic.trace runs the differentiable trace
(autodiff.py) and the value returned here back-propagates to the coefficients through
ort_trace_pupil_vjp. The reductions (mean, sqrt) are torch ops on the device.
"""

from __future__ import annotations

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
        optic.trace(Hx, Hy, wavelength, num_rays, distribution)
        x = optic.surface_group.x[surface_number, :].flatten()
        y = optic.surface_group.y[surface_number, :].flatten()
        r2 = (x - torch.mean(x)) ** 2 + (y - torch.mean(y)) ** 2
        return torch.sqrt(torch.mean(r2))


rms_spot_size = RayOperand.rms_spot_size
