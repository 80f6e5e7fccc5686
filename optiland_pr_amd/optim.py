"""Adam over device-resident Zernike coefficients, fused with the lens update.

The reference's torch optimiser loop (optimization/optimizer/torch/base.py:95-154) calls
torch.optim.Adam's step and then, at the next trace, writes the new coefficient values into
the lens (ZernikeCoefficientVariable.update_value, variable/zernike_coeff.py:71-95); here the
trace reads coefficients from the lowered lens's device tables, so every step needs their
patch (DeviceLens.patch_coefficients: one launch) after torch's fused Adam (two launches:
the step-count increment and the update). ZernikeAdam does all three in ONE launch
(ort_adam_patch_zernike): torch.optim.Adam's update of each coefficient, written into the
parameter tensor, its exp_avg / exp_avg_sq, the lens's term table and the surface's Cartesian
blocks. The next trace then skips its own patch (DeviceLens.coefficients_current). The update
is torch's fused Adam's arithmetic for doubles (tests/test_gpu_optim.py compares the
coefficient trajectory with torch.optim.Adam(fused=True) bit for bit).

Parameters must be the device-resident coefficient tensors of the lenses' Zernike surfaces
(geometry.coefficients = tensor on the GPU, requires_grad) -- as config 5 holds them.
Capturable: no host synchronisation, kernel arguments by value (a HIP graph replays it).
"""

from __future__ import annotations

import ctypes as C

import torch

from . import _native


class ZernikeAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, maximize=False; weight_decay the L2 form) for the
    device-resident Zernike coefficients of `lenses`: each parameter tensor updated once per
    step, by one fused launch per lowered lens that holds some of them.

    As torch.optim.Adam: a parameter without a gradient is skipped (the rest of its group
    still steps), and every parameter keeps its own state -- "step", "exp_avg",
    "exp_avg_sq" in self.state[p] (the step count a device double). An optic traced under
    several keys (wavelengths, records) holds one lowered lens per key, all reading the
    same tensors: the tensor is updated in the launch of the first lens holding it, and the
    other lenses' tables are marked stale, so their next trace re-patches them from it."""

    def __init__(self, params, lenses, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.lenses = list(lenses)
        self._plans = {}

    def _device_lenses(self):
        for lens in self.lenses:
            for dl in getattr(lens, "_lowered", {}).values():
                if getattr(dl.table, "device_coeffs", None):
                    yield dl

    def _state(self, p):
        st = self.state[p]
        if not st:
            if not (p.is_cuda and p.dtype == torch.float64 and p.is_contiguous()):
                raise ValueError("ZernikeAdam: contiguous float64 device coefficient tensors")
            # (made once: a plan built inside a graph capture -- new grad tensors -- must
            # not capture a fill that every replay would repeat)
            st["step"] = torch.zeros((), dtype=torch.float64, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @staticmethod
    def _key(t):
        """A coefficient tensor by its memory (a detached view of a parameter -- what a
        geometry may hold -- is the parameter's storage)"""
        return (t.data_ptr(), t.numel())

    def _plan(self, dl, group, params):
        """The launch arguments for one lens (by value): the tensors of `params` it holds,
        each at its (one) term-row offset."""
        mine = {}
        for off, t in dl.table.device_coeffs:
            mine.setdefault(self._key(t), off)
        items = [(mine[self._key(p)], p) for p in params if self._key(p) in mine]
        beta1, beta2 = group["betas"]
        hyper = (float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
                 float(group["weight_decay"]))
        key = (id(dl), hyper, tuple((off, p.data_ptr(), p.grad.data_ptr()) for off, p in items))
        hit = self._plans.get(key)
        if hit is not None:
            return hit
        if len(items) > _native.ADAM_MAX_TENSORS:
            raise ValueError(f"at most {_native.ADAM_MAX_TENSORS} coefficient tensors per lens")
        a = _native.ort_adam_params()
        a.n_tensors = len(items)
        for k, (off, p) in enumerate(items):
            st = self._state(p)
            a.param[k] = p.data_ptr()
            a.grad[k] = p.grad.data_ptr()
            a.exp_avg[k] = st["exp_avg"].data_ptr()
            a.exp_avg_sq[k] = st["exp_avg_sq"].data_ptr()
            a.step[k] = st["step"].data_ptr()
            a.row0[k] = int(off)
            a.count[k] = p.numel()
        a.lr, a.beta1, a.beta2, a.eps, a.weight_decay = hyper
        hit = (a, [p for _, p in items])
        self._plans[key] = hit
        return hit

    @torch.no_grad()
    def step(self, closure=None):
        from .raytrace import _stream_handle

        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _native.load()
        lenses = list(self._device_lenses())
        updated = {}  # tensor key -> the lens whose launch updated it
        for group in self.param_groups:
            # (torch.optim.Adam skips the parameters without a gradient, not the group)
            params = [p for p in group["params"] if p.grad is not None]
            for dl in lenses:
                todo = [p for p in params if self._key(p) not in updated]
                if not todo:
                    break
                a, done = self._plan(dl, group, todo)
                if not done:
                    continue
                rc = lib.ort_adam_patch_zernike(C.byref(dl.c), C.byref(a), _stream_handle())
                _native.check(rc, "ort_adam_patch_zernike")
                for p in done:
                    updated[self._key(p)] = dl
        # which lowered lenses hold the new values: a lens whose every updated tensor was
        # updated by its own launch (each at one offset) is current; one that holds a tensor
        # another lens's launch updated -- or the same tensor on two surfaces -- re-patches
        # at its next trace (DeviceLens.patch_coefficients)
        for dl in lenses:
            ids = [self._key(t) for _, t in dl.table.device_coeffs]
            hit = [updated[i] for i in ids if i in updated]
            if not hit:
                continue
            if all(h is dl for h in hit) and len(set(ids)) == len(ids):
                dl.coefficients_current()
            else:
                dl.invalidate_patch()
        return loss
