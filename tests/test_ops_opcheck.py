"""The custom ops are self-describing: the lowered lens reaches them as
tensors (ops.lens_args: the nine tables, the ort_lens scalars), the backward formulas are ops
themselves (ort::trace_sequential_vjp, ort::trace_pupil_vjp, ort::rms_spot_vjp), so
torch.library.opcheck's schema / fake-tensor / autograd-registration / AOT-dispatch checks
pass, and torch.compile(fullgraph=True) traces a function that calls the trace. CPU key
here (the host build of the trace core); tests/test_gpu_opcheck.py runs the CUDA key.

The lens key (a handle of the DeviceLens / HostLens that holds the host-side schedule
caches) is only a cache key: a key that names no live object of these tensors makes the op
rebuild the lens from the tensors (test_rebuilt_from_tensors)."""

import numpy as np
import pytest
import torch

from optiland_pr_amd import _abi, host, ops
from optiland_pr_amd.lowering import lower_surface_group
from tests._cases import build_lens
from tests.test_gpu_adjoint import _leaves
from tests.test_seam_adapter import _generated

FIELDS = ("x", "y", "z", "L", "M", "N", "i", "opd")


def _traced(spec):
    """(kind, lens surface index) -> (kind, traced-surface index): the object is not traced"""
    return [(k, si - 1) for k, si in spec]


def _seq_args(name, spec=(), n_rays=8, requires_grad=True):
    lens = build_lens(name)
    leaves = _leaves(torch, lens, list(spec))
    table = lower_surface_group(lens.surface_group, [lens.primary_wavelength], record=True)
    table.final_mat = -1  # SurfaceGroup.trace: no image-space propagate
    hl = host.HostLens(table)
    L, meta, ft, key = ops.lens_args(hl)
    rays = _generated(torch, lens, 0.0, 1.0, lens.primary_wavelength, n_rays, "cpu", "hexapolar")
    fields = [getattr(rays, a).detach().clone().requires_grad_(requires_grad) for a in FIELDS]
    args = (L, meta, ft, key, fields, None, leaves, ops.encode_spec(_traced(spec)), 0, False)
    return hl, args


def _pupil_args(name, spec=(), n_p=37):
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.lowering import segment_params

    lens = build_lens(name)
    leaves = _leaves(torch, lens, list(spec))
    table = lower_surface_group(lens.surface_group, [lens.primary_wavelength])
    hl = host.HostLens(table)
    L, meta, ft, key = ops.lens_args(hl)
    seg = np.stack([segment_params(lens, 0.0, h, 0) for h in (0.0, 1.0)])
    seg_t = torch.from_numpy(np.frombuffer(seg.astype(_abi.SEGMENT).tobytes(), dtype=np.uint8)
                             .copy())
    d = RandomDistribution(seed=3)
    d.generate_points(n_p)
    px = torch.as_tensor(np.asarray(d.x, dtype=np.float64))
    py = torch.as_tensor(np.asarray(d.y, dtype=np.float64))
    n = n_p * len(seg)
    args = (L, meta, ft, key, seg_t, None, px, py, leaves, ops.encode_spec(_traced(spec)),
            [n, n_p, 0, 0, 0], 0)
    return hl, args


def _assert_opcheck(op, args):
    res = torch.library.opcheck(op, args)
    assert all(v == "SUCCESS" for v in res.values()), res


@pytest.mark.parametrize("name,spec", [
    ("cooke", ()),
    ("cooke", (("radius", 1), ("thickness", 2))),
    ("tma_fringe", (("zernike", 1), ("zernike", 2))),
])
def test_opcheck_trace_sequential_cpu(name, spec):
    _, args = _seq_args(name, spec)
    _assert_opcheck(torch.ops.ort.trace_sequential.default, args)


@pytest.mark.parametrize("name,spec", [
    ("cooke", ()),
    ("tma_fringe", (("zernike", 1), ("zernike", 3))),
])
def test_opcheck_trace_pupil_cpu(name, spec):
    _, args = _pupil_args(name, spec)
    _assert_opcheck(torch.ops.ort.trace_pupil.default, args)


def test_opcheck_rms_spot_cpu():
    g = np.random.default_rng(1)
    x = torch.as_tensor(g.normal(size=101)).requires_grad_(True)
    y = torch.as_tensor(g.normal(size=101) + 2.0).requires_grad_(True)
    _assert_opcheck(torch.ops.ort.rms_spot.default, (x, y))
    rms, stats = torch.ops.ort.rms_spot(x, y)
    xn, yn = x.detach().numpy(), y.detach().numpy()
    ref = np.sqrt(np.mean((xn - xn.mean()) ** 2 + (yn - yn.mean()) ** 2))
    np.testing.assert_allclose(float(rms.detach()), ref, rtol=1e-14)
    rms.backward()
    np.testing.assert_allclose(x.grad.numpy(), (xn - xn.mean()) / (101 * ref), rtol=1e-12)


def test_opcheck_vjp_ops_cpu():
    """The backward ops on their own (the arguments the forward's autograd formula passes;
    no second derivatives: the inputs do not require grad)."""
    hl, args = _seq_args("tma_fringe", (("zernike", 1),))
    L, meta, ft, key, fields, w, params, spec, start, prw = args
    outs = torch.ops.ort.trace_sequential(*args)
    zp, st, ftan, n_param = ops.tangent_tables(hl.table, ops._spec_pairs(spec), params)
    tabs = ops._tables_cpu(zp, st, ftan, ops.slot_need(hl.table, zp, st, ftan))
    cot = [torch.ones_like(outs[0]), torch.ones_like(outs[1])] + [None] * 6
    vargs = ([t.detach() for t in L], meta, ft, key, [f.detach() for f in fields], None,
             outs[9].detach(), outs[8].detach(), cot, None, tabs, n_param, _abi.VJP_ADJOINT,
             0, False, True)
    _assert_opcheck(torch.ops.ort.trace_sequential_vjp.default, vargs)


def test_rebuilt_from_tensors():
    """A key that names no live lens of these tensors: the op rebuilds the lens from the
    tensors themselves and traces the same bits."""
    hl, args = _seq_args("cooke", requires_grad=False)
    a = torch.ops.ort.trace_sequential(*args)
    copies = [t.clone() for t in args[0]]  # other storage: the key's lens does not match
    b = torch.ops.ort.trace_sequential(copies, *args[1:])
    for u, v in zip(a[:9], b[:9], strict=True):
        assert torch.equal(u, v)


def test_compile_fullgraph_trace_sequential_cpu():
    """torch.compile(fullgraph=True) of a function that traces and reduces: no graph break
    (the op is opaque, its fake kernel gives the shapes), same values as eager."""
    hl, args = _seq_args("cooke", requires_grad=False)
    L, meta, ft, key, fields, w, params, spec, start, prw = args

    def f(L, fields):
        out = torch.ops.ort.trace_sequential(L, meta, ft, key, fields, None, [], [], 0, False)
        return out[0].sum() + out[1].square().sum(), out[7]

    eager = f(L, fields)
    compiled = torch.compile(f, fullgraph=True, backend="aot_eager")(L, fields)
    for u, v in zip(eager, compiled, strict=True):
        assert torch.equal(u, v)


def test_trace_pupil_fused_rms_cpu():
    """plan_meta's want_rms (the rms spot size computed by the trace op, its gradient folded
    into the trace's VJP as ort_vjp_params.rms_stats / rms_grad) against the same trace
    followed by ort::rms_spot: value and coefficient gradients agree."""
    spec = (("zernike", 1), ("zernike", 3))
    _, args = _pupil_args("tma_fringe", spec, n_p=53)
    L, meta, ft, key, seg_t, apod, px, py, leaves, sp, pmeta, pkey = args
    fused = torch.ops.ort.trace_pupil(L, meta, ft, key, seg_t, apod, px, py, leaves, sp,
                                      pmeta + [1], pkey)
    assert fused[10].dim() == 0 and fused[11].numel() == 5
    g_fused = torch.autograd.grad(fused[10], leaves)
    plain = torch.ops.ort.trace_pupil(*args)
    assert plain[10].numel() == 0
    rms = torch.ops.ort.rms_spot(plain[0], plain[1])[0]
    g_plain = torch.autograd.grad(rms, leaves)
    np.testing.assert_allclose(float(fused[10].detach()), float(rms.detach()), rtol=1e-14)
    for a, b in zip(g_fused, g_plain, strict=True):
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-12, atol=1e-18)


def test_opcheck_trace_pupil_fused_rms_cpu():
    _, args = _pupil_args("tma_fringe", (("zernike", 1),), n_p=29)
    args = (*args[:10], args[10] + [1], args[11])
    _assert_opcheck(torch.ops.ort.trace_pupil.default, args)
