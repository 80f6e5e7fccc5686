"""CPU: the custom-op boundary (ops.py) and the adapter's gradient rules, without a GPU.

* torch.ops.ort.trace_sequential / trace_pupil are registered with the schemas the
  adapter and the native front-end call; trace_sequential has a CPU kernel (the host build,
  liboptiland_host.so) that takes only a HostLens handle, trace_pupil none (the dispatcher
  refuses a CPU tensor);
* ops.tangent_tables lays the parameter kinds out as ort_vjp_params expects;
* adapter._grad_params: which lens values are differentiated, which hand the call back to
  the reference loop (Unsupported), which are ignored (the reference's be.grad_mode makes
  every be.array a requires-grad leaf; only values reaching a torch.nn.Parameter count).
"""

import numpy as np
import pytest
import torch

from optiland_pr_amd import _abi, adapter, ops
from optiland_pr_amd.lowering import lower_surface_group
from optiland_pr_amd.samples import CookeTriplet, ThreeMirrorAnastigmat


def test_ops_registered():
    """The ops take the lowered lens itself (its tables as tensors, the ort_lens scalars),
    not a handle: fake-tensor propagation, torch.compile and
    torch.export see every input; the backward formulas are ops too."""
    s1 = str(torch.ops.ort.trace_sequential.default._schema)
    s2 = str(torch.ops.ort.trace_pupil.default._schema)
    for s in (s1, s2):
        assert "Tensor[] lens" in s and "SymInt[] lens_meta" in s and "float final_thickness" in s
        assert "Tensor[] params" in s
    assert "Tensor[] rays" in s1 and "bool per_ray_w" in s1
    assert s1.count("Tensor") >= 10 + 4  # 10 outputs, lens / rays / w / params inputs
    assert "Tensor seg" in s2 and "Tensor? apod" in s2
    for name in ("trace_sequential_vjp", "trace_pupil_vjp", "rms_spot", "rms_spot_vjp"):
        assert hasattr(torch.ops.ort, name)
    assert len(ops.LENS_META) == 10


def test_rms_spot_refuses_mismatched_inputs():
    """the op checks dtype, size and device before any pointer reaches the
    kernels (here through the fake / meta path, no GPU needed)."""
    x = torch.zeros(8, dtype=torch.float64, device="meta")
    with pytest.raises(ValueError, match="points"):
        torch.ops.ort.rms_spot(x, torch.zeros(7, dtype=torch.float64, device="meta"))
    with pytest.raises(ValueError, match="float64"):
        torch.ops.ort.rms_spot(x, torch.zeros(8, dtype=torch.float32, device="meta"))


def test_spec_roundtrip():
    pairs = [("zernike", 0), ("radius", 3), ("conic", 1), ("thickness", 2), ("vertex", 5)]
    assert ops._spec_pairs(ops.encode_spec(pairs)) == pairs


def test_tangent_tables_kinds():
    tma = ThreeMirrorAnastigmat()
    table = lower_surface_group(tma.surface_group, [0.587])
    S = table.n_surfaces
    n_z = int(table.surfaces[1]["n_coef"])
    params = [torch.zeros(n_z), torch.zeros(()), torch.zeros(()), torch.zeros(())]
    pairs = [("zernike", 1), ("radius", 0), ("vertex", 2), ("thickness", S - 1)]
    zp, surf, final, n_param = ops.tangent_tables(table, pairs, params)
    assert n_param == n_z + 3
    base = int(table.surfaces[1]["coef_off"])
    assert list(zp[base:base + n_z]) == list(range(n_z))
    assert np.all(zp[:base] == -1)
    assert surf[n_z, 0, 0] == 1.0 and surf[n_z].sum() == 1.0
    assert surf[n_z + 1, 2, 2] == 1.0 and surf[n_z + 1].sum() == 1.0
    assert final[n_z + 2] == 1.0  # the image surface's thickness: the final propagate
    with pytest.raises(ValueError):
        ops.tangent_tables(table, [("zernike", S - 1)], [torch.zeros(n_z)])  # the image plane


def _cooke_group():
    return CookeTriplet().surface_group


def test_grad_params_collects_differentiable_values():
    sg = _cooke_group()
    R = torch.tensor(50.0, dtype=torch.float64, requires_grad=True)
    sg.surfaces[3].geometry.radius = R
    z = torch.tensor(float(sg.surfaces[4].geometry.cs.z), dtype=torch.float64, requires_grad=True)
    sg.surfaces[4].geometry.cs.z = z * 1.0
    got = adapter._grad_params(sg)
    assert [(k, si) for k, si, _ in got] == [("radius", 2), ("vertex", 3)]
    with torch.no_grad():
        assert adapter._grad_params(sg) == []


def test_grad_params_refuses_undifferentiated_values(monkeypatch):
    sg = _cooke_group()
    sg.surfaces[2].geometry.cs.ry = torch.tensor(0.0, dtype=torch.float64, requires_grad=True)
    with pytest.raises(adapter.Unsupported, match="cs.ry"):
        adapter._grad_params(sg)
    # under the reference's grad mode a plain requires-grad leaf is a be.array artifact
    monkeypatch.setattr(adapter, "_grad_mode_on", lambda: True)
    assert adapter._grad_params(sg) == []
    # ... unless it depends on a trainable parameter
    p = torch.nn.Parameter(torch.tensor(0.0, dtype=torch.float64))
    sg.surfaces[2].geometry.cs.ry = p * 2.0
    with pytest.raises(adapter.Unsupported, match="cs.ry"):
        adapter._grad_params(sg)


def test_reaches_parameter_shared_memo():
    p = torch.nn.Parameter(torch.tensor(1.0, dtype=torch.float64))
    leaf = torch.tensor(2.0, dtype=torch.float64, requires_grad=True)
    a = leaf * 3.0
    b = a + p
    c = a * 2.0
    memo = {}
    assert adapter._reaches_parameter(b, memo)
    assert not adapter._reaches_parameter(c, memo)  # a's subgraph memoised as "no"
    assert adapter._reaches_parameter(p, memo)
    assert not adapter._reaches_parameter(leaf, memo)


def test_seq_vjp_entry_declared():
    import re

    from tests.conftest import REPO

    with open(f"{REPO}/include/optiland_rt.h") as f:
        text = f.read()
    assert re.search(r"int ort_trace_sequential_vjp\(", text)
    assert re.search(r"int ort_trace_spot\(", text)
    m = re.search(r"#define ORT_ABI_VERSION (\d+)", text)
    assert m and int(m.group(1)) == _abi.ABI_VERSION >= 13


def test_verify_max_sched_matches_header():
    import re

    from optiland_pr_amd import raytrace
    from tests.conftest import REPO

    with open(f"{REPO}/include/optiland_rt.h") as f:
        text = f.read()
    m = re.search(r"#define ORT_VERIFY_MAX_SCHED (\d+)", text)
    assert m and int(m.group(1)) == raytrace.VERIFY_MAX_SCHED
    for field in ("verify_stats", "verify_prev_flag", "verify_flag", "sched_out"):
        assert re.search(rf"\b{field};", text)
        assert field in [f for f, _ in __import__("optiland_pr_amd._native", fromlist=["x"]).ort_options._fields_]


def test_flops_per_ray_counts_newton_schedule():
    """bench._flops_per_ray: RT-asph (config 3) with the verified schedule of one update per
    asphere (two sag + normal evaluations of 66 flops with 3 coefficients); None for
    surface kinds it does not count (Zernike without a schedule)."""
    import numpy as np

    import bench
    from optiland_pr_amd import _abi
    from optiland_pr_amd.lowering import lower_surface_group
    from optiland_pr_amd.samples import ReverseTelephotoAsphere, ThreeMirrorAnastigmat

    t = lower_surface_group(ReverseTelephotoAsphere().surface_group, [0.4861, 0.5876, 0.6563])
    asph = t.surfaces["geometry"] == _abi.GEOM_EVEN_ASPHERE
    assert int(asph.sum()) == 2
    f0 = bench._flops_per_ray(t, np.where(asph, 0, 0))
    f1 = bench._flops_per_ray(t, np.where(asph, 1, 0))
    assert f1 - f0 == 2 * (66 + 8)  # one more evaluation and one update per asphere
    assert f1 == 1634
    tma = lower_surface_group(ThreeMirrorAnastigmat().surface_group, [0.587])
    assert bench._flops_per_ray(tma, np.zeros(tma.n_surfaces)) is None


def test_segment_cache_invalidation():
    """raytrace._cached_segments: reused for an unchanged optic, recomputed when anything
    segment_params reads changes (fields / vignetting, aperture, stop, object, lens bytes);
    no caching when the primary wavelength is not the traced one."""
    import numpy as np

    from optiland_pr_amd import raytrace
    from optiland_pr_amd.lowering import pupil_scalars, segment_params
    from optiland_pr_amd.samples import CookeTriplet

    class DL:
        fingerprint = b"lens-a"

    lens = CookeTriplet()
    wl = lens.primary_wavelength
    Hx, Hy = np.zeros(2), np.array([0.0, 1.0])
    a = raytrace._cached_segments(lens, DL, wl, Hx, Hy)
    assert raytrace._cached_segments(lens, DL, wl, Hx, Hy) is a
    EPL, EPD = pupil_scalars(lens)
    ref = np.stack([segment_params(lens, 0.0, h, 0, EPL, EPD) for h in (0.0, 1.0)])
    assert a.tobytes() == ref.tobytes()
    for edit in (lambda: setattr(lens.fields.fields[-1], "vy", 0.2),
                 lambda: setattr(lens.aperture, "value", lens.aperture.value * 1.1),
                 lambda: setattr(lens.surface_group.surfaces[2], "is_stop",
                                 not lens.surface_group.surfaces[2].is_stop),
                 lambda: setattr(DL, "fingerprint", b"lens-b")):
        edit()
        b = raytrace._cached_segments(lens, DL, wl, Hx, Hy)
        assert b is not a
        a = b
    other = wl + 0.01
    assert raytrace._segment_key(lens, DL, other, Hx, Hy) is None
