"""GPU: Newton schedules verified on the device (newton_mode="device": verify-and-re-trace
launches, or ort_newton_fixup + conditional re-launches; raytrace._run_device): the same schedules and bit-identical rays
as the host-verified path, a wrong cached schedule corrected on the device (too long:
the exact stop index; too short: grown, then exact), the settled schedule written back
to the host cache, and errors raised at the next check (check_all_pending)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("needs the MI355X")
    from optiland_pr_amd import _native

    _native.load()
    return torch


def _trace(lens, mode, n=4096, hy=1.0, wl=0.5876):
    from optiland_pr_amd.distribution import RandomDistribution

    d = RandomDistribution(seed=3)
    d.generate_points(n)
    lens.newton_mode = mode
    rays = lens.trace(0.0, hy, wl, num_rays=n, distribution=d)
    return {a: getattr(rays, a).cpu().numpy() for a in ("x", "y", "z", "L", "M", "N", "opd")}


def _dlens(lens, wl):
    from optiland_pr_amd.raytrace import lens_for

    return lens_for(lens, [wl])


@pytest.mark.parametrize("name", ["rt_asph", "tma_fringe"])
def test_device_mode_equals_reference(torch, name):
    from optiland_pr_amd import raytrace
    from tests._cases import build_lens

    wl = 0.5876 if name == "rt_asph" else 0.587
    ref_lens, lens = build_lens(name), build_lens(name)
    ref = _trace(ref_lens, "reference", wl=wl)
    first = _trace(lens, "device", wl=wl)  # cold cache: host-verified
    again = _trace(lens, "device", wl=wl)  # warm: device-verified, no host read
    dl = _dlens(lens, wl)
    assert dl.last_schedule_dev is not None and dl.pending
    raytrace.check_all_pending()
    for a in ref:
        np.testing.assert_array_equal(first[a], ref[a], err_msg=a)
        np.testing.assert_array_equal(again[a], ref[a], err_msg=a)


@pytest.mark.parametrize("path", ["verify_retrace", "fixup_run_if"])
@pytest.mark.parametrize("offset", [+5, -1, -2])
def test_device_fixup_corrects_a_wrong_schedule(torch, offset, path, monkeypatch):
    """Seed the warm cache with a wrong schedule: the device rounds settle it to the
    reference's stop index and the rays equal the host-verified trace -- through the
    verify-and-re-trace launches (ort_options.verify_*, one launch per round) and through
    the two-launch rounds (ort_newton_fixup + run_if) that larger schedules take."""
    from optiland_pr_amd import raytrace
    from tests._cases import build_lens

    if path == "fixup_run_if":
        monkeypatch.setattr(raytrace, "VERIFY_MAX_SCHED", 0)

    ref_lens, lens = build_lens("rt_asph"), build_lens("rt_asph")
    ref = _trace(ref_lens, "reference")
    _trace(lens, "reference")
    dl = _dlens(lens, 0.5876)
    good = {k: v.copy() for k, v in dl.sched_cache.items() if k != "_default"}
    for k, v in good.items():  # a wrong warm schedule
        bad = v.copy()
        for s in dl.newton:
            bad[s] = max(0, int(v[s]) + offset)
        dl.sched_cache[k] = bad
    dl._dev_sched.clear()
    got = _trace(lens, "device")
    raytrace.check_all_pending()
    for a in ref:
        np.testing.assert_array_equal(got[a], ref[a], err_msg=a)
    for k, v in good.items():  # the settled device schedule is back in the host cache
        assert np.array_equal(dl.sched_cache[k], v), (k, dl.sched_cache[k], v)


def test_device_mode_gradients_equal_reference(torch):
    """The config-5 step in device mode: the same loss and gradients as host-verified."""
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.operands import RayOperand
    from optiland_pr_amd import raytrace
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    d = RandomDistribution(seed=0)
    d.generate_points(65536)
    res = {}
    for mode in ("reference", "device"):
        lens = ThreeMirrorAnastigmat()
        lens.newton_mode = mode
        leaves = []
        for si in (1, 2, 3):
            g = lens.surface_group.surfaces[si].geometry
            t = torch.tensor(np.asarray(g.coefficients), dtype=torch.float64, device="cuda",
                             requires_grad=True)
            g.coefficients = t
            leaves.append(t)
        for _ in range(3):  # warm, then device-verified steps
            for t in leaves:
                t.grad = None
            loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, 65536, 0.587, d)
            loss.backward()
        raytrace.check_all_pending()
        res[mode] = (float(loss.detach()), np.concatenate([t.grad.cpu().numpy() for t in leaves]))
    assert res["device"][0] == res["reference"][0]
    np.testing.assert_array_equal(res["device"][1], res["reference"][1])


def test_device_mode_range_error_surfaces_at_check(torch):
    from optiland_pr_amd import raytrace
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    lens = ThreeMirrorAnastigmat()
    _trace(lens, "device", n=64, wl=0.587)
    _trace(lens, "device", n=64, wl=0.587)  # warm
    raytrace.check_all_pending()
    for s in lens.surface_group.surfaces[1:4]:
        s.geometry.norm_radius = 0.5
    lens.invalidate()
    with pytest.raises(ValueError, match="Zernike coordinates must be normalized"):
        _trace(lens, "device", n=64, wl=0.587)
        raytrace.check_all_pending()


def test_newton_finish_state_for_the_next_call(torch):
    """ort_newton_finish (ABI v17) on hand-made round buffers: the status of the last round
    that ran lands in status_out, every status word is zeroed, every statistics byte is
    0xFF and the schedule is copied out -- the state the next call's rounds start from."""
    import ctypes as C

    from optiland_pr_amd import _native
    from optiland_pr_amd.raytrace import _ptr, _stream_handle
    from tests._cases import build_lens

    lens = build_lens("rt_asph")
    _trace(lens, "reference")
    dl = _dlens(lens, 0.5876)
    S = dl.table.n_surfaces
    R, n_groups = 3, 2
    nb = n_groups * S * 24
    stats = torch.randint(0, 255, (R + 1, nb), dtype=torch.uint8, device="cuda")
    # round 1 ran (flags[0] == 1), round 2 did not (flags[1] == 0): the last status is [1]
    flags = torch.tensor([1, 0, 0, 9], dtype=torch.int32, device="cuda")
    statuses = torch.tensor([4, 1, 2, 8], dtype=torch.int32, device="cuda")
    status_out = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    sched = torch.arange(n_groups * S, dtype=torch.int32, device="cuda")
    copy = torch.full((n_groups * S,), -7, dtype=torch.int32, device="cuda")
    rc = _native.load().ort_newton_finish(C.byref(dl.c), n_groups, _ptr(stats), R, 0,
                                          _ptr(sched), _ptr(flags), _ptr(statuses),
                                          _ptr(status_out), _ptr(copy), _stream_handle())
    _native.check(rc, "ort_newton_finish")
    torch.cuda.synchronize()
    assert int(status_out) == 1
    assert flags.tolist() == [1, 0, 0, 0]  # flags[R] = flags[R - 1]: nothing ran to check
    assert statuses.tolist() == [0, 0, 0, 0]
    assert bool((stats == 255).all())
    assert torch.equal(copy, sched)


def test_device_rounds_reuse_their_buffers(torch):
    """Consecutive device-verified calls on the same round buffers (ort_newton_finish leaves
    them initialised for the next call, no per-call fills): three wrong warm schedules in a
    row, each settled to the reference's, each call's rays equal to the host-verified
    trace, and the settled schedule the backward keeps is each call's own copy."""
    from optiland_pr_amd import raytrace
    from tests._cases import build_lens

    ref_lens, lens = build_lens("rt_asph"), build_lens("rt_asph")
    ref = _trace(ref_lens, "reference")
    _trace(lens, "reference")
    dl = _dlens(lens, 0.5876)
    good = {k: v.copy() for k, v in dl.sched_cache.items() if k != "_default"}
    copies = []
    for offset in (+5, -1, +2, 0):
        for k, v in good.items():
            bad = v.copy()
            for s in dl.newton:
                bad[s] = max(0, int(v[s]) + offset)
            dl.sched_cache[k] = bad
        dl._dev_sched.clear()
        got = _trace(lens, "device")
        assert dl.last_schedule_private
        copies.append(dl.last_schedule_dev)
        raytrace.check_all_pending()
        for a in ref:
            np.testing.assert_array_equal(got[a], ref[a], err_msg=f"{a} offset {offset}")
        for k, v in good.items():
            assert np.array_equal(dl.sched_cache[k], v), (offset, k, dl.sched_cache[k], v)
    assert len({c.data_ptr() for c in copies}) == len(copies)  # one live copy per call
    for c in copies:
        assert torch.equal(c, copies[0])


@pytest.mark.parametrize("path", ["verify_retrace", "fixup_run_if"])
@pytest.mark.parametrize("offset", [+5, -1])
def test_taped_rounds_stride_and_correct(torch, offset, path, monkeypatch):
    """The config-5 step (taped forward, fused rms) with more rays than one grid of the
    verify rounds covers (kVerifyGrid = 1024 workgroups = 262,144 rays; 600,000 here, so
    the F_STRIDE kernels loop): a wrong warm schedule is corrected by re-traces in those
    rounds -- the verify-and-re-trace launches, or the two-launch rounds (ort_newton_fixup +
    a run_if re-launch, also on the grid-stride kernel) -- and loss and gradients equal the
    host-verified step bit for bit."""
    from optiland_pr_amd import raytrace

    if path == "fixup_run_if":
        monkeypatch.setattr(raytrace, "VERIFY_MAX_SCHED", 0)
    from optiland_pr_amd.distribution import RandomDistribution
    from optiland_pr_amd.operands import RayOperand
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    n = 600_000
    d = RandomDistribution(seed=5)
    d.generate_points(n)
    res = {}
    for mode in ("reference", "device"):
        lens = ThreeMirrorAnastigmat()
        lens.newton_mode = mode
        leaves = []
        for si in (1, 2, 3):
            g = lens.surface_group.surfaces[si].geometry
            t = torch.tensor(np.asarray(g.coefficients), dtype=torch.float64, device="cuda",
                             requires_grad=True)
            g.coefficients = t
            leaves.append(t)

        def step():
            for t in leaves:
                t.grad = None
            loss = RayOperand.rms_spot_size(lens, -1, 0.0, 1.0, n, 0.587, d)
            loss.backward()
            return loss

        step()  # warm (host-verified)
        if mode == "device":
            dl = _dlens(lens, 0.587)
            for k, v in list(dl.sched_cache.items()):
                if k == "_default":
                    continue
                bad = v.copy()
                for s in dl.newton:
                    bad[s] = max(0, int(v[s]) + offset)
                dl.sched_cache[k] = bad
            dl._dev_sched.clear()
        loss = step()
        raytrace.check_all_pending()
        res[mode] = (float(loss.detach()), np.concatenate([t.grad.cpu().numpy() for t in leaves]))
    assert res["device"][0] == res["reference"][0]
    np.testing.assert_array_equal(res["device"][1], res["reference"][1])
