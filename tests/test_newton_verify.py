"""Host logic of the Newton speculate-and-verify protocol (raytrace.DeviceLens.verify), on
hand-made ort_newton_stat records -- no GPU. The reference's rule it reproduces: a trace
call stops at the first stop index k whose GLOBAL test passes (newton_raphson.py:148,
k >= 0 updates; grid_sag.py:128, k >= 1 updates), else after max_iter updates."""

import numpy as np
import pytest

from optiland_pr_amd import _abi
from optiland_pr_amd.raytrace import DeviceLens


class _Table:
    def __init__(self, kinds, max_iter):
        self.surfaces = np.zeros(len(kinds), dtype=_abi.SURFACE)
        self.surfaces["geometry"] = kinds
        self.surfaces["max_iter"] = max_iter
        self.n_surfaces = len(kinds)


def _lens(kinds, max_iter=100):
    dl = DeviceLens.__new__(DeviceLens)  # host half only: no device upload
    dl.table = _Table(kinds, max_iter)
    dl.newton = [i for i, g in enumerate(kinds) if g in _abi.NEWTON_GEOMETRIES]
    dl.sched_cache = {}
    return dl


def _stats(n_groups, S, passed, last_bad, base=0):
    """passed[(g, s)] = stop indices whose test passed for every ray (absolute k)."""
    st = np.zeros((n_groups, S), dtype=_abi.NEWTON_STAT)
    st["conv_mask"] = 0
    st["last_bad"] = -1
    for (g, s), ks in passed.items():
        m = 0
        for k in ks:
            if base <= k < base + _abi.CONV_WINDOW:
                m |= 1 << (k - base)
        st[g, s]["conv_mask"][0] = m & (2**64 - 1)
        st[g, s]["conv_mask"][1] = m >> 64
    for (g, s), v in last_bad.items():
        st[g, s]["last_bad"] = v
    return st


EVEN, GRID, PLANE = _abi.GEOM_EVEN_ASPHERE, _abi.GEOM_GRID_SAG, _abi.GEOM_PLANE


def test_exact_schedule_accepted():
    dl = _lens([PLANE, EVEN])
    sched = np.array([[0, 2]], dtype=np.int32)
    # passed at k = 2 (and only there), failed at 0, 1
    ok, new, need = dl.verify(sched, {0: _stats(1, 2, {(0, 1): [2]}, {(0, 1): 1})})
    assert ok and need is None and new[0, 1] == 2


def test_early_stop_detected():
    dl = _lens([EVEN])
    sched = np.array([[3]], dtype=np.int32)
    ok, new, need = dl.verify(sched, {0: _stats(1, 1, {(0, 0): [1, 2, 3]}, {(0, 0): 0})})
    assert not ok and need is None and new[0, 0] == 1


def test_schedule_too_short_grows():
    dl = _lens([EVEN])
    sched = np.array([[2]], dtype=np.int32)
    ok, new, _ = dl.verify(sched, {0: _stats(1, 1, {}, {(0, 0): 2})})
    assert not ok and new[0, 0] == 8


def test_nan_ray_forces_max_iter():
    """One NaN ray never passes (np.max propagates NaN): max_iter updates, accepted with
    no passed bit anywhere in [0, 100) -- all inside the first window."""
    dl = _lens([EVEN], max_iter=100)
    sched = np.array([[100]], dtype=np.int32)
    ok, new, need = dl.verify(sched, {0: _stats(1, 1, {}, {(0, 0): 100})})
    assert ok and need is None and new[0, 0] == 100


def test_grid_needs_at_least_one_update():
    """grid_sag.py:111-129 makes one update before its first test: U = 0 (e.g. a schedule
    cached for a zero-coefficient asphere at the same index) is refused."""
    dl = _lens([PLANE, GRID])
    sched = np.array([[0, 0]], dtype=np.int32)
    ok, new, _ = dl.verify(sched, {0: _stats(1, 2, {}, {})})
    assert not ok and new[0, 1] == 1


def test_stop_index_beyond_64_is_seen():
    """A grid that converges after 70 updates (past the old 64-bit mask)."""
    dl = _lens([GRID], max_iter=100)
    sched = np.array([[100]], dtype=np.int32)
    ok, new, need = dl.verify(sched, {0: _stats(1, 1, {(0, 0): list(range(70, 101))},
                                               {(0, 0): 69})})
    assert not ok and need is None and new[0, 0] == 70


def test_second_window_requested_and_used():
    """max_iter 300: indices >= 128 need a second launch with conv_base = 128."""
    dl = _lens([EVEN], max_iter=300)
    sched = np.array([[300]], dtype=np.int32)
    passed = {(0, 0): list(range(150, 301))}
    w0 = _stats(1, 1, passed, {(0, 0): 149}, base=0)
    ok, new, need = dl.verify(sched, {0: w0})
    assert need == 128
    w1 = _stats(1, 1, passed, {(0, 0): 149}, base=128)
    ok, new, need = dl.verify(sched, {0: w0, 128: w1})
    assert not ok and need is None and new[0, 0] == 150


def test_first_mismatch_per_group_only():
    """Later surfaces of a group depend on the earlier ones' updates: only the first
    mismatch of a group is corrected per round."""
    dl = _lens([EVEN, EVEN])
    sched = np.array([[3, 3], [2, 2]], dtype=np.int32)
    passed = {(0, 0): [1, 2, 3], (0, 1): [1, 2, 3], (1, 0): [2], (1, 1): [1, 2]}
    ok, new, _ = dl.verify(sched, {0: _stats(2, 2, passed, {(0, 0): 0, (1, 0): 1})})
    assert not ok
    assert new.tolist() == [[1, 3], [2, 1]]


@pytest.mark.parametrize("cached,expect", [(0, 1), (500, 100), (5, 5)])
def test_initial_schedule_clamped_to_legal_counts(cached, expect):
    dl = _lens([PLANE, GRID], max_iter=100)
    dl.sched_cache[("k",)] = np.array([0, cached], dtype=np.int32)
    assert int(dl.initial_schedule([("k",)])[0, 1]) == expect
