"""CPU: which VJP mode a lens gets (host logic; the kernels run in test_gpu_adjoint.py)."""


def test_standard_zernike_takes_adjoint_within_the_tape():
    """standard / noll Zernike surfaces carry SURF_SLOPE_INEXACT (their Newton slope omits
    the normalisation constant, zernike.py:163-231); the adjoint is exact on them while
    every surface's schedule fits the tape (U <= ADJ_HIST), the forward-mode VJP serves a
    longer one. Surfaces with an exact slope keep the adjoint whatever U."""
    import numpy as np

    from optiland_pr_amd import _abi, autodiff
    from tests._cases import build_lens
    from optiland_pr_amd.lowering import lower_surface_group

    for name, inexact in (("tma_standard", True), ("tma_noll", True), ("tma_fringe", False),
                          ("rt_asph", False), ("cooke", False)):
        lens = build_lens(name)
        table = lower_surface_group(lens.surface_group, [lens.primary_wavelength])
        flags = (table.surfaces["flags"] & _abi.SURF_SLOPE_INEXACT) != 0
        geo = table.surfaces["geometry"]
        assert np.array_equal(flags, inexact & (geo == _abi.GEOM_ZERNIKE)), name
        assert autodiff.vjp_mode(table) == _abi.VJP_ADJOINT, name
        S = table.n_surfaces
        newton = geo >= _abi.GEOM_EVEN_ASPHERE
        for U in (0, 1, _abi.ADJ_HIST, _abi.ADJ_HIST + 1, 100):
            sched = np.where(newton, U, -1).astype(np.int32).reshape(1, S).repeat(3, 0)
            want = (_abi.VJP_UNROLLED if inexact and U > _abi.ADJ_HIST
                    else _abi.VJP_ADJOINT)
            assert autodiff.vjp_mode(table, sched) == want, (name, U)
        assert autodiff.inexact_updates(table, None) == 0


def test_more_slots_than_the_adjoint_holds_take_unrolled_mode():
    """The adjoint keeps its per-block slot partials in LDS (ORT_VJP_ADJOINT_MAX_SLOTS =
    3 S + n_zern + 1 + n_mono at most, include/optiland_rt.h): a lens with more Zernike terms than
    that takes the forward-mode VJP instead of a refused launch."""
    import re
    from pathlib import Path

    import numpy as np

    from optiland_pr_amd import _abi, autodiff
    from tests._cases import build_lens
    from optiland_pr_amd.lowering import lower_surface_group

    hdr = Path(__file__).resolve().parents[1] / "include" / "optiland_rt.h"
    m = re.search(r"#define ORT_VJP_ADJOINT_MAX_SLOTS (\d+)", hdr.read_text())
    assert m and int(m.group(1)) == _abi.VJP_ADJOINT_MAX_SLOTS
    lens = build_lens("tma_fringe")
    table = lower_surface_group(lens.surface_group, [lens.primary_wavelength])
    assert autodiff.vjp_mode(table) == _abi.VJP_ADJOINT
    S = table.n_surfaces
    # Zernike terms the adjoint still holds (the Cartesian surfaces' monomial slots, ABI v18,
    # count too)
    from optiland_pr_amd.ops import mono_slot_count

    room = _abi.VJP_ADJOINT_MAX_SLOTS - (3 * S + 1 + mono_slot_count(table, table.zern))
    z = table.zern
    big = np.concatenate([z] * (room // len(z) + 1))[:room + 1]
    table.zern = big
    assert autodiff.vjp_mode(table) == _abi.VJP_UNROLLED
    table.zern = big[:room]
    assert autodiff.vjp_mode(table) == _abi.VJP_ADJOINT
