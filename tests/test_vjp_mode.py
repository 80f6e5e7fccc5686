"""CPU: which VJP mode a lens gets (host logic; the kernels run in test_gpu_adjoint.py)."""


def test_standard_zernike_keeps_unrolled_mode():
    from optiland_pr_amd import _abi, autodiff
    from tests._cases import build_lens
    from optiland_pr_amd.lowering import lower_surface_group

    for name, want in (("tma_standard", _abi.VJP_UNROLLED), ("tma_noll", _abi.VJP_UNROLLED),
                       ("tma_fringe", _abi.VJP_ADJOINT), ("cooke", _abi.VJP_ADJOINT)):
        lens = build_lens(name)
        table = lower_surface_group(lens.surface_group, [lens.primary_wavelength])
        assert autodiff.vjp_mode(table) == want, name


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
