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
