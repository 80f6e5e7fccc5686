"""The drop-in adapter lowers REFERENCE Optiland objects into exactly the table bytes the
native host API produces (CPU; runs only where /root/reference is importable, i.e. in
the build container -- skipped on the GPU box)."""

import os
import sys

import numpy as np
import pytest

from tests.conftest import REPO

REF = "/root/reference"


@pytest.fixture(scope="module")
def ref():
    if not os.path.isdir(os.path.join(REF, "optiland")):
        pytest.skip("reference not present")
    sys.dont_write_bytecode = True  # never write __pycache__ into the reference tree
    for p in (os.path.join(REPO, "tests", "golden", "shims"), REF):
        if p not in sys.path:
            sys.path.insert(0, p)
    import optiland.backend as be
    from optiland.samples import objectives

    be.set_backend("numpy")
    return objectives


@pytest.mark.parametrize("name,wls", [("DoubleGauss", [0.4861, 0.5876]),
                                      ("CookeTriplet", [0.55]),
                                      ("ReverseTelephoto", [0.5876, 0.6563])])
def test_reference_lowering_equals_native(ref, name, wls):
    from optiland_pr_amd import samples
    from optiland_pr_amd.adapter import lower_reference_group
    from optiland_pr_amd.lowering import lower_surface_group

    ref_lens = getattr(ref, name)()
    native = getattr(samples, name)()
    a = lower_reference_group(ref_lens.surface_group, wls)
    b = lower_surface_group(native.surface_group, wls)
    assert a.surfaces.tobytes() == b.surfaces.tobytes()
    assert a.cs_ops.tobytes() == b.cs_ops.tobytes()
    np.testing.assert_array_equal(a.n_tab, b.n_tab)
    np.testing.assert_array_equal(a.alpha_tab, b.alpha_tab)
    assert a.final_mat == b.final_mat and a.final_thickness == b.final_thickness


@pytest.mark.parametrize("name", ["freeform", "tma_fringe", "rt_asph", "cooke_shapes",
                                  "cooke_aperture", "forbes", "forbes_q2d", "paraxial_lens",
                                  "paraxial_mirror", "phase_plate", "grating_flat",
                                  "grating_curved", "grating_reflective", "grating_tilted",
                                  "grid_lens", "cooke_abbe", "uv_projection"])
def test_reference_lowering_equals_native_newton(ref, name):
    """Newton geometries (incl. the freeform kinds): the adapter's lowering of the
    reference lens equals the native lens's bytes, coefficient blocks included."""
    import sys

    from optiland_pr_amd.adapter import lower_reference_group
    from optiland_pr_amd.lowering import lower_surface_group
    from optiland_pr_amd.samples import GOLDEN_LENSES

    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import gen_golden

    builder = gen_golden.CASES[name][0]
    ref_lens = builder()
    native = GOLDEN_LENSES[name]()
    wls = [0.55]
    a = lower_reference_group(ref_lens.surface_group, wls)
    b = lower_surface_group(native.surface_group, wls)
    assert a.surfaces.tobytes() == b.surfaces.tobytes()
    assert a.cs_ops.tobytes() == b.cs_ops.tobytes()
    np.testing.assert_array_equal(a.coef, b.coef)
    assert a.zern.tobytes() == b.zern.tobytes()
