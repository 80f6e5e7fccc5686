"""Shared helpers: rebuild a golden case with the NATIVE host API (optiland_pr_amd)."""

import numpy as np

from optiland_pr_amd import _abi
from optiland_pr_amd.lowering import lower_surface_group, segment_params
from optiland_pr_amd.samples import GOLDEN_LENSES


def native_case(name, meta, record=False):
    """-> (optic, LensTable, segments [n_pairs] (field-major, then wavelength), keys)."""
    lens = GOLDEN_LENSES[name]()
    wls = meta["wavelengths"]
    table = lower_surface_group(lens.surface_group, wls, record=record)
    EPL, EPD = lens.paraxial.EPL(), lens.paraxial.EPD()
    segs = []
    for hx, hy in meta["fields"]:
        for wi in range(len(wls)):
            segs.append(segment_params(lens, hx, hy, wi, EPL, EPD))
    return lens, table, np.stack(segs)


# golden cases whose every traced surface is closed-form (plane / conic): the oracle and
# the HIP kernel reproduce the reference bit for bit there
CLOSED_FORM = ("cooke", "dg", "rt", "cooke_aperture", "decentered")
NEWTON = ("rt_asph", "rt_odd", "tma_fringe", "tma_standard", "tma_noll", "freeform")
ALL_CASES = CLOSED_FORM + NEWTON

FIELDS = _abi.RAY_FIELDS
