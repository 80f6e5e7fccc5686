"""Shared helpers: rebuild a golden case with the NATIVE host API (optiland_pr_amd)."""

import os

import numpy as np

from optiland_pr_amd import _abi
from optiland_pr_amd.lowering import (lower_apodization, lower_surface_group, pupil_scalars,
                                      segment_params)
from optiland_pr_amd.samples import GOLDEN_LENSES


JSON_LENSES = {"json_cooke": "cooke_triplet", "json_heliar": "heliar",
               "json_rt": "reverse_telephoto"}


def build_lens(name):
    """Native lens of a golden case: a sample class, or a reference JSON lens file read
    with the native loader (optiland_pr_amd.lensio)."""
    if name in JSON_LENSES:
        from optiland_pr_amd.lensio import load_optiland_json

        return load_optiland_json(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                               "golden", "lenses", JSON_LENSES[name] + ".json"))
    return GOLDEN_LENSES[name]()


def native_case(name, meta, record=False):
    """-> (optic, LensTable, segments [n_pairs] (field-major, then wavelength), keys)."""
    lens = build_lens(name)
    wls = meta["wavelengths"]
    table = lower_surface_group(lens.surface_group, wls, record=record)
    table.apod = lower_apodization(lens)
    EPL, EPD = pupil_scalars(lens)
    segs = []
    for hx, hy in meta["fields"]:
        for wi in range(len(wls)):
            segs.append(segment_params(lens, hx, hy, wi, EPL, EPD))
    return lens, table, np.stack(segs)


# golden cases whose every traced surface is closed-form (plane / conic): the oracle and
# the HIP kernel reproduce the reference bit for bit there
CLOSED_FORM = ("cooke", "dg", "rt", "cooke_aperture", "cooke_shapes", "decentered", "json_cooke",
               "json_heliar", "json_rt", "cooke_pih", "finite_pih", "paraxial_lens",
               "paraxial_mirror", "grating_flat", "grating_curved", "grating_reflective",
               "grating_tilted", "uv_projection", "apod_gaussian", "apod_cos2", "apod_hann",
               "apod_poly", "apod_supergauss", "apod_tukey", "apod_uniform", "cooke_abbe")
NEWTON = ("rt_asph", "rt_odd", "tma_fringe", "tma_standard", "tma_noll", "freeform",
          "forbes", "forbes_q2d", "phase_plate", "grid_lens", "nurbs_lens")
ALL_CASES = CLOSED_FORM + NEWTON

FIELDS = _abi.RAY_FIELDS
