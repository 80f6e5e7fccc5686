"""Lens JSON I/O (optiland_pr_amd.lensio, the reference's Optic.to_dict / from_dict
schema, optic/optic.py:649-713). The reference's sample files (tests/golden/lenses,
copied from its docs/samples) are pinned through the golden cases json_* (oracle and GPU
parity against the reference's own from_dict + trace); here: round trips preserve the
lowered table bytes for every golden lens, and malformed inputs raise."""

import json

import numpy as np
import pytest

from optiland_pr_amd.lensio import optic_from_dict, optic_to_dict
from optiland_pr_amd.lowering import lower_surface_group
from tests._cases import ALL_CASES, build_lens


@pytest.mark.parametrize("name", ALL_CASES)
def test_round_trip_preserves_lowering(name):
    lens = build_lens(name)
    data = json.loads(json.dumps(optic_to_dict(lens)))  # through real JSON text
    back = optic_from_dict(data)
    wls = [0.55]
    a = lower_surface_group(lens.surface_group, wls)
    b = lower_surface_group(back.surface_group, wls)
    assert a.fingerprint() == b.fingerprint()
    assert back.paraxial.EPD() == lens.paraxial.EPD()
    assert back.paraxial.EPL() == lens.paraxial.EPL()
    assert back.field_type == lens.field_type
    np.testing.assert_array_equal(back.fields.y_fields, lens.fields.y_fields)
    assert back.wavelengths.get_wavelengths() == lens.wavelengths.get_wavelengths()


def test_unsupported_inputs_raise():
    data = optic_to_dict(build_lens("cooke"))
    bad = json.loads(json.dumps(data))
    bad["surface_group"]["surfaces"][1]["geometry"]["type"] = "BogusGeometry"
    with pytest.raises(ValueError, match="geometry type"):
        optic_from_dict(bad)
    bad = json.loads(json.dumps(data))
    bad["surface_group"]["surfaces"][1]["coating"] = {"type": "SimpleCoating"}
    with pytest.raises(ValueError, match="coating"):
        optic_from_dict(bad)
    bad = json.loads(json.dumps(data))
    bad["surface_group"]["surfaces"][1]["material_post"] = {"type": "Material", "name": "XYZ"}
    with pytest.raises(ValueError):
        optic_from_dict(bad)
