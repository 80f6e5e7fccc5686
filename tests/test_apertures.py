"""Physical apertures (CPU): the native classes, lowered to aperture programs and
evaluated by the oracle, against the reference's own contains() masks
(tests/golden/apertures.npz / apertures.json from gen_golden.py --apertures); dict
round trips; lowering flags."""

import json
import os

import numpy as np
import pytest

from oracle import trace_np
from optiland_pr_amd import _abi
from optiland_pr_amd.apertures import (
    BaseAperture,
    EllipticalAperture,
    FileAperture,
    PolygonAperture,
    RadialAperture,
    RectangularAperture,
    program_depth,
)
from tests.conftest import REPO, load_golden

NAMES = ("radial", "offset_radial", "ellipse", "rect", "polygon", "union", "intersection",
         "difference", "nested")


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(REPO, "tests", "golden", "apertures.json")) as f:
        return load_golden("apertures"), json.load(f)


@pytest.mark.parametrize("name", NAMES)
def test_contains_matches_reference(golden, name):
    g, dicts = golden
    ap = BaseAperture.from_dict(dicts[name])
    got = trace_np.aperture_contains(ap.program(), g["x"], g["y"])
    assert np.array_equal(got, g[name]), (name, int(np.sum(got != g[name])))


@pytest.mark.parametrize("name", NAMES)
def test_dict_round_trip(golden, name):
    _, dicts = golden
    ap = BaseAperture.from_dict(dicts[name])
    again = BaseAperture.from_dict(json.loads(json.dumps(ap.to_dict())))
    assert again.program() == ap.program()


def test_operators_and_depth():
    a, b, c = RadialAperture(2), RectangularAperture(-1, 1, -1, 1), EllipticalAperture(1, 2)
    prog = ((a | b) - c).program()
    ops = [int(v) for v in prog if int(v) in (_abi.AP_UNION, _abi.AP_DIFFERENCE)]
    assert int(prog[10]) == _abi.AP_UNION and int(prog[-1]) == _abi.AP_DIFFERENCE
    assert ops[-1] == _abi.AP_DIFFERENCE and program_depth(prog) == 2
    assert type(a + b).__name__ == "UnionAperture" and type(a & b).__name__ == "IntersectionAperture"


def test_file_aperture(tmp_path):
    p = tmp_path / "ap.txt"
    p.write_text("// x y\n0 0\n2 0\n2 1\n0 1\n")
    ap = FileAperture(str(p))
    assert np.array_equal(ap.x, [0, 2, 2, 0]) and np.array_equal(ap.y, [0, 0, 1, 1])
    ins = trace_np.aperture_contains(ap.program(), np.array([1.0, 3.0]), np.array([0.5, 0.5]))
    assert ins.tolist() == [True, False]
    bad = tmp_path / "bad.txt"
    bad.write_text("1 2 3\n4 5 6\n")
    with pytest.raises(ValueError):
        FileAperture(str(bad))


def test_lowering_flags():
    from optiland_pr_amd.lowering import lower_surface_group
    from optiland_pr_amd.samples import CookeTripletShapes

    lens = CookeTripletShapes()
    t = lower_surface_group(lens.surface_group, [0.55])
    flags = t.surfaces["flags"]
    prog_rows = np.flatnonzero(flags & _abi.SURF_APERTURE_PROG)
    assert prog_rows.tolist() == [0, 1, 2, 3, 5]  # traced-surface indices of s1-s4, s6
    for si in prog_rows:
        s = t.surfaces[si]
        prog = t.coef[int(s["ap_off"]):int(s["ap_off"]) + int(s["ap_len"])]
        ap = lens.surface_group.surfaces[si + 1].aperture
        assert prog.tolist() == [float(v) for v in ap.program()]


def test_polygon_requires_matching_lengths():
    with pytest.raises(ValueError):
        PolygonAperture([0, 1, 2], [0, 1])
