"""The REFERENCE's NURBS lens (tests/golden/gen_golden.py nurbs_lens: a bicubic fit of a conic
in front, an explicit rational net behind, nurbs_geometry.py) traced by the reference's own
Optic.trace, first as it is and then with the drop-in installed (adapter.install(): the
NumPy backend's rays served by the op's CPU kernel, the host build of ort_nurbs.h); prints
one JSON line with both image planes and adapter.STATS. Launched by
tests/test_reference_install.py in the build container (the reference is not on the GPU
box):

    python tests/refrun/nurbs_run.py
"""

import json
import os
import sys

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "tests", "golden", "shims"),
          "/root/reference", REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

import gen_golden  # noqa: E402

from optiland_pr_amd import adapter  # noqa: E402

FIELDS = ("x", "y", "z", "L", "M", "N", "i", "opd")


def trace(lens):
    out = []
    for hx, hy in ((0.0, 0.0), (0.0, 1.0), (0.6, 0.6)):
        r = lens.trace(hx, hy, 0.55, num_rays=16, distribution="hexapolar")
        out.append({a: np.asarray(getattr(r, a), dtype=np.float64).tolist() for a in FIELDS})
    return out


def main():
    ref = trace(gen_golden.nurbs_lens())
    adapter.install()
    got = trace(gen_golden.nurbs_lens())
    print(json.dumps({"reference": ref, "installed": got, "stats": adapter.STATS}))


if __name__ == "__main__":
    main()
