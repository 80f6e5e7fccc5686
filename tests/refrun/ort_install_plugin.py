"""pytest plugin for running the REFERENCE's own test files with the drop-in installed
(tests/test_reference_install.py launches them; never loaded on the GPU box).
It lives outside the `tests` package: the reference's own tests are a package named `tests`.

Loaded with `-p ort_install_plugin` (tests/refrun on PYTHONPATH): patches optiland's SurfaceGroup.trace with
adapter.install() before any test runs, and at the end writes which path served the trace
calls (adapter.STATS: the op's CUDA / CPU kernels, or the reference's own loop) into the
directory named by ORT_INSTALL_STATS, one JSON file per process (pytest-xdist workers each
write their own).
"""

import json
import os


def pytest_configure(config):
    from optiland_pr_amd import adapter

    adapter.install()


def pytest_unconfigure(config):
    from optiland_pr_amd import adapter

    out = os.environ.get("ORT_INSTALL_STATS")
    if out:
        with open(os.path.join(out, f"{os.getpid()}.json"), "w") as f:
            json.dump({**adapter.STATS, "reasons": adapter.REASONS}, f)
