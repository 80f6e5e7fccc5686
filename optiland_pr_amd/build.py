"""Build the HIP extension in-tree: optiland_pr_amd/lib/liboptiland_rt.so (gfx950).

    python -m optiland_pr_amd.build

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU container too.
The .so is git-ignored but travels to the GPU box with the repo snapshot.
"""

from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "liboptiland_rt.so")
SOURCES = [os.path.join(HERE, "csrc", "ort_trace.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", "ort_core.h"),
                  os.path.join(REPO, "include", "optiland_rt.h")]

# -ffp-contract=off: no a*b+c fusion, so each +,-,*,/ rounds exactly as NumPy does.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17", "-fPIC",
               "-shared", "-Wno-unused-result"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build the MI355X trace core)")


def needs_build():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + ".tmp"
    cmd = [hipcc(), *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), "-o", tmp, *SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
