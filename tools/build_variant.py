"""Build an A/B variant of liboptiland_rt.so that differs only in one kernel TU (default
the closed-form kernel's, ort_k_closed.hip): compile that TU with extra -D flags and link
it with the main build's other objects. Measurement tooling (tools/ab.sh), not product.

usage: python tools/build_variant.py NAME [--tu ort_k_trace.hip[,ort_k_closed.hip,...]]
           [--from-rev GIT_REV] [-DFLAG ...]
       -> optiland_pr_amd/lib/variants/NAME.so
--from-rev: the swapped TUs (and the headers they include) as they were at GIT_REV -- an
A/B of the current build against an earlier commit's kernels, for TUs whose argument
structs did not change in between.
"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from optiland_pr_amd import build  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
tu_name = "ort_k_closed.hip"
if flags[:1] == ["--tu"]:
    tu_name, flags = flags[1], flags[2:]
src_dir, inc_dir = None, os.path.join(REPO, "include")
if flags[:1] == ["--from-rev"]:
    import tempfile

    rev, flags = flags[1], flags[2:]
    tmp = tempfile.mkdtemp(prefix="ort_rev_")
    subprocess.run(f"git -C {REPO} archive {rev} optiland_pr_amd/csrc include | tar -x -C {tmp}",
                   shell=True, check=True)
    src_dir, inc_dir = os.path.join(tmp, "optiland_pr_amd", "csrc"), os.path.join(tmp, "include")
build.build()  # the main objects must be current
obj_main = os.path.join(build.LIB_DIR, "obj")
vdir = os.path.join(build.LIB_DIR, "variants")
os.makedirs(vdir, exist_ok=True)
tus = tu_name.split(",")
new = []
for t in tus:  # each swapped TU compiled with the extra flags
    obj = os.path.join(vdir, f"obj_{name}_{t.split('.')[0]}.o")
    subprocess.run([build.hipcc(), *build.HIPCC_FLAGS, *flags, "-I", inc_dir, "-c", "-o", obj,
                    os.path.join(src_dir or build.CSRC, t)], check=True)
    new.append(obj)
objs = [o for o in glob.glob(os.path.join(obj_main, "*.o"))
        if os.path.basename(o) not in {t + ".o" for t in tus}] + new
out = os.path.join(vdir, name + ".so")
subprocess.run([build.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs],
               check=True)
print(out)
