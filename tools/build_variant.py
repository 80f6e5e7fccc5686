"""Build an A/B variant of liboptiland_rt.so that differs only in one kernel TU (default
the closed-form kernel's, ort_k_closed.hip): compile that TU with extra -D flags and link
it with the main build's other objects. Measurement tooling (tools/ab.sh), not product.

usage: python tools/build_variant.py NAME [--tu ort_k_trace.hip[,ort_k_closed.hip,...]] [-DFLAG ...]
       -> optiland_pr_amd/lib/variants/NAME.so
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
build.build()  # the main objects must be current
obj_main = os.path.join(build.LIB_DIR, "obj")
vdir = os.path.join(build.LIB_DIR, "variants")
os.makedirs(vdir, exist_ok=True)
tus = tu_name.split(",")
new = []
for t in tus:  # each swapped TU compiled with the extra flags
    obj = os.path.join(vdir, f"obj_{name}_{t.split('.')[0]}.o")
    subprocess.run([build.hipcc(), *build.HIPCC_FLAGS, *flags, "-I",
                    os.path.join(REPO, "include"), "-c", "-o", obj,
                    os.path.join(build.CSRC, t)], check=True)
    new.append(obj)
objs = [o for o in glob.glob(os.path.join(obj_main, "*.o"))
        if os.path.basename(o) not in {t + ".o" for t in tus}] + new
out = os.path.join(vdir, name + ".so")
subprocess.run([build.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs],
               check=True)
print(out)
