"""Build an A/B variant of liboptiland_rt.so that differs only in one kernel TU (default
the closed-form kernel's, ort_k_closed.hip): compile that TU with extra -D flags and link
it with the main build's other objects. Measurement tooling (tools/ab.sh), not product.

usage: python tools/build_variant.py NAME [--tu ort_k_trace.hip] [-DFLAG ...]
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
tu = os.path.join(build.CSRC, tu_name)
obj = os.path.join(vdir, f"obj_{name}_{tu_name.split('.')[0]}.o")
subprocess.run([build.hipcc(), *build.HIPCC_FLAGS, *flags, "-I", os.path.join(REPO, "include"),
                "-c", "-o", obj, tu], check=True)
objs = [o for o in glob.glob(os.path.join(obj_main, "*.o")) if os.path.basename(o) != tu_name + ".o"] + [obj]
out = os.path.join(vdir, name + ".so")
subprocess.run([build.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs],
               check=True)
print(out)
