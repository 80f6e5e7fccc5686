"""Build an A/B variant of liboptiland_rt.so that differs only in the closed-form kernel
TU (ort_k_closed.hip): compile that TU with extra -D flags and link it with the main
build's other objects. Measurement tooling (tools/ab.sh), not product.

usage: python tools/build_variant.py NAME [-DFLAG ...]  -> optiland_pr_amd/lib/variants/NAME.so
"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from optiland_pr_amd import build  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
build.build()  # the main objects must be current
obj_main = os.path.join(build.LIB_DIR, "obj")
vdir = os.path.join(build.LIB_DIR, "variants")
os.makedirs(vdir, exist_ok=True)
tu = os.path.join(build.CSRC, "ort_k_closed.hip")
obj = os.path.join(vdir, f"obj_{name}_closed.o")
subprocess.run([build.hipcc(), *build.HIPCC_FLAGS, *flags, "-I", os.path.join(REPO, "include"),
                "-c", "-o", obj, tu], check=True)
objs = [o for o in glob.glob(os.path.join(obj_main, "*.o")) if "ort_k_closed" not in o] + [obj]
out = os.path.join(vdir, name + ".so")
subprocess.run([build.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs],
               check=True)
print(out)
