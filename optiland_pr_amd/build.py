"""Build the native libraries in-tree:

  optiland_pr_amd/lib/liboptiland_rt.so    the HIP trace core for gfx950 (hipcc)
  optiland_pr_amd/lib/liboptiland_host.so  its host build, the CPU dispatch key of the torch
                                           custom ops (g++ -fopenmp, include/optiland_host.h)

    python -m optiland_pr_amd.build

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU container too.
The .so files are git-ignored but travel to the GPU box with the repo snapshot.
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
HOST_LIB_PATH = os.path.join(LIB_DIR, "liboptiland_host.so")
CSRC = os.path.join(HERE, "csrc")
# one translation unit per kernel family, compiled in parallel, linked into one .so
SOURCES = [os.path.join(CSRC, f) for f in (
    "ort_api.hip", "ort_k_closed.hip", "ort_k_trace.hip", "ort_k_trace_mono.hip", "ort_k_trace_tape.hip", "ort_k_trace_rec.hip",
    "ort_k_trace_w.hip", "ort_k_vjp.hip", "ort_k_vjp1.hip", "ort_k_vjp2.hip", "ort_k_vjp4.hip", "ort_k_geom.hip",
    "ort_k_adj.hip", "ort_k_adj2.hip", "ort_k_adj4.hip", "ort_k_adj2r.hip", "ort_k_adj4r.hip", "ort_k_pupil.hip", "ort_k_trace_ia.hip",
    "ort_k_spot.hip", "ort_k_wavefront.hip")]
HEADERS = [os.path.join(CSRC, "ort_core.h"), os.path.join(CSRC, "ort_kernels.h"), os.path.join(CSRC, "ort_fastpath.h"),
           os.path.join(CSRC, "ort_adjoint.h"), os.path.join(CSRC, "ort_pupil.h"),
           os.path.join(CSRC, "ort_sincos_table.h"), os.path.join(CSRC, "ort_material.h"), os.path.join(CSRC, "ort_interact.h"), os.path.join(CSRC, "ort_reduce.h"),
           os.path.join(CSRC, "ort_sweep.h"), os.path.join(CSRC, "ort_nurbs.h"),
           os.path.join(REPO, "include", "optiland_rt.h")]
DEPS = SOURCES + HEADERS
HOST_SOURCES = [os.path.join(CSRC, "ort_host.cpp")]
HOST_DEPS = HOST_SOURCES + [os.path.join(CSRC, f) for f in ("ort_core.h", "ort_sweep.h",
                                                           "ort_material.h", "ort_interact.h",
                                                           "ort_nurbs.h")] + [
    os.path.join(REPO, "include", "optiland_rt.h"), os.path.join(REPO, "include", "optiland_host.h")]
# the host build keeps the kernels' rounding: no contraction of a*b+c (as -ffp-contract=off
# on hipcc), no fast-math
HOST_FLAGS = ["-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-fPIC", "-shared",
              "-std=c++17", "-Wall", "-Wno-unknown-pragmas"]

# -ffp-contract=off: no a*b+c fusion, so each +,-,*,/ rounds exactly as NumPy does.
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17", "-fPIC",
               "-Wno-unused-result"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build the MI355X trace core)")


def needs_build(out=None, deps=None):
    out = out or LIB_PATH
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in (deps or DEPS))


def _start_host_build(force=False, verbose=False):
    """Start the g++ build of liboptiland_host.so (None when it is up to date)."""
    if not force and not needs_build(HOST_LIB_PATH, HOST_DEPS):
        return None
    os.makedirs(LIB_DIR, exist_ok=True)
    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    cmd = [cxx, *HOST_FLAGS, "-I", os.path.join(REPO, "include"), "-o", HOST_LIB_PATH + ".tmp",
           *HOST_SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    return subprocess.Popen(cmd)


def _finish_host_build(proc):
    if proc is None:
        return
    if proc.wait() != 0:
        raise subprocess.CalledProcessError(proc.returncode, "g++ ort_host.cpp")
    os.replace(HOST_LIB_PATH + ".tmp", HOST_LIB_PATH)


def build_host(force=False, verbose=False):
    """Compile liboptiland_host.so alone (the CPU dispatch key)."""
    _finish_host_build(_start_host_build(force, verbose))
    return HOST_LIB_PATH


def build(force=False, verbose=False, out=None, extra_flags=(), jobs=None):
    """Compile every translation unit (in parallel) and link liboptiland_rt.so; the host
    library liboptiland_host.so is compiled alongside (default output only).
    out / extra_flags: build a variant library elsewhere (A/B timing)."""
    host = None if out else _start_host_build(force, verbose)
    out = out or LIB_PATH
    if not force and not needs_build(out):
        _finish_host_build(host)
        return out
    obj_dir = os.path.join(os.path.dirname(out), "obj" + ("" if out == LIB_PATH else "_" +
                           os.path.splitext(os.path.basename(out))[0]))
    os.makedirs(obj_dir, exist_ok=True)
    cc = hipcc()
    inc = ["-I", os.path.join(REPO, "include")]
    procs, objs = [], []
    jobs = jobs or min(len(SOURCES), max(1, os.cpu_count() or 1), 16)
    pending = list(SOURCES)
    failed = None
    # a translation unit is recompiled when it or a header is newer than its object, or when
    # the flags changed (force: every unit)
    flag_file = os.path.join(obj_dir, "flags.txt")
    flags_now = " ".join([*HIPCC_FLAGS, *extra_flags])
    same_flags = os.path.exists(flag_file) and open(flag_file).read() == flags_now
    newest_hdr = max(os.path.getmtime(h) for h in HEADERS)

    def fresh(src, obj):
        return (not force and same_flags and os.path.exists(obj)
                and os.path.getmtime(obj) > max(os.path.getmtime(src), newest_hdr))

    while pending or procs:
        while pending and len(procs) < jobs:
            src = pending.pop(0)
            obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
            objs.append(obj)
            if fresh(src, obj):
                continue
            cmd = [cc, *HIPCC_FLAGS, *extra_flags, *inc, "-c", "-o", obj, src]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((subprocess.Popen(cmd), src))
        if not procs:
            continue
        p, src = procs.pop(0)
        if p.wait() != 0:
            failed = src
    if failed:
        raise subprocess.CalledProcessError(1, f"hipcc {failed}")
    with open(flag_file, "w") as f:
        f.write(flags_now)
    tmp = out + ".tmp"
    cmd = [cc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    _finish_host_build(host)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
