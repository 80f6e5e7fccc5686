"""C ABI checks (CPU): struct layouts match the header, the library loads and exports
every entry point include/optiland_rt.h declares. No compute calls (no GPU here)."""

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from optiland_pr_amd import _abi, _native
from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "optiland_rt.h")

STRUCTS = {
    "ort_surface": (_abi.SURFACE, None),
    "ort_cs_op": (_abi.CS_OP, None),
    "ort_zernike_term": (_abi.ZERNIKE_TERM, None),
    "ort_segment": (_abi.SEGMENT, None),
    "ort_apodization": (_abi.APODIZATION, None),
    "ort_newton_stat": (_abi.NEWTON_STAT, None),
    "ort_lens": (None, _native.ort_lens),
    "ort_rays": (None, _native.ort_rays),
    "ort_batch": (None, _native.ort_batch),
    "ort_options": (None, _native.ort_options),
    "ort_vjp_params": (None, _native.ort_vjp_params),
    "ort_adam_params": (None, _native.ort_adam_params),
    "ort_pupil": (None, _native.ort_pupil),
    "ort_spot_layout": (None, _native.ort_spot_layout),
    "ort_wavefront_ref": (None, _native.ort_wavefront_ref),
}


def _c_layout(tmp_path):
    src = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(){"]
    for name, (dt, cs) in STRUCTS.items():
        fields = dt.names if dt is not None else [f[0] for f in cs._fields_]
        src.append(f'printf("{name} sizeof %zu\\n", sizeof({name}));')
        for f in fields:
            src.append(f'printf("{name} {f} %zu\\n", offsetof({name}, {f}));')
    src.append("return 0;}")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(c)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    lay = {}
    for line in out.splitlines():
        s, f, v = line.split()
        lay[(s, f)] = int(v)
    return lay


def test_struct_layouts_match_header(tmp_path):
    lay = _c_layout(tmp_path)
    for name, (dt, cs) in STRUCTS.items():
        if dt is not None:
            assert dt.itemsize == lay[(name, "sizeof")], name
            for f in dt.names:
                assert dt.fields[f][1] == lay[(name, f)], (name, f)
        else:
            assert ctypes.sizeof(cs) == lay[(name, "sizeof")], name
            for f, _ in cs._fields_:
                assert getattr(cs, f).offset == lay[(name, f)], (name, f)


def test_enums_match_header():
    text = open(HEADER).read()
    for cname, pyval in [("ORT_GEOM_PLANE", _abi.GEOM_PLANE), ("ORT_GEOM_STANDARD", _abi.GEOM_STANDARD),
                         ("ORT_GEOM_EVEN_ASPHERE", _abi.GEOM_EVEN_ASPHERE),
                         ("ORT_GEOM_ODD_ASPHERE", _abi.GEOM_ODD_ASPHERE),
                         ("ORT_GEOM_ZERNIKE", _abi.GEOM_ZERNIKE),
                         ("ORT_CS_TRANSLATE", _abi.CS_TRANSLATE), ("ORT_CS_ROT_X", _abi.CS_ROT_X),
                         ("ORT_CS_ROT_Y", _abi.CS_ROT_Y), ("ORT_CS_ROT_Z", _abi.CS_ROT_Z),
                         ("ORT_GEN_INFINITE", _abi.GEN_INFINITE), ("ORT_GEN_FINITE", _abi.GEN_FINITE),
                         ("ORT_GEN_TELECENTRIC", _abi.GEN_TELECENTRIC),
                         ("ORT_APOD_UNIFORM", _abi.APOD_UNIFORM),
                         ("ORT_APOD_GAUSSIAN", _abi.APOD_GAUSSIAN),
                         ("ORT_APOD_COSINE_SQUARED", _abi.APOD_COSINE_SQUARED),
                         ("ORT_APOD_HANN", _abi.APOD_HANN),
                         ("ORT_APOD_POLYNOMIAL", _abi.APOD_POLYNOMIAL),
                         ("ORT_APOD_SUPER_GAUSSIAN", _abi.APOD_SUPER_GAUSSIAN),
                         ("ORT_APOD_TUKEY", _abi.APOD_TUKEY),
                         ("ORT_NEWTON_SCHEDULE", _abi.NEWTON_SCHEDULE),
                         ("ORT_NEWTON_WAVE", _abi.NEWTON_WAVE),
                         ("ORT_VJP_UNROLLED", _abi.VJP_UNROLLED),
                         ("ORT_VJP_ADJOINT", _abi.VJP_ADJOINT),
                         ("ORT_PUPIL_UNIFORM", _abi.PUPIL_UNIFORM),
                         ("ORT_PUPIL_HEXAPOLAR", _abi.PUPIL_HEXAPOLAR),
                         ("ORT_PUPIL_RANDOM", _abi.PUPIL_RANDOM),
                         ("ORT_PUPIL_RING", _abi.PUPIL_RING),
                         ("ORT_PUPIL_LINE_X", _abi.PUPIL_LINE_X),
                         ("ORT_PUPIL_LINE_Y", _abi.PUPIL_LINE_Y),
                         ("ORT_PUPIL_CROSS", _abi.PUPIL_CROSS)]:
        m = re.search(rf"{cname}\s*=\s*(\d+)", text)
        assert m and int(m.group(1)) == pyval, cname
    for cname, pyval in [("ORT_SURF_REFLECTIVE", _abi.SURF_REFLECTIVE),
                         ("ORT_SURF_RADIUS_INF", _abi.SURF_RADIUS_INF),
                         ("ORT_SURF_APERTURE", _abi.SURF_APERTURE),
                         ("ORT_SURF_RECORD", _abi.SURF_RECORD),
                         ("ORT_STATUS_ZERNIKE_RANGE", _abi.STATUS_ZERNIKE_RANGE)]:
        m = re.search(rf"{cname}\s*=\s*1u\s*<<\s*(\d+)", text)
        assert m and (1 << int(m.group(1))) == pyval, cname
    assert re.search(r"#define ORT_ABI_VERSION (\d+)", text).group(1) == str(_abi.ABI_VERSION)
    assert re.search(r"#define ORT_MAX_SURFACES (\d+)", text).group(1) == str(_abi.MAX_SURFACES)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("HIP extension not built (run __graft_entry__.build())")
    lib = _native.load()
    declared = set(re.findall(r"^int(?:64_t)? (ort_\w+)\(", open(HEADER).read(), re.M))
    assert declared == set(_native.EXPORTS)
    for sym in declared:
        assert hasattr(lib, sym), sym
    assert lib.ort_abi_version() == _abi.ABI_VERSION


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_native.NativeLibraryError):
        _native.load(str(tmp_path / "nope.so"))


def test_host_library_exports_every_declared_symbol():
    """liboptiland_host.so (the CPU dispatch key) exports every entry point
    include/optiland_host.h declares, at the declared version."""
    if not os.path.exists(_native.HOST_LIB_PATH):
        pytest.skip("host library not built (run __graft_entry__.build())")
    lib = _native.load_host()
    text = open(os.path.join(REPO, "include", "optiland_host.h")).read()
    declared = set(re.findall(r"^(?:int|void)(?:64_t)? (ort_host_\w+)\(", text, re.M))
    assert declared == set(_native.HOST_EXPORTS)
    for sym in declared:
        assert hasattr(lib, sym), sym
    v = re.search(r"#define ORT_HOST_ABI_VERSION (\d+)", text).group(1)
    assert lib.ort_host_abi_version() == int(v) == _native.HOST_ABI_VERSION


def test_missing_host_library_fails_loudly(tmp_path):
    with pytest.raises(_native.NativeLibraryError):
        _native.load_host(str(tmp_path / "nope.so"))
