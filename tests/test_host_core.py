"""The trace core's per-ray arithmetic (csrc/ort_core.h, the functions the HIP kernels
call) compiled for the HOST with g++ -ffp-contract=off behind tests/native/trace_main.cpp,
traced over the golden lens cases and checked against the reference's outputs
(tests/golden/*.npz) -- so a mistake in the shared math shows up in the CPU suite, not
only on the metered GPU -- and once more under AddressSanitizer + UBSan (SURVEY.md 4,
build test item 2).

Tolerances are the GPU parity tests': closed-form lenses bit-exact in x, y, z, L, M, N,
opd (intensity rtol 1e-12: the absorption exponent is accumulated and exponentiated
once); Newton lenses 1e-9 mm / 1e-11 with the reference's update counts.
"""

import os
import shutil
import subprocess

import numpy as np
import pytest

from tests._cases import native_case
from tests.conftest import REPO, load_golden

SRC = os.path.join(REPO, "tests", "native", "trace_main.cpp")
FIELDS = ("x", "y", "z", "L", "M", "N", "i", "opd")

CLOSED = ("cooke", "dg", "rt", "cooke_aperture", "cooke_shapes", "decentered", "json_heliar",
          "cooke_pih", "finite_pih", "uv_projection", "apod_gaussian", "apod_tukey",
          "cooke_abbe")
NEWTON = ("rt_asph", "rt_odd", "tma_fringe", "tma_standard", "tma_noll", "freeform",
          "forbes", "forbes_q2d", "nurbs_lens")


def _build(tmp_path_factory, name, flags):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    out = tmp_path_factory.mktemp(name) / "trace_main"
    subprocess.run(["g++", "-std=c++17", "-ffp-contract=off", *flags, "-o", str(out), SRC],
                   check=True)
    return str(out)


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    return _build(tmp_path_factory, "host", ["-O2"])


@pytest.fixture(scope="module")
def exe_san(tmp_path_factory):
    return _build(tmp_path_factory, "san", ["-O1", "-g", "-fno-omit-frame-pointer",
                                            "-fsanitize=address,undefined",
                                            "-fno-sanitize-recover=undefined"])


def host_trace(exe, table, segs, px, py, record=False, start=0):
    """-> (rays dict, updates [n_seg][S], status, records [S][8][n] or None)."""
    S = table.n_surfaces
    n_p = len(px)
    n = len(segs) * n_p
    apod = table.apod
    head = np.array([S, len(table.cs_ops), len(table.coef), len(table.zern),
                     table.n_tab.shape[0], table.n_tab.shape[1], table.final_mat, len(segs),
                     n_p, 0, start, int(record), int(apod is not None), 0, 0, 0],
                    dtype=np.int64)
    parts = [head.tobytes(), np.float64(table.final_thickness).tobytes(),
             table.surfaces.tobytes(), table.cs_ops.tobytes(),
             np.ascontiguousarray(table.coef, dtype=np.float64).tobytes(),
             table.zern.tobytes(),
             np.ascontiguousarray(table.n_tab, dtype=np.float64).tobytes(),
             np.ascontiguousarray(table.alpha_tab, dtype=np.float64).tobytes(),
             np.ascontiguousarray(table.optics).tobytes(),
             np.ascontiguousarray(segs).tobytes()]
    if apod is not None:
        parts.append(np.ascontiguousarray(apod).tobytes())
    parts += [np.ascontiguousarray(px, dtype=np.float64).tobytes(),
              np.ascontiguousarray(py, dtype=np.float64).tobytes()]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([exe], input=b"".join(parts), capture_output=True, env=env)
    assert p.returncode == 0, p.stderr.decode()[-3000:]
    buf = p.stdout
    rays = np.frombuffer(buf, dtype=np.float64, count=8 * n).reshape(8, n)
    off = 8 * n * 8
    ups = np.frombuffer(buf, dtype=np.int32, count=len(segs) * S, offset=off).reshape(len(segs), S)
    off += len(segs) * S * 4
    status = int(np.frombuffer(buf, dtype=np.int32, count=1, offset=off)[0])
    off += 4
    rec = None
    if record:
        rec = np.frombuffer(buf, dtype=np.float64, count=S * 8 * n, offset=off).reshape(S, 8, n)
    return dict(zip(FIELDS, rays, strict=True)), ups, status, rec


def _check(name, got, g, exact):
    for a in FIELDS:
        if a == "i":
            np.testing.assert_allclose(got[a], g[a], rtol=1e-12, err_msg=f"{name} i")
        elif exact:
            np.testing.assert_array_equal(got[a], g[a], err_msg=f"{name} {a}")
        else:
            tol = 1e-11 if a in ("L", "M", "N") else 1e-9
            np.testing.assert_allclose(got[a], g[a], rtol=0, atol=tol, err_msg=f"{name} {a}")


@pytest.mark.parametrize("name", CLOSED + NEWTON)
def test_host_core_matches_reference(exe, golden_index, name):
    meta = golden_index[name]
    g = load_golden(name)
    _, table, segs = native_case(name, meta)
    got, ups, status, _ = host_trace(exe, table, segs, g["Px"], g["Py"])
    assert status == 0
    _check(name, got, g, name in CLOSED)
    ref = g["newton_updates"]  # [pair][surface incl. object], -1 = not a Newton surface
    for p in range(len(segs)):
        for si in range(table.n_surfaces):
            if ups[p, si] >= 0:
                assert ref[p][si + 1] == ups[p, si], (name, p, si)


def test_host_core_records_bit_exact(exe, golden_index):
    """DoubleGauss per-surface records (standard_surface.py:266-286)."""
    meta = golden_index["dg"]
    g = load_golden("dg")
    _, table, segs = native_case("dg", meta, record=True)
    _, _, _, rec = host_trace(exe, table, segs, g["Px"], g["Py"], record=True)
    n_p = len(g["Px"])
    ref = g["records"]  # [pair][surface][8][n_p]
    for p in range(len(segs)):
        for si in range(table.n_surfaces):
            for f in range(8):
                got = rec[si, f, p * n_p:(p + 1) * n_p]
                if f == 6:
                    np.testing.assert_allclose(got, ref[p, si + 1, f], rtol=1e-12)
                else:
                    np.testing.assert_array_equal(got, ref[p, si + 1, f])


def test_host_core_matches_oracle_extreme_operands(exe):
    """Rays from outside the lens, grazing and on-vertex pupil points: the core and the
    oracle agree bit for bit, NaN masks included (misses, TIR)."""
    from oracle import trace_np
    from optiland_pr_amd.lowering import lower_surface_group, segment_params
    from optiland_pr_amd.samples import CookeTriplet

    lens = CookeTriplet()
    table = lower_surface_group(lens.surface_group, [0.55])
    seg = np.stack([segment_params(lens, 0.0, 1.0, 0)])
    px = np.array([0.0, 1.0, -1.0, 3.0, 1e-300, -0.0, 0.999999999, 25.0])
    py = np.array([0.0, 0.0, 1.0, 3.0, 5e-324, 1.0, 0.0, -25.0])
    got, _, _, _ = host_trace(exe, table, seg, px, py)
    ref = trace_np.trace_segment(table, trace_np.generate_rays(seg[0], px, py), 0).rays
    for a in FIELDS:
        r = getattr(ref, a)
        assert np.array_equal(np.isnan(got[a]), np.isnan(r)), a
        m = ~np.isnan(r)
        if a == "i":
            np.testing.assert_allclose(got[a][m], r[m], rtol=1e-12)
        else:
            np.testing.assert_array_equal(got[a][m], r[m], err_msg=a)


@pytest.mark.parametrize("name", ["cooke_aperture", "rt_asph", "tma_fringe", "apod_tukey"])
def test_host_core_sanitized(exe_san, golden_index, name):
    """The same driver under AddressSanitizer + UndefinedBehaviorSanitizer: no invalid
    access or UB in the shared per-ray code, and the same answers."""
    meta = golden_index[name]
    g = load_golden(name)
    _, table, segs = native_case(name, meta, record=True)
    got, _, status, _ = host_trace(exe_san, table, segs, g["Px"], g["Py"], record=True)
    assert status == 0
    _check(name, got, g, name in CLOSED or name.startswith("apod"))
