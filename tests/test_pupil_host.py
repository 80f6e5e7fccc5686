"""Device pupil sampling (csrc/ort_pupil.h) compiled for the host with g++ and checked
against the reference's own samples (tests/golden/distributions.npz) and against
correctly rounded sin / cos (mpmath, 200 bits). CPU only; the GPU build runs the same
source (tests/test_gpu_pupil.py)."""

import os
import shutil
import subprocess

import numpy as np
import pytest

from optiland_pr_amd import pupil
from tests.conftest import REPO, load_golden

SRC = os.path.join(REPO, "tests", "native", "pupil_main.cpp")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    out = tmp_path_factory.mktemp("pupil") / "pupil_main"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(out), SRC],
                   check=True)
    return str(out)


def _run(exe, kind, n, seed=None):
    spec, t = pupil.host_spec(kind, n, seed)
    rs = t.get("row_start", np.zeros(0, np.int64))
    rc = t.get("row_col", np.zeros((0, 2), np.int64))
    ch = t.get("rng_chunk", np.zeros((0, 4), np.uint64))
    ln = t.get("rng_lane", np.zeros((0, 4), np.uint64))
    head = np.array([spec["kind"], spec["positive_only"], spec["n"], spec["n_points"],
                     spec["n_rows"], len(ch)], dtype=np.int64)
    blob = b"".join(a.astype(np.int64 if a.dtype != np.uint64 else np.uint64).tobytes()
                    for a in (head, rs, rc, ch, ln))
    out = subprocess.run([exe, "pupil"], input=blob, capture_output=True, check=True).stdout
    xy = np.frombuffer(out, dtype=np.float64).reshape(-1, 2)
    assert len(xy) == spec["n_points"]
    return xy[:, 0], xy[:, 1]


GRID = [("uniform", 33), ("uniform", 128), ("line_x", 21), ("line_y", 20),
        ("positive_line_x", 9), ("positive_line_y", 10), ("cross", 21), ("cross", 20)]
TRIG = [("hexapolar", 6), ("hexapolar", 17), ("ring", 13)]


@pytest.mark.parametrize("kind,n", GRID)
def test_grid_kinds_bit_exact(exe, kind, n):
    g = load_golden("distributions")
    x, y = _run(exe, kind, n)
    assert np.array_equal(x, g[f"{kind}_{n}_x"]) and np.array_equal(y, g[f"{kind}_{n}_y"])


@pytest.mark.parametrize("kind,n", TRIG)
def test_trig_kinds_within_one_ulp(exe, kind, n):
    g = load_golden("distributions")
    x, y = _run(exe, kind, n)
    for got, ref in ((x, g[f"{kind}_{n}_x"]), (y, g[f"{kind}_{n}_y"])):
        assert np.all(np.abs(got - ref) <= 2 * np.spacing(np.abs(ref)))
        assert np.mean(got == ref) > 0.97


def test_random_matches_numpy_generator(exe):
    """seed 7, 1000 points: the PCG64 draws are numpy's bit for bit (radii and angles
    recomputed from numpy's own uniform draws), cos / sin within one ulp."""
    g = load_golden("distributions")
    x, y = _run(exe, "random", 1000, seed=7)
    rng = np.random.default_rng(7)
    r = rng.uniform(size=1000)
    t = rng.uniform(0, 2 * np.pi, size=1000)
    ref_x, ref_y = g["random_1000_x"], g["random_1000_y"]
    assert np.array_equal(ref_x, np.sqrt(r) * np.cos(t))  # the golden is this formula
    # one ulp of cos / sin, scaled by sqrt(r) and rounded again: <= 2 ulp of the product
    assert np.all(np.abs(x - ref_x) <= 2 * np.spacing(np.abs(ref_x)))
    assert np.all(np.abs(y - ref_y) <= 2 * np.spacing(np.abs(ref_y)))
    assert np.mean((x == ref_x) & (y == ref_y)) > 0.97


def test_random_chunk_boundaries(exe):
    """n not a multiple of the 256-draw chunk, angles starting mid-chunk."""
    x, y = _run(exe, "random", 777, seed=123)
    rng = np.random.default_rng(123)
    r = rng.uniform(size=777)
    t = rng.uniform(0, 2 * np.pi, size=777)
    rx, ry = np.sqrt(r) * np.cos(t), np.sqrt(r) * np.sin(t)
    assert np.all(np.abs(x - rx) <= 2 * np.spacing(np.abs(rx)))
    assert np.all(np.abs(y - ry) <= 2 * np.spacing(np.abs(ry)))


def test_sincos_correctly_rounded(exe):
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.prec = 200
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.uniform(0, 2 * np.pi, 20000), np.arange(257) * np.pi / 128,
                         [0.0, 2 * np.pi, 1e-300, 5e-324, np.pi / 2, np.pi, 1.5 * np.pi]])
    out = subprocess.run([exe, "sincos"], input=xs.tobytes(), capture_output=True,
                         check=True).stdout
    sc = np.frombuffer(out, dtype=np.float64).reshape(-1, 2)
    for x, (s, c) in zip(xs, sc, strict=True):
        X = mpmath.mpf(float(x))
        assert s == float(mpmath.sin(X)) and c == float(mpmath.cos(X)), x.hex()


def test_pcg64_tables_reproduce_numpy_draws():
    """pure-Python replay of the device's jump arithmetic vs numpy's uniform draws."""
    state, inc = pupil.pcg64_state(42)
    n = 600
    chunk, lane = pupil.pcg64_tables(state, inc, n)
    ref = np.random.default_rng(42).uniform(size=2 * n)
    M = (1 << 128) - 1

    def u(s):
        hi, lo = s >> 64, s & 0xFFFFFFFFFFFFFFFF
        xv, rot = hi ^ lo, hi >> 58
        v = ((xv >> rot) | (xv << ((64 - rot) & 63))) & 0xFFFFFFFFFFFFFFFF
        return (v >> 11) * (1.0 / 9007199254740992.0)

    for k in list(range(0, n, 37)) + [n - 1]:
        c, l = k >> 8, k & 255
        A = int(lane[l, 0]) | (int(lane[l, 1]) << 64)
        C = int(lane[l, 2]) | (int(lane[l, 3]) << 64)
        s_r = int(chunk[c, 0]) | (int(chunk[c, 1]) << 64)
        s_t = int(chunk[c, 2]) | (int(chunk[c, 3]) << 64)
        assert u((A * s_r + C) & M) == ref[k]
        assert u((A * s_t + C) & M) == ref[n + k]


def test_point_counts():
    for kind, n in GRID + TRIG:
        g = load_golden("distributions")
        assert pupil.n_points(kind, n) == g[f"{kind}_{n}_x"].size
