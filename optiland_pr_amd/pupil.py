"""Pupil distributions sampled on the device (ort_generate_pupil).

RealRayTracer.trace with a distribution NAME (the reference's create_distribution
strings, distribution.py:378-408) no longer builds the points with NumPy on the host and
copies them to the GPU: the host prepares a few KB of tables (the uniform grid's row
table, PCG64 jump tables for "random") and one launch writes px, py into HBM. Grid kinds
(uniform, line_x/y, positive_line_x/y, cross) are bit-identical to NumPy; ring,
hexapolar and random use correctly rounded cos / sin (NumPy's glibc cos / sin is
within 0.55 ulp and differs from the correctly rounded value for ~0.3% of angles).

"random" keeps the reference's semantics (a fresh numpy.random.default_rng(None) per
call, distribution.py:144-158): the seed is drawn from OS entropy, the PCG64 stream is
numpy's exactly (draws u_k = (next64 >> 11) 2^-53, radii from draws 0..n-1, angles from
draws n..2n-1), so a seed reproduces numpy's generator bit for bit in u.
"""

from __future__ import annotations

import ctypes as C
import secrets

import numpy as np

from . import _abi, _native

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

KINDS = {
    "uniform": (_abi.PUPIL_UNIFORM, 0),
    "hexapolar": (_abi.PUPIL_HEXAPOLAR, 0),
    "random": (_abi.PUPIL_RANDOM, 0),
    "ring": (_abi.PUPIL_RING, 0),
    "line_x": (_abi.PUPIL_LINE_X, 0),
    "line_y": (_abi.PUPIL_LINE_Y, 0),
    "positive_line_x": (_abi.PUPIL_LINE_X, 1),
    "positive_line_y": (_abi.PUPIL_LINE_Y, 1),
    "cross": (_abi.PUPIL_CROSS, 0),
}

PCG_MULT = 0x2360ED051FC65DA44385DF649FCCF645
MASK128 = (1 << 128) - 1
CHUNK = 256


def n_points(kind, n):
    """Points the reference's distribution generates for argument n."""
    k, _ = KINDS[kind]
    if k == _abi.PUPIL_UNIFORM:
        return int(uniform_rows(n)[0][-1])
    if k == _abi.PUPIL_HEXAPOLAR:
        return 1 + 3 * n * (n + 1)
    if k == _abi.PUPIL_CROSS:
        return 2 * n - 1 if n % 2 == 1 else 2 * n
    return n


_ROWS = {}


def uniform_rows(n):
    """distribution.py:161-186 grid mask -> (cumulative point counts [rows + 1],
    row_start [rows], row_col [rows][2] = (grid row, first column)); rows without
    points are skipped. The mask of each row is contiguous (checked)."""
    if n in _ROWS:
        return _ROWS[n]
    x = np.linspace(-1, 1, n)
    starts, cols = [], []
    total = 0
    for i in range(n):
        m = x ** 2 + x[i] ** 2 <= 1
        cnt = int(m.sum())
        if cnt == 0:
            continue
        j = np.flatnonzero(m)
        if j[-1] - j[0] + 1 != cnt:
            raise AssertionError("non-contiguous uniform grid row")
        starts.append(total)
        cols.append((i, int(j[0])))
        total += cnt
    out = (np.array(starts + [total], dtype=np.int64), np.array(starts, dtype=np.int64),
           np.array(cols, dtype=np.int64).reshape(-1, 2))
    _ROWS[n] = out
    return out


def _affine_pow(d, inc):
    """(A, C) with state_{k+d} = A state_k + C (mod 2^128) for the PCG64 LCG."""
    A, Cc = 1, 0
    a, c = PCG_MULT, inc
    while d:
        if d & 1:
            A, Cc = (A * a) & MASK128, (Cc * a + c) & MASK128
        a, c = (a * a) & MASK128, (c * a + c) & MASK128
        d >>= 1
    return A, Cc


def _split(v):
    return v & 0xFFFFFFFFFFFFFFFF, v >> 64


def pcg64_tables(state, inc, n):
    """chunk table [ceil(n/256)][4] (state before draw 256c, before draw n + 256c) and
    lane table [256][4] (the map advanced l + 1 steps) for ort_pupil.rng_*."""
    n_chunks = max(1, -(-n // CHUNK))
    A256, C256 = _affine_pow(CHUNK, inc)
    An, Cn = _affine_pow(n, inc)
    chunk = np.zeros((n_chunks, 4), dtype=np.uint64)
    s_r = state
    s_t = (An * state + Cn) & MASK128
    for c in range(n_chunks):
        chunk[c] = (*_split(s_r), *_split(s_t))
        s_r = (A256 * s_r + C256) & MASK128
        s_t = (A256 * s_t + C256) & MASK128
    lane = np.zeros((CHUNK, 4), dtype=np.uint64)
    A, Cc = PCG_MULT, inc
    for l in range(CHUNK):
        lane[l] = (*_split(A), *_split(Cc))
        A, Cc = (A * PCG_MULT) & MASK128, (Cc * PCG_MULT + inc) & MASK128
    return chunk, lane


def pcg64_state(seed):
    """numpy.random.default_rng(seed)'s PCG64 (state, increment)."""
    st = np.random.default_rng(seed).bit_generator.state["state"]
    return int(st["state"]), int(st["inc"])


def host_spec(kind, n, seed=None):
    """-> (fields of ort_pupil without device pointers, host tables dict)."""
    if kind not in KINDS:
        raise ValueError("Invalid distribution type.")
    k, pos = KINDS[kind]
    tables = {}
    n_rows = 0
    if k == _abi.PUPIL_UNIFORM:
        cum, starts, cols = uniform_rows(n)
        tables["row_start"], tables["row_col"] = starts, cols
        n_rows = len(starts)
    npts = n_points(kind, n)
    if k == _abi.PUPIL_RANDOM:
        if seed is None:
            seed = secrets.randbits(64)
        state, inc = pcg64_state(seed)
        tables["rng_chunk"], tables["rng_lane"] = pcg64_tables(state, inc, npts)
    return dict(kind=k, positive_only=pos, n=int(n), n_points=int(npts), n_rows=n_rows), tables


_DEV = {}


def device_pupil(kind, n, device, seed=None, stream=None):
    """px, py (float64 device tensors) of distribution `kind` with argument n, generated
    by ort_generate_pupil. Deterministic kinds are cached per (kind, n, device)."""
    from .raytrace import _stream_handle

    key = (kind, int(n), str(device))
    if kind != "random" and key in _DEV:
        return _DEV[key]
    spec, tables = host_spec(kind, n, seed)
    dev_t = {name: torch.from_numpy(arr.view(np.int64).copy()).to(device)
             for name, arr in tables.items()}
    p = _native.ort_pupil(spec["kind"], spec["positive_only"], spec["n"], spec["n_points"],
                          spec["n_rows"], 0,
                          *(dev_t[f].data_ptr() if f in dev_t else None
                            for f in ("row_start", "row_col", "rng_chunk", "rng_lane")))
    npts = spec["n_points"]
    px = torch.empty(npts, dtype=torch.float64, device=device)
    py = torch.empty(npts, dtype=torch.float64, device=device)
    lib = _native.load()
    rc = lib.ort_generate_pupil(C.byref(p), C.c_void_p(px.data_ptr() if npts else None),
                                C.c_void_p(py.data_ptr() if npts else None),
                                _stream_handle() if stream is None else stream)
    _native.check(rc, "ort_generate_pupil")
    if kind != "random":
        _DEV[key] = (px, py)
    # the tables may be freed now: the caching allocator hands their blocks only to later
    # work on this stream, which runs after the launch
    return px, py


# distributions generated on the device by default: bit-identical to NumPy, or random
# by definition (a fresh generator per call); hexapolar and ring keep NumPy's cos / sin
# (host-generated once per (kind, n) and cached on the device) so the default trace stays
# bit-exact against the reference
DEVICE_KINDS = ("uniform", "line_x", "line_y", "positive_line_x", "positive_line_y", "cross",
                "random")
_HOST = {}


def pupil_arrays(distribution, num, device):
    """(px, py) device tensors for Optic.trace / SpotDiagram: a distribution name is
    sampled on the device (DEVICE_KINDS) or generated once on the host and cached; a
    distribution object's arrays are copied to the device once and reused while the
    object keeps the same arrays."""
    from .distribution import BaseDistribution, create_distribution

    if isinstance(distribution, str):
        if distribution in DEVICE_KINDS:
            return device_pupil(distribution, num, device)
        key = (distribution, int(num), str(device))
        if key not in _HOST:
            d = create_distribution(distribution)
            d.generate_points(num)
            _HOST[key] = tuple(torch.as_tensor(np.asarray(v, dtype=np.float64), device=device)
                               for v in (d.x, d.y))
        return _HOST[key]
    if not isinstance(distribution, BaseDistribution) and not hasattr(distribution, "x"):
        raise ValueError("Invalid distribution type.")
    x, y = distribution.x, distribution.y
    c = getattr(distribution, "_ort_device", None)
    if c is not None and c[0] is x and c[1] is y and c[2] == str(device):
        return c[3], c[4]
    px = torch.as_tensor(np.asarray(x, dtype=np.float64), device=device)
    py = torch.as_tensor(np.asarray(y, dtype=np.float64), device=device)
    try:
        distribution._ort_device = (x, y, str(device), px, py)
    except AttributeError:  # pragma: no cover - objects without a __dict__
        pass
    return px, py
