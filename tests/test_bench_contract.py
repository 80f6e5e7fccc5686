"""bench.py's JSON contract on the host (no GPU): the roofline objects every config's line
carries, from the committed PMC summaries under profiles/."""

import bench

ROOFLINE_KEYS = {"bound", "achieved", "peak", "unit", "frac", "traffic"}


def _w(**kw):
    base = dict(kernel="k", bytes_per_launch=None, flops_per_ray=None, pmc_file=None,
                rays=1_000_000)
    base.update(kw)
    return bench.Workload(**base)


def test_hbm_roofline_from_committed_pmc():
    w = _w(bytes_per_launch=80_000_000, pmc_file="hbm_traffic.json")
    r = bench._roofline(w, 0.068)
    assert ROOFLINE_KEYS <= set(r)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["achieved"] - 80e6 / 0.068e-3 / 1e9) < 1e-9
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-12
    # rocprofv3 bytes equal the algorithmic bytes to 0.3% (profiles/hbm_traffic.json)
    assert abs(r["traffic"] / 80e6 - 1) < 3e-3


def test_config4_traffic_scaled_to_the_rank_share():
    w = _w(bytes_per_launch=3_920_000_000, pmc_file="hbm_traffic_c4.json", traffic_scale=0.5)
    r = bench._roofline(w, 4.0)
    assert abs(r["traffic"] / 3.92e9 - 1) < 3e-3


def test_config5_adjoint_roofline():
    R, S = 1_000_000, 4
    w = _w(pmc_file="hbm_traffic_c5.json", vjp_ms=1.1, tape_bytes_per_launch=S * 11 * 8 * R,
           algorithmic_bytes_per_launch=S * 11 * 8 * R + 64 * R + 31 * 8 * (R // 64))
    r = bench._roofline(w, 1.95)
    assert ROOFLINE_KEYS <= set(r)
    assert r["bound"] == "fp64_valu" and r["kernel_ms"] == 1.1 and r["step_device_ms"] == 1.95
    assert r["achieved"] > 0 and 0 < r["frac"] < 1
    # the taped forward writes the tape, the adjoint reads it once (S x 11 doubles per ray)
    assert r["tape_bytes_per_launch"] == 352_000_000
    assert r["algorithmic_bytes_per_launch"] > r["tape_bytes_per_launch"]


def test_launch_bound_spot_config_has_null_rates():
    r = bench._roofline(_w(spot=True), 0.023)
    assert ROOFLINE_KEYS <= set(r) and r["achieved"] is None and r["bound"] == "launch"


def test_config5_tape_bytes_follow_the_schedule():
    """The adjoint reads 7 tape rows per traced surface plus min(U, 4) Newton iterates per
    Newton surface (the rows the taped forward writes): the TMA with one update per mirror
    reads 31 rows x 8 B per ray."""
    from types import SimpleNamespace

    import numpy as np

    from optiland_pr_amd.lowering import lower_surface_group
    from optiland_pr_amd.samples import ThreeMirrorAnastigmat

    lens = ThreeMirrorAnastigmat()
    table = lower_surface_group(lens.surface_group, [0.587])
    S = table.n_surfaces
    U = np.array([1 if g == 4 else 0 for g in table.surfaces["geometry"]])
    lens._lowered = {"k": SimpleNamespace(table=table, sched_cache={"_default": U})}
    assert bench._tape_read_bytes(lens, 1_000_000) == (7 * S + int((U > 0).sum())) * 8 * 1_000_000
    assert bench._tape_read_bytes(lens, 1_000_000) == 31 * 8 * 1_000_000
