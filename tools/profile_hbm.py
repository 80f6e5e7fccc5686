"""Summarise rocprofv3 runs of bench.py into profiles/ (test/measurement tooling).

usage: python tools/profile_hbm.py <round tag> <kernel-trace dir> [<pmc dir> ...]

Writes profiles/<tag>_kernel_stats.csv (copy of the kernel stats) and, when PMC runs
with FETCH_SIZE / WRITE_SIZE are given, profiles/hbm_traffic.json with the HBM bytes per
launch of the trace kernel. gfx950 correction (MI355X_MICROARCH.md 'HBM'): FETCH_SIZE
reports half of the bytes of WIDE (16 B/lane) coalesced reads; the trace kernel reads
8 B/lane (uncalibrated width), so both the raw and the x2 figures are recorded, and the
calibration kernel (generate_kernel: 16 B/ray read, 64 B/ray written, same widths) is
reported beside it.
"""
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    tag, ktrace = sys.argv[1], sys.argv[2]
    pmc_dirs = sys.argv[3:]
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(ktrace, "**", "*kernel_stats.csv"), recursive=True)
    for f in stats:
        shutil.copy(f, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    res = {}
    for d in pmc_dirs:
        for r in _rows(os.path.join(d, "**", "*counter_collection.csv")):
            k = r.get("Kernel_Name", "")
            if "trace_kernel" not in k and "generate_kernel" not in k:
                continue
            name = "trace_kernel" if "trace_kernel" in k else "generate_kernel"
            ctr = r.get("Counter_Name")
            val = float(r.get("Counter_Value", "nan"))
            res.setdefault(name, {}).setdefault(ctr, []).append(val)
    summary = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in res.items()}
    if summary:
        t = summary.get("trace_kernel", {})
        fetch = t.get("FETCH_SIZE")
        write = t.get("WRITE_SIZE")
        out = {"per_dispatch_kilobytes": summary}
        if fetch is not None and write is not None:
            out["bytes_per_launch_raw"] = (fetch + write) * 1024
            out["bytes_per_launch"] = (2 * fetch + write) * 1024
            out["note"] = "FETCH_SIZE x2 gfx950 correction applied to bytes_per_launch"
        with open(os.path.join(prof, "hbm_traffic.json"), "w") as fh:
            json.dump(out, fh, indent=1)
        with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as fh:
            json.dump(out, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
