"""Summarise rocprofv3 runs of bench.py into profiles/ (measurement tooling, not product).

usage: python tools/profile_hbm.py <round tag> <kernel-trace dir | -> [<pmc dir> ...]
                                  [--traffic NAME]   (default hbm_traffic.json)
                                  [--kernel SUBSTR]  (default: the trace kernels)

Writes
  profiles/<tag>_kernel_stats.csv   copy of rocprofv3 --kernel-trace --stats summary
  profiles/<tag>_pmc_summary.json   per-dispatch averages of every PMC counter seen for
                                    the trace kernel
  profiles/hbm_traffic.json         what bench.py reads: HBM bytes and hardware FP64
                                    FLOPs per launch of the trace kernel

gfx950 corrections (MI355X_MICROARCH.md 'HBM'): FETCH_SIZE reports half of the bytes of
wide coalesced reads -- verified for this kernel's 8 B/lane pupil reads: raw FETCH_SIZE
is 7.9 MB for 16 MB of Px/Py, so bytes_per_launch uses 2 x FETCH_SIZE + WRITE_SIZE
(in KiB). SQ_INSTS_VALU_FLOPS_FP64 counts per wave-instruction: x 64 lanes.
"""
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_KEYS = ("trace_kernel", "trace_closed_kernel")


def main():
    argv = list(sys.argv)
    traffic = "hbm_traffic.json"
    if "--traffic" in argv:
        i = argv.index("--traffic")
        traffic = argv[i + 1]
        del argv[i:i + 2]
    keys = KERNEL_KEYS
    if "--kernel" in argv:
        i = argv.index("--kernel")
        keys = (argv[i + 1],)
        del argv[i:i + 2]
    sys.argv = argv
    tag, ktrace = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    if ktrace != "-":
        for f in glob.glob(os.path.join(ktrace, "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    acc = {}
    for d in sys.argv[3:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if not any(k in r.get("Kernel_Name", "") for k in keys):
                    continue
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    per = {c: sum(v) / len(v) for c, v in acc.items()}
    if not per:
        print(f"no PMC rows for {keys}")
        return
    out = {"per_dispatch": per}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        out["bytes_per_launch_raw"] = (per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024
        out["bytes_per_launch"] = (2 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024
    if "SQ_INSTS_VALU_FLOPS_FP64" in per:
        out["fp64_flops_per_launch"] = per["SQ_INSTS_VALU_FLOPS_FP64"] * 64
    if "SQ_INSTS_VALU" in per and "SQ_WAVES" in per:
        out["valu_insts_per_wave"] = per["SQ_INSTS_VALU"] / per["SQ_WAVES"]
    out["source"] = f"rocprofv3 PMC passes, round tag {tag}"
    with open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    with open(os.path.join(prof, traffic), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
