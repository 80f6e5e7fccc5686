"""Per-kernel PMC summary from rocprofv3 --pmc CSV directories, one line of averages over
the dispatches of a kernel whose duration is at least --min-us (so e.g. the taped
forward's full trace is separated from its early-exit verify rounds, which share the
kernel symbol). Measurement tooling, not product.

usage: python tools/pmc_kernel.py KERNEL_SUBSTR DIR [DIR ...] [--min-us 50] [--out F.json]
           [--source TEXT] [--rays N]
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def collect(key, dirs, min_us):
    per = defaultdict(list)
    regs, name, durs = {}, None, []
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            disp = defaultdict(dict)
            for r in csv.DictReader(open(f)):
                if key not in r["Kernel_Name"]:
                    continue
                name = r["Kernel_Name"]
                e = disp[r["Dispatch_Id"]]
                e[r["Counter_Name"]] = float(r["Counter_Value"])
                e["_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                for k in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size",
                          "LDS_Block_Size", "Workgroup_Size", "Grid_Size"):
                    regs[k] = r.get(k)
            for e in disp.values():
                if e["_us"] < min_us:
                    continue
                durs.append(e["_us"])
                for c, v in e.items():
                    if not c.startswith("_"):
                        per[c].append(v)
    return name, regs, {c: sum(v) / len(v) for c, v in sorted(per.items())}, durs


def derive(c, rays=None):
    der = {}
    w = c.get("SQ_WAVES")
    if w:
        for k, n in (("SQ_INSTS_VALU", "valu_insts_per_wave"), ("SQ_INSTS_SALU", "salu_insts_per_wave"),
                     ("SQ_INSTS_SMEM", "smem_insts_per_wave"), ("SQ_INSTS_BRANCH", "branch_insts_per_wave"),
                     ("SQ_INSTS_VMEM", "vmem_insts_per_wave"), ("SQ_INSTS_LDS", "lds_insts_per_wave")):
            if k in c:
                der[n] = c[k] / w
        f64 = [c.get(f"SQ_INSTS_VALU_{k}_F64") for k in ("ADD", "MUL", "FMA", "TRANS")]
        if all(v is not None for v in f64):
            der["fp64_valu_insts_per_wave"] = sum(f64) / w
    cyc = c.get("SQ_WAVE_CYCLES")
    if cyc:
        for k, n in (("SQ_WAIT_INST_ANY", "wait_inst_any_frac"), ("SQ_WAIT_ANY", "wait_any_frac"),
                     ("SQ_ACTIVE_INST_ANY", "active_inst_any_frac"),
                     ("SQ_ACTIVE_INST_VALU", "active_valu_frac"),
                     ("SQ_ACTIVE_INST_SCA", "active_sca_frac")):
            if k in c:
                der[n] = c[k] / cyc
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # gfx950: FETCH_SIZE reports half of wide coalesced reads (tools/profile_hbm.py)
        der["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    if "SQ_INSTS_VALU_FLOPS_FP64" in c:
        der["fp64_flops_per_launch"] = c["SQ_INSTS_VALU_FLOPS_FP64"] * 64
        if rays:
            der["hw_fp64_flops_per_ray"] = der["fp64_flops_per_launch"] / rays
    return der


def main():
    argv = list(sys.argv[1:])
    opts = {"--min-us": "50", "--out": None, "--source": "", "--rays": None}
    for k in list(opts):
        if k in argv:
            i = argv.index(k)
            opts[k] = argv[i + 1]
            del argv[i:i + 2]
    key, dirs = argv[0], argv[1:]
    name, regs, c, durs = collect(key, dirs, float(opts["--min-us"]))
    der = derive(c, float(opts["--rays"]) if opts["--rays"] else None)
    out = {"source": opts["--source"], "kernel": name, "registers": regs,
           "dispatches": len(durs), "mean_us_under_counters": sum(durs) / max(1, len(durs)),
           "counters": c, "derived": der}
    if opts["--out"]:
        with open(opts["--out"], "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("kernel", "registers", "dispatches",
                                          "mean_us_under_counters")}, indent=None))
    print(json.dumps({k: round(v, 4) if v < 10 else round(v) for k, v in der.items()}, indent=1))


if __name__ == "__main__":
    main()
