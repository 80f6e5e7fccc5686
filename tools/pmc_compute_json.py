"""Per-dispatch compute counters of one kernel from rocprofv3 --pmc CSV directories, as the
JSON bench.py reads for `roofline_fp64.hw_counted` (measurement tooling, not product).

usage: python tools/pmc_compute_json.py OUT.json KERNEL_SUBSTR "source text" DIR [DIR ...]
         [--rays N] [--algorithmic-flops F]
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    argv = list(sys.argv[1:])
    opts = {}
    for k in ("--rays", "--algorithmic-flops"):
        if k in argv:
            i = argv.index(k)
            opts[k] = float(argv[i + 1])
            del argv[i:i + 2]
    out, key, source, dirs = argv[0], argv[1], argv[2], argv[3:]
    acc = defaultdict(list)
    regs, name = {}, None
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if key not in r["Kernel_Name"]:
                    continue
                name = r["Kernel_Name"]
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
                for k in ("VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size",
                          "LDS_Block_Size", "Workgroup_Size", "Grid_Size"):
                    if k in r:
                        regs[k] = r[k]
    c = {k: sum(v) / len(v) for k, v in sorted(acc.items())}
    w = c.get("SQ_WAVES")
    der = {}
    if w:
        der["valu_insts_per_wave"] = c.get("SQ_INSTS_VALU", 0) / w
        f64 = [c.get(f"SQ_INSTS_VALU_{k}_F64") for k in ("ADD", "MUL", "FMA", "TRANS")]
        if all(v is not None for v in f64):
            der["fp64_valu_insts_per_wave"] = sum(f64) / w
        if "SQ_INSTS_SALU" in c:
            der["salu_insts_per_wave"] = c["SQ_INSTS_SALU"] / w
        if "SQ_INSTS_BRANCH" in c:
            der["branch_insts_per_wave"] = c["SQ_INSTS_BRANCH"] / w
    if "--rays" in opts and "SQ_INSTS_VALU_FLOPS_FP64" in c:
        der["rays_per_launch"] = opts["--rays"]
        der["hw_fp64_flops_per_ray"] = c["SQ_INSTS_VALU_FLOPS_FP64"] * 64 / opts["--rays"]
        if "--algorithmic-flops" in opts:
            der["algorithmic_flops_per_ray"] = opts["--algorithmic-flops"]
            der["hw_over_algorithmic"] = der["hw_fp64_flops_per_ray"] / opts["--algorithmic-flops"]
    cyc = c.get("SQ_WAVE_CYCLES")
    if cyc:
        for k, n in (("SQ_WAIT_INST_ANY", "wait_inst_any_frac"), ("SQ_WAIT_ANY", "wait_any_frac"),
                     ("SQ_ACTIVE_INST_VALU", "active_valu_frac"),
                     ("SQ_ACTIVE_INST_SCA", "active_sca_frac")):
            if k in c:
                der[n] = c[k] / cyc
    with open(out, "w") as f:
        json.dump({"source": source, "kernel": name, "registers": regs, "counters": c,
                   "derived": der}, f, indent=1)
    print(json.dumps(der, indent=1))


if __name__ == "__main__":
    main()
