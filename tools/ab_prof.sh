#!/bin/bash
# Kernel-level A/B: rocprofv3 kernel stats of one bench config per library variant.
# usage: AB_ARGS="--config 5 --steps 10 --warmup 2" bash tools/ab_prof.sh KERNEL_SUBSTR libA.so libB.so ...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
k=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "$@"; do
  d=gpurun_out/abp_${v%.so}
  ORT_LIB_PATH=optiland_pr_amd/lib/variants/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --no-cpu ${AB_ARGS:---steps 100 --warmup 10} > $d.log 2>&1 || exit $?
  python3 - "$d" "$k" "$v" <<'PY' | tee -a gpurun_out/ab.log
import csv, glob, sys
d, k, v = sys.argv[1:4]
for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Name"]:
            print(v, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
