#!/bin/bash
# A/B kernel variants: timing (2 reps, interleaved) + one PMC pass (VALU / SALU counts) each.
# usage (GPU box): bash tools/ab_pmc.sh A.so B.so ...   (files in optiland_pr_amd/lib/variants)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for rep in 1 2; do
  for v in "$@"; do
    ms=$(ORT_LIB_PATH=optiland_pr_amd/lib/variants/$v timeout -k 10 300 python bench.py --no-cpu --steps 100 --warmup 10 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms']*1e3,2), 'us', '%.3e'%d['value'])")
    rc=$?
    echo "$v rep$rep $ms" | tee -a gpurun_out/ab.log
    [ $rc -ne 0 ] && exit $rc
  done
done
for v in "$@"; do
  ORT_LIB_PATH=optiland_pr_amd/lib/variants/$v timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/pmc_$v -o run -- python3 bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/pmc_$v.log 2>&1 || exit $?
done
exit 0
