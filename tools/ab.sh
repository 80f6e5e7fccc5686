#!/bin/bash
# A/B kernel timing: bash tools/ab.sh libX.so libY.so ... (files in optiland_pr_amd/lib/variants)
# AB_ARGS: bench.py arguments (default: config 2, 100 steps)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    ms=$(ORT_LIB_PATH=optiland_pr_amd/lib/variants/$v timeout -k 10 300 python bench.py --no-cpu ${AB_ARGS:---steps 100 --warmup 10} 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d.get('roofline',{}).get('kernel_ms',float('nan'))*1e3,2), 'us', 'step', round(d['ms_per_step'],4), 'ms', '%.3e'%d['value'])")
    rc=$?
    echo "$v rep$rep $ms" | tee -a gpurun_out/ab.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
