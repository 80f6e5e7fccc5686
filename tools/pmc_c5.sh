#!/bin/bash
# Config 5 (TMA optimisation step): PMC passes for the adjoint kernel (HBM bytes, FP64
# FLOPs, VALU instructions), then the config 5 bench line; afterwards on the build host:
#   python tools/profile_hbm.py r02_config5 - gpurun_out/pmc_c5_* --kernel adj_kernel \
#       --traffic hbm_traffic_c5.json
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
run() { local n=$1; shift; echo "== $n"; timeout -k 10 300 "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
B="python3 bench.py --no-cpu --config 5 --eager --steps 3 --warmup 1"
run pmc_c5_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_c5_fetch -o run -- $B
run pmc_c5_write rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_c5_write -o run -- $B
run pmc_c5_valu rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_c5_valu -o run -- $B
# stall breakdown (optional: bash tools/pmc_c5.sh stall)
if [ "${1:-}" = stall ]; then
  run pmc_c5_stall rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_c5_stall -o run -- $B
fi
