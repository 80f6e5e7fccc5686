#!/bin/bash
# Compute-side counters of the config 3 Newton trace kernel (trace_kernel<81>: VALU
# instructions, FP64 FLOPs by kind, issue / stall cycles), one rocprofv3 pass per group
# (gfx950 limits: <= 8 SQ counters per pass); then on the build host:
#   python tools/pmc_summary.py gpurun_out/pmc_c3_* > profiles/r03_config3_pmc_compute.json
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
run() { local n=$1; shift; echo "== $n"; timeout -k 10 300 "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python3 bench.py --no-cpu --config 3 --steps 3 --warmup 1"
run pmc_c3_valu rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_c3_valu -o run -- $B
run pmc_c3_stall rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_c3_stall -o run -- $B
run pmc_c3_issue rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/pmc_c3_issue -o run -- $B
