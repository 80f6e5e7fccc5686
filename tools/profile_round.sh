#!/bin/bash
# Full profile pass for the current kernel: kernel-trace stats + PMC (HBM bytes, FP64
# FLOPs, VALU, stalls). Output under gpurun_out/; then on the build host:
#   python tools/profile_hbm.py <tag> gpurun_out/prof gpurun_out/pmc_*
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
B="python3 bench.py --no-cpu --steps 200 --warmup 5"
run() { local n=$1; shift; echo "== $n"; timeout -k 10 300 "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
mkdir -p gpurun_out
run rocprof rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- $B
run pmc_fetch rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- $B
run pmc_write rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- $B
run pmc_valu rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_valu -o run -- $B
run pmc_stall rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_stall -o run -- $B
run bench python3 bench.py
