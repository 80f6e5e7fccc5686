#!/bin/bash
# Round 6: where config 5's taped forward / adjoint and config 3's Newton kernel wait --
# the scalar data / instruction caches (SQC), scalar memory and SALU cycles, and the stall
# breakdown -- one rocprofv3 pass per counter group, each under its own hard time limit.
# Afterwards, on the build host: python tools/pmc_kernel.py KERNEL gpurun_out/pmc6_*
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
run() { local n=$1; shift; echo "== $n"; timeout -s KILL 150 "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
P="--kernel-trace --output-format csv"
for c in 5 3; do
  if [ $c = 5 ]; then B="python3 bench.py --no-cpu --config 5 --eager --steps 3 --warmup 1 --ramp-steps 0"; else B="python3 bench.py --no-cpu --config 3 --steps 2 --warmup 1 --ramp-steps 0"; fi
  run pmc6_c${c}_sqc rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES GRBM_GUI_ACTIVE $P -d gpurun_out/pmc6_c${c}_sqc -o run -- $B
  run pmc6_c${c}_smem rocprofv3 --pmc SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES $P -d gpurun_out/pmc6_c${c}_smem -o run -- $B
  run pmc6_c${c}_stall rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES $P -d gpurun_out/pmc6_c${c}_stall -o run -- $B
  run pmc6_c${c}_valu rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE $P -d gpurun_out/pmc6_c${c}_valu -o run -- $B
done
echo END_OK
