#!/bin/bash
# Config 5 (TMA optimisation step): PMC passes for its two big kernels -- the adjoint
# adj_kernel<4,2,false> and the taped forward trace_kernel<1108> -- one rocprofv3 pass per
# counter group (gfx950 limits: <= 8 SQ, <= 4 TCC counters per pass): HBM bytes, FP64 FLOPs
# by kind, VALU / SALU / LDS / branch instructions, issue and stall cycles. Afterwards, on
# the build host:
#   python tools/pmc_compute_json.py profiles/r05_config5_adj_pmc.json adj_kernel "..." gpurun_out/pmc_c5_*
#   python tools/pmc_compute_json.py profiles/r05_config5_fwd_pmc.json 'trace_kernelILj1108' "..." gpurun_out/pmc_c5_*
#   python tools/profile_hbm.py r05_config5 - gpurun_out/pmc_c5_* --kernel adj_kernel --traffic hbm_traffic_c5.json
set -u
cd "$(dirname "$0")/.."
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
run() { local n=$1; shift; echo "== $n"; timeout -k 10 300 "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -2 gpurun_out/$n.log; [ $rc -eq 0 ] || exit $rc; }
B="python3 bench.py --no-cpu --config 5 --eager --steps 3 --warmup 1 --ramp-steps 0"
P="--kernel-trace --output-format csv"
run pmc_c5_fetch rocprofv3 --pmc FETCH_SIZE $P -d gpurun_out/pmc_c5_fetch -o run -- $B
run pmc_c5_write rocprofv3 --pmc WRITE_SIZE $P -d gpurun_out/pmc_c5_write -o run -- $B
run pmc_c5_valu rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE $P -d gpurun_out/pmc_c5_valu -o run -- $B
run pmc_c5_stall rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES $P -d gpurun_out/pmc_c5_stall -o run -- $B
run pmc_c5_issue rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS $P -d gpurun_out/pmc_c5_issue -o run -- $B
exit 0
