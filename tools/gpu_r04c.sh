#!/bin/bash
# round 4 (c): GPU tests on the 3-wave unparked adjoint; config 5 line + kernel stats;
# config 5 adjoint PMC (HBM bytes, VALU); config 3 Newton variants under the VALU counters
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --config 5 --no-cpu --steps 200 --warmup 5 > gpurun_out/c5_graph.log 2>&1 || exit $?
tail -1 gpurun_out/c5_graph.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 5 > gpurun_out/prof_c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --config 3 --no-cpu --steps 10 --warmup 2 > gpurun_out/prof_c3.log 2>&1 || exit $?
bash tools/pmc_c5.sh || exit $?
for v in tr_nofast tr_fast tr_fast_w6; do
  ORT_LIB_PATH=optiland_pr_amd/lib/variants/$v.so timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmc_c3v_$v -o run -- python3 bench.py --no-cpu --config 3 --steps 2 --warmup 1 > gpurun_out/pmc_c3v_$v.log 2>&1 || exit $?
  echo "$v done"
done
AB_ARGS="--config 5 --eager --steps 30 --warmup 3" bash tools/ab.sh adj_z0.so adj_z16.so || exit $?
