#!/bin/bash
# round 4: GPU tests, config 5 graph vs eager, adjoint A/B (config 5), Newton fast pass A/B (config 3)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/c5_graph.log 2>&1 || exit $?
tail -1 gpurun_out/c5_graph.log | cut -c1-700
timeout -k 10 300 python3 bench.py --config 5 --no-cpu --eager --steps 100 --warmup 5 > gpurun_out/c5_eager.log 2>&1 || exit $?
tail -1 gpurun_out/c5_eager.log | cut -c1-300
AB_ARGS="--config 5 --steps 30 --warmup 3" bash tools/ab.sh adj_w4park.so adj_w4np.so adj_w3np.so adj_w2np.so || exit $?
AB_ARGS="--config 3 --steps 10 --warmup 2" bash tools/ab.sh tr_nofast.so tr_fast.so tr_fast_w6.so
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 5 > gpurun_out/prof_c5.log 2>&1 || exit $?
