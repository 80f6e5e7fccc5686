#!/bin/bash
# round 4 (i): Newton iterates taped straight from the loop -- GPU tests, config 5 line;
# the coefficient adjoint's cost (timing variant)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --config 5 --no-cpu --steps 200 --warmup 5 > gpurun_out/c5_graph.log 2>&1 || exit $?
tail -1 gpurun_out/c5_graph.log | cut -c1-300
rm -f gpurun_out/ab.log
AB_ARGS="--config 5 --steps 100 --warmup 3" bash tools/ab.sh adj_w3.so adj_ms.so adj_nocoef.so || exit $?
