#!/bin/bash
# round 4 (d): GPU tests (adjoint with LDS Zernike accumulators), the fast-pass probe,
# config 5 line, adjoint PMC passes
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
ORT_LIB_PATH=optiland_pr_amd/lib/variants/tr_probe.so timeout -k 10 300 python3 tools/fast_probe.py > gpurun_out/fast_probe.log 2>&1 || exit $?
cat gpurun_out/fast_probe.log
timeout -k 10 300 python3 bench.py --config 5 --no-cpu --steps 200 --warmup 5 > gpurun_out/c5_graph.log 2>&1 || exit $?
tail -1 gpurun_out/c5_graph.log | cut -c1-300
bash tools/pmc_c5.sh || exit $?
