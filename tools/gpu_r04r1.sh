#!/bin/bash
# round 4 (r1): final build -- GPU tests, then the bench lines of configs 1-5 and their
# rocprofv3 kernel statistics (tools/bench_configs.sh prof)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/bench_configs.sh prof
