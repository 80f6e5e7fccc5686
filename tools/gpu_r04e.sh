#!/bin/bash
# round 4 (e): GPU tests, every config's bench line (CPU baselines included) with rocprofv3
# kernel stats, and the config 3 kernel's compute counters
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
bash tools/bench_configs.sh prof || exit $?
bash tools/pmc_c3.sh || exit $?
