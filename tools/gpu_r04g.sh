#!/bin/bash
# round 4 (g): per-surface patch kernel -- GPU tests, config 5 line + kernel stats + PMC
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --config 5 --no-cpu --steps 200 --warmup 5 > gpurun_out/c5_graph.log 2>&1 || exit $?
tail -1 gpurun_out/c5_graph.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_c5g
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5g -o run -- python3 bench.py --config 5 --no-cpu --steps 50 --warmup 5 > gpurun_out/prof_c5g.log 2>&1 || exit $?
head -6 gpurun_out/prof_c5g/run_kernel_stats.csv | cut -c1-160
rm -rf gpurun_out/pmc_c5_*
bash tools/pmc_c5.sh || exit $?
