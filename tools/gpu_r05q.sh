#!/bin/bash
# round 5 (q): the 5-wave config-3 build -- GPU suite, config 3 and 5 bench lines, the
# config-3 HBM passes (the spill writes gone?) and its compute counters
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config 3 --steps 10 --warmup 2 > gpurun_out/bench_c3.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --config 5 --steps 100 --warmup 5 > gpurun_out/bench_c5.log 2>&1 || exit $?
bash tools/pmc_c3.sh || exit $?
bash tools/pmc_configs.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --config 3 --no-cpu --steps 5 --warmup 1 > gpurun_out/prof_c3.log 2>&1
