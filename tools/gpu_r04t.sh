#!/bin/bash
# round 4 (t): final build with the taped forward at 5 waves -- GPU tests, smoke, the
# default bench line and the config 5 line
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-250
timeout -k 10 300 python3 bench.py --config 5 --steps 100 --warmup 5 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | cut -c1-250
