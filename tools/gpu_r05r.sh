#!/bin/bash
# round 5 (r): the rms finish as the second workgroup of ort_newton_finish_rms (13 launches
# per config-5 step): GPU suite, config 5 bench line and kernel trace
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_r.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --config 5 --steps 100 --warmup 5 > gpurun_out/bench_c5r.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5r -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5r.log 2>&1
