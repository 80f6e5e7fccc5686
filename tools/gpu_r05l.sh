#!/bin/bash
# round 5 (l): slope-form Newton updates (+ prefetching verify rounds, parallel finish):
# GPU suite, config 3 and config 5 benches, kernel stats of both
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --config 3 --steps 10 --warmup 2 > gpurun_out/c3_l$rep.json 2> gpurun_out/c3_l$rep.err || exit $?
  timeout -k 10 300 python3 bench.py --no-cpu --config 5 --steps 200 --warmup 10 > gpurun_out/c5_l$rep.json 2> gpurun_out/c5_l$rep.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5l -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5l.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3l -o run -- python3 bench.py --config 3 --no-cpu --steps 10 --warmup 2 > gpurun_out/prof_c3l.log 2>&1
