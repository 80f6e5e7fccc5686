#!/bin/bash
# round 5 (k): verify-round schedule prefetch, parallel newton_finish, rms finish beside
# the finish launch (side stream): GPU suite, config 5 bench x2, kernel trace
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_k.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --config 5 --steps 200 --warmup 10 > gpurun_out/c5_k$rep.json 2> gpurun_out/c5_k$rep.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5k -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5k.log 2>&1
