#!/bin/bash
# round 4 (k): ort_newton_finish / pointer patch / static backward seed -- GPU tests,
# smoke, the default bench line, config 5 line and its rocprofv3 kernel statistics
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 300 python3 bench.py --config 5 --steps 100 --warmup 5 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 3 > gpurun_out/prof_c5.log 2>&1 || exit $?
tail -1 gpurun_out/prof_c5.log | cut -c1-200
