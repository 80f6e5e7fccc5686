#!/bin/bash
# round-4 first GPU pass: parity tests, smoke, default bench, config 5 bench + kernel stats
set -u
cd "$(dirname "$0")/.."
bash tools/gpu_session.sh testsall smoke bench || exit $?
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --config 5 --steps 100 --warmup 5 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -2 gpurun_out/bench_c5.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --no-cpu --steps 20 --warmup 2 > gpurun_out/prof_c5.log 2>&1
echo "prof rc=$?"
