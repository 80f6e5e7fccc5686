#!/bin/bash
# round 5 (w): config 5 bench line, kernel trace and PMC passes on the hybrid-slope build
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 400 python3 bench.py --config 5 --steps 100 --warmup 5 > gpurun_out/bench_c5.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5w -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5w.log 2>&1 || exit $?
bash tools/pmc_c5.sh || exit $?
echo W_OK
