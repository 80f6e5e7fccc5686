#!/bin/bash
# round 4 (q): ort_rms_spot with 1024 chunks for its one pair -- GPU tests, A/B of the
# chunk count on config 5
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/ab.log
AB_ARGS="--config 5 --steps 100 --warmup 3" bash tools/ab.sh rms256.so rms1024.so || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 3 > gpurun_out/prof_c5.log 2>&1 || exit $?
tail -1 gpurun_out/prof_c5.log | cut -c1-200
