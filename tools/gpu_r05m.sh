#!/bin/bash
# round 5 (m): slope-form Newton updates with compile-time evaluation modes: parity tests,
# config 3 / config 5 benches, kernel stats
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_config_sizes.py tests/test_gpu_autograd.py tests/test_gpu_device_verify.py > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_m.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --config 3 --steps 10 --warmup 2 > gpurun_out/c3_m$rep.json 2> gpurun_out/c3_m$rep.err || exit $?
  timeout -k 10 300 python3 bench.py --no-cpu --config 5 --steps 200 --warmup 10 > gpurun_out/c5_m$rep.json 2> gpurun_out/c5_m$rep.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5m -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5m.log 2>&1
