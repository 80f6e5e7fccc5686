#!/bin/bash
# round 5 (j): verify rounds on a kVerifyGrid grid (F_STRIDE), 1024-thread rms finish,
# no per-step fill in ZernikeAdam: the whole GPU suite, config 5 bench, kernel stats
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_device_verify.py tests/test_gpu_autograd.py > gpurun_out/pytest_j1.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_j1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_j.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_j.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu --config 5 --steps 200 --warmup 10 > gpurun_out/c5_j$rep.json 2> gpurun_out/c5_j$rep.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5j -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5j.log 2>&1
