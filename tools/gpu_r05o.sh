#!/bin/bash
# round 5 (o): A/B prev (95725da, slope-form updates) vs conic (+ one-reciprocal conic
# terms, host RN(1/R^2)): parity tests on the new build, then config 3 and config 5
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_config_sizes.py tests/test_gpu_autograd.py tests/test_gpu_device_verify.py tests/test_gpu_adjoint.py > gpurun_out/pytest_o.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_o.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--config 3 --steps 10 --warmup 2" bash tools/ab.sh prev.so conic.so || exit $?
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab.sh prev.so conic.so vg256.so || exit $?
