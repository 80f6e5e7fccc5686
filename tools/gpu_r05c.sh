#!/bin/bash
# round 5 (c): the monomial-basis coefficient adjoint -- its GPU parity tests (adjoint vs
# forward mode, autograd goldens, config 5's 1M-ray gradient, the captured step), then an
# A/B of config 5 against the unrolled-Horner build (zunroll) at 3 and 4 waves per SIMD
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_adjoint.py tests/test_gpu_autograd.py tests/test_gpu_graph_step.py "tests/test_gpu_config_sizes.py" > gpurun_out/pytest_c.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_c.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--config 5 --steps 100 --warmup 10" bash tools/ab.sh zunroll.so mono3.so mono4.so || exit $?
