#!/bin/bash
# round 5 (h): the fused Adam + patch (optim.ZernikeAdam): its GPU tests, then config 5 with
# it (default) and with torch's fused Adam (--torch-adam), kernel stats of the default
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_graph_step.py tests/test_gpu_autograd.py > gpurun_out/pytest_h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_h.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--config 5 --steps 100 --warmup 10" bash tools/ab.sh adam.so || exit $?
AB_ARGS="--config 5 --steps 100 --warmup 10 --torch-adam" bash tools/ab.sh adam.so || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5h -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5h.log 2>&1
