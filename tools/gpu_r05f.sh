#!/bin/bash
# round 5 (f): two-launch parameter reduction; taped-forward occupancy A/B (5 waves =
# main, 4 waves without scratch, 6 waves); config 5 kernel stats of the main build
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_adjoint.py tests/test_gpu_autograd.py tests/test_gpu_graph_step.py tests/test_gpu_config_sizes.py > gpurun_out/pytest_f.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_f.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--config 5 --steps 100 --warmup 10" bash tools/ab.sh main.so fwd4.so fwd6.so || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5f -o run -- python3 bench.py --config 5 --no-cpu --steps 100 --warmup 5 > gpurun_out/prof_c5f.log 2>&1
