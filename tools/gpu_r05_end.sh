#!/bin/bash
# round 5 end (1 of 2): the GPU suite, smoke(), bench lines of configs 1-5 with their
# kernel stats (tools/gpu_r05_pmc.sh: the PMC passes). Output under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_end.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_end.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_end.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_end.log; [ $rc -eq 0 ] || exit $rc
bash tools/bench_configs.sh prof || exit $?
echo END_OK
