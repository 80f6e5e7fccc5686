#!/bin/bash
# round 5 (v): Zernike slopes from the Cartesian gradient off the axis disc (hyb, this
# build) vs the reference's eps-guarded polar chain everywhere (chain): GPU suite on this
# build, then config 5 A/B
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_v.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_v.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--config 5 --steps 200 --warmup 10" bash tools/ab.sh hyb.so chain.so || exit $?
