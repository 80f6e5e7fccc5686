#!/bin/bash
# round 5 (d): config 5 A/B of the monomial-basis adjoint at 3 / 4 waves per SIMD, then
# PC sampling (rocprofv3 host-trap) of configs 5 and 3
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
AB_ARGS="--config 5 --steps 100 --warmup 10" bash tools/ab.sh mono3.so mono4.so || exit $?
bash tools/pcsamp.sh 5 || exit $?
bash tools/pcsamp.sh 3 || exit $?
