#!/bin/bash
# round 4 (s): occupancy A/B after the non-temporal stores and block partials -- taped
# forward at 5 waves, adjoint at 4 waves, against the build's choice (config 5)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
AB_ARGS="--config 5 --steps 100 --warmup 3" bash tools/ab.sh base.so tape5.so adj4.so || exit $?
