#!/bin/bash
# round 5 (b): A/B of the degree-specialised (unrolled) Cartesian Zernike Horner schemes
# against the start-of-round build: config 5 step + adjoint launch, then config 3 trace
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
AB_ARGS="--config 5 --steps 100 --warmup 10" bash tools/ab.sh base.so zunroll.so || exit $?
