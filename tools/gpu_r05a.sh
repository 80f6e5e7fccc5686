#!/bin/bash
# round 5 (a): config 5 counters of the current build (adjoint + taped forward: HBM bytes,
# VALU / SALU / LDS, stalls), then an A/B of the adjoint without its coefficient pass
# (timing only: how much of the launch the Zernike coefficient adjoint costs)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
bash tools/pmc_c5.sh || exit $?
AB_ARGS="--config 5 --steps 100 --warmup 10" bash tools/ab.sh base.so nocoef.so
