#!/bin/bash
# round 4 (h): what the Zernike coefficient adjoint costs (timing variant)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
rm -f gpurun_out/ab.log
AB_ARGS="--config 5 --steps 100 --warmup 3" bash tools/ab.sh adj_w3.so adj_nocoef.so || exit $?
